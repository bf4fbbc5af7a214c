// Encoder internals shared by encoder.hip (scoring) and encoder_train.hip (training forward/backward).
#pragma once
#include <vector>

#include "common.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace tmk {

constexpr int HID = 64;   // hid_dim supported by this build (reference default --hid_dim 64)
constexpr int TILE_ROWS = 32;

__host__ __device__ constexpr int r16(int x) { return (x + 15) & ~15; }

struct Lin {
    const float4 *w;  // packed [nt][nq][64 lanes] float4
    const float *b;   // [nt*16] zero padded
    int nt, nq, nout, k;
};

struct EncW {
    int de, dn, kev, kdep;
    Lin ev, g1, g2, w1, w2, a1, a2, m1, m2, d1, d2;
    const float *m3w, *m3b, *d3w, *d3b, *freq, *phase;
    // lin_event bias plus the K steps q >= qt (all time features) at dt = 0: walk position 2 is
    // relative to itself, so those steps are the constant cos(phase) (walk_kernel's slot pass)
    const float *evc;
    int qt;
    // lin_event's folded time steps alone (evc - bias, fp64 sum rounded once): the table-mode slot pass,
    // whose edge-table row already carries the bias
    const float *devc;
    // fused walk kernel (eval, hid_dim 64): layers folded at pack time in fp64 (tm_weights_pack).  With
    // H = event_gcn's relu'd hidden layer of both branches, F = blockdiag(g2, g2) H + [bg2; bg2];
    // W1D = W1 blockdiag(g2,g2), b1d = W1 [bg2;bg2] + b1 (so Wp = W1 F_2 + b1 = W1D H_2 + b1d),
    // G = W2 blockdiag(g2,g2), beta = W2 [bg2;bg2] + b2 (Q_i = W2 F_i + b2 = G H_i + beta).  The score
    // Wp . Q_i = V . H_i + cw with V = G^T Wp = kv H_2 + v0 (kv = G^T W1D, v0 = G^T b1d) and
    // cw = Wp . beta = u . H_2 + c0 (u = W1D^T beta, c0 = b1d . beta); attention.MLP.0 of the
    // attention output = P2 + alpha_0 R_0 + alpha_1 R_1 with P2 = A1D H_2 + cp, R_i = A1G H_i
    // (A1D = a1 blockdiag(g2,g2), A1G = a1 G, cp = a1 [bg2;bg2] + a1 beta + ba1; alpha_0 + alpha_1 = 1);
    // M1A2 = MLP.0[:, :h] a2, tc[c] = MLP.0[:, h + c] + bm1 + MLP.0[:, :h] ba2 (row 12: no category).
    Lin kv, a1d, a1g, m1a2;
    const float *v0, *u, *c0, *cp, *tc;
    // zero node features (tm_weights_set_node_zero; FoldLay KVZ ...): the same layers on U = H[:64] = H[64:]
    Lin kvz, a1dz, a1gz;
    const float *v0z, *uz;
    // constructor variants (explainer_new.py:103-105, :121, :141): tg = use_temporal_guidance (0: the plain
    // Attention, no time weighting of the scores), dep = use_dependency_aware_sampling (0: no gate)
    int tg = 1, dep = 1;
    // hid_dim and the final MLP's width (hm = h + 12 with the one-hot category feature, h without:
    // if_cat_feature, explainer_new.py:121-125); the fused walk kernel covers h = 64 with the category
    int h = 64, hm = 76, cat = 1;
};

// ------------------------------------------------------------------ MFMA tile GEMM
// out[16mt.., 16nt..] = X[16*MT rows][ldx] (LDS) * W^T (packed, streamed from L2).
// Each wave owns column tiles nt = wave, wave + nw, ... and sweeps all MT row tiles for
// them, two column tiles at a time: per 16-deep K step it loads 2 weight fragments (the
// next step's are prefetched into registers) and MT activation fragments (ds_read_b128)
// and issues 8*MT MFMAs.  The epilogue gets (mt, nt, acc) with acc[r] = D[4*(lane>>4)+r][lane&15].
template <int MT, class Epi>
__device__ __forceinline__ void gemm(const float *X, int ldx, const Lin &L, Epi epi) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int arow = lane & 15, akoff = 4 * (lane >> 4);
    const int nq = L.nq;
    for (int nt0 = wave; nt0 < L.nt; nt0 += 2 * nw) {
        const int nt1 = nt0 + nw;
        const bool has1 = nt1 < L.nt;
        floatx4 acc0[MT], acc1[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            acc0[m] = floatx4{0.f, 0.f, 0.f, 0.f};
            acc1[m] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        const float4 *wb0 = L.w + (size_t)nt0 * nq * 64 + lane;
        const float4 *wb1 = L.w + (size_t)(has1 ? nt1 : nt0) * nq * 64 + lane;
        const float *xa = X + arow * ldx + akoff;
        float4 b0 = wb0[0], b1 = wb1[0];
        for (int q = 0; q < nq; ++q) {
            float4 n0 = b0, n1 = b1;
            if (q + 1 < nq) {
                n0 = wb0[(q + 1) * 64];
                n1 = wb1[(q + 1) * 64];
            }
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const float4 a = *reinterpret_cast<const float4 *>(xa + m * 16 * ldx + 16 * q);
                acc0[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b0.x, acc0[m], 0, 0, 0);
                acc1[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b1.x, acc1[m], 0, 0, 0);
                acc0[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b0.y, acc0[m], 0, 0, 0);
                acc1[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b1.y, acc1[m], 0, 0, 0);
                acc0[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b0.z, acc0[m], 0, 0, 0);
                acc1[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b1.z, acc1[m], 0, 0, 0);
                acc0[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b0.w, acc0[m], 0, 0, 0);
                acc1[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b1.w, acc1[m], 0, 0, 0);
            }
            b0 = n0;
            b1 = n1;
        }
#pragma unroll
        for (int m = 0; m < MT; ++m) epi(m, nt0, acc0[m]);
        if (has1) {
#pragma unroll
            for (int m = 0; m < MT; ++m) epi(m, nt1, acc1[m]);
        }
    }
}

__device__ __forceinline__ int erow(int mt, int r) { return mt * 16 + 4 * ((threadIdx.x & 63) >> 4) + r; }
__device__ __forceinline__ int ecol(int nt) { return nt * 16 + (threadIdx.x & 15); }

// cos(t * w + phi) with the multiply and add rounded separately, as torch does
// (TimeEncode.forward, explainer_new.py:56-58); never contracted into an fma.
__device__ __forceinline__ float time_cos(float t, float w, float phi) { return cos_rd(__fadd_rn(__fmul_rn(t, w), phi)); }

__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// The dependency gate's logit d3 . G2 over its h2 = h/2 features in ONE fixed order, shared by the
// LDS-tiled kernels and the register-resident gate_reg_kernel (h2 = 32) so their gates agree bit for bit:
// part k (k = 0..3) is an fma chain over features 16t + 4k + r (t < h2/16 rounded up, r = 0..3) and
// z = (part0 + part1) + (part2 + part3).
__device__ __forceinline__ float gate_part(const float *g2, const float *w3, int k, int h2 = 32) {
    float p = 0.f;
    for (int t = 0; 16 * t < h2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) p = __builtin_fmaf(g2[16 * t + 4 * k + r], w3[16 * t + 4 * k + r], p);
    return p;
}
// LDS form: 8 lanes per row (sub = lane & 7), the row's relu'd G2 at g2 (zero padded to a multiple of 16;
// w3 likewise); the result in every lane
__device__ __forceinline__ float gate_logit_lds(const float *g2, const float *w3, int sub, int h2 = 32) {
    float v = sub < 4 ? gate_part(g2, w3, sub, h2) : 0.f;
    v += __shfl_xor(v, 1, 8);
    v += __shfl_xor(v, 2, 8);
    return v;
}

// Folded region at the start of tm_weights::buf (float offsets; hid_dim 64): the fused walk kernel's
// packs and vectors (EncW::w1d ...), then the reference layers in tm_weights_create's order.
struct FoldLay {
    static constexpr int KV = 0, V0 = KV + 8 * 8 * 256, U = V0 + 128, C0 = U + 128, A1D = C0 + 4, CP = A1D + 4 * 8 * 256,
                         A1G = CP + 64, M1A2 = A1G + 4 * 8 * 256, TC = M1A2 + 5 * 4 * 256,
                         // the zero-node-feature forms (H_s = H_t = U, so H = [U; U] and every layer reading H
                         // takes the sum of its two column halves; kv and v0 also sum their two row halves, the
                         // score V . H_i becoming VZ . U_i with VZ = V[:64] + V[64:])
                         KVZ = (TC + 13 * 80 + 63) & ~63, A1DZ = KVZ + 4 * 4 * 256, A1GZ = A1DZ + 4 * 4 * 256,
                         V0Z = A1GZ + 4 * 4 * 256, UZ = V0Z + 64, SIZE = (UZ + 64 + 63) & ~63;
    // fold32 scratch (row-major fp32 matrices before packing)
    static constexpr int S_KV = 0, S_A1D = S_KV + 128 * 128, S_A1G = S_A1D + 64 * 128, S_M1A2 = S_A1G + 64 * 128,
                         S_KVZ = S_M1A2 + 76 * 64, S_A1DZ = S_KVZ + 64 * 64, S_A1GZ = S_A1DZ + 64 * 64,
                         S_SIZE = S_A1GZ + 64 * 64;
    // fold64 scratch (stage 1): a1 W2, a1 b2, W1D = W1 blockdiag(g2,g2), G = W2 blockdiag(g2,g2), b1d, beta
    static constexpr int S64_A1W2 = 0, S64_A1B2 = S64_A1W2 + 64 * 128, S64_W1D = S64_A1B2 + 64,
                         S64_G = S64_W1D + 128 * 128, S64_B1D = S64_G + 128 * 128, S64_BETA = S64_B1D + 128,
                         S64_SIZE = S64_BETA + 128;
};

// Transposed weight packs for the backward's data-gradient GEMMs (dX = dY W = dY (W^T)^T), same
// fragment format as the forward packs; no biases.  evT holds only lin_event's time-feature columns.
struct EncWT {
    Lin evT, g1T, g2T, w1T, w2T, a1T, a2T, m1T, m2T;
    Lin d1T, d2T;   // dependency gate: d1T holds only the time-feature columns of edge_dependency_gcn.0
};

// Dropout keep-masks of the training forward, uint8 [n_walks][drop_cols(h, hm)]: attention weights alpha
// (TemporalAwareAttention.dropout, explainer_new.py:839) in columns 0..1, the attention MLP's hidden layer
// (:780) in the h columns from DROP_H and the final MLP's hidden layer (:122) in the hm columns from
// DROP_H + h; 1 = kept (scaled by 1/(1-p)), 0 = dropped.  Rows padded to 16 columns (144 for the default
// hid_dim 64 with the category feature).  The plain Attention (use_temporal_guidance=False, :12-43) has
// neither of the first two dropouts: their columns are ignored then.
constexpr int DROP_A = 0, DROP_H = 2;
__host__ __device__ constexpr int drop_cols(int h, int hm) { return r16(DROP_H + h + hm); }
static_assert(drop_cols(HID, HID + 12) == 144, "dropout mask columns");

// ------------------------------------------------------------------ register-resident MFMA chains (shared by the
// fused walk kernel and the register-resident training kernels)
// out[t] = W tile t * x  over the flattened (t, q) sequence, weights prefetched PF steps ahead in
// a rotating register buffer; sched_barrier pins each step so the loads stay PF steps ahead instead
// of being hoisted (which would need NTO*NQ registers).
constexpr int PF = 3;

// The lane index laundered through an opaque asm: loads addressed with it cannot be hoisted out of
// the pass loop by LICM (hoisting every loop-invariant weight/bias load costs ~300 registers).
__device__ __forceinline__ int lane_id() {
    int l = threadIdx.x & 63;
    asm volatile("" : "+v"(l));
    return l;
}

// Weight fragments are read with buffer loads: the fragment's byte offset is a compile-time SGPR
// operand (s_mov, scalar pipe) instead of a 64-bit VGPR address add per fragment.  The lane offset
// goes through lane_id() so the loads stay inside the pass loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wrsrc(const float4 *w) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float4 *>(w), (short)0, 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ float4 wload(__amdgpu_buffer_rsrc_t r, int vo, int f4) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, f4 * 16, 0));
}

template <int NTO, int NQ>
struct PairOrder {   // fragment i of the pair order -> (tile, K step)
    static constexpr int NP = NTO / 2, NPF = 2 * NP * NQ;
    static constexpr int t(int i) { return i < NPF ? 2 * (i / (2 * NQ)) + (i & 1) : NTO - 1; }
    static constexpr int q(int i) { return i < NPF ? (i % (2 * NQ)) / 2 : i - NPF; }
};

// NQL = the pack's K steps (L.nq); NQ <= NQL of them are multiplied (the leading ones).  Tile pairs (t, t+1)
// with their K steps inside and the two tiles' MFMAs interleaved (no MFMA waits on the accumulator of the one
// before it: 32-cycle issue, 40-cycle dependent latency); an odd last tile alone.  Every tile accumulates its
// K steps in the same order as a tile-by-tile loop (same results).
template <int NTO, int NQ, int NQL = NQ>
__device__ __forceinline__ void rgemm(const Lin &L, const floatx4 (&x)[NQ], floatx4 (&o)[NTO]) {
    using O = PairOrder<NTO, NQ>;
    const auto wr = wrsrc(L.w);
    const int vo = lane_id() * 16;
    constexpr int N = NTO * NQ, D = PF < N ? PF : N;
    auto off = [](int i) { return (O::t(i) * NQL + O::q(i)) * 64; };
#pragma unroll
    for (int t = 0; t < NTO; ++t) o[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    float4 buf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) buf[i] = wload(wr, vo, off(i));
#pragma unroll
    for (int k = 0; k < O::NP * NQ; ++k) {
        const int i = 2 * k, t = O::t(i), q = O::q(i);
        const float4 w0 = buf[i % D];
        if (i + D < N) buf[i % D] = wload(wr, vo, off(i + D));
        const float4 w1 = buf[(i + 1) % D];
        if (i + 1 + D < N) buf[(i + 1) % D] = wload(wr, vo, off(i + 1 + D));
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.x, x[q].x, o[t], 0, 0, 0);
        o[t + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.x, x[q].x, o[t + 1], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.y, x[q].y, o[t], 0, 0, 0);
        o[t + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.y, x[q].y, o[t + 1], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.z, x[q].z, o[t], 0, 0, 0);
        o[t + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.z, x[q].z, o[t + 1], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.w, x[q].w, o[t], 0, 0, 0);
        o[t + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.w, x[q].w, o[t + 1], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (NTO % 2) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = O::NPF + q;
            const float4 w = buf[i % D];
            if (i + D < N) buf[i % D] = wload(wr, vo, off(i + D));
            o[NTO - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, x[q].x, o[NTO - 1], 0, 0, 0);
            o[NTO - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, x[q].y, o[NTO - 1], 0, 0, 0);
            o[NTO - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, x[q].z, o[NTO - 1], 0, 0, 0);
            o[NTO - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, x[q].w, o[NTO - 1], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// the register-resident event_gcn forward of the training step (encoder_train.hip) for these dims: launched
// on s (true), or no instance (false: the caller runs gcn_kernel)
bool launch_gcn_fwd_reg(const EncW &P, int node_zero, int64_t n_rows, const float *n_feat, const float *e_feat, const int32_t *node6,
                        const int32_t *eid3, const float *ts3, const float *cnt, float *F, hipStream_t s);

}  // namespace tmk

using tmk::Lin;
using tmk::EncW;

struct tm_weights {
    int device;
    int de, dn, h;
    float *buf;
    size_t n_floats;
    EncW P;
    // the caller's node-feature table is all zeros (tm_weights_set_node_zero): the fused eval kernel computes
    // one event_gcn branch, the other being bit-identical
    int node_zero = 0;
    // a process-wide stamp (tm_weights_bump: every create / repack / variant / node-zero change takes the next
    // value of one global counter): caches of values computed from the weights (the drop-in's gate factors per
    // edge id, the pipeline's per-edge-id tables) key on it, and no two weight states -- of this object or of
    // another one later allocated at the same address -- ever share a stamp
    uint64_t version = 0;
    // per linear: raw tensor index, nout, k
    struct Spec {
        Lin *lin;
        int wi, nout, k;
    };
    std::vector<Spec> specs;
    std::vector<std::pair<int, float **>> vecs;
    // training: transposed packs (encoder_train.hip)
    tmk::EncWT T;
    float *tbuf = nullptr;
    size_t t_floats = 0;
    // fold scratch (tm_weights_pack): fp64 a1 W2 [h][2h] and fp32 row-major folded matrices before packing
    double *fold64 = nullptr;
    float *fold32 = nullptr;
};

void tm_weights_bump(tm_weights *w);   // encoder.hip: w->version = the next process-wide stamp

// encoder_train.hip: transposed packs (tm_weights_create / _free) and the one-launch packing of every tensor
int train_packs_create(tm_weights *w);
void pack_all_weights(tm_weights *w, const float *const *t, hipStream_t s);   // every pack, one launch (+ evc)
void train_packs_free(tm_weights *w);

static inline hipStream_t S_(void *s) { return (hipStream_t)s; }
