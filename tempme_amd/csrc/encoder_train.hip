// TempME motif encoder, training: backward kernels on gfx950.
//
// Reference (dharunm236/TempME): the explainer's training step temp_exp_main.py:605-632 back-propagates
// through TempME.forward (models/explainer_new.py:174-201: event features, event_gcn x2 :79-96,
// TemporalAwareAttention :789-846 with dropout on alpha :839 and in its MLP :780, the category one-hot
// and MLP :122-125 with dropout, sigmoid).  The reference leaves that to autograd; here the forward
// runs gcn_kernel + head_kernel (encoder.hip, dropout keep-masks applied in the head) and the backward
// is two LDS-tiled MFMA kernels that recompute the forward of their tile and run its chain rule:
//
//   head_bwd_kernel  per 32 walks: attention + MLP head forward again (from the stored F rows), then
//                    d imp -> d logit -> MLP -> one-hot split -> attention MLP -> softmax / temporal
//                    scaling -> W1 / W2 -> dF [walk][position][2h]
//   gcn_bwd_kernel   per 32 walk positions: event features, lin_event, both event_gcn branches again,
//                    then dF -> MLP.2 -> ReLU -> MLP.0 -> the two ReLU branches -> d lin_event ->
//                    d time features -> (-sin) for the time encoder's frequency / phase
//
// Every data-gradient GEMM (dX = dY W) runs on MFMA against transposed weight packs (EncWT, packed
// alongside the forward packs).  Each kernel also writes, per layer, the (dY, X) row pairs of its tile;
// wgrad_partial_kernel + wgrad_reduce_kernel then form every weight gradient dW = dY^T X (and bias
// gradient, a column of ones appended to X) over all rows in two launches (tm_encoder_wgrad).
#include <cstdlib>
#include <string>

#include "encoder_common.h"

namespace tmk {

// ------------------------------------------------------------------ weight packing (one launch)
// Every packed tensor of tm_weights -- the forward fragment packs, the transposed packs of the backward
// and the zero-padded bias / vector copies -- is one job of a single launch (the training step repacks
// after every optimizer step).  Fragment job: packed element (o, c) = src[o * so + c * sc] in
// the fragment order the MFMA tiles read (see EncW / gemm); copy job (nt = 0): dst[i] = i < nout ? src[i] : 0 for i < k (k = padded length).
struct PackJob {
    const float *src;
    float *dst;
    int32_t so, sc, nout, k, nt, nq;
    int64_t begin;
};
constexpr int MAX_PACK_JOBS = 56;
struct PackJobs {
    PackJob j[MAX_PACK_JOBS];
    int32_t n;
    int64_t total;
};

__global__ void pack_jobs_kernel(PackJobs J) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < J.total; i += (int64_t)gridDim.x * blockDim.x) {
        int b = 0;
        while (b + 1 < J.n && i >= J.j[b + 1].begin) ++b;
        const PackJob &p = J.j[b];
        const int64_t e = i - p.begin;
        if (p.nt == 0) {
            p.dst[e] = e < p.nout ? p.src[e] : 0.f;
            continue;
        }
        const int s = e & 3, l = (e >> 2) & 63;
        const int64_t tq = e >> 8;
        const int q = (int)(tq % p.nq), t = (int)(tq / p.nq);
        const int o = 16 * t + (l & 15), c = 16 * q + 4 * (l >> 4) + s;
        p.dst[e] = (o < p.nout && c < p.k) ? p.src[(int64_t)o * p.so + (int64_t)c * p.sc] : 0.f;
    }
}

// evc[f] = b[f] + sum_{k >= 16 qt} W[f][k] * cos(0 * w + phi): one wave per output feature, fp64
// partial sums combined in a fixed butterfly order, one rounding to fp32 (walk_kernel's slot pass);
// devc[f] = the same sum without the bias (the table-mode slot pass: the edge-table row carries the bias)
__global__ void __launch_bounds__(64) evc_par_kernel(const float *__restrict__ W, const float *__restrict__ b,
                                                     const float *__restrict__ phase, int de, int dn, int kev, int qt,
                                                     float *__restrict__ out, float *__restrict__ dout) {
    const int f = blockIdx.x, lane = threadIdx.x;
    double acc = 0.0;
    if (f < dn)
        for (int k = 16 * qt + lane; k < kev; k += 64) acc += (double)W[(int64_t)f * kev + k] * (double)cos_rd(phase[k - de - 3]);
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) {
        out[f] = f < dn ? (float)(acc + (double)b[f]) : 0.f;
        dout[f] = f < dn ? (float)acc : 0.f;
    }
}

// ------------------------------------------------------------------ folded layers of the fused walk kernel
// (EncW::w1d ..., tmk::FoldLay), fp64 products of the reference's fp32 weights rounded once.  Raw tensors
// t[] in tm_weights_pack's order: 4/5 event_conv.MLP.2 (g2), 6/7 attention.W1, 8/9 attention.W2,
// 10/11 attention.MLP.0 (a1), 12/13 attention.MLP.3|2 (a2), 14/15 MLP.0 (m1).  h = 64.
struct FoldIn {
    const float *g2w, *g2b, *w1, *b1, *w2, *b2, *a1, *ba1, *a2, *ba2, *m1, *bm1;
};

// X blockdiag(g2, g2)[o][k] = sum_{j < 64} X[o][64 (k >= 64) + j] g2[j][k % 64];  X [bg2; bg2][o]
template <class Row>
__device__ __forceinline__ double fold_bd(const FoldIn &F, Row row, int k) {
    double acc = 0.0;
    const int base = k >= 64 ? 64 : 0, kk = k % 64;
    for (int j = 0; j < 64; ++j) acc += (double)row(base + j) * (double)F.g2w[j * 64 + kk];
    return acc;
}
template <class Row>
__device__ __forceinline__ double fold_bv(const FoldIn &F, Row row) {
    double acc = 0.0;
    for (int j = 0; j < 128; ++j) acc += (double)row(j) * (double)F.g2b[j % 64];
    return acc;
}

// stage 1 (fp64 scratch): a1 W2 [64][128], a1 b2 [64], W1D [128][128], G [128][128], b1d [128], beta [128]
constexpr int FOLD1_N = 64 * 128 + 64 + 2 * 128 * 128 + 2 * 128;
__global__ void __launch_bounds__(256) fold1_kernel(FoldIn F, double *__restrict__ s64) {
    using L = FoldLay;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 64 * 128) {
        const int o = i / 128, k = i % 128;
        double acc = 0.0;
        for (int j = 0; j < 128; ++j) acc += (double)F.a1[o * 128 + j] * (double)F.w2[j * 128 + k];
        s64[L::S64_A1W2 + i] = acc;
        return;
    }
    i -= 64 * 128;
    if (i < 64) {
        double acc = 0.0;
        for (int j = 0; j < 128; ++j) acc += (double)F.a1[i * 128 + j] * (double)F.b2[j];
        s64[L::S64_A1B2 + i] = acc;
        return;
    }
    i -= 64;
    if (i < 128 * 128) {
        const int o = i / 128, k = i % 128;
        s64[L::S64_W1D + i] = fold_bd(F, [&](int j) { return F.w1[o * 128 + j]; }, k);
        return;
    }
    i -= 128 * 128;
    if (i < 128 * 128) {
        const int o = i / 128, k = i % 128;
        s64[L::S64_G + i] = fold_bd(F, [&](int j) { return F.w2[o * 128 + j]; }, k);
        return;
    }
    i -= 128 * 128;
    if (i < 128) {
        s64[L::S64_B1D + i] = fold_bv(F, [&](int j) { return F.w1[i * 128 + j]; }) + (double)F.b1[i];
        return;
    }
    i -= 128;
    if (i < 128) s64[L::S64_BETA + i] = fold_bv(F, [&](int j) { return F.w2[i * 128 + j]; }) + (double)F.b2[i];
}

// stage 2: the packed matrices (fp32 row-major into s32, packed afterwards) and the vectors (into buf)
constexpr int FOLD2_N = 128 * 128 + 2 * 64 * 128 + 76 * 64 + 128 + 128 + 1 + 64 + 13 * 80 + 3 * 64 * 64 + 64 + 64;
__global__ void __launch_bounds__(256) fold2_kernel(FoldIn F, const double *__restrict__ s64, float *__restrict__ s32,
                                                    float *__restrict__ buf) {
    using L = FoldLay;
    const double *W1D = s64 + L::S64_W1D, *G = s64 + L::S64_G, *b1d = s64 + L::S64_B1D, *beta = s64 + L::S64_BETA;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 128 * 128) {                                 // kv = G^T W1D
        const int o = i / 128, k = i % 128;
        double acc = 0.0;
        for (int j = 0; j < 128; ++j) acc += G[j * 128 + o] * W1D[j * 128 + k];
        s32[L::S_KV + i] = (float)acc;
        return;
    }
    i -= 128 * 128;
    if (i < 64 * 128) {                                  // A1D = a1 blockdiag(g2, g2)
        const int o = i / 128, k = i % 128;
        s32[L::S_A1D + i] = (float)fold_bd(F, [&](int j) { return F.a1[o * 128 + j]; }, k);
        return;
    }
    i -= 64 * 128;
    if (i < 64 * 128) {                                  // A1G = (a1 W2) blockdiag(g2, g2)
        const int o = i / 128, k = i % 128;
        s32[L::S_A1G + i] = (float)fold_bd(F, [&](int j) { return s64[L::S64_A1W2 + o * 128 + j]; }, k);
        return;
    }
    i -= 64 * 128;
    if (i < 76 * 64) {                                   // M1A2 = m1[:, :64] a2 [76][64]
        const int o = i / 64, k = i % 64;
        double acc = 0.0;
        for (int j = 0; j < 64; ++j) acc += (double)F.m1[o * 76 + j] * (double)F.a2[j * 64 + k];
        s32[L::S_M1A2 + i] = (float)acc;
        return;
    }
    i -= 76 * 64;
    if (i < 128) {                                       // v0 = G^T b1d
        double acc = 0.0;
        for (int j = 0; j < 128; ++j) acc += G[j * 128 + i] * b1d[j];
        buf[L::V0 + i] = (float)acc;
        return;
    }
    i -= 128;
    if (i < 128) {                                       // u = W1D^T beta
        double acc = 0.0;
        for (int j = 0; j < 128; ++j) acc += W1D[j * 128 + i] * beta[j];
        buf[L::U + i] = (float)acc;
        return;
    }
    i -= 128;
    if (i < 1) {                                         // c0 = b1d . beta
        double acc = 0.0;
        for (int j = 0; j < 128; ++j) acc += b1d[j] * beta[j];
        buf[L::C0] = (float)acc;
        return;
    }
    i -= 1;
    if (i < 64) {                                        // cp = a1 [bg2;bg2] + a1 W2 [bg2;bg2] + a1 b2 + ba1
        const double a = fold_bv(F, [&](int j) { return F.a1[i * 128 + j]; });
        const double g = fold_bv(F, [&](int j) { return s64[L::S64_A1W2 + i * 128 + j]; });
        buf[L::CP + i] = (float)(a + g + s64[L::S64_A1B2 + i] + (double)F.ba1[i]);
        return;
    }
    i -= 64;
    if (i < 13 * 80) {                                   // tc[c][o] = m1[o][64 + c] + bm1[o] + m1[o][:64] ba2
        const int c = i / 80, o = i % 80;
        float v = 0.f;
        if (o < 76) {
            double acc = (double)F.bm1[o];
            for (int j = 0; j < 64; ++j) acc += (double)F.m1[o * 76 + j] * (double)F.ba2[j];
            if (c < 12) acc += (double)F.m1[o * 76 + 64 + c];
            v = (float)acc;
        }
        buf[L::TC + i] = v;
        return;
    }
    i -= 13 * 80;
    // zero-node-feature forms: U = H[:64] = H[64:], so a layer X reading H is X[:, :64] + X[:, 64:] on U;
    // kv and v0 also fold their row halves (the score V . H = (V[:64] + V[64:]) . U).  fp64 sums, one rounding
    if (i < 64 * 64) {                                   // KVZ = (G[:, o] + G[:, o+64])^T (W1D[:, k] + W1D[:, k+64])
        const int o = i / 64, k = i % 64;
        double acc = 0.0;
        for (int j = 0; j < 128; ++j)
            acc += (G[j * 128 + o] + G[j * 128 + o + 64]) * (W1D[j * 128 + k] + W1D[j * 128 + k + 64]);
        s32[L::S_KVZ + i] = (float)acc;
        return;
    }
    i -= 64 * 64;
    if (i < 64 * 64) {                                   // A1DZ = A1D[:, :64] + A1D[:, 64:]
        const int o = i / 64, k = i % 64;
        const auto row = [&](int j) { return F.a1[o * 128 + j]; };
        s32[L::S_A1DZ + i] = (float)(fold_bd(F, row, k) + fold_bd(F, row, k + 64));
        return;
    }
    i -= 64 * 64;
    if (i < 64 * 64) {                                   // A1GZ = A1G[:, :64] + A1G[:, 64:]
        const int o = i / 64, k = i % 64;
        const auto row = [&](int j) { return s64[L::S64_A1W2 + o * 128 + j]; };
        s32[L::S_A1GZ + i] = (float)(fold_bd(F, row, k) + fold_bd(F, row, k + 64));
        return;
    }
    i -= 64 * 64;
    if (i < 64) {                                        // v0z = v0[:64] + v0[64:]
        double acc = 0.0;
        for (int j = 0; j < 128; ++j) acc += (G[j * 128 + i] + G[j * 128 + i + 64]) * b1d[j];
        buf[L::V0Z + i] = (float)acc;
        return;
    }
    i -= 64;
    if (i < 64) {                                        // uz = u[:64] + u[64:]
        double acc = 0.0;
        for (int j = 0; j < 128; ++j) acc += (W1D[j * 128 + i] + W1D[j * 128 + i + 64]) * beta[j];
        buf[L::UZ + i] = (float)acc;
    }
}

// ------------------------------------------------------------------ head backward
// Row strides for hid_dim h and the final MLP's width hm (h + 12 with the category feature, h without);
// KM = r16(hm).  The default constructor: h = 64, KM = 80.
struct HeadBwdOut {
    float *imp;     // [n]          recomputed sigmoid output (nullable)
    float *dlogit;  // [n]          d logit                         (MLP.5: with M2)
    float *M2;      // [n][h]       relu(MLP.3 ...)
    float *dM2;     // [n][h]       d MLP.3 pre-activation          (with M1d)
    float *M1d;     // [n][KM]      dropout(relu(MLP.0 x))
    float *dM1;     // [n][KM]      d MLP.0 pre-activation          (with X)
    float *X;       // [n][KM]      [attention out | one-hot(cat)]  (attention out alone without the category)
    float *dY2;     // [n][h]       d attention.MLP.3 output        (with H1d)
    float *H1d;     // [n][h]       dropout(relu(attention.MLP.0 O))
    float *dH1;     // [n][h]       d attention.MLP.0 pre-activation (with O)
    float *O;       // [n][2h]      src + sum alpha' Wq
    float *dP;      // [n][2h]      d W1(src)                       (with F[:, 2])
    float *dQ;      // [2][n][2h]   d W2(tgt_k)                     (with F[:, k])
    float *dF;      // [n][3][2h]   d [U_s | U_t] per walk position
};

// LDS of head_bwd_kernel<TR> (TR walks per workgroup): Qb [2TR][LD], Wp / Ob [TR][LD], H1 / M2 [TR][LDH],
// Xb / M1 [TR][LDM]
__host__ __device__ constexpr size_t head_bwd_lds_floats(int h, int hm, int TR) {
    return (size_t)TR * (4 * (2 * h + 8) + 2 * (h + 8) + 2 * (r16(hm) + 8));
}

// TR = 16 walks per workgroup (head_bwd_tr; the template also takes 32)
template <int TR>
__global__ void __launch_bounds__(256) head_bwd_kernel(EncW P, EncWT T, int64_t n_walks, int64_t walks_per_group,
                                                       int32_t W, const float *__restrict__ F,
                                                       const float *__restrict__ ts3, const double *__restrict__ cut,
                                                       const int32_t *__restrict__ cat, const float *__restrict__ stdv,
                                                       const uint8_t *__restrict__ drop, float dscale,
                                                       const float *__restrict__ d_imp, HeadBwdOut o) {
    static_assert(TR == 32 || TR == 16, "head_bwd_kernel: 16 or 32 walks per workgroup");
    constexpr int MT1 = TR / 16, MT2 = TR / 8;   // row tiles of TR and 2 TR rows
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int h = P.h, D2 = 2 * h, LD = D2 + 8, LDH = h + 8, KM = r16(P.hm), LDM = KM + 8;
    const int dcols = drop_cols(h, P.hm), DM = DROP_H + h;
    float *Qb = smem;              // [2TR][LD] W2(F0 | F1)            -> dQ
    float *Wp = Qb + 2 * TR * LD;  // [TR][LD]  W1(F2)                 -> dP      (Wp..Ob: F0|F1 staging)
    float *Ob = Wp + TR * LD;      // [TR][LD]  F2 -> O                -> dO
    float *H1 = Ob + TR * LD;      // [TR][LDH] H1d                    -> dH1
    float *Xb = H1 + TR * LDH;     // [TR][LDM] X                      -> dY2
    float *M1 = Xb + TR * LDM;     // [TR][LDM] M1d                    -> dM1
    float *M2 = M1 + TR * LDM;     // [TR][LDH] M2                     -> dM2
    __shared__ float s_mult[64], s_score[64], s_alpha[64], s_alphad[64], s_dsr[64], s_dl[32];
    __shared__ int32_t s_cat[32];
    const int64_t w0 = (int64_t)blockIdx.x * TR;
    const int tid = threadIdx.x;
    const float kscale = drop ? dscale : 1.f;              // d(dropout(relu(z)))/dz where the output is > 0
    const float kscale_h = drop && P.tg ? dscale : 1.f;    // attention.MLP hidden: no Dropout in plain Attention
    auto valid = [&](int w) { return w0 + w < n_walks; };
    auto keep = [&](int w, int col) -> float {
        if (!drop) return 1.f;
        return (valid(w) && drop[(w0 + w) * dcols + col]) ? dscale : 0.f;
    };
    auto keep_att = [&](int w, int col) -> float { return P.tg ? keep(w, col) : 1.f; };

    // ---- forward again: Q = W2 [F0; F1], Wp = W1 F2, scores, softmax, dropout, O
    float *Tb = Wp;
    for (int i = tid; i < 2 * TR * (D2 / 4); i += blockDim.x) {
        const int row = i / (D2 / 4), c4 = i % (D2 / 4), p = row / TR, w = row % TR;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (valid(w)) v = reinterpret_cast<const float4 *>(F + ((w0 + w) * 3 + p) * D2)[c4];
        *reinterpret_cast<float4 *>(Tb + row * LD + 4 * c4) = v;
    }
    if (tid < 2 * TR) {
        const int w = tid >> 1, p = tid & 1;
        float tw = 1.f;   // plain Attention: the scores unscaled
        if (P.tg && valid(w)) {
            const int64_t gw = w0 + w, g = gw / walks_per_group, b = (gw % walks_per_group) / W;
            const float c = (float)cut[g * (walks_per_group / W) + b];
            tw = expf(-fabsf(c - ts3[gw * 3 + p]) / (stdv[g] + 1e-6f));
        }
        s_mult[tid] = P.tg ? __fadd_rn(0.7f, __fmul_rn(0.3f, tw)) : 1.f;   // 1.0 - 0.3 + 0.3 * time_weight (:835-836)
    }
    if (tid < TR) s_cat[tid] = valid(tid) ? cat[w0 + tid] : -1;
    __syncthreads();
    gemm<MT2>(Tb, LD, P.w2, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) Qb[erow(mt, r) * LD + c] = acc[r] + P.w2.b[c];
    });
    __syncthreads();
    for (int i = tid; i < TR * (D2 / 4); i += blockDim.x) {
        const int w = i / (D2 / 4), c4 = i % (D2 / 4);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (valid(w)) v = reinterpret_cast<const float4 *>(F + ((w0 + w) * 3 + 2) * D2)[c4];
        *reinterpret_cast<float4 *>(Ob + w * LD + 4 * c4) = v;
    }
    __syncthreads();
    gemm<MT1>(Ob, LD, P.w1, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) Wp[erow(mt, r) * LD + c] = acc[r] + P.w1.b[c];
    });
    __syncthreads();
    {   // 4 lanes per (walk, position); groups past TR walks sum nothing
        const int pair = tid >> 2, sub = tid & 3, w = pair >> 1, p = pair & 1;
        const int cend = w < TR ? D2 : 0;
        float s = 0.f;
        for (int c = sub; c < cend; c += 4) s += Wp[w * LD + c] * Qb[(p * TR + w) * LD + c];
        s += __shfl_xor(s, 1, 4);
        s += __shfl_xor(s, 2, 4);
        if (sub == 0 && w < TR) s_score[pair] = s * s_mult[pair];
    }
    __syncthreads();
    if (tid < TR) {
        const float s0 = s_score[2 * tid], s1 = s_score[2 * tid + 1], mx = fmaxf(s0, s1);
        const float e0 = expf(s0 - mx), e1 = expf(s1 - mx), sum = e0 + e1;
        const float a0 = e0 / sum, a1 = e1 / sum;
        s_alpha[2 * tid] = a0;
        s_alpha[2 * tid + 1] = a1;
        s_alphad[2 * tid] = a0 * keep_att(tid, DROP_A);
        s_alphad[2 * tid + 1] = a1 * keep_att(tid, DROP_A + 1);
    }
    __syncthreads();
    for (int i = tid; i < TR * D2; i += blockDim.x) {
        const int w = i / D2, c = i % D2;
        const float a = s_alphad[2 * w] * Qb[w * LD + c] + s_alphad[2 * w + 1] * Qb[(TR + w) * LD + c];
        const float v = Ob[w * LD + c] + a;
        Ob[w * LD + c] = v;
        if (valid(w)) o.O[(w0 + w) * D2 + c] = v;
    }
    __syncthreads();
    gemm<MT1>(Ob, LD, P.a1, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            const float v = relu(acc[r] + P.a1.b[c]) * keep_att(row, DROP_H + c);
            H1[row * LDH + c] = v;
            if (valid(row)) o.H1d[(w0 + row) * h + c] = v;
        }
    });
    __syncthreads();
    gemm<MT1>(H1, LDH, P.a2, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) Xb[erow(mt, r) * LDM + c] = acc[r] + P.a2.b[c];
    });
    if (P.cat) {   // one-hot category after the attention output (:308-315)
        for (int i = tid; i < TR * 16; i += blockDim.x) {
            const int w = i >> 4, c = i & 15;
            Xb[w * LDM + h + c] = (c < 12 && s_cat[w] == c) ? 1.f : 0.f;
        }
    }
    __syncthreads();
    for (int i = tid; i < TR * KM; i += blockDim.x) {
        const int w = i / KM, c = i % KM;
        if (valid(w)) o.X[(w0 + w) * KM + c] = Xb[w * LDM + c];
    }
    gemm<MT1>(Xb, LDM, P.m1, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            const float v = c < P.m1.nout ? relu(acc[r] + P.m1.b[c]) * keep(row, DM + c) : 0.f;
            M1[row * LDM + c] = v;
            if (valid(row)) o.M1d[(w0 + row) * KM + c] = v;
        }
    });
    __syncthreads();
    gemm<MT1>(M1, LDM, P.m2, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            const float v = relu(acc[r] + P.m2.b[c]);
            M2[row * LDH + c] = v;
            if (valid(row)) o.M2[(w0 + row) * h + c] = v;
        }
    });
    __syncthreads();
    {
        const int w = tid >> 3, sub = tid & 7;
        const int cend = w < TR ? h : 0;
        float s = 0.f;
        for (int c = sub; c < cend; c += 8) s += M2[w * LDH + c] * P.m3w[c];
        s += __shfl_xor(s, 1, 8);
        s += __shfl_xor(s, 2, 8);
        s += __shfl_xor(s, 4, 8);
        if (sub == 0 && w < TR) {
            float dl = 0.f;
            if (valid(w)) {
                const float y = 1.f / (1.f + expf(-(s + P.m3b[0])));
                dl = d_imp[w0 + w] * (1.f - y) * y;   // sigmoid backward
                if (o.imp) o.imp[w0 + w] = y;
                o.dlogit[w0 + w] = dl;
            }
            s_dl[w] = dl;
        }
    }
    __syncthreads();

    // ---- backward through the MLP head
    for (int i = tid; i < TR * h; i += blockDim.x) {
        const int w = i / h, c = i % h;
        const float v = M2[w * LDH + c] > 0.f ? s_dl[w] * P.m3w[c] : 0.f;
        M2[w * LDH + c] = v;
        if (valid(w)) o.dM2[(w0 + w) * h + c] = v;
    }
    __syncthreads();
    gemm<MT1>(M2, LDH, T.m2T, [&](int mt, int nt, floatx4 acc) {   // d M1d = dM2 P3
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            const float v = (c < P.m1.nout && M1[row * LDM + c] > 0.f) ? acc[r] * kscale : 0.f;
            M1[row * LDM + c] = v;
            if (valid(row)) o.dM1[(w0 + row) * KM + c] = v;
        }
    });
    __syncthreads();
    gemm<MT1>(M1, LDM, T.m1T, [&](int mt, int nt, floatx4 acc) {   // d X = dM1 P0; keep the attention part
        const int c = ecol(nt);
        if (c < h) {
            for (int r = 0; r < 4; ++r) {
                const int row = erow(mt, r);
                Xb[row * LDM + c] = acc[r];
                if (valid(row)) o.dY2[(w0 + row) * h + c] = acc[r];
            }
        }
    });
    __syncthreads();
    gemm<MT1>(Xb, LDM, T.a2T, [&](int mt, int nt, floatx4 acc) {   // d H1d = dY2 A3
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            const float v = H1[row * LDH + c] > 0.f ? acc[r] * kscale_h : 0.f;
            H1[row * LDH + c] = v;
            if (valid(row)) o.dH1[(w0 + row) * h + c] = v;
        }
    });
    __syncthreads();
    gemm<MT1>(H1, LDH, T.a1T, [&](int mt, int nt, floatx4 acc) {   // d O = dH1 A0
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) Ob[erow(mt, r) * LD + c] = acc[r];
    });
    __syncthreads();
    {   // d alpha'_k = dO . Wq_k
        const int pair = tid >> 2, sub = tid & 3, w = pair >> 1, p = pair & 1;
        const int cend = w < TR ? D2 : 0;
        float s = 0.f;
        for (int c = sub; c < cend; c += 4) s += Ob[w * LD + c] * Qb[(p * TR + w) * LD + c];
        s += __shfl_xor(s, 1, 4);
        s += __shfl_xor(s, 2, 4);
        if (sub == 0 && w < TR) s_score[pair] = s;
    }
    __syncthreads();
    if (tid < TR) {   // dropout, softmax and temporal-scaling backward
        const float a0 = s_alpha[2 * tid], a1 = s_alpha[2 * tid + 1];
        const float g0 = s_score[2 * tid] * keep_att(tid, DROP_A), g1 = s_score[2 * tid + 1] * keep_att(tid, DROP_A + 1);
        const float dot = g0 * a0 + g1 * a1;
        s_dsr[2 * tid] = (g0 - dot) * a0 * s_mult[2 * tid];
        s_dsr[2 * tid + 1] = (g1 - dot) * a1 * s_mult[2 * tid + 1];
    }
    __syncthreads();
    for (int i = tid; i < TR * D2; i += blockDim.x) {
        const int w = i / D2, c = i % D2;
        const float q0 = Qb[w * LD + c], q1 = Qb[(TR + w) * LD + c], wp = Wp[w * LD + c], dO = Ob[w * LD + c];
        const float ds0 = s_dsr[2 * w], ds1 = s_dsr[2 * w + 1];
        const float dq0 = s_alphad[2 * w] * dO + ds0 * wp, dq1 = s_alphad[2 * w + 1] * dO + ds1 * wp;
        const float dp = ds0 * q0 + ds1 * q1;
        Qb[w * LD + c] = dq0;
        Qb[(TR + w) * LD + c] = dq1;
        Wp[w * LD + c] = dp;
        if (valid(w)) {
            o.dQ[(w0 + w) * D2 + c] = dq0;
            o.dQ[(n_walks + w0 + w) * D2 + c] = dq1;
            o.dP[(w0 + w) * D2 + c] = dp;
        }
    }
    __syncthreads();
    gemm<MT2>(Qb, LD, T.w2T, [&](int mt, int nt, floatx4 acc) {   // dF0, dF1 = dQ W2
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r), p = row / TR, w = row % TR;
            if (valid(w)) o.dF[((w0 + w) * 3 + p) * D2 + c] = acc[r];
        }
    });
    gemm<MT1>(Wp, LD, T.w1T, [&](int mt, int nt, floatx4 acc) {   // dF2 = dO + dP W1
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            if (valid(row)) o.dF[((w0 + row) * 3 + 2) * D2 + c] = acc[r] + Ob[row * LD + c];
        }
    });
}

// ------------------------------------------------------------------ event_gcn backward
struct GcnBwdOut {
    float *ev;    // [R][kev16]     event features                    (lin_event: with dlev)
    float *AB;    // [R][2][dn16]   [x_s + relu(a) | x_t + relu(b)]     (MLP.0: with dZ)
    float *H;     // [R][2][64]     relu(MLP.0 .)                       (MLP.2: with dF)
    float *dZ;    // [R][2][64]     d MLP.0 pre-activation
    float *dlev;  // [R][dn16]      d lin_event output
    float *g;     // [R][dn16]      d time feature * -sin(dt w + phi)   (phase: sum; freq: dt^T g)
    float *dt;    // [R]            dt of the row (relative to walk position 2)
};

// ZN (zero node features): A = B, H_s = H_t and the relu masks agree, so every branch sum folds before its GEMM:
// dZ_s + dZ_t = ((dU_s + dU_t) M2) * [z > 0] and d lev = ((dZ_s + dZ_t) M0) * [a > 0] run on 32 rows instead of 64.
// The weight-gradient row pairs become (dZ_s + dZ_t, A) for MLP.0 and (dU_s + dU_t, H) for MLP.2: o.AB / o.H hold
// A / H in half 0, o.dZ holds dZ_s + dZ_t in half 0 and dU_s + dU_t in half 1 (tm_encoder_wgrad's ZN jobs).
template <bool ZN = false>
__global__ void __launch_bounds__(256) gcn_bwd_kernel(EncW P, EncWT T, int64_t n_rows, const float *__restrict__ n_feat,
                                                      const float *__restrict__ e_feat,
                                                      const int32_t *__restrict__ node6, const int32_t *__restrict__ eid3,
                                                      const float *__restrict__ ts3, const float *__restrict__ cnt,
                                                      const float *__restrict__ dF, GcnBwdOut o) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int de = P.de, dn = P.dn, kev = P.kev, kev16 = r16(kev), dn16 = r16(dn);
    const int h = P.h, ldx = kev16 + 8, ldab = dn16 + 8, ldh = h + 8;
    const int xsz = max(TILE_ROWS * ldx, 2 * TILE_ROWS * ldh);
    float *X = smem;                                     // [32][ldx]  event features -> dU [64][ldh]
    float *dU = X;
    float *AB = X + xsz;                                 // [64][ldab] hs rows 0..31, ht rows 32..63 -> d lev
    float *Hb = AB + 2 * TILE_ROWS * ldab;               // [64][ldh]  z = relu(MLP.0 .) -> dZ
    uint8_t *MK = reinterpret_cast<uint8_t *>(Hb + 2 * TILE_ROWS * ldh);   // [64][dn16] relu masks of a / b
    __shared__ int32_t s_eid[TILE_ROWS], s_ns[TILE_ROWS], s_nt[TILE_ROWS];
    __shared__ float s_dt[TILE_ROWS], s_cnt[TILE_ROWS * 3];
    const int64_t row0 = (int64_t)blockIdx.x * TILE_ROWS;
    const int tid = threadIdx.x;
    auto valid = [&](int r) { return row0 + r < n_rows; };
    if (tid < TILE_ROWS) {
        const int64_t r = row0 + tid;
        if (r < n_rows) {
            const int64_t w = r / 3;
            const int p = (int)(r % 3);
            s_eid[tid] = eid3[w * 3 + p];
            s_ns[tid] = node6[w * 6 + 2 * p];
            s_nt[tid] = node6[w * 6 + 2 * p + 1];
            s_dt[tid] = ts3[w * 3 + 2] - ts3[w * 3 + p];
            for (int q = 0; q < 3; ++q) s_cnt[tid * 3 + q] = cnt[w * 9 + p * 3 + q];
            o.dt[r] = s_dt[tid];
        } else {
            s_eid[tid] = 0; s_ns[tid] = 0; s_nt[tid] = 0; s_dt[tid] = 0.f;
            for (int q = 0; q < 3; ++q) s_cnt[tid * 3 + q] = 0.f;
        }
    }
    __syncthreads();
    for (int i = tid; i < TILE_ROWS * kev16; i += blockDim.x) {
        const int r = i / kev16, c = i % kev16;
        float v = 0.f;
        if (valid(r)) {
            if (c < de) v = e_feat[(int64_t)s_eid[r] * de + c];
            else if (c < de + 3) v = s_cnt[r * 3 + (c - de)];
            else if (c < kev) v = time_cos(s_dt[r], P.freq[c - de - 3], P.phase[c - de - 3]);
            o.ev[(row0 + r) * kev16 + c] = v;
        }
        X[r * ldx + c] = v;
    }
    __syncthreads();
    gemm<2>(X, ldx, P.ev, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            float hs = 0.f, ht = 0.f;
            uint8_t ma = 0, mb = 0;
            if (c < dn) {
                const float L = acc[r] + P.ev.b[c];
                const float xs = ZN ? 0.f : n_feat[(int64_t)s_ns[row] * dn + c];
                const float xt = ZN ? 0.f : n_feat[(int64_t)s_nt[row] * dn + c];
                const float a = xt + L, b = xs + L;
                hs = xs + relu(a);
                ht = xt + relu(b);
                ma = a > 0.f;
                mb = b > 0.f;
            }
            AB[row * ldab + c] = hs;
            MK[row * dn16 + c] = ma;
            if (!ZN) {
                AB[(row + TILE_ROWS) * ldab + c] = ht;
                MK[(row + TILE_ROWS) * dn16 + c] = mb;
            }
            if (valid(row)) {
                o.AB[((row0 + row) * 2) * dn16 + c] = hs;
                if (!ZN) o.AB[((row0 + row) * 2 + 1) * dn16 + c] = ht;
            }
        }
    });
    __syncthreads();
    if (ZN) {   // dU_s + dU_t in rows 0..31, also the MLP.2 weight-gradient rows (o.dZ half 1)
        for (int i = tid; i < TILE_ROWS * h; i += blockDim.x) {
            const int r = i / h, c = i % h;
            float v = 0.f;
            if (valid(r)) {
                v = dF[(row0 + r) * (2 * h) + c] + dF[(row0 + r) * (2 * h) + h + c];
                o.dZ[((row0 + r) * 2 + 1) * h + c] = v;
            }
            dU[r * ldh + c] = v;
        }
    } else {
        for (int i = tid; i < 2 * TILE_ROWS * h; i += blockDim.x) {   // dU: d U_s rows 0..31, d U_t rows 32..63
            const int row = i / h, c = i % h, r = row % TILE_ROWS, half = row / TILE_ROWS;
            dU[row * ldh + c] = valid(r) ? dF[(row0 + r) * (2 * h) + half * h + c] : 0.f;
        }
    }
    auto g1_epi = [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r), rr = row % TILE_ROWS, half = row / TILE_ROWS;
            const float v = relu(acc[r] + P.g1.b[c]);
            Hb[row * ldh + c] = v;
            if (valid(rr)) o.H[((row0 + rr) * 2 + half) * h + c] = v;
        }
    };
    if constexpr (ZN) gemm<2>(AB, ldab, P.g1, g1_epi);
    else gemm<4>(AB, ldab, P.g1, g1_epi);
    __syncthreads();
    auto g2_epi = [&](int mt, int nt, floatx4 acc) {   // dZ = (dU M2) * [z > 0]
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r), rr = row % TILE_ROWS, half = row / TILE_ROWS;
            const float v = Hb[row * ldh + c] > 0.f ? acc[r] : 0.f;
            Hb[row * ldh + c] = v;
            if (valid(rr)) o.dZ[((row0 + rr) * 2 + half) * h + c] = v;
        }
    };
    if constexpr (ZN) gemm<2>(dU, ldh, T.g2T, g2_epi);
    else gemm<4>(dU, ldh, T.g2T, g2_epi);
    __syncthreads();
    // d lev = (dZ_s M0) * [a > 0] + (dZ_t M0) * [b > 0]; rows r and r + 32 of one column land in the same
    // lane (row tiles mt and mt + 2, in that order), so the sum needs no synchronisation.  ZN: one product.
    float *DL = AB;
    auto lev_epi = [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            const float v = MK[row * dn16 + c] ? acc[r] : 0.f;
            if (ZN) {
                DL[row * ldab + c] = v;
                if (valid(row)) o.dlev[(row0 + row) * dn16 + c] = v;
            } else if (mt < 2) {
                DL[row * ldab + c] = v;
            } else {
                const int rr = row - TILE_ROWS;
                const float s = DL[rr * ldab + c] + v;
                DL[rr * ldab + c] = s;
                if (valid(rr)) o.dlev[(row0 + rr) * dn16 + c] = s;
            }
        }
    };
    if constexpr (ZN) gemm<2>(Hb, ldh, T.g1T, lev_epi);
    else gemm<4>(Hb, ldh, T.g1T, lev_epi);
    __syncthreads();
    gemm<2>(DL, ldab, T.evT, [&](int mt, int nt, floatx4 acc) {   // d time features -> * -sin(dt w + phi)
        const int j = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            if (!valid(row)) continue;
            float gv = 0.f;
            if (j < dn) gv = -acc[r] * sinf(__fadd_rn(__fmul_rn(s_dt[row], P.freq[j]), P.phase[j]));
            o.g[(row0 + row) * dn16 + j] = gv;
        }
    });
}


// Register-resident event_gcn backward (hid_dim 64, dn with 11 tiles, lin_event with NQE K steps): the same
// computation as gcn_bwd_kernel in the fused walk kernel's orientation -- weights are the MFMA A operand
// (forward packs P.ev / P.g1 and the transposed packs T.g2T / T.g1T / T.evT), one wave's 16 walk positions the
// B operand's columns, so the whole chain (recomputed lin_event, both event_gcn branches, dZ, d lev, the
// time-feature gradient) stays in registers with no LDS and no barriers; the (d pre-activation, input) row
// pairs the weight gradients need are stored as they are produced.  Every tile accumulates its K steps in
// the LDS kernel's order; the time-feature gradient's sin is the branch-free sin_rd (common.h, |error| ~1e-7;
// ocml's sinf carries a Payne-Hanek slow path).
struct GcnRow {
    int64_t r, rc;   // this lane's row (walk position) and its clamped index
    bool valid;
    float dt;
};

// The front of the register-resident event_gcn kernels for one wave's 16 walk positions: event features,
// lin_event, A / B and event_gcn's first layer (pre-activation) of both branches; BWD also stores the event
// features and A / B rows and dt for the weight gradients and returns the relu masks of a / b as bits.
// tabw / tabp: the workgroup's LDS tables of the time encoder's frequency / phase on the event-feature axis.
template <int NQE, bool BWD, bool ZN = false>
__device__ __forceinline__ GcnRow gcn_front(const EncW &P, int64_t n_rows, const float *__restrict__ n_feat,
                                            const float *__restrict__ e_feat, const int32_t *__restrict__ node6,
                                            const int32_t *__restrict__ eid3, const float *__restrict__ ts3,
                                            const float *__restrict__ cnt, float4 *tabw, float4 *tabp,
                                            const GcnBwdOut *o, floatx4 (&Hs)[4], floatx4 (&Ht)[4], uint64_t &ma,
                                            uint64_t &mb) {
    constexpr int NTD = 11, KE = 16 * NQE, DN = 16 * NTD;
    const int lane = threadIdx.x & 63, col = lane & 15, g = lane_id() >> 4;
    const int64_t r0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16;
    const int64_t r = r0 + col;
    const bool valid = r < n_rows;                       // a wave past the end computes row n_rows - 1, stores nothing
    const int64_t rc = valid ? r : n_rows - 1;           // clamped: every load in bounds, stores skipped
    const int64_t w = rc / 3;
    const int p = (int)(rc % 3);
    const int de = P.de, dn = P.dn, kev = P.kev;
    const int32_t e = eid3[rc], ns = node6[w * 6 + 2 * p], nt = node6[w * 6 + 2 * p + 1];
    const float dt = ts3[w * 3 + 2] - ts3[w * 3 + p];
    const float c0 = cnt[rc * 3], c1 = cnt[rc * 3 + 1], c2 = cnt[rc * 3 + 2];
    if (BWD && valid && g == 0) o->dt[r] = dt;
    // 1. event features (B fragments: lane group g holds features 16 q + 4 g + s of column col) -> lin_event.
    // Branch-free: the edge-feature float4 (clamped index), the counts and the cos are all formed and the
    // lane's value selected; the time encoder's frequency / phase come from an LDS table laid out on the
    // event-feature axis (zero outside the time block)
    for (int i = threadIdx.x; i < NQE * 16; i += blockDim.x) {
        const int ti = i - de - 3;
        reinterpret_cast<float *>(tabw)[i] = (ti >= 0 && ti < dn) ? P.freq[ti] : 0.f;
        reinterpret_cast<float *>(tabp)[i] = (ti >= 0 && ti < dn) ? P.phase[ti] : 0.f;
    }
    __syncthreads();
    const float4 *er = reinterpret_cast<const float4 *>(e_feat + (int64_t)e * de);
    floatx4 X[NQE];
#pragma unroll
    for (int q = 0; q < NQE; ++q) {
        const float4 ef4 = er[min(4 * q + g, de / 4 - 1)], w4 = tabw[4 * q + g], p4 = tabp[4 * q + g];
        const float ef[4] = {ef4.x, ef4.y, ef4.z, ef4.w}, wv[4] = {w4.x, w4.y, w4.z, w4.w}, pv[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int k = 16 * q + 4 * g + s;
            float c = time_cos(dt, wv[s], pv[s]);
            asm volatile("" : "+v"(c));
            float v = k < kev ? c : 0.f;
            if (k < de + 3) v = k == de ? c0 : k == de + 1 ? c1 : c2;
            if (k < de) v = ef[s];
            X[q][s] = v;
        }
        if (BWD && valid)
            *reinterpret_cast<float4 *>(o->ev + r * KE + 16 * q + 4 * g) = make_float4(X[q][0], X[q][1], X[q][2], X[q][3]);
    }
    floatx4 L[NTD];
    rgemm<NTD, NQE, NQE>(P.ev, X, L);
#pragma unroll
    for (int t = 0; t < NTD; ++t) {
        const float4 b = *reinterpret_cast<const float4 *>(P.ev.b + 16 * t + 4 * g);
        L[t] = floatx4{L[t][0] + b.x, L[t][1] + b.y, L[t][2] + b.z, L[t][3] + b.w};
    }
    // 2. A = x_s + relu(x_t + L), B = x_t + relu(x_s + L) (:93-96) K step by K step into event_gcn's first
    // layer for both branches (one weight fragment feeds both); relu masks of a / b kept as bits
    // ZN (zero node features): A = B, one branch (Ht, mb unused)
    const float4 *nrs = reinterpret_cast<const float4 *>(n_feat + (int64_t)(ZN ? 0 : ns) * dn);
    const float4 *nrt = reinterpret_cast<const float4 *>(n_feat + (int64_t)(ZN ? 0 : nt) * dn);
    const auto wg1 = wrsrc(P.g1.w);
    const int vo = lane_id() * 16;
#pragma unroll
    for (int t = 0; t < 4; ++t) Hs[t] = Ht[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    ma = mb = 0;
    float4 wq[2][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) wq[0][t] = wload(wg1, vo, (t * NTD + 0) * 64);
#pragma unroll
    for (int q = 0; q < NTD; ++q) {
        if (q + 1 < NTD) {
#pragma unroll
            for (int t = 0; t < 4; ++t) wq[(q + 1) & 1][t] = wload(wg1, vo, (t * NTD + q + 1) * 64);
        }
        const int f4 = min(4 * q + g, dn / 4 - 1);
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 xs4 = ZN ? z4 : nrs[f4], xt4 = ZN ? z4 : nrt[f4];
        const float xs[4] = {xs4.x, xs4.y, xs4.z, xs4.w}, xt[4] = {xt4.x, xt4.y, xt4.z, xt4.w};
        floatx4 A, Bq;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int c = 16 * q + 4 * g + s;
            const float l = L[q][s], a = xt[s] + l, b = xs[s] + l;
            const bool in = q < NTD - 1 || c < dn;     // 161 <= dn <= 176: only the last tile has padding
            A[s] = in ? xs[s] + relu(a) : 0.f;
            Bq[s] = in ? xt[s] + relu(b) : 0.f;
            if (BWD) {
                ma |= (uint64_t)(in && a > 0.f) << (4 * q + s);
                mb |= (uint64_t)(in && b > 0.f) << (4 * q + s);
            }
        }
        if (BWD && valid) {
            *reinterpret_cast<float4 *>(o->AB + (r * 2) * DN + 16 * q + 4 * g) = make_float4(A[0], A[1], A[2], A[3]);
            if (!ZN)
                *reinterpret_cast<float4 *>(o->AB + (r * 2 + 1) * DN + 16 * q + 4 * g) = make_float4(Bq[0], Bq[1], Bq[2], Bq[3]);
        }
        if constexpr (ZN) {
#pragma unroll
            for (int t = 0; t < 4; ++t) Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wq[q & 1][t].x, A.x, Hs[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 4; ++t) Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wq[q & 1][t].y, A.y, Hs[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 4; ++t) Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wq[q & 1][t].z, A.z, Hs[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 4; ++t) Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wq[q & 1][t].w, A.w, Hs[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            continue;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float4 wv = wq[q & 1][t];
            Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.x, A.x, Hs[t], 0, 0, 0);
            Ht[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.x, Bq.x, Ht[t], 0, 0, 0);
            Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.y, A.y, Hs[t], 0, 0, 0);
            Ht[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.y, Bq.y, Ht[t], 0, 0, 0);
            Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.z, A.z, Hs[t], 0, 0, 0);
            Ht[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.z, Bq.z, Ht[t], 0, 0, 0);
            Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.w, A.w, Hs[t], 0, 0, 0);
            Ht[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv.w, Bq.w, Ht[t], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    // the relu masks as VGPR bit fields (opaque to the compiler: it would otherwise keep every compare's lane
    // mask alive in SGPR pairs until step 6 and spill the scalar file)
    if (BWD) {
        uint32_t ma0 = (uint32_t)ma, ma1 = (uint32_t)(ma >> 32), mb0 = (uint32_t)mb, mb1 = (uint32_t)(mb >> 32);
        asm volatile("" : "+v"(ma0), "+v"(ma1), "+v"(mb0), "+v"(mb1));
        ma = ((uint64_t)ma1 << 32) | ma0;
        mb = ((uint64_t)mb1 << 32) | mb0;
    }
    return GcnRow{r, rc, valid, dt};
}

// the zero-node-feature tail of gcn_bwd_reg_kernel (steps 3-7 on one branch)
template <int NQE>
__device__ __forceinline__ void gcn_bwd_reg_zn(const EncW &P, const EncWT &T, const GcnRow &rw, const float *__restrict__ dF,
                                               const GcnBwdOut &o, const floatx4 (&Hs)[4], uint64_t ma) {
    constexpr int NTD = 11, DN = 16 * NTD, H = HID;
    const int g = lane_id() >> 4, vo = lane_id() * 16, dn = P.dn;
    const int64_t r = rw.r, rc = rw.rc;
    const bool valid = rw.valid;
    const float dt = rw.dt;
    uint32_t mz = 0;
    floatx4 dU[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const float4 b = *reinterpret_cast<const float4 *>(P.g1.b + 16 * t + 4 * g);
        const float bb[4] = {b.x, b.y, b.z, b.w};
        floatx4 z;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            z[s] = relu(Hs[t][s] + bb[s]);
            mz |= (uint32_t)(z[s] > 0.f) << (4 * t + s);
        }
        const float4 us = *reinterpret_cast<const float4 *>(dF + rc * (2 * H) + 16 * t + 4 * g);
        const float4 ut = *reinterpret_cast<const float4 *>(dF + rc * (2 * H) + H + 16 * t + 4 * g);
        const float4 su = make_float4(us.x + ut.x, us.y + ut.y, us.z + ut.z, us.w + ut.w);
        dU[t] = floatx4{valid ? su.x : 0.f, valid ? su.y : 0.f, valid ? su.z : 0.f, valid ? su.w : 0.f};
        if (valid) {
            *reinterpret_cast<float4 *>(o.H + (r * 2) * H + 16 * t + 4 * g) = make_float4(z[0], z[1], z[2], z[3]);
            *reinterpret_cast<float4 *>(o.dZ + (r * 2 + 1) * H + 16 * t + 4 * g) = su;
        }
    }
    asm volatile("" : "+v"(mz));
    floatx4 dZ[4];
    rgemm<4, 4, 4>(T.g2T, dU, dZ);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int s = 0; s < 4; ++s) dZ[t][s] = (mz >> (4 * t + s)) & 1u ? dZ[t][s] : 0.f;
        if (valid)
            *reinterpret_cast<float4 *>(o.dZ + (r * 2) * H + 16 * t + 4 * g) = make_float4(dZ[t][0], dZ[t][1], dZ[t][2], dZ[t][3]);
    }
    const auto wg1t = wrsrc(T.g1T.w);
    floatx4 DL[NTD];
#pragma unroll
    for (int t = 0; t < NTD; ++t) {
        float4 wf[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) wf[q] = wload(wg1t, vo, (t * 4 + q) * 64);
        floatx4 as = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            as = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].x, dZ[q].x, as, 0, 0, 0);
            as = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].y, dZ[q].y, as, 0, 0, 0);
            as = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].z, dZ[q].z, as, 0, 0, 0);
            as = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].w, dZ[q].w, as, 0, 0, 0);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) DL[t][s] = (ma >> (4 * t + s)) & 1u ? as[s] : 0.f;
        if (valid)
            *reinterpret_cast<float4 *>(o.dlev + r * DN + 16 * t + 4 * g) = make_float4(DL[t][0], DL[t][1], DL[t][2], DL[t][3]);
        __builtin_amdgcn_sched_barrier(0);
    }
    floatx4 GT[NTD];
    rgemm<NTD, NTD, NTD>(T.evT, DL, GT);
    if (valid) {
#pragma unroll
        for (int t = 0; t < NTD; ++t) {
            float gv[4];
            const float4 f4 = *reinterpret_cast<const float4 *>(P.freq + 16 * t + 4 * g);
            const float4 h4 = *reinterpret_cast<const float4 *>(P.phase + 16 * t + 4 * g);
            const float fv[4] = {f4.x, f4.y, f4.z, f4.w}, hv[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int j = 16 * t + 4 * g + s;
                gv[s] = (t < NTD - 1 || j < dn) ? -GT[t][s] * sin_rd(__fadd_rn(__fmul_rn(dt, fv[s]), hv[s])) : 0.f;
            }
            *reinterpret_cast<float4 *>(o.g + r * DN + 16 * t + 4 * g) = make_float4(gv[0], gv[1], gv[2], gv[3]);
        }
    }
}

// ZN: one branch; dZ_s + dZ_t = (M2^T (dU_s + dU_t)) * [z > 0] and d lev = (M0^T (dZ_s + dZ_t)) * [a > 0] (the
// masks agree), stored as gcn_bwd_kernel<true> stores them (o.dZ half 0 = the dZ sum, half 1 = the dU sum)
template <int NQE, bool ZN = false>
__global__ void __launch_bounds__(256, 2) gcn_bwd_reg_kernel(EncW P, EncWT T, int64_t n_rows,
                                                              const float *__restrict__ n_feat,
                                                              const float *__restrict__ e_feat,
                                                              const int32_t *__restrict__ node6,
                                                              const int32_t *__restrict__ eid3,
                                                              const float *__restrict__ ts3,
                                                              const float *__restrict__ cnt,
                                                              const float *__restrict__ dF, GcnBwdOut o) {
    constexpr int NTD = 11, DN = 16 * NTD, H = HID;
    __shared__ float4 tabw[NQE * 4], tabp[NQE * 4];
    const int g = lane_id() >> 4;
    const int vo = lane_id() * 16;
    const int dn = P.dn;
    floatx4 Hs[4], Ht[4];
    uint64_t ma, mb;
    const GcnRow rw = gcn_front<NQE, true, ZN>(P, n_rows, n_feat, e_feat, node6, eid3, ts3, cnt, tabw, tabp, &o, Hs,
                                               Ht, ma, mb);
    const int64_t r = rw.r, rc = rw.rc;
    const bool valid = rw.valid;
    const float dt = rw.dt;
    // 3. z = relu(MLP.0 . + b) of both branches (stored: MLP.2's inputs); 4. dU = dF (the head's gradient);
    // 5. dZ = (M2^T dU) * [z > 0]
    if constexpr (ZN) {
        gcn_bwd_reg_zn<NQE>(P, T, rw, dF, o, Hs, ma);
        return;
    }
    uint32_t mz = 0;
    floatx4 dUs[4], dUt[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const float4 b = *reinterpret_cast<const float4 *>(P.g1.b + 16 * t + 4 * g);
        const float bb[4] = {b.x, b.y, b.z, b.w};
        floatx4 zs, zt;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            zs[s] = relu(Hs[t][s] + bb[s]);
            zt[s] = relu(Ht[t][s] + bb[s]);
            mz |= (uint32_t)(zs[s] > 0.f) << (4 * t + s);
            mz |= (uint32_t)(zt[s] > 0.f) << (16 + 4 * t + s);
        }
        if (valid) {
            *reinterpret_cast<float4 *>(o.H + (r * 2) * H + 16 * t + 4 * g) = make_float4(zs[0], zs[1], zs[2], zs[3]);
            *reinterpret_cast<float4 *>(o.H + (r * 2 + 1) * H + 16 * t + 4 * g) = make_float4(zt[0], zt[1], zt[2], zt[3]);
        }
        const float4 us = *reinterpret_cast<const float4 *>(dF + rc * (2 * H) + 16 * t + 4 * g);
        const float4 ut = *reinterpret_cast<const float4 *>(dF + rc * (2 * H) + H + 16 * t + 4 * g);
        dUs[t] = floatx4{valid ? us.x : 0.f, valid ? us.y : 0.f, valid ? us.z : 0.f, valid ? us.w : 0.f};
        dUt[t] = floatx4{valid ? ut.x : 0.f, valid ? ut.y : 0.f, valid ? ut.z : 0.f, valid ? ut.w : 0.f};
    }
    asm volatile("" : "+v"(mz));
    floatx4 dZs[4], dZt[4];
    rgemm<4, 4, 4>(T.g2T, dUs, dZs);
    rgemm<4, 4, 4>(T.g2T, dUt, dZt);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            dZs[t][s] = (mz >> (4 * t + s)) & 1u ? dZs[t][s] : 0.f;
            dZt[t][s] = (mz >> (16 + 4 * t + s)) & 1u ? dZt[t][s] : 0.f;
        }
        if (valid) {
            *reinterpret_cast<float4 *>(o.dZ + (r * 2) * H + 16 * t + 4 * g) = make_float4(dZs[t][0], dZs[t][1], dZs[t][2], dZs[t][3]);
            *reinterpret_cast<float4 *>(o.dZ + (r * 2 + 1) * H + 16 * t + 4 * g) = make_float4(dZt[t][0], dZt[t][1], dZt[t][2], dZt[t][3]);
        }
    }
    // 6. d lev = (M0^T dZ_s) * [a > 0] + (M0^T dZ_t) * [b > 0], tile by tile (one fragment feeds both branches)
    const auto wg1t = wrsrc(T.g1T.w);
    floatx4 DL[NTD];
#pragma unroll
    for (int t = 0; t < NTD; ++t) {
        float4 wf[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) wf[q] = wload(wg1t, vo, (t * 4 + q) * 64);
        floatx4 as = floatx4{0.f, 0.f, 0.f, 0.f}, at = as;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            as = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].x, dZs[q].x, as, 0, 0, 0);
            at = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].x, dZt[q].x, at, 0, 0, 0);
            as = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].y, dZs[q].y, as, 0, 0, 0);
            at = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].y, dZt[q].y, at, 0, 0, 0);
            as = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].z, dZs[q].z, as, 0, 0, 0);
            at = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].z, dZt[q].z, at, 0, 0, 0);
            as = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].w, dZs[q].w, as, 0, 0, 0);
            at = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[q].w, dZt[q].w, at, 0, 0, 0);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float vs = (ma >> (4 * t + s)) & 1u ? as[s] : 0.f, vt = (mb >> (4 * t + s)) & 1u ? at[s] : 0.f;
            DL[t][s] = vs + vt;
        }
        if (valid)
            *reinterpret_cast<float4 *>(o.dlev + r * DN + 16 * t + 4 * g) = make_float4(DL[t][0], DL[t][1], DL[t][2], DL[t][3]);
        __builtin_amdgcn_sched_barrier(0);
    }
    // 7. d time features = lin_event's time columns^T d lev, times -sin(dt w + phi)
    floatx4 GT[NTD];
    rgemm<NTD, NTD, NTD>(T.evT, DL, GT);
    if (valid) {
#pragma unroll
        for (int t = 0; t < NTD; ++t) {
            float gv[4];
            const float4 f4 = *reinterpret_cast<const float4 *>(P.freq + 16 * t + 4 * g);
            const float4 h4 = *reinterpret_cast<const float4 *>(P.phase + 16 * t + 4 * g);
            const float fv[4] = {f4.x, f4.y, f4.z, f4.w}, hv[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int j = 16 * t + 4 * g + s;
                gv[s] = (t < NTD - 1 || j < dn) ? -GT[t][s] * sin_rd(__fadd_rn(__fmul_rn(dt, fv[s]), hv[s])) : 0.f;
            }
            *reinterpret_cast<float4 *>(o.g + r * DN + 16 * t + 4 * g) = make_float4(gv[0], gv[1], gv[2], gv[3]);
        }
    }
}


// Register-resident event_gcn forward for the training step (hid_dim 64, 11 node tiles): F = [MLP(A) | MLP(B)]
// per walk position (explainer_new.py:79-96), the front of gcn_bwd_reg_kernel plus MLP.2, with gcn_kernel's
// accumulation order (the same F; tm_encoder_train_fwd keeps it for the head and the backward).
template <int NQE, bool ZN = false>
__global__ void __launch_bounds__(256, 2) gcn_fwd_reg_kernel(EncW P, int64_t n_rows, const float *__restrict__ n_feat,
                                                              const float *__restrict__ e_feat,
                                                              const int32_t *__restrict__ node6,
                                                              const int32_t *__restrict__ eid3,
                                                              const float *__restrict__ ts3,
                                                              const float *__restrict__ cnt, float *__restrict__ F) {
    constexpr int H = HID;
    __shared__ float4 tabw[NQE * 4], tabp[NQE * 4];
    const int g = lane_id() >> 4;
    floatx4 Hs[4], Ht[4];
    uint64_t ma, mb;
    const GcnRow rw = gcn_front<NQE, false, ZN>(P, n_rows, n_feat, e_feat, node6, eid3, ts3, cnt, tabw, tabp, nullptr,
                                                Hs, Ht, ma, mb);
    if constexpr (ZN) {   // F = [MLP(A) | MLP(A)]
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float4 b = *reinterpret_cast<const float4 *>(P.g1.b + 16 * t + 4 * g);
            Hs[t] = floatx4{relu(Hs[t][0] + b.x), relu(Hs[t][1] + b.y), relu(Hs[t][2] + b.z), relu(Hs[t][3] + b.w)};
        }
        floatx4 Fs[4];
        rgemm<4, 4, 4>(P.g2, Hs, Fs);
        if (rw.valid) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float4 b = *reinterpret_cast<const float4 *>(P.g2.b + 16 * t + 4 * g);
                const float4 v = make_float4(Fs[t][0] + b.x, Fs[t][1] + b.y, Fs[t][2] + b.z, Fs[t][3] + b.w);
                *reinterpret_cast<float4 *>(F + rw.r * (2 * H) + 16 * t + 4 * g) = v;
                *reinterpret_cast<float4 *>(F + rw.r * (2 * H) + H + 16 * t + 4 * g) = v;
            }
        }
        return;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const float4 b = *reinterpret_cast<const float4 *>(P.g1.b + 16 * t + 4 * g);
        Hs[t] = floatx4{relu(Hs[t][0] + b.x), relu(Hs[t][1] + b.y), relu(Hs[t][2] + b.z), relu(Hs[t][3] + b.w)};
        Ht[t] = floatx4{relu(Ht[t][0] + b.x), relu(Ht[t][1] + b.y), relu(Ht[t][2] + b.z), relu(Ht[t][3] + b.w)};
    }
    floatx4 Fs[4], Ft[4];
    rgemm<4, 4, 4>(P.g2, Hs, Fs);
    rgemm<4, 4, 4>(P.g2, Ht, Ft);
    if (rw.valid) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float4 b = *reinterpret_cast<const float4 *>(P.g2.b + 16 * t + 4 * g);
            *reinterpret_cast<float4 *>(F + rw.r * (2 * H) + 16 * t + 4 * g) =
                make_float4(Fs[t][0] + b.x, Fs[t][1] + b.y, Fs[t][2] + b.z, Fs[t][3] + b.w);
            *reinterpret_cast<float4 *>(F + rw.r * (2 * H) + H + 16 * t + 4 * g) =
                make_float4(Ft[t][0] + b.x, Ft[t][1] + b.y, Ft[t][2] + b.z, Ft[t][3] + b.w);
        }
    }
}

// ------------------------------------------------------------------ weight gradients: dW = dY^T X over rows
// One launch computes every weight / bias gradient of the encoder from the (dY, X) row pairs the two
// backward kernels wrote: job j covers a 64 x 64 block of dW_j over CHUNK rows (column block 0 also sums dY's
// columns: the bias gradient); the workgroup stages WG_SR-row slabs of dY and X in LDS and each wave runs a
// 16 x 64 strip on MFMA (k = rows), then stores its partial block.  A second launch sums
// the partials of every output element in a fixed order (deterministic; no atomics).
constexpr int WG_CHUNK = 1024, WG_LDS_LD = 80, MAX_WG_JOBS = 14, MAX_WG_TGTS = 12;
// a workgroup's partial: its 64 x 64 block of dW, then (column block 0 only) the 64 dY column sums of its rows
constexpr int WG_PART = 4096 + 64;
struct WgJob {
    const float *y, *x;
    int32_t ldy, ldx, O, I, bias, OB, IB, R, vec;
    int64_t wg_begin, part_begin;
};
struct WgTarget {
    float *w, *b;
    int32_t O, I, bias, j0, nj;
    int64_t out_begin;
};
struct WgPlan {
    WgJob job[MAX_WG_JOBS];
    WgTarget tgt[MAX_WG_TGTS];
    int32_t njob, ntgt;
    int64_t total_wg, total_out;
};

// slab staging: 64 rows x 64 columns of dY (cols o0..) and X (cols i0.., the ones column at I), one
// float4 per (thread, k) when the job's rows are 16-byte aligned (vec), else scalars
template <int SR>
struct Slab {
    float4 y[SR / 16], x[SR / 16];
};

__device__ __forceinline__ float4 ld_cols(const float *p, int64_t row_off, int c0, int ncol, bool vec, bool ones,
                                          bool rv) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!rv) return v;
    float e[4] = {0.f, 0.f, 0.f, 0.f};
    if (vec && c0 + 3 < ncol) {
        v = *reinterpret_cast<const float4 *>(p + row_off + c0);
        e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w;
    } else {
        for (int k = 0; k < 4; ++k)
            if (c0 + k < ncol) e[k] = p[row_off + c0 + k];
    }
    if (ones)
        for (int k = 0; k < 4; ++k)
            if (c0 + k == ncol) e[k] = 1.f;
    return make_float4(e[0], e[1], e[2], e[3]);
}

template <int SR>
__device__ __forceinline__ void slab_load(const WgJob &J, int r0, int r_end, int o0, int i0, Slab<SR> &sl) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < SR / 16; ++k) {
        const int e = tid + 256 * k, row = e >> 4, c = (e & 15) * 4, r = r0 + row;
        const bool rv = r < r_end;
        sl.y[k] = ld_cols(J.y, (int64_t)r * J.ldy, o0 + c, J.O, J.vec, false, rv);
        sl.x[k] = ld_cols(J.x, (int64_t)r * J.ldx, i0 + c, J.I, J.vec, false, rv);
    }
}

template <int SR>
__device__ __forceinline__ void slab_store(const Slab<SR> &sl, float *Ys, float *Xs) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < SR / 16; ++k) {
        const int e = tid + 256 * k, row = e >> 4, c = (e & 15) * 4;
        *reinterpret_cast<float4 *>(Ys + row * WG_LDS_LD + c) = sl.y[k];
        *reinterpret_cast<float4 *>(Xs + row * WG_LDS_LD + c) = sl.x[k];
    }
}

// rows per LDS slab: 16 (20 KB of LDS per workgroup, so the workgroups a CU holds are set by waves, not LDS):
// 64-row slabs (80 KB, two workgroups per CU) ran this kernel 0.238 ms per launch, 32 rows 0.167, 16 rows 0.143 --
// 36.1k -> 38.9k trained edges/s (round 5, tools/train_ab.sh, profiles/r05_train_tiles_ab.txt)
constexpr int WG_SR = 16;
__global__ void __launch_bounds__(256) wgrad_partial_kernel(WgPlan P, float *__restrict__ part) {
    constexpr int SR = WG_SR;
    __shared__ __attribute__((aligned(16))) float Ys[2][SR * WG_LDS_LD], Xs[2][SR * WG_LDS_LD];
    const int64_t bid = blockIdx.x;
    int j = 0;
    while (j + 1 < P.njob && bid >= P.job[j + 1].wg_begin) ++j;
    const WgJob &J = P.job[j];
    const int64_t local = bid - J.wg_begin;
    const int nb = J.OB * J.IB;
    const int chunk = (int)(local / nb), tb = (int)(local % nb), ob = tb / J.IB, ib = tb % J.IB;
    const int o0 = ob * 64, i0 = ib * 64;
    const int r_begin = chunk * WG_CHUNK, r_end = min(J.R, r_begin + WG_CHUNK);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, m = lane & 15;
    // the bias gradient (dY's column sums) on the VALU in column block 0, from the A values the MFMAs read; the
    // block's MFMA column tiles past I are skipped (a time-encoder job has one column)
    const bool bias_blk = ib == 0;
    const int nt = min(4, (J.I - i0 + 15) >> 4);
    float ysum = 0.f;
    floatx4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    // double-buffered: slab k+1 is loaded into registers while slab k's MFMAs run from LDS
    Slab<SR> sl;
    slab_load<SR>(J, r_begin, r_end, o0, i0, sl);
    slab_store<SR>(sl, Ys[0], Xs[0]);
    __syncthreads();
    int buf = 0;
    for (int r0 = r_begin; r0 < r_end; r0 += SR) {
        const bool more = r0 + SR < r_end;
        if (more) slab_load<SR>(J, r0 + SR, r_end, o0, i0, sl);
        const float *Y = Ys[buf], *X = Xs[buf];
#pragma unroll 4
        for (int s = 0; s < SR / 4; ++s) {
            const float a = Y[(4 * s + g) * WG_LDS_LD + 16 * wave + m];
            if (bias_blk) ysum += a;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (t >= nt) break;
                const float b = X[(4 * s + g) * WG_LDS_LD + 16 * t + m];
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
            }
        }
        if (more) slab_store<SR>(sl, Ys[buf ^ 1], Xs[buf ^ 1]);
        __syncthreads();
        buf ^= 1;
    }
    float *out = part + J.part_begin + local * WG_PART;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(16 * wave + 4 * g + r) * 64 + 16 * t + m] = acc[t][r];
    if (bias_blk) {
        ysum += __shfl_xor(ysum, 16);
        ysum += __shfl_xor(ysum, 32);
        if (g == 0) out[4096 + 16 * wave + m] = ysum;
    }
}


__global__ void wgrad_reduce_kernel(WgPlan P, const float *__restrict__ part) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < P.total_out; e += (int64_t)gridDim.x * blockDim.x) {
        int t = 0;
        while (t + 1 < P.ntgt && e >= P.tgt[t + 1].out_begin) ++t;
        const WgTarget &T = P.tgt[t];
        const int ia = T.I + T.bias;
        const int64_t le = e - T.out_begin;
        const int o = (int)(le / ia), i = (int)(le % ia);
        float s = 0.f;
        for (int jj = 0; jj < T.nj; ++jj) {
            const WgJob &J = P.job[T.j0 + jj];
            const int nchunk = (J.R + WG_CHUNK - 1) / WG_CHUNK, nb = J.OB * J.IB;
            const bool wcol = i < T.I;
            const int tb = (o / 64) * J.IB + (wcol ? i / 64 : 0);
            const float *p = part + J.part_begin + (int64_t)tb * WG_PART + (wcol ? (o % 64) * 64 + (i % 64) : 4096 + o % 64);
            for (int c = 0; c < nchunk; ++c) s += p[(int64_t)c * nb * WG_PART];
        }
        if (i < T.I) T.w[(int64_t)o * T.I + i] = s;
        else T.b[o] = s;
    }
}


// ------------------------------------------------------------------ explanation (training)
// retrieve_edge_imp_node with the dependency gate in training mode (explainer_new.py:354-406):
//   gate_train_fwd_kernel   per 32 walk positions: X = [E[e] | cos(t w + phi)], gate MLP with its two
//                           dropouts, z, gate = 0.5 + 0.5 sigmoid(z); keeps X, G1, G2 for the backward
//   explain_train_kernel    per (group, event): LDS hash scatter-max of imp_w * gate over the walk edge
//                           ids, gathered at the subgraph edge ids -> p (before beta_sample / mask)
//   explain_train_bwd_kernel per (group, event): d p -> d dense (scatter-add) -> split evenly among the
//                           tied maxima -> d imp (sum over a walk's 3 positions), d gate
//   gate_train_bwd_kernel   per 32 positions: d gate -> d z -> .6 -> relu/dropout -> .3 -> relu/dropout
//                           -> d time features -> * -sin(t w + phi)
struct ExplIO {
    float *X, *G1, *G2, *z, *gate, *d_gate, *dz, *dG2, *dG1, *g, *t;
};

__global__ void __launch_bounds__(256) gate_train_fwd_kernel(EncW P, int64_t n_rows, const float *__restrict__ e_feat,
                                                             const int32_t *__restrict__ eid3,
                                                             const float *__restrict__ ts3,
                                                             const uint8_t *__restrict__ keep1,
                                                             const uint8_t *__restrict__ keep2, float sc1, float sc2,
                                                             ExplIO o) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int h = P.h, H2 = h / 2;
    const int de = P.de, kdep = P.kdep, kd16 = r16(kdep), ldx = kd16 + 8, ldg = r16(h) + 8, ldg2 = r16(H2) + 8;
    float *X = smem, *G1 = X + TILE_ROWS * ldx, *G2 = G1 + TILE_ROWS * ldg;
    __shared__ int32_t s_e[TILE_ROWS];
    __shared__ float s_t[TILE_ROWS];
    const int64_t r0 = (int64_t)blockIdx.x * TILE_ROWS;
    const int tid = threadIdx.x;
    auto valid = [&](int r) { return r0 + r < n_rows; };
    if (!P.dep) {   // use_dependency_aware_sampling=False: no gate (:366-386 skipped), walk_imp = graphlet_imp
        if (tid < TILE_ROWS && valid(tid)) o.gate[r0 + tid] = 1.f;
        return;
    }
    if (tid < TILE_ROWS) {
        s_e[tid] = valid(tid) ? eid3[r0 + tid] : 0;
        s_t[tid] = valid(tid) ? ts3[r0 + tid] : 0.f;    // raw event time (:371)
        if (valid(tid)) o.t[r0 + tid] = s_t[tid];
    }
    __syncthreads();
    for (int i = tid; i < TILE_ROWS * kd16; i += blockDim.x) {
        const int r = i / kd16, c = i % kd16;
        float v = 0.f;
        if (valid(r)) {
            if (c < de) v = e_feat[(int64_t)s_e[r] * de + c];
            else if (c < kdep) v = time_cos(s_t[r], P.freq[c - de], P.phase[c - de]);
            o.X[(r0 + r) * kd16 + c] = v;
        }
        X[r * ldx + c] = v;
    }
    __syncthreads();
    gemm<2>(X, ldx, P.d1, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            float v = relu(acc[r] + P.d1.b[c]);
            if (keep1) v = (valid(row) && keep1[(r0 + row) * h + c]) ? v * sc1 : 0.f;
            G1[row * ldg + c] = v;
            if (valid(row)) o.G1[(r0 + row) * h + c] = v;
        }
    });
    __syncthreads();
    gemm<2>(G1, ldg, P.d2, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            float v = relu(acc[r] + P.d2.b[c]);
            if (keep2) v = (valid(row) && c < H2 && keep2[(r0 + row) * H2 + c]) ? v * sc2 : 0.f;
            G2[row * ldg2 + c] = v;
            if (valid(row) && c < H2) o.G2[(r0 + row) * H2 + c] = v;
        }
    });
    __syncthreads();
    const int r = tid >> 3, sub = tid & 7;
    const float sv = gate_logit_lds(G2 + r * ldg2, P.d3w, sub, H2);
    if (sub == 0 && valid(r)) {
        const float z = sv + P.d3b[0];
        o.z[r0 + r] = z;
        o.gate[r0 + r] = 0.5f + 0.5f * (1.f / (1.f + expf(-z)));
    }
}

// open-addressing LDS hash of one event's walk edge ids -> max of imp_w * gate (float bits; values > 0)
__device__ __forceinline__ void expl_hash_build(int nrow, const int32_t *e3, const float *imp_ev, const float *gate_ev,
                                                int hbits, int32_t *hkey, uint32_t *hval) {
    const int hsize = 1 << hbits;
    for (int i = threadIdx.x; i < hsize; i += blockDim.x) {
        hkey[i] = -1;
        hval[i] = 0u;
    }
    __syncthreads();
    for (int r = threadIdx.x; r < nrow; r += blockDim.x) {
        const int32_t key = e3[r];
        const float v = imp_ev[r / 3] * gate_ev[r];
        uint32_t hh = ((uint32_t)key * 0x9E3779B1u) >> (32 - hbits);
        while (true) {
            const int32_t prev = atomicCAS(&hkey[hh], -1, key);
            if (prev == -1 || prev == key) break;
            hh = (hh + 1) & (hsize - 1);
        }
        atomicMax(&hval[hh], __float_as_uint(v));
    }
    __syncthreads();
}

__device__ __forceinline__ int expl_hash_find(int32_t key, int hbits, const int32_t *hkey) {
    const int hsize = 1 << hbits;
    uint32_t hh = ((uint32_t)key * 0x9E3779B1u) >> (32 - hbits);
    while (true) {
        const int32_t k = hkey[hh];
        if (k == key) return (int)hh;
        if (k == -1) return -1;
        hh = (hh + 1) & (hsize - 1);
    }
}

__global__ void __launch_bounds__(256) explain_train_kernel(int32_t W, int32_t N, int32_t hbits,
                                                            const int32_t *__restrict__ eid3,
                                                            const float *__restrict__ imp,
                                                            const float *__restrict__ gate,
                                                            const int32_t *__restrict__ sub1_eid,
                                                            const int32_t *__restrict__ sub2_eid,
                                                            float *__restrict__ p1, float *__restrict__ p2,
                                                            const int32_t *__restrict__ sub1_node = nullptr,
                                                            const int32_t *__restrict__ sub2_node = nullptr,
                                                            float *__restrict__ keep1 = nullptr,
                                                            float *__restrict__ keep2 = nullptr) {
    extern __shared__ __attribute__((aligned(16))) int32_t hkey[];
    uint32_t *hval = reinterpret_cast<uint32_t *>(hkey + (1 << hbits));
    const int64_t ge = blockIdx.x;
    const int nrow = 3 * W;
    expl_hash_build(nrow, eid3 + ge * nrow, imp + ge * W, gate + ge * nrow, hbits, hkey, hval);
    const int n1 = N, n2 = N * N;
    for (int i = threadIdx.x; i < n1 + n2; i += blockDim.x) {
        const bool h1 = i < n1;
        const int64_t o = h1 ? ge * n1 + i : ge * n2 + (i - n1);
        const int hh = expl_hash_find(h1 ? sub1_eid[o] : sub2_eid[o], hbits, hkey);
        const float p = hh >= 0 ? __uint_as_float(hval[hh]) : 0.f;   // ids no walk passes through: 0
        if (h1) p1[o] = p;
        else p2[o] = p;
        if (keep1) {   // the padding mask of :400-404 (node 0 -> weight 0), as a factor
            if (h1) keep1[o] = sub1_node[o] == 0 ? 0.f : 1.f;
            else keep2[o] = sub2_node[o] == 0 ? 0.f : 1.f;
        }
    }
}

__global__ void __launch_bounds__(256) explain_train_bwd_kernel(int32_t W, int32_t N, int32_t hbits,
                                                                const int32_t *__restrict__ eid3,
                                                                const float *__restrict__ imp,
                                                                const float *__restrict__ gate,
                                                                const int32_t *__restrict__ sub1_eid,
                                                                const int32_t *__restrict__ sub2_eid,
                                                                const float *__restrict__ dp1,
                                                                const float *__restrict__ dp2,
                                                                float *__restrict__ d_imp, float *__restrict__ d_gate) {
    extern __shared__ __attribute__((aligned(16))) int32_t hkey[];
    const int hsize = 1 << hbits;
    uint32_t *hval = reinterpret_cast<uint32_t *>(hkey + hsize);
    int32_t *hcnt = reinterpret_cast<int32_t *>(hval + hsize);
    float *hd = reinterpret_cast<float *>(hcnt + hsize);
    const int64_t ge = blockIdx.x;
    const int nrow = 3 * W;
    const int32_t *e3 = eid3 + ge * nrow;
    const float *imp_ev = imp + ge * W, *gate_ev = gate + ge * nrow;
    for (int i = threadIdx.x; i < hsize; i += blockDim.x) {
        hcnt[i] = 0;
        hd[i] = 0.f;
    }
    expl_hash_build(nrow, e3, imp_ev, gate_ev, hbits, hkey, hval);
    // number of positions attaining each maximum; d dense[e] = sum of d p over the slots gathering e
    for (int r = threadIdx.x; r < nrow; r += blockDim.x) {
        const int hh = expl_hash_find(e3[r], hbits, hkey);
        if (__float_as_uint(imp_ev[r / 3] * gate_ev[r]) == hval[hh]) atomicAdd(&hcnt[hh], 1);
    }
    const int n1 = N, n2 = N * N;
    for (int i = threadIdx.x; i < n1 + n2; i += blockDim.x) {
        const bool h1 = i < n1;
        const int64_t o = h1 ? ge * n1 + i : ge * n2 + (i - n1);
        const int hh = expl_hash_find(h1 ? sub1_eid[o] : sub2_eid[o], hbits, hkey);
        if (hh >= 0) atomicAdd(&hd[hh], h1 ? dp1[o] : dp2[o]);
    }
    __syncthreads();
    for (int w = threadIdx.x; w < W; w += blockDim.x) {
        const float iw = imp_ev[w];
        float di = 0.f;
        for (int k = 0; k < 3; ++k) {
            const int r = 3 * w + k;
            const int hh = expl_hash_find(e3[r], hbits, hkey);
            const float gt = gate_ev[r];
            float dv = 0.f;
            if (__float_as_uint(iw * gt) == hval[hh]) dv = hd[hh] / (float)hcnt[hh];
            di += dv * gt;
            d_gate[ge * nrow + r] = dv * iw;
        }
        d_imp[ge * W + w] = di;
    }
}

__global__ void __launch_bounds__(256) gate_train_bwd_kernel(EncW P, EncWT T, int64_t n_rows, const uint8_t *keep1,
                                                             const uint8_t *keep2, float sc1, float sc2, ExplIO o) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int h = P.h, H2 = h / 2, H2p = r16(H2);
    const int dn = P.dn, dn16 = r16(dn), ldg = r16(h) + 8, ldg2 = H2p + 8;
    float *G1 = smem, *G2 = G1 + TILE_ROWS * ldg;
    __shared__ float s_dz[TILE_ROWS], s_t[TILE_ROWS];
    const int64_t r0 = (int64_t)blockIdx.x * TILE_ROWS;
    const int tid = threadIdx.x;
    auto valid = [&](int r) { return r0 + r < n_rows; };
    const float k1 = keep1 ? sc1 : 1.f, k2 = keep2 ? sc2 : 1.f;
    if (tid < TILE_ROWS) {
        float dz = 0.f, t = 0.f;
        if (valid(tid)) {
            const float sg = 1.f / (1.f + expf(-o.z[r0 + tid]));
            dz = o.d_gate[r0 + tid] * 0.5f * (1.f - sg) * sg;   // gate = 0.5 + 0.5 sigmoid(z)
            t = o.t[r0 + tid];
            o.dz[r0 + tid] = dz;
        }
        s_dz[tid] = dz;
        s_t[tid] = t;
    }
    for (int i = tid; i < TILE_ROWS * h; i += blockDim.x) {
        const int r = i / h, c = i % h;
        G1[r * ldg + c] = valid(r) ? o.G1[(r0 + r) * h + c] : 0.f;
    }
    __syncthreads();
    for (int i = tid; i < TILE_ROWS * H2p; i += blockDim.x) {   // dG2 = dz d3 * [G2 > 0] * keep (K padding 0)
        const int r = i / H2p, c = i % H2p;
        const float g2 = (valid(r) && c < H2) ? o.G2[(r0 + r) * H2 + c] : 0.f;
        const float v = g2 > 0.f ? s_dz[r] * P.d3w[c] * k2 : 0.f;
        G2[r * ldg2 + c] = v;
        if (valid(r) && c < H2) o.dG2[(r0 + r) * H2 + c] = v;
    }
    __syncthreads();
    gemm<2>(G2, ldg2, T.d2T, [&](int mt, int nt, floatx4 acc) {   // dG1 = (dG2 W.3) * [G1 > 0] * keep
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            const float v = G1[row * ldg + c] > 0.f ? acc[r] * k1 : 0.f;
            G1[row * ldg + c] = v;
            if (valid(row)) o.dG1[(r0 + row) * h + c] = v;
        }
    });
    __syncthreads();
    gemm<2>(G1, ldg, T.d1T, [&](int mt, int nt, floatx4 acc) {   // d time features -> * -sin(t w + phi)
        const int j = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            if (!valid(row)) continue;
            float gv = 0.f;
            if (j < dn) gv = -acc[r] * sinf(__fadd_rn(__fmul_rn(s_t[row], P.freq[j]), P.phase[j]));
            o.g[(r0 + row) * dn16 + j] = gv;
        }
    });
}

}  // namespace tmk

using namespace tmk;

// ------------------------------------------------------------------ host side
int train_packs_create(tm_weights *w) {
    const int de = w->de, dn = w->dn, h = w->h, h2 = 2 * h, hm = w->P.hm, kev = de + 3 + dn;
    (void)kev;
    struct D {
        Lin *lin;
        int nout, k;
    } ds[] = {{&w->T.evT, dn, dn}, {&w->T.g1T, dn, h}, {&w->T.g2T, h, h},   {&w->T.w1T, h2, h2}, {&w->T.w2T, h2, h2},
              {&w->T.a1T, h2, h},  {&w->T.a2T, h, h},  {&w->T.m1T, hm, hm}, {&w->T.m2T, hm, h},
              {&w->T.d1T, dn, h},  {&w->T.d2T, h, h / 2}};
    size_t total = 0;
    std::vector<size_t> off;
    for (auto &d : ds) {
        d.lin->nt = r16(d.nout) / 16;
        d.lin->nq = r16(d.k) / 16;
        d.lin->nout = d.nout;
        d.lin->k = d.k;
        d.lin->b = nullptr;
        off.push_back(total);
        total += (size_t)d.lin->nt * d.lin->nq * 256;
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(w->device) != hipSuccess || hipMalloc(&w->tbuf, total * sizeof(float)) != hipSuccess ||
        hipMemset(w->tbuf, 0, total * sizeof(float)) != hipSuccess) {
        (void)hipSetDevice(prev);
        w->tbuf = nullptr;
        return fail(TM_E_HIP, "tm_weights_create: allocation of the transposed packs failed");
    }
    (void)hipSetDevice(prev);
    w->t_floats = total;
    for (size_t i = 0; i < off.size(); ++i) ds[i].lin->w = reinterpret_cast<const float4 *>(w->tbuf + off[i]);
    return TM_OK;
}

void pack_all_weights(tm_weights *w, const float *const *t, hipStream_t s) {
    const int de = w->de, dn = w->dn, h = w->h, h2 = 2 * h, hm = w->P.hm, kev = de + 3 + dn;
    PackJobs P{};
    int64_t total = 0;
    auto frag = [&](const Lin &lin, const float *src, int so, int sc) {
        PackJob &p = P.j[P.n++];
        p.src = src;
        p.dst = const_cast<float *>(reinterpret_cast<const float *>(lin.w));
        p.so = so;
        p.sc = sc;
        p.nout = lin.nout;
        p.k = lin.k;
        p.nt = lin.nt;
        p.nq = lin.nq;
        p.begin = total;
        total += (int64_t)p.nt * p.nq * 256;
    };
    auto copy = [&](const float *src, const float *dst, int n, int npad) {
        PackJob &p = P.j[P.n++];
        p.src = src;
        p.dst = const_cast<float *>(dst);
        p.nout = n;
        p.k = npad;
        p.nt = 0;
        p.begin = total;
        total += npad;
    };
    for (auto &sp : w->specs) {           // forward packs of W[nout][k] and their biases
        frag(*sp.lin, t[sp.wi], sp.k, 1);
        copy(t[sp.wi + 1], sp.lin->b, sp.nout, sp.lin->nt * 16);
    }
    copy(t[18], w->P.m3w, h, r16(h));
    copy(t[19], w->P.m3b, 1, 4);
    copy(t[24], w->P.d3w, h / 2, r16(h / 2));
    copy(t[25], w->P.d3b, 1, 4);
    copy(t[26], w->P.freq, dn, r16(dn));
    copy(t[27], w->P.phase, dn, r16(dn));
    // transposed packs of W[nout][k] (so = 1, sc = k); evT takes lin_event's time-feature columns only
    frag(w->T.evT, t[0] + de + 3, 1, kev);
    frag(w->T.g1T, t[2], 1, dn);
    frag(w->T.g2T, t[4], 1, h);
    frag(w->T.w1T, t[6], 1, h2);
    frag(w->T.w2T, t[8], 1, h2);
    frag(w->T.a1T, t[10], 1, h2);
    frag(w->T.a2T, t[12], 1, h);
    frag(w->T.m1T, t[14], 1, hm);
    frag(w->T.m2T, t[16], 1, hm);
    frag(w->T.d1T, t[20] + de, 1, de + dn);
    frag(w->T.d2T, t[22], 1, h);
    // the fused walk kernel's folded layers (hid_dim 64): fp64 products first, then packed with the rest
    const bool fold = h == HID && w->P.cat && w->fold64 && w->fold32;
    if (fold) {
        using L = FoldLay;
        const FoldIn F{t[4], t[5], t[6], t[7], t[8], t[9], t[10], t[11], t[12], t[13], t[14], t[15]};
        fold1_kernel<<<dim3((FOLD1_N + 255) / 256), 256, 0, s>>>(F, w->fold64);
        fold2_kernel<<<dim3((FOLD2_N + 255) / 256), 256, 0, s>>>(F, w->fold64, w->fold32, w->buf);
        frag(w->P.kv, w->fold32 + L::S_KV, h2, 1);
        frag(w->P.a1d, w->fold32 + L::S_A1D, h2, 1);
        frag(w->P.a1g, w->fold32 + L::S_A1G, h2, 1);
        frag(w->P.m1a2, w->fold32 + L::S_M1A2, h, 1);
        frag(w->P.kvz, w->fold32 + L::S_KVZ, h, 1);
        frag(w->P.a1dz, w->fold32 + L::S_A1DZ, h, 1);
        frag(w->P.a1gz, w->fold32 + L::S_A1GZ, h, 1);
    }
    P.total = total;
    pack_jobs_kernel<<<dim3((unsigned)std::min<int64_t>((total + 255) / 256, 1024)), 256, 0, s>>>(P);
    evc_par_kernel<<<dim3(r16(dn)), 64, 0, s>>>(t[0], t[1], t[27], de, dn, kev, w->P.qt, const_cast<float *>(w->P.evc),
                                                const_cast<float *>(w->P.devc));
}

void train_packs_free(tm_weights *w) {
    if (w->tbuf) (void)hipFree(w->tbuf);
    w->tbuf = nullptr;
}

// walks per head_bwd_kernel workgroup: 16 (0 = the tiles exceed the LDS).  32-walk workgroups (110 KB of LDS at
// hid_dim 64: one per CU) ran 0.224 ms per launch, 16-walk ones (55 KB, two per CU) 0.175 (round 5,
// profiles/r05_train_tiles_ab.txt)
static int head_bwd_tr(const EncW &P) {
    return sizeof(float) * head_bwd_lds_floats(P.h, P.hm, 16) <= 160 * 1024 ? 16 : 0;
}
static size_t gcn_bwd_lds(const EncW &P) {
    const int ldx = r16(P.kev) + 8, ldab = r16(P.dn) + 8, ldh = r16(P.h) + 8;
    const size_t xsz = std::max(TILE_ROWS * ldx, 2 * TILE_ROWS * ldh);
    return sizeof(float) * (xsz + 2 * TILE_ROWS * ldab + 2 * TILE_ROWS * ldh) + 2 * TILE_ROWS * r16(P.dn);
}

// Whether the training kernels (tm_encoder_train_fwd / _bwd, tm_explain_train_fwd / _bwd) have an
// instance for these encoder dims: hid_dim a multiple of 16 up to 256 whose tiles fit the LDS.
extern "C" int tm_encoder_train_supported(int32_t de, int32_t dn, int32_t h, int32_t cat) {
    if (de <= 0 || dn <= 0 || h <= 0 || h % 16 || h > 256) return 0;
    EncW P{};
    P.de = de;
    P.dn = dn;
    P.kev = de + 3 + dn;
    P.kdep = de + dn;
    P.h = h;
    P.hm = cat ? h + 12 : h;
    const size_t lim = 160 * 1024;
    const size_t gate = sizeof(float) * TILE_ROWS * (r16(P.kdep) + 8 + r16(h) + 8 + r16(h / 2) + 8);
    return head_bwd_tr(P) && gcn_bwd_lds(P) <= lim && gate <= lim ? 1 : 0;
}

// the register-resident event_gcn backward runs (the dims it has an instance for; the LDS-tiled one otherwise)
static bool gcn_bwd_uses_reg(const tm_weights *w) {
    const EncW &P = w->P;
    const int nqe = r16(P.kev) / 16;
    return P.h == HID && r16(P.dn) == 176 && P.dn % 4 == 0 && P.de % 4 == 0 && nqe >= 11 && nqe <= 14 &&
           P.g1.nt == 4 && P.g1.nq == 11 && w->T.g2T.nt == 4 && w->T.g1T.nt == 11 && w->T.g1T.nq == 4 &&
           w->T.evT.nt == 11 && w->T.evT.nq == 11 && P.ev.nq == nqe;
}

extern "C" int tm_encoder_bwd(const tm_weights *w, const float *n_feat, const float *e_feat, int32_t n_groups,
                              int32_t B, int32_t W, const int32_t *node6, const int32_t *eid3, const float *ts3,
                              const int32_t *cat, const double *cut, const float *cnt, const uint8_t *drop,
                              float drop_scale, const void *workspace, const float *d_imp, const tm_encoder_grad_io *io,
                              void *stream) {
    if (!w || !io || n_groups < 0 || B < 0 || W < 0) return fail(TM_E_ARG, "tm_encoder_bwd: bad arguments");
    const int64_t n_walks = (int64_t)n_groups * B * W;
    if (n_walks == 0) return TM_OK;
    if (!n_feat || !e_feat || !node6 || !eid3 || !ts3 || !cat || !cut || !cnt || !workspace || !d_imp)
        return fail(TM_E_ARG, "tm_encoder_bwd: NULL pointer");
    if (!io->dlogit || !io->M2 || !io->dM2 || !io->M1d || !io->dM1 || !io->X || !io->dY2 || !io->H1d || !io->dH1 ||
        !io->O || !io->dP || !io->dQ || !io->dF || !io->ev || !io->AB || !io->H || !io->dZ || !io->dlev || !io->g ||
        !io->dt)
        return fail(TM_E_ARG, "tm_encoder_bwd: NULL output buffer");
    if (!w->tbuf) return fail(TM_E_ARG, "tm_encoder_bwd: weights have no transposed packs");
    const EncW &P = w->P;
    const int tr = head_bwd_tr(P);
    const size_t lh = sizeof(float) * head_bwd_lds_floats(P.h, P.hm, tr), lg = gcn_bwd_lds(P);
    if (P.h % 16 || !tr || lg > 160 * 1024) return fail(TM_E_UNSUPPORTED, "tm_encoder_bwd: LDS budget exceeded");
    hipStream_t s = S_(stream);
    const float *F = reinterpret_cast<const float *>(workspace);
    const float *stdv = F + n_walks * 3 * 2 * P.h;
    HeadBwdOut ho{io->imp, io->dlogit, io->M2, io->dM2, io->M1d, io->dM1, io->X, io->dY2, io->H1d, io->dH1, io->O,
                  io->dP,  io->dQ,     io->dF};
    hipEvent_t pe = prof_begin(s);
    head_bwd_kernel<16><<<dim3((unsigned)((n_walks + 15) / 16)), 256, lh, s>>>(
        P, w->T, n_walks, (int64_t)B * W, W, F, ts3, cut, cat, stdv, drop, drop_scale, d_imp, ho);
    TM_CHECK_LAUNCH();
    prof_end("head_bwd_kernel", s, pe);
    const int64_t n_rows = n_walks * 3;
    GcnBwdOut go{io->ev, io->AB, io->H, io->dZ, io->dlev, io->g, io->dt};
    pe = prof_begin(s);
    const int nqe = r16(P.kev) / 16;
    // register-resident instance: hid_dim 64, 11 node-feature tiles (dn 161..176, a multiple of 4), lin_event
    // with 11..14 K steps; the LDS-tiled kernel otherwise
    const bool reg = gcn_bwd_uses_reg(w);
    if (reg) {
        const unsigned blocks = (unsigned)((n_rows + 63) / 64);
#define TM_BWD_REG(Q)                                                                                              \
        (w->node_zero ? gcn_bwd_reg_kernel<Q, true><<<dim3(blocks), 256, 0, s>>>(P, w->T, n_rows, n_feat, e_feat, node6, \
                                                                                 eid3, ts3, cnt, io->dF, go)          \
                      : gcn_bwd_reg_kernel<Q, false><<<dim3(blocks), 256, 0, s>>>(P, w->T, n_rows, n_feat, e_feat, node6, \
                                                                                  eid3, ts3, cnt, io->dF, go))
        if (nqe == 11) TM_BWD_REG(11);
        else if (nqe == 12) TM_BWD_REG(12);
        else if (nqe == 13) TM_BWD_REG(13);
        else TM_BWD_REG(14);
#undef TM_BWD_REG
    } else if (w->node_zero) {
        gcn_bwd_kernel<true><<<dim3((unsigned)((n_rows + TILE_ROWS - 1) / TILE_ROWS)), 256, lg, s>>>(
            P, w->T, n_rows, n_feat, e_feat, node6, eid3, ts3, cnt, io->dF, go);
    } else {
        gcn_bwd_kernel<false><<<dim3((unsigned)((n_rows + TILE_ROWS - 1) / TILE_ROWS)), 256, lg, s>>>(
            P, w->T, n_rows, n_feat, e_feat, node6, eid3, ts3, cnt, io->dF, go);
    }
    TM_CHECK_LAUNCH();
    prof_end("gcn_bwd_kernel", s, pe);
    return TM_OK;
}

// the register-resident event_gcn training forward (gcn_fwd_reg_kernel) for the dims it has an instance for:
// 8 % faster per training step than the LDS-tiled gcn_kernel / gcn_bwd_kernel (round 5, tools/train_flags_ab.sh)
bool tmk::launch_gcn_fwd_reg(const EncW &P, int node_zero, int64_t n_rows, const float *n_feat, const float *e_feat,
                             const int32_t *node6, const int32_t *eid3, const float *ts3, const float *cnt, float *F,
                             hipStream_t s) {
    const int nqe = r16(P.kev) / 16;
    if (!(P.h == HID && r16(P.dn) == 176 && P.dn % 4 == 0 && P.de % 4 == 0 && nqe >= 11 && nqe <= 14 &&
          P.ev.nt == 11 && P.ev.nq == nqe && P.g1.nt == 4 && P.g1.nq == 11 && P.g2.nt == 4 && P.g2.nq == 4))
        return false;
    const unsigned blocks = (unsigned)((n_rows + 63) / 64);
#define TM_FWD_REG(Q)                                                                                              \
    (node_zero ? gcn_fwd_reg_kernel<Q, true><<<dim3(blocks), 256, 0, s>>>(P, n_rows, n_feat, e_feat, node6, eid3, ts3, \
                                                                          cnt, F)                                    \
               : gcn_fwd_reg_kernel<Q, false><<<dim3(blocks), 256, 0, s>>>(P, n_rows, n_feat, e_feat, node6, eid3, ts3, \
                                                                           cnt, F))
    if (nqe == 11) TM_FWD_REG(11);
    else if (nqe == 12) TM_FWD_REG(12);
    else if (nqe == 13) TM_FWD_REG(13);
    else TM_FWD_REG(14);
#undef TM_FWD_REG
    return true;
}

// Shared driver of the weight-gradient launches: jobs (dY, X, rows) and targets (dW, db, job range).
static int run_wgrad(const tm_wgrad_job *jobs, int njob, const tm_wgrad_target *tgts, int ntgt, hipStream_t s,
                     const char *what) {
    if (njob <= 0 || njob > MAX_WG_JOBS || ntgt <= 0 || ntgt > MAX_WG_TGTS)
        return fail(TM_E_ARG, std::string(what) + ": job / target count out of range");
    WgPlan P{};
    P.njob = njob;
    int64_t wg = 0, pb = 0;
    for (int j = 0; j < njob; ++j) {
        const tm_wgrad_job &d = jobs[j];
        if (!d.dy || !d.x || d.O <= 0 || d.I <= 0 || d.R < 0 || d.ldy < d.O || d.ldx < d.I)
            return fail(TM_E_ARG, std::string(what) + ": bad job " + std::to_string(j));
        WgJob &J = P.job[j];
        J.y = d.dy; J.x = d.x; J.ldy = d.ldy; J.ldx = d.ldx; J.O = d.O; J.I = d.I; J.R = d.R;
        J.bias = 1;   // every job adds its dY column sums to its target's bias gradient
        // float4 staging when both row arrays are 16-byte aligned row by row
        J.vec = (d.ldy % 4 == 0 && d.ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(d.dy) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(d.x) & 15) == 0) ? 1 : 0;
        J.OB = (d.O + 63) / 64;
        J.IB = (d.I + 63) / 64;   // the bias column is not a column of X (column block 0 sums dY)
        J.wg_begin = wg;
        J.part_begin = pb;
        const int64_t nchunk = (d.R + WG_CHUNK - 1) / WG_CHUNK;
        wg += nchunk * J.OB * J.IB;
        pb += nchunk * J.OB * J.IB * WG_PART;
    }
    P.total_wg = wg;
    P.ntgt = ntgt;
    int64_t ob = 0;
    for (int t = 0; t < ntgt; ++t) {
        const tm_wgrad_target &d = tgts[t];
        if (!d.w || !d.b || d.first_job < 0 || d.n_jobs <= 0 || d.first_job + d.n_jobs > njob)
            return fail(TM_E_ARG, std::string(what) + ": bad target " + std::to_string(t));
        WgTarget &T = P.tgt[t];
        T.j0 = d.first_job;
        T.nj = d.n_jobs;
        T.w = d.w;
        T.b = d.b;
        T.O = jobs[T.j0].O;
        T.I = jobs[T.j0].I;
        for (int j = T.j0; j < T.j0 + T.nj; ++j)
            if (jobs[j].O != T.O || jobs[j].I != T.I)
                return fail(TM_E_ARG, std::string(what) + ": jobs of one target differ in shape");
        T.bias = 1;
        T.out_begin = ob;
        ob += (int64_t)T.O * (T.I + 1);
    }
    P.total_out = ob;
    if (wg == 0) {   // no rows: every gradient is zero
        for (int t = 0; t < ntgt; ++t) {
            TM_HIP(hipMemsetAsync(P.tgt[t].w, 0, sizeof(float) * P.tgt[t].O * P.tgt[t].I, s));
            TM_HIP(hipMemsetAsync(P.tgt[t].b, 0, sizeof(float) * P.tgt[t].O, s));
        }
        return TM_OK;
    }
    float *part = reinterpret_cast<float *>(scratch((size_t)pb * sizeof(float), s));
    if (!part) return fail(TM_E_HIP, std::string(what) + ": scratch allocation failed");
    hipEvent_t pe = prof_begin(s);
    // (a transposed-LDS form of the partials, 2 x 2 tiles per wave, measured 1.3 % slower per training step in
    // round 5: tools/patches/training_variants.patch)
    wgrad_partial_kernel<<<dim3((unsigned)wg), 256, 0, s>>>(P, part);
    TM_CHECK_LAUNCH();
    prof_end("wgrad_partial_kernel", s, pe);
    pe = prof_begin(s);
    wgrad_reduce_kernel<<<dim3((unsigned)std::min<int64_t>((ob + 255) / 256, 1024)), 256, 0, s>>>(P, part);
    TM_CHECK_LAUNCH();
    prof_end("wgrad_reduce_kernel", s, pe);
    return TM_OK;
}

extern "C" int tm_wgrad(const tm_wgrad_job *jobs, int32_t n_jobs, const tm_wgrad_target *targets, int32_t n_targets,
                        void *stream) {
    if (!jobs || !targets) return fail(TM_E_ARG, "tm_wgrad: NULL arguments");
    return run_wgrad(jobs, n_jobs, targets, n_targets, S_(stream), "tm_wgrad");
}

extern "C" int tm_encoder_wgrad(const tm_weights *w, int32_t n_groups, int32_t B, int32_t W,
                                const tm_encoder_grad_io *io, const void *workspace, float *const *grads,
                                void *stream) {
    if (!w || !io || !workspace || !grads || n_groups < 0 || B < 0 || W < 0)
        return fail(TM_E_ARG, "tm_encoder_wgrad: bad arguments");
    for (int i = 0; i < TM_N_ENC_GRADS; ++i)
        if (!grads[i]) return fail(TM_E_ARG, "tm_encoder_wgrad: NULL gradient " + std::to_string(i));
    const int64_t n64 = (int64_t)n_groups * B * W;
    if (n64 * 3 * 2 > INT32_MAX) return fail(TM_E_UNSUPPORTED, "tm_encoder_wgrad: too many walks per call");
    const int n = (int)n64, R = 3 * n, h = w->h, h2 = 2 * h, hm = w->P.hm;
    const int dn = w->dn, kev = w->P.kev, KE = r16(kev), DN = r16(dn), KM = r16(hm);
    const float *F = reinterpret_cast<const float *>(workspace);
    // zero node features (gcn_bwd_kernel<true>): one row pair per position for MLP.0 / MLP.2, the branch sums
    const bool zn = w->node_zero;   // both event_gcn backward kernels have the zero-node form
    const tm_wgrad_job zn0{io->dZ, io->AB, 2 * h, 2 * DN, h, dn, R}, zn2{io->dZ + h, io->H, 2 * h, 2 * h, h, h, R};
    const tm_wgrad_job jobs[] = {
        {io->dlev, io->ev, DN, KE, dn, kev, R},            // lin_event
        zn ? zn0 : tm_wgrad_job{io->dZ, io->AB, h, DN, h, dn, 2 * R},   // event_conv.MLP.0
        zn ? zn2 : tm_wgrad_job{io->dF, io->H, h, h, h, h, 2 * R},      // event_conv.MLP.2
        {io->dP, F + 2 * h2, h2, 3 * h2, h2, h2, n},       // attention.W1 (x = F[:, 2])
        {io->dQ, F, h2, 3 * h2, h2, h2, n},                // attention.W2, position 0
        {io->dQ + (int64_t)n * h2, F + h2, h2, 3 * h2, h2, h2, n},   // position 1
        {io->dH1, io->O, h, h2, h, h2, n},                 // attention.MLP.0
        {io->dY2, io->H1d, h, h, h, h, n},                 // attention.MLP.3
        {io->dM1, io->X, KM, KM, hm, hm, n},               // MLP.0
        {io->dM2, io->M1d, h, KM, h, hm, n},               // MLP.3
        {io->dlogit, io->M2, 1, h, 1, h, n},               // MLP.5
        {io->g, io->dt, DN, 1, dn, 1, R},                  // time encoder: freq (x = dt), phase (ones)
    };
    const tm_wgrad_target tgts[] = {{grads[0], grads[1], 0, 1},   {grads[2], grads[3], 1, 1},
                                    {grads[4], grads[5], 2, 1},   {grads[6], grads[7], 3, 1},
                                    {grads[8], grads[9], 4, 2},   {grads[10], grads[11], 6, 1},
                                    {grads[12], grads[13], 7, 1}, {grads[14], grads[15], 8, 1},
                                    {grads[16], grads[17], 9, 1}, {grads[18], grads[19], 10, 1},
                                    {grads[20], grads[21], 11, 1}};
    return run_wgrad(jobs, (int)(sizeof(jobs) / sizeof(jobs[0])), tgts, (int)(sizeof(tgts) / sizeof(tgts[0])),
                     S_(stream), "tm_encoder_wgrad");
}

static int expl_hbits(int W) {
    int hb = 6;
    while ((1 << hb) < 2 * 3 * W) ++hb;
    return hb;
}

static int explain_train_fwd(const tm_weights *w, const float *e_feat, int32_t n_groups, int32_t B, int32_t W,
                             int32_t N, const int32_t *eid3, const float *ts3, const float *imp, const int32_t *sub1_eid,
                             const int32_t *sub2_eid, const uint8_t *keep1, const uint8_t *keep2, float scale1,
                             float scale2, const tm_explain_grad_io *io, float *p1, float *p2, const int32_t *sub1_node,
                             const int32_t *sub2_node, float *pad1, float *pad2, void *stream);

extern "C" int tm_explain_train_fwd(const tm_weights *w, const float *e_feat, int32_t n_groups, int32_t B, int32_t W,
                                    int32_t N, const int32_t *eid3, const float *ts3, const float *imp,
                                    const int32_t *sub1_eid, const int32_t *sub2_eid, const uint8_t *keep1,
                                    const uint8_t *keep2, float scale1, float scale2, const tm_explain_grad_io *io,
                                    float *p1, float *p2, void *stream) {
    return explain_train_fwd(w, e_feat, n_groups, B, W, N, eid3, ts3, imp, sub1_eid, sub2_eid, keep1, keep2, scale1,
                             scale2, io, p1, p2, nullptr, nullptr, nullptr, nullptr, stream);
}

extern "C" int tm_explain_train_fwd_pad(const tm_weights *w, const float *e_feat, int32_t n_groups, int32_t B,
                                        int32_t W, int32_t N, const int32_t *eid3, const float *ts3, const float *imp,
                                        const int32_t *sub1_eid, const int32_t *sub2_eid, const uint8_t *keep1,
                                        const uint8_t *keep2, float scale1, float scale2,
                                        const tm_explain_grad_io *io, float *p1, float *p2,
                                        const int32_t *sub1_node, const int32_t *sub2_node, float *pad1, float *pad2,
                                        void *stream) {
    if (!sub1_node || !sub2_node || !pad1 || !pad2) return fail(TM_E_ARG, "tm_explain_train_fwd_pad: NULL pointer");
    return explain_train_fwd(w, e_feat, n_groups, B, W, N, eid3, ts3, imp, sub1_eid, sub2_eid, keep1, keep2, scale1,
                             scale2, io, p1, p2, sub1_node, sub2_node, pad1, pad2, stream);
}

static int explain_train_fwd(const tm_weights *w, const float *e_feat, int32_t n_groups, int32_t B, int32_t W,
                             int32_t N, const int32_t *eid3, const float *ts3, const float *imp, const int32_t *sub1_eid,
                             const int32_t *sub2_eid, const uint8_t *keep1, const uint8_t *keep2, float scale1,
                             float scale2, const tm_explain_grad_io *io, float *p1, float *p2, const int32_t *sub1_node,
                             const int32_t *sub2_node, float *pad1, float *pad2, void *stream) {
    if (!w || !io || n_groups < 0 || B < 0 || W <= 0 || N <= 0) return fail(TM_E_ARG, "tm_explain_train_fwd: bad arguments");
    const int64_t rows = (int64_t)n_groups * B;
    if (rows == 0) return TM_OK;
    if (!e_feat || !eid3 || !ts3 || !imp || !sub1_eid || !sub2_eid || !p1 || !p2 || !io->X || !io->G1 || !io->G2 ||
        !io->z || !io->gate || !io->t)
        return fail(TM_E_ARG, "tm_explain_train_fwd: NULL pointer");
    const int hb = expl_hbits(W);
    if (hb > 12) return fail(TM_E_UNSUPPORTED, "tm_explain_train_fwd: too many walks per event");
    const EncW &P = w->P;
    hipStream_t s = S_(stream);
    const int64_t R = rows * 3 * W;
    ExplIO o{io->X, io->G1, io->G2, io->z, io->gate, io->d_gate, io->dz, io->dG2, io->dG1, io->g, io->t};
    const size_t lds = sizeof(float) * (TILE_ROWS * (r16(P.kdep) + 8) + TILE_ROWS * (r16(P.h) + 8) + TILE_ROWS * (r16(P.h / 2) + 8));
    if (lds > 160 * 1024) return fail(TM_E_UNSUPPORTED, "tm_explain_train_fwd: LDS budget exceeded");
    hipEvent_t pe = prof_begin(s);
    gate_train_fwd_kernel<<<dim3((unsigned)((R + TILE_ROWS - 1) / TILE_ROWS)), 256, lds, s>>>(
        P, R, e_feat, eid3, ts3, keep1, keep2, scale1, scale2, o);
    TM_CHECK_LAUNCH();
    prof_end("gate_train_fwd_kernel", s, pe);
    pe = prof_begin(s);
    explain_train_kernel<<<dim3((unsigned)rows), 256, 2 * sizeof(int32_t) * (1u << hb), s>>>(
        W, N, hb, eid3, imp, io->gate, sub1_eid, sub2_eid, p1, p2, sub1_node, sub2_node, pad1, pad2);
    TM_CHECK_LAUNCH();
    prof_end("explain_train_kernel", s, pe);
    return TM_OK;
}

extern "C" int tm_explain_train_bwd(const tm_weights *w, int32_t n_groups, int32_t B, int32_t W, int32_t N,
                                    const int32_t *eid3, const float *ts3, const float *imp, const int32_t *sub1_eid,
                                    const int32_t *sub2_eid, const uint8_t *keep1, const uint8_t *keep2, float scale1,
                                    float scale2, const float *dp1, const float *dp2, const tm_explain_grad_io *io,
                                    float *d_imp, float *const *grads, void *stream) {
    (void)ts3;
    if (!w || !io || !grads || n_groups < 0 || B < 0 || W <= 0 || N <= 0)
        return fail(TM_E_ARG, "tm_explain_train_bwd: bad arguments");
    for (int i = 0; i < 8; ++i)
        if (!grads[i]) return fail(TM_E_ARG, "tm_explain_train_bwd: NULL gradient " + std::to_string(i));
    const int64_t rows = (int64_t)n_groups * B;
    if (!eid3 || !imp || !sub1_eid || !sub2_eid || !dp1 || !dp2 || !d_imp || !io->X || !io->G1 || !io->G2 ||
        !io->z || !io->gate || !io->d_gate || !io->dz || !io->dG2 || !io->dG1 || !io->g || !io->t)
        return fail(TM_E_ARG, "tm_explain_train_bwd: NULL pointer");
    const int64_t R64 = rows * 3 * W;
    if (R64 > INT32_MAX) return fail(TM_E_UNSUPPORTED, "tm_explain_train_bwd: too many walk positions");
    const int hb = expl_hbits(W);
    if (hb > 12) return fail(TM_E_UNSUPPORTED, "tm_explain_train_bwd: too many walks per event");
    const EncW &P = w->P;
    hipStream_t s = S_(stream);
    ExplIO o{io->X, io->G1, io->G2, io->z, io->gate, io->d_gate, io->dz, io->dG2, io->dG1, io->g, io->t};
    if (rows > 0) {
        hipEvent_t pe = prof_begin(s);
        explain_train_bwd_kernel<<<dim3((unsigned)rows), 256, 4 * sizeof(int32_t) * (1u << hb), s>>>(
            W, N, hb, eid3, imp, io->gate, sub1_eid, sub2_eid, dp1, dp2, d_imp, io->d_gate);
        TM_CHECK_LAUNCH();
        prof_end("explain_train_bwd_kernel", s, pe);
        if (P.dep) {   // no gate without dependency-aware sampling: d imp is the whole backward
            const size_t lds = sizeof(float) * (TILE_ROWS * (r16(P.h) + 8) + TILE_ROWS * (r16(P.h / 2) + 8));
            pe = prof_begin(s);
            gate_train_bwd_kernel<<<dim3((unsigned)((R64 + TILE_ROWS - 1) / TILE_ROWS)), 256, lds, s>>>(
                P, w->T, R64, keep1, keep2, scale1, scale2, o);
            TM_CHECK_LAUNCH();
            prof_end("gate_train_bwd_kernel", s, pe);
        }
    }
    // without the gate its tensors and the time encoder get no gradient from this path: zero rows below
    const int R = P.dep ? (int)R64 : 0, h = w->h, dn = w->dn, kdep = P.kdep;
    const tm_wgrad_job jobs[] = {
        {io->dG1, io->X, h, r16(kdep), h, kdep, R},        // edge_dependency_gcn.0
        {io->dG2, io->G1, h / 2, h, h / 2, h, R},          // .3
        {io->dz, io->G2, 1, h / 2, 1, h / 2, R},           // .6
        {io->g, io->t, r16(dn), 1, dn, 1, R},              // time encoder: freq (x = t), phase (ones)
    };
    const tm_wgrad_target tgts[] = {{grads[0], grads[1], 0, 1}, {grads[2], grads[3], 1, 1}, {grads[4], grads[5], 2, 1},
                                    {grads[6], grads[7], 3, 1}};
    return run_wgrad(jobs, 4, tgts, 4, s, "tm_explain_train_bwd");
}

// ------------------------------------------------------------------ kl_loss, prior = 'empirical'
// explainer_new.py:432-448 for the G groups of one step (the reference's three per-side calls, summed):
// per (group g, event b) one wave computes, in fp64,
//   p = clamp(prob, 1e-6, 1-1e-6);  s = mean_w p;  m_k = mean_{w: cat=k} p  (0 for an empty category)
//   A = (1-s) log((1-s)/(1-target+1e-6) + 1e-6),  E_k = s m_k log(s m_k/(target null_k + 1e-6) + 1e-6)
// and the event's share of the group's .mean() over the broadcast [B, 12]: (A + mean_k E_k) / B,
// plus d(sum over groups)/d prob for its W walks (zero where the clamp is active), so the loss and
// its whole backward are a few launches instead of ~150 small ones.
__global__ void __launch_bounds__(64) kl_loss_kernel(int32_t B, int32_t W, const float *__restrict__ prob,
                                                     const int32_t *__restrict__ cat,
                                                     const float *__restrict__ null12, float target,
                                                     float *__restrict__ partial, float *__restrict__ dprob) {
    __shared__ double ssum[64], bins[12], dcat[12];
    __shared__ int cnts[12];
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;                 // group * B + event
    const float *p = prob + row * W;
    const int32_t *c = cat + row * W;
    if (tid < 12) {
        bins[tid] = 0.0;
        cnts[tid] = 0;
    }
    __syncthreads();
    double acc = 0.0;
    for (int w = tid; w < W; w += 64) {
        const double v = fmin(fmax((double)p[w], 1e-6), 1.0 - 1e-6);
        acc += v;
        const int k = c[w];
        if (k >= 0 && k < 12) {
            atomicAdd(&bins[k], v);
            atomicAdd(&cnts[k], 1);
        }
    }
    ssum[tid] = acc;
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) {
        if (tid < o) ssum[tid] += ssum[tid + o];
        __syncthreads();
    }
    const double s = ssum[0] / W;
    const double c1 = 1.0 - (double)target + 1e-6;
    const double u = (1.0 - s) / c1 + 1e-6;
    // per-category value and d/d(emp_k), lanes 0..11
    double ek = 0.0, dek = 0.0, mk = 0.0;
    if (tid < 12) {
        mk = cnts[tid] ? bins[tid] / cnts[tid] : 0.0;
        const double emp = s * mk, nk = (double)target * (double)null12[tid] + 1e-6, v = emp / nk + 1e-6;
        ek = emp * log(v);
        dek = log(v) + emp / (v * nk);
    }
    double se = ek, sdm = dek * mk;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
        se += __shfl_xor(se, o, 16);
        sdm += __shfl_xor(sdm, o, 16);
    }
    se = __shfl(se, 0);
    sdm = __shfl(sdm, 0);
    const double a = (1.0 - s) * log(u), dads = -log(u) - (1.0 - s) / (u * c1);
    if (tid == 0) partial[row] = (float)((a + se / 12.0) / B);
    // d/dp_w = (1/W) [dA/ds / B + sum_k dE_k/demp_k m_k / (12 B)] + dE_{c(w)}/demp s / (12 B n_{c(w)})
    const double base = (dads / B + sdm / (12.0 * B)) / W;
    if (tid < 12) dcat[tid] = cnts[tid] ? dek * s / (12.0 * B * cnts[tid]) : 0.0;
    __syncthreads();
    for (int w = tid; w < W; w += 64) {
        const float pw = p[w];
        const int k = c[w];
        double g = base + ((k >= 0 && k < 12) ? dcat[k] : 0.0);
        if (!(pw >= 1e-6f && pw <= 1.f - 1e-6f)) g = 0.0;      // clamp's backward
        dprob[row * W + w] = (float)g;
    }
}

// ------------------------------------------------------------------ Beta rsample glue (explainer_new.py:420-430)
// Beta(clamp(10 p, min=1), clamp(10 (1 - p), min=1)).rsample() as torch evaluates it, minus its chain of small
// launches: the concentrations (and the Dirichlet total) of the [n, 2] Dirichlet torch samples, in one
// launch; and the backward after torch._dirichlet_grad, in one launch.  Same fp32 operations and order as
// torch's autograd graph, so the results are bitwise the torch path's (tests/test_gpu_explain_train.py).
__global__ void beta_params_kernel(int64_t n, const float *__restrict__ p, float2 *__restrict__ conc,
                                   float2 *__restrict__ total) {
#pragma clang fp contract(off)   // torch rounds every product and sum separately: no fma contraction
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float a0 = p[i] * 10.f, b0 = (1.f - p[i]) * 10.f;
        const float a = a0 < 1.f ? 1.f : a0, b = b0 < 1.f ? 1.f : b0;   // clamp(min=1), NaN propagates
        conc[i] = make_float2(a, b);
        const float t = a + b;
        total[i] = make_float2(t, t);
    }
}

// dp from d out (out = x0 * pad), x [n, 2] the Dirichlet sample, d [n, 2] = torch._dirichlet_grad(x, conc, total):
// Dirichlet backward with grad_output (g0, 0), select, clamp (self >= min) and the two scalings
__global__ void beta_rsample_bwd_kernel(int64_t n, const float *__restrict__ g, const float *__restrict__ pad,
                                        const float2 *__restrict__ x, const float2 *__restrict__ d,
                                        const float *__restrict__ p, float *__restrict__ dp) {
#pragma clang fp contract(off)   // ga * 10 + -(gb * 10) would otherwise become one fma (autograd adds two rounded terms)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float g0 = g[i] * pad[i];
        const float2 xv = x[i], dv = d[i];
        const float sx = xv.x * g0 + xv.y * 0.f;
        const float gc0 = dv.x * (g0 - sx), gc1 = dv.y * (0.f - sx);
        const float pv = p[i];
        const float ga = (pv * 10.f >= 1.f) ? gc0 : 0.f;
        const float gb = ((1.f - pv) * 10.f >= 1.f) ? gc1 : 0.f;
        dp[i] = ga * 10.f + -(gb * 10.f);
    }
}

extern "C" int tm_beta_params(const float *p, int64_t n, float *conc, float *total, void *stream) {
    if (n < 0) return fail(TM_E_ARG, "tm_beta_params: bad size");
    if (n == 0) return TM_OK;
    if (!p || !conc || !total) return fail(TM_E_ARG, "tm_beta_params: NULL pointer");
    hipStream_t s = S_(stream);
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    beta_params_kernel<<<grid, 256, 0, s>>>(n, p, reinterpret_cast<float2 *>(conc), reinterpret_cast<float2 *>(total));
    TM_CHECK_LAUNCH();
    return TM_OK;
}

extern "C" int tm_beta_rsample_bwd(const float *g, const float *pad, const float *x, const float *d, const float *p,
                                   int64_t n, float *dp, void *stream) {
    if (n < 0) return fail(TM_E_ARG, "tm_beta_rsample_bwd: bad size");
    if (n == 0) return TM_OK;
    if (!g || !pad || !x || !d || !p || !dp) return fail(TM_E_ARG, "tm_beta_rsample_bwd: NULL pointer");
    hipStream_t s = S_(stream);
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    beta_rsample_bwd_kernel<<<grid, 256, 0, s>>>(n, g, pad, reinterpret_cast<const float2 *>(x),
                                                 reinterpret_cast<const float2 *>(d), p, dp);
    TM_CHECK_LAUNCH();
    return TM_OK;
}

extern "C" int tm_kl_loss(const float *prob, const int32_t *cat, const float *null12, float target, int32_t n_groups,
                          int32_t B, int32_t W, float *partial, float *dprob, void *stream) {
    if (n_groups < 0 || B < 0 || W <= 0) return fail(TM_E_ARG, "tm_kl_loss: bad arguments");
    if (n_groups == 0 || B == 0) return TM_OK;
    if (!prob || !cat || !null12 || !partial || !dprob) return fail(TM_E_ARG, "tm_kl_loss: NULL pointer");
    hipStream_t s = S_(stream);
    hipEvent_t pe = prof_begin(s);
    kl_loss_kernel<<<dim3((unsigned)((int64_t)n_groups * B)), 64, 0, s>>>(B, W, prob, cat, null12, target, partial,
                                                                          dprob);
    TM_CHECK_LAUNCH();
    prof_end("kl_loss_kernel", s, pe);
    return TM_OK;
}
