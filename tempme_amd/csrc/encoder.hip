// TempME motif encoder + edge-importance retrieval on gfx950 (fp32 MFMA, v_mfma_f32_16x16x4_f32).
//
// Reference (dharunm236/TempME, models/explainer_new.py):
//   forward :174-201  event features (:176-179, time :318-330, TimeEncode :45-59), node features
//                     (:343-352), event_gcn x2 (:79-96, lin_event shared), TemporalAwareAttention
//                     (:789-846, batch-global std :828), one-hot category (:308-315), MLP + sigmoid
//   retrieve_edge_imp_node :354-406 (dependency gate :367-386, scatter-max :389, gather :392-393,
//                     beta_sample eval :420-430, padding mask :400-404)
//
// Kernels (one launch each):
//   std_kernel      per group: unbiased std of |cut - t| over the [B,W,2] walk times (f64 accumulate)
//   gcn_kernel      per 32 walk-positions: [E(e)|cnt|cos(dt*w+phi)] -> lin_event -> (A,B) -> MLP -> F rows
//   head_kernel     per 32 walks: W1/W2 attention with temporal scaling, softmax, MLP, one-hot, MLP, sigmoid
//   gate_pos_kernel per 32 walk positions of the call: dependency-gate MLP -> walk_imp
//   explain_hash_kernel  per (group, event): LDS hash scatter-max of walk_imp over the walk edge ids,
//                   gather at subgraph edge ids, Beta mean, node==0 mask
// Every dense projection runs on MFMA with the packed weight stream read from L2 and the
// activations staged in LDS (row stride K16+8 floats: conflict-free ds_read_b128).
#include <algorithm>
#include <atomic>
#include <cstring>
#include <vector>

#include "encoder_common.h"

namespace tmk {

// ------------------------------------------------------------------ std over |cut - t| per group
// sum over the workgroup (fixed order: wave butterflies, then the waves' partials in order)
__device__ __forceinline__ double block_sum(double v, double *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
    for (int k = 0; k < nw; ++k) s += red[k];
    return s;
}

// one 1024-thread workgroup per group; thread w takes walk w's two |cut - t| values (int32 indexing)
__global__ void __launch_bounds__(1024) std_kernel(int32_t B, int32_t W, const double *__restrict__ cut,
                                                   const float *__restrict__ ts3, float *__restrict__ std_out) {
    __shared__ double red[16];
    const int64_t g = blockIdx.x;
    const int32_t nw = B * W;
    const int64_t n = (int64_t)nw * 2;
    const float *t = ts3 + g * (int64_t)nw * 3;
    const double *cg = cut + g * B;
    double s = 0.0;
    for (int32_t w = threadIdx.x; w < nw; w += blockDim.x) {
        const float c = (float)cg[w / W];
        s += (double)fabsf(c - t[w * 3]) + (double)fabsf(c - t[w * 3 + 1]);
    }
    const double mean = block_sum(s, red) / (double)n;
    double v = 0.0;
    for (int32_t w = threadIdx.x; w < nw; w += blockDim.x) {
        const float c = (float)cg[w / W];
        const double d0 = (double)fabsf(c - t[w * 3]) - mean, d1 = (double)fabsf(c - t[w * 3 + 1]) - mean;
        v += d0 * d0 + d1 * d1;
    }
    const double var = block_sum(v, red);
    if (threadIdx.x == 0) std_out[g] = n > 1 ? (float)sqrt(var / (double)(n - 1)) : __builtin_nanf("");
}

// std_kernel for one group whose B <= 256 cut times come as a kernel argument (tm_dropin_forward): the same
// sums in the same order as std_kernel, and the cut times written to cut_out for the kernels that follow
// on the stream
struct CutArg {
    double v[256];
};

// Launched with 1 + ceil(n_pos / 1024) workgroups when the drop-in's gate-factor cache is on: workgroups 1.. are
// gate_cache_lookup's (1024 walk positions each), and workgroup 0 also zeroes the miss counter of the side's next
// call (the counters alternate per call, so this call's lookup and gate kernels keep theirs).  B = 0: no cut times.
__device__ __forceinline__ void gate_cache_lookup(int64_t i, const int32_t *__restrict__ eid, const float *__restrict__ ts,
                                                  const unsigned long long *__restrict__ cache, int64_t n_cache,
                                                  float *__restrict__ gf, int32_t *__restrict__ list,
                                                  uint32_t *__restrict__ list_n, int64_t n_pos);
struct GateLookup {
    int64_t n_pos, n_cache;
    const int32_t *eid;
    const float *ts;
    const unsigned long long *cache;
    float *gf;
    int32_t *list;
    uint32_t *cnt, *cnt_next;
};

// workgroup 0's part: the cut times to cut_out and the group's std
__device__ __forceinline__ void std_cut_body(int32_t B, int32_t W, const CutArg &c, const float *__restrict__ ts3,
                                             double *__restrict__ cut_out, float *__restrict__ std_out, int32_t do_std,
                                             const GateLookup &gl) {
    __shared__ double red[16];
    if (threadIdx.x == 0 && gl.cnt_next) *gl.cnt_next = 0u;
    if ((int)threadIdx.x < B) cut_out[threadIdx.x] = c.v[threadIdx.x];
    if (!do_std || B == 0) return;
    const int32_t nw = B * W;
    const int64_t n = (int64_t)nw * 2;
    double s = 0.0, v = 0.0, mean;
    constexpr int SR = 16;                              // walks per thread held in registers
    if (nw <= SR * (int32_t)blockDim.x) {
        // every |cut - t| of the thread requested at once (one memory latency, not one per walk), kept for the
        // second pass; the same walks per thread and the same sums in the same order as below
        float a0[SR], a1[SR];
#pragma unroll
        for (int k = 0; k < SR; ++k) {
            const int32_t w = (int32_t)threadIdx.x + k * (int32_t)blockDim.x;
            a0[k] = a1[k] = 0.f;
            if (w < nw) {
                const float cc = (float)c.v[w / W];
                a0[k] = fabsf(cc - ts3[w * 3]);
                a1[k] = fabsf(cc - ts3[w * 3 + 1]);
            }
        }
#pragma unroll
        for (int k = 0; k < SR; ++k)
            if ((int32_t)threadIdx.x + k * (int32_t)blockDim.x < nw) s += (double)a0[k] + (double)a1[k];
        mean = block_sum(s, red) / (double)n;
#pragma unroll
        for (int k = 0; k < SR; ++k)
            if ((int32_t)threadIdx.x + k * (int32_t)blockDim.x < nw) {
                const double d0 = (double)a0[k] - mean, d1 = (double)a1[k] - mean;
                v += d0 * d0 + d1 * d1;
            }
    } else {
        for (int32_t w = threadIdx.x; w < nw; w += blockDim.x) {
            const float cc = (float)c.v[w / W];
            s += (double)fabsf(cc - ts3[w * 3]) + (double)fabsf(cc - ts3[w * 3 + 1]);
        }
        mean = block_sum(s, red) / (double)n;
        for (int32_t w = threadIdx.x; w < nw; w += blockDim.x) {
            const float cc = (float)c.v[w / W];
            const double d0 = (double)fabsf(cc - ts3[w * 3]) - mean, d1 = (double)fabsf(cc - ts3[w * 3 + 1]) - mean;
            v += d0 * d0 + d1 * d1;
        }
    }
    const double var = block_sum(v, red);
    if (threadIdx.x == 0) std_out[0] = n > 1 ? (float)sqrt(var / (double)(n - 1)) : __builtin_nanf("");
}

__global__ void __launch_bounds__(1024) std_cut_kernel(int32_t B, int32_t W, CutArg c, const float *__restrict__ ts3,
                                                       double *__restrict__ cut_out, float *__restrict__ std_out,
                                                       int32_t do_std, GateLookup gl) {
    if (blockIdx.x > 0) {
        gate_cache_lookup((int64_t)(blockIdx.x - 1) * blockDim.x + threadIdx.x, gl.eid, gl.ts, gl.cache, gl.n_cache, gl.gf,
                          gl.list, gl.cnt, gl.n_pos);
        return;
    }
    std_cut_body(B, W, c, ts3, cut_out, std_out, do_std, gl);
}

// ------------------------------------------------------------------ event_gcn: 32 walk-positions per block
// F[row] = [MLP(x_s + relu(x_t + L)) | MLP(x_t + relu(x_s + L))],  L = lin_event([E(e) | cnt | cos(dt)])
// ZN (zero node features, tm_weights_set_node_zero): A = B, so MLP.0 / MLP.2 run on the 32 A rows and both halves
// of F get the same (bit-identical) values
template <bool ZN = false>
__global__ void __launch_bounds__(256) gcn_kernel(EncW P, int64_t n_rows, const float *__restrict__ n_feat,
                                                  const float *__restrict__ e_feat, const int32_t *__restrict__ node6,
                                                  const int32_t *__restrict__ eid3, const float *__restrict__ ts3,
                                                  const float *__restrict__ cnt, float *__restrict__ F) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int de = P.de, dn = P.dn, kev = P.kev, kev16 = r16(kev), dn16 = r16(dn);
    const int h = P.h, ldx = kev16 + 8, ldab = dn16 + 8, ldh = r16(h) + 8;
    const int xsz = max(TILE_ROWS * ldx, 2 * TILE_ROWS * ldh);
    float *X = smem;                                  // [32][ldx]      event features
    float *AB = X + xsz;                              // [64][ldab]     A rows 0..31, B rows 32..63
    float *H = X;                                     // [64][ldh]      aliases X after lin_event
    __shared__ int32_t s_eid[TILE_ROWS], s_ns[TILE_ROWS], s_nt[TILE_ROWS];
    __shared__ float s_dt[TILE_ROWS], s_cnt[TILE_ROWS * 3];
    const int64_t row0 = (int64_t)blockIdx.x * TILE_ROWS;
    const int tid = threadIdx.x;
    if (tid < TILE_ROWS) {
        const int64_t r = row0 + tid;
        if (r < n_rows) {
            const int64_t w = r / 3;
            const int p = (int)(r % 3);
            s_eid[tid] = eid3[w * 3 + p];
            s_ns[tid] = node6[w * 6 + 2 * p];       // src nodes: columns 0, 2, 4 (:348)
            s_nt[tid] = node6[w * 6 + 2 * p + 1];   // tgt nodes: columns 1, 3, 5 (:349)
            s_dt[tid] = ts3[w * 3 + 2] - ts3[w * 3 + p];   // relative to walk position 2 (:326)
            for (int q = 0; q < 3; ++q) s_cnt[tid * 3 + q] = cnt[w * 9 + p * 3 + q];
        } else {
            s_eid[tid] = 0; s_ns[tid] = 0; s_nt[tid] = 0; s_dt[tid] = 0.f;
            for (int q = 0; q < 3; ++q) s_cnt[tid * 3 + q] = 0.f;
        }
    }
    __syncthreads();
    for (int i = tid; i < TILE_ROWS * kev16; i += blockDim.x) {
        const int r = i / kev16, c = i % kev16;
        float v = 0.f;
        if (row0 + r < n_rows) {
            if (c < de) v = e_feat[(int64_t)s_eid[r] * de + c];
            else if (c < de + 3) v = s_cnt[r * 3 + (c - de)];
            else if (c < kev) v = time_cos(s_dt[r], P.freq[c - de - 3], P.phase[c - de - 3]);
        }
        X[r * ldx + c] = v;
    }
    __syncthreads();
    // L = lin_event(X); A = x_s + relu(x_t + L); B = x_t + relu(x_s + L)
    gemm<2>(X, ldx, P.ev, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            float a = 0.f, b = 0.f;
            if (c < dn) {
                const float L = acc[r] + P.ev.b[c];
                const float xs = ZN ? 0.f : n_feat[(int64_t)s_ns[row] * dn + c];
                const float xt = ZN ? 0.f : n_feat[(int64_t)s_nt[row] * dn + c];
                a = xs + relu(xt + L);
                b = xt + relu(xs + L);
            }
            AB[row * ldab + c] = a;
            if (!ZN) AB[(row + TILE_ROWS) * ldab + c] = b;
        }
    });
    __syncthreads();
    auto g1_epi = [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) H[erow(mt, r) * ldh + c] = relu(acc[r] + P.g1.b[c]);
    };
    if constexpr (ZN) gemm<2>(AB, ldab, P.g1, g1_epi);
    else gemm<4>(AB, ldab, P.g1, g1_epi);
    __syncthreads();
    auto g2_epi = [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            const int rr = row & (TILE_ROWS - 1), half = row >> 5;
            const int64_t gr = row0 + rr;
            if (gr < n_rows && c < h) {
                const float v = acc[r] + P.g2.b[c];
                F[gr * (2 * h) + half * h + c] = v;
                if (ZN) F[gr * (2 * h) + h + c] = v;
            }
        }
    };
    if constexpr (ZN) gemm<2>(H, ldh, P.g2, g2_epi);
    else gemm<4>(H, ldh, P.g2, g2_epi);
}

// ------------------------------------------------------------------ attention head + final MLP: TR walks per block
// TR = 32, or 16 where the 32-walk tiles exceed the LDS (hid_dim above 152)
template <int TR>
__global__ void __launch_bounds__(256) head_kernel(EncW P, int64_t n_walks, int64_t walks_per_group, int32_t W,
                                                   const float *__restrict__ F, const float *__restrict__ ts3,
                                                   const double *__restrict__ cut, const int32_t *__restrict__ cat,
                                                   const float *__restrict__ stdv, float *__restrict__ out,
                                                   const uint8_t *__restrict__ drop = nullptr, float dscale = 1.f) {
    // drop (training forward, nullable): keep-masks [n_walks][DROP_COLS]; kept values are scaled by dscale
    static_assert(TR == 32 || TR == 16, "head_kernel: 16 or 32 walks per workgroup");
    constexpr int MT1 = TR / 16, MT2 = TR / 8;   // row tiles of TR and 2 TR rows
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int h = P.h, D2 = 2 * h, LD = D2 + 8, LDM = r16(P.hm) + 8, LDH = r16(h) + 8;
    float *T = smem;                  // [64][LD]  positions 0,1 (rows p*32 + w)  -> later S, P
    float *Q = T + 2 * TR * LD;  // [64][LD]  W2(tgt)
    float *S = T;                     // [32][LD]  position 2
    float *Pp = T + TR * LD;   // [32][LD]  W1(src) -> later O
    float *H1 = Q;                    // [32][LDH]
    float *X = S;                     // [32][LDM]
    float *M1 = Pp;                   // [32][LDM]
    float *M2 = Q;                    // [32][LDH]
    __shared__ float s_score[TR * 2], s_tw[TR * 2], s_alpha[TR * 2];
    __shared__ int32_t s_cat[TR];
    const int64_t w0 = (int64_t)blockIdx.x * TR;
    const int tid = threadIdx.x;
    // stage positions 0,1
    for (int i = tid; i < 2 * TR * (D2 / 4); i += blockDim.x) {
        const int row = i / (D2 / 4), c4 = i % (D2 / 4), p = row / TR, w = row % TR;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (w0 + w < n_walks) v = reinterpret_cast<const float4 *>(F + ((w0 + w) * 3 + p) * D2)[c4];
        *reinterpret_cast<float4 *>(T + row * LD + 4 * c4) = v;
    }
    if (tid < TR * 2) {
        const int w = tid >> 1, p = tid & 1;
        const int64_t gw = w0 + w;
        float tw = 0.f;
        if (gw < n_walks) {
            const int64_t g = gw / walks_per_group, b = (gw % walks_per_group) / W;
            const float c = (float)cut[g * (walks_per_group / W) + b];
            const float diff = fabsf(c - ts3[gw * 3 + p]);
            tw = P.tg ? expf(-diff / (stdv[g] + 1e-6f)) : 1.f;   // plain Attention: 0.7 + 0.3 * 1 == 1 exactly
        }
        s_tw[tid] = tw;
    }
    if (tid < TR) s_cat[tid] = (w0 + tid < n_walks) ? cat[w0 + tid] : -1;
    __syncthreads();
    gemm<MT2>(T, LD, P.w2, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) Q[erow(mt, r) * LD + c] = acc[r] + P.w2.b[c];
    });
    __syncthreads();
    // stage position 2 into S (T is dead)
    for (int i = tid; i < TR * (D2 / 4); i += blockDim.x) {
        const int w = i / (D2 / 4), c4 = i % (D2 / 4);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (w0 + w < n_walks) v = reinterpret_cast<const float4 *>(F + ((w0 + w) * 3 + 2) * D2)[c4];
        *reinterpret_cast<float4 *>(S + w * LD + 4 * c4) = v;
    }
    __syncthreads();
    gemm<MT1>(S, LD, P.w1, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) Pp[erow(mt, r) * LD + c] = acc[r] + P.w1.b[c];
    });
    __syncthreads();
    // scores[w][p] = <W1 src, W2 tgt_p>, 4 lanes per dot product
    {
        const int pair = tid >> 2, sub = tid & 3, w = pair >> 1, p = pair & 1;
        const int cend = w < TR ? D2 : 0;   // lane groups past TR walks sum nothing
        float s = 0.f;
        for (int c = sub; c < cend; c += 4) s += Pp[w * LD + c] * Q[(p * TR + w) * LD + c];
        s += __shfl_xor(s, 1, 4);
        s += __shfl_xor(s, 2, 4);
        if (sub == 0 && w < TR) {
            // scores * (1.0 - 0.3 + 0.3 * time_weight)   (:835-836)
            const float m = __fadd_rn(0.7f, __fmul_rn(0.3f, s_tw[pair]));
            s_score[pair] = s * m;
        }
    }
    __syncthreads();
    if (tid < TR) {
        const float s0 = s_score[2 * tid], s1 = s_score[2 * tid + 1], mx = fmaxf(s0, s1);
        const float e0 = expf(s0 - mx), e1 = expf(s1 - mx), sum = e0 + e1;
        float a0 = e0 / sum, a1 = e1 / sum;
        if (drop && P.tg) {   // alpha = self.dropout(alpha)  (:839); the plain Attention has no dropout
            const uint8_t *dm = drop + (w0 + tid < n_walks ? w0 + tid : 0) * drop_cols(h, P.hm) + DROP_A;
            a0 = dm[0] ? a0 * dscale : 0.f;
            a1 = dm[1] ? a1 * dscale : 0.f;
        }
        s_alpha[2 * tid] = a0;
        s_alpha[2 * tid + 1] = a1;
    }
    __syncthreads();
    // O = src + alpha . Wq   (into Pp)
    for (int i = tid; i < TR * D2; i += blockDim.x) {
        const int w = i / D2, c = i % D2;
        const float o = s_alpha[2 * w] * Q[w * LD + c] + s_alpha[2 * w + 1] * Q[(TR + w) * LD + c];
        Pp[w * LD + c] = S[w * LD + c] + o;
    }
    __syncthreads();
    gemm<MT1>(Pp, LD, P.a1, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            float v = relu(acc[r] + P.a1.b[c]);
            if (drop && P.tg)   // TemporalAwareAttention.MLP's Dropout (:780); Attention.MLP has none (:18)
                v = drop[(w0 + row < n_walks ? w0 + row : 0) * drop_cols(h, P.hm) + DROP_H + c] ? v * dscale : 0.f;
            H1[row * LDH + c] = v;
        }
    });
    __syncthreads();
    // X = [attention MLP out | one-hot(cat)]
    gemm<MT1>(H1, LDH, P.a2, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) X[erow(mt, r) * LDM + c] = acc[r] + P.a2.b[c];
    });
    if (P.cat) {   // one-hot category after the attention output (compute_catogory_feautres :308-315)
        for (int i = tid; i < TR * 16; i += blockDim.x) {
            const int w = i >> 4, c = i & 15;
            X[w * LDM + h + c] = (c < 12 && s_cat[w] == c) ? 1.f : 0.f;
        }
    }
    __syncthreads();
    gemm<MT1>(X, LDM, P.m1, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) {
            const int row = erow(mt, r);
            float v = c < P.m1.nout ? relu(acc[r] + P.m1.b[c]) : 0.f;
            if (drop && c < P.m1.nout)
                v = drop[(w0 + row < n_walks ? w0 + row : 0) * drop_cols(h, P.hm) + DROP_H + h + c] ? v * dscale : 0.f;
            M1[row * LDM + c] = v;
        }
    });
    __syncthreads();
    gemm<MT1>(M1, LDM, P.m2, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) M2[erow(mt, r) * LDH + c] = relu(acc[r] + P.m2.b[c]);
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
        if (sub == 0 && w < TR && w0 + w < n_walks) {
            const float z = s + P.m3b[0];
            out[w0 + w] = 1.f / (1.f + expf(-z));
        }
    }
}

// ------------------------------------------------------------------ edge importance: one block per (group, event)
__device__ __forceinline__ uint32_t hash_eid(int32_t e) { return (uint32_t)e * 0x9E3779B1u; }

// Per walk position, 32 flattened (group, event, position) rows per workgroup: the dependency gate
// (:367-386) on MFMA from LDS tiles and walk_imp = graphlet_imp * (0.5 + 0.5 * gate) (:364, :386).  A
// launch covers every position of the call, so a single reference batch (3 W x B positions) still fills
// the chip; the per-(group, event) scatter-max and gather follow in explain_hash_kernel.
__global__ void __launch_bounds__(256) gate_pos_kernel(EncW P, int64_t n_rows, int32_t W,
                                                       const float *__restrict__ e_feat,
                                                       const int32_t *__restrict__ eid3, const float *__restrict__ ts3,
                                                       const float *__restrict__ imp, float *__restrict__ wv) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int de = P.de, kdep = P.kdep, kd16 = r16(kdep), ldx = kd16 + 8, ldg = r16(P.h) + 8, ldg2 = r16(P.h / 2) + 8;
    float *X = smem;                       // [32][ldx]
    float *G1 = X + TILE_ROWS * ldx;       // [32][ldg]
    float *G2 = G1 + TILE_ROWS * ldg;      // [32][ldg2]
    __shared__ int32_t s_eid[TILE_ROWS];
    __shared__ float s_t[TILE_ROWS];
    const int tid = threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.x * TILE_ROWS;
    const int64_t W3 = 3 * (int64_t)W;
    if (!P.dep) {                          // no dependency gate (tm_weights_variant): walk_imp = graphlet_imp
        if (tid < TILE_ROWS && c0 + tid < n_rows) {
            const int64_t r = c0 + tid;
            wv[r] = imp ? imp[(r / W3) * W + (r % W3) / 3] : 1.f;
        }
        return;
    }
    if (tid < TILE_ROWS) {
        const int64_t r = c0 + tid;
        s_eid[tid] = r < n_rows ? eid3[r] : 0;
        s_t[tid] = r < n_rows ? ts3[r] : 0.f;   // raw event time (:371), not dt
    }
    __syncthreads();
    for (int i = tid; i < TILE_ROWS * kd16; i += blockDim.x) {
        const int r = i / kd16, c = i % kd16;
        float v = 0.f;
        if (c0 + r < n_rows) {
            if (c < de) v = e_feat[(int64_t)s_eid[r] * de + c];
            else if (c < kdep) v = time_cos(s_t[r], P.freq[c - de], P.phase[c - de]);
        }
        X[r * ldx + c] = v;
    }
    __syncthreads();
    gemm<2>(X, ldx, P.d1, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) G1[erow(mt, r) * ldg + c] = relu(acc[r] + P.d1.b[c]);
    });
    __syncthreads();
    gemm<2>(G1, ldg, P.d2, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) G2[erow(mt, r) * ldg2 + c] = relu(acc[r] + P.d2.b[c]);
    });
    __syncthreads();
    const int r = tid >> 3, sub = tid & 7;
    const float sc = gate_logit_lds(G2 + r * ldg2, P.d3w, sub, P.h / 2);
    const int64_t gr = c0 + r;
    if (sub == 0 && gr < n_rows) {
        const float gate = 1.f / (1.f + expf(-(sc + P.d3b[0])));
        // imp == nullptr: the gate factor alone (tm_dropin_forward), multiplied by graphlet_imp later in
        // explain_hash_kernel -- the same two roundings in the same order
        const float fac = 0.5f + 0.5f * gate;
        wv[gr] = imp ? imp[(gr / W3) * W + (gr % W3) / 3] * fac : fac;
    }
}

// One workgroup per (group, event): scatter-max of the 3 W walk_imp values onto their edge ids (LDS
// open-addressing table; atomicMax on the float bits, values >= 0), then the gather at the subgraph's
// hop-1 / hop-2 edge ids, the Beta mean (eval) and the padding mask (:388-406, :420-430).
__device__ __forceinline__ void explain_hash_row(int64_t ge, int32_t W, int32_t N, int32_t hbits,
                                                 const int32_t *__restrict__ eid3, const float *__restrict__ wv,
                                                 const float *__restrict__ imp, const int32_t *__restrict__ sub1_node,
                                                 const int32_t *__restrict__ sub1_eid,
                                                 const int32_t *__restrict__ sub2_node,
                                                 const int32_t *__restrict__ sub2_eid, float *__restrict__ out1,
                                                 float *__restrict__ out2, float *__restrict__ keep1 = nullptr,
                                                 float *__restrict__ keep2 = nullptr) {
    extern __shared__ __attribute__((aligned(16))) int32_t hsm[];
    const int hsize = 1 << hbits;
    int32_t *hkey = hsm;
    uint32_t *hval = reinterpret_cast<uint32_t *>(hkey + hsize);
    const int tid = threadIdx.x, nrow = 3 * W;
    for (int i = tid; i < hsize; i += blockDim.x) {
        hkey[i] = -1;
        hval[i] = 0u;
    }
    __syncthreads();
    for (int i = tid; i < nrow; i += blockDim.x) {
        const int32_t key = eid3[ge * nrow + i];
        // wv = walk_imp, or (imp != nullptr) the gate factor of tm_dropin_forward times graphlet_imp
        const float v = imp ? imp[ge * W + i / 3] * wv[ge * nrow + i] : wv[ge * nrow + i];
        uint32_t h = hash_eid(key) >> (32 - hbits);
        while (true) {
            const int32_t prev = atomicCAS(&hkey[h], -1, key);
            if (prev == -1 || prev == key) break;
            h = (h + 1) & (hsize - 1);
        }
        atomicMax(&hval[h], __float_as_uint(v));   // v >= 0: uint order == float order
    }
    __syncthreads();
    // gather at the subgraph edge ids, Beta mean (eval), padding mask
    const int n1 = N, n2 = N * N;
    for (int i = tid; i < n1 + n2; i += blockDim.x) {
        const bool h1 = i < n1;
        const int64_t o = h1 ? ge * n1 + i : ge * n2 + (i - n1);
        const int32_t key = h1 ? sub1_eid[o] : sub2_eid[o];
        const int32_t nd = h1 ? sub1_node[o] : sub2_node[o];
        uint32_t h = hash_eid(key) >> (32 - hbits);
        float p = 0.f;   // edges no walk touched: scatter fill value 0
        while (true) {
            const int32_t k = hkey[h];
            if (k == key) {
                p = __uint_as_float(hval[h]);
                break;
            }
            if (k == -1) break;
            h = (h + 1) & (hsize - 1);
        }
        if (keep1) {   // training=True (beta_sample's rsample follows in torch): p and the padding mask
            if (h1) {
                out1[o] = p;
                keep1[o] = nd == 0 ? 0.f : 1.f;
            } else {
                out2[o] = p;
                keep2[o] = nd == 0 ? 0.f : 1.f;
            }
            continue;
        }
        const float a = fmaxf(p * 10.f, 1.f), b = fmaxf((1.f - p) * 10.f, 1.f);
        const float v = nd == 0 ? 0.f : a / (a + b);
        if (h1) out1[o] = v;
        else out2[o] = v;
    }
}

__global__ void __launch_bounds__(256) explain_hash_kernel(int32_t W, int32_t N, int32_t hbits,
                                                           const int32_t *__restrict__ eid3,
                                                           const float *__restrict__ wv,
                                                           const float *__restrict__ imp,
                                                           const int32_t *__restrict__ sub1_node,
                                                           const int32_t *__restrict__ sub1_eid,
                                                           const int32_t *__restrict__ sub2_node,
                                                           const int32_t *__restrict__ sub2_eid,
                                                           float *__restrict__ out1, float *__restrict__ out2) {
    explain_hash_row(blockIdx.x, W, N, hbits, eid3, wv, imp, sub1_node, sub1_eid, sub2_node, sub2_eid, out1, out2);
}

// the three sides of one reference batch in one launch (retrieve_explanation), each side's inputs at
// their own addresses (device-pack views), the outputs concatenated [3 B, N] / [3 B, N^2]
struct ExplainSides {
    const float *gf[3], *imp[3];
    const int32_t *eid3[3], *s1n[3], *s1e[3], *s2n[3], *s2e[3];
};

__global__ void __launch_bounds__(256) explain_hash3_kernel(ExplainSides a, int32_t B, int32_t W, int32_t N,
                                                            int32_t hbits, float *__restrict__ out1,
                                                            float *__restrict__ out2, float *__restrict__ keep1,
                                                            float *__restrict__ keep2) {
    const int s = blockIdx.x / B;
    // per-side pointers shifted so that row index (s B + b) addresses row b of side s
    const int64_t sh = (int64_t)s * B;
    explain_hash_row(blockIdx.x, W, N, hbits, a.eid3[s] - sh * 3 * W, a.gf[s] - sh * 3 * W, a.imp[s] - sh * W,
                     a.s1n[s] - sh * N, a.s1e[s] - sh * N, a.s2n[s] - sh * N * N, a.s2e[s] - sh * N * N, out1, out2,
                     keep1, keep2);
}

// ------------------------------------------------------------------ fused register-resident walk encoder
// Weights are the MFMA A operand (16 output features per tile, packed as above); activations are
// the B operand with one walk position per column: lane l holds features 16q + 4(l>>4) + {0..3} of
// column l&15.  The D tile of one layer is then exactly the B fragment of K-step q = tile of the
// next layer, so the whole chain stays in registers.  A wave owns 16 hop-1 slots (columns):
// position 2 (shared by the M walks of a slot: same e1, t1, v1, root, edge counts, dt = 0) is
// encoded once per slot, positions 0/1 once per walk.
#define TM_W_ADDR(i) ((((i) / NQ) * nq + ((i) % NQ)) * 64)

// two column sets through the same weights (one weight load feeds both)
template <int NTO, int NQ>
__device__ __forceinline__ void rgemm2(const Lin &L, const floatx4 (&x)[NQ], const floatx4 (&y)[NQ],
                                       floatx4 (&o)[NTO], floatx4 (&p)[NTO]) {
    const auto wr = wrsrc(L.w);
    const int vo = lane_id() * 16;
    constexpr int nq = NQ;
    constexpr int N = NTO * NQ, D = PF < N ? PF : N;
#pragma unroll
    for (int t = 0; t < NTO; ++t) {
        o[t] = floatx4{0.f, 0.f, 0.f, 0.f};
        p[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    float4 buf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) buf[i] = wload(wr, vo, TM_W_ADDR(i));
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int t = i / NQ, q = i % NQ;
        const float4 w = buf[i % D];
        if (i + D < N) buf[i % D] = wload(wr, vo, TM_W_ADDR(i + D));
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, x[q].x, o[t], 0, 0, 0);
        p[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, y[q].x, p[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, x[q].y, o[t], 0, 0, 0);
        p[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, y[q].y, p[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, x[q].z, o[t], 0, 0, 0);
        p[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, y[q].z, p[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, x[q].w, o[t], 0, 0, 0);
        p[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, y[q].w, p[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Weight layout of the fused walk kernel (hid_dim 64, 11 node-feature tiles): float offsets into
// tm_weights::buf -- the folded region (FoldLay) first, then the reference layers in
// tm_weights_create's order; compile-time for a kernel instance (NQE = lin_event's K steps), so every
// weight fragment is one buffer load off a single resource with a constant offset.  The host checks the
// live pointers against it before the launch (walk_layout_ok).
template <int NQE>
struct WalkLay {
    static constexpr int EV = FoldLay::SIZE, EVB = EV + 11 * NQE * 256, G1 = EVB + 176, G1B = G1 + 4 * 11 * 256,
                         G2 = G1B + 64, G2B = G2 + 4 * 4 * 256, W1 = G2B + 64, W1B = W1 + 8 * 8 * 256, W2 = W1B + 128,
                         W2B = W2 + 8 * 8 * 256, A1 = W2B + 128, A1B = A1 + 4 * 8 * 256, A2 = A1B + 64,
                         A2B = A2 + 4 * 4 * 256, M1 = A2B + 64, M1B = M1 + 5 * 5 * 256, M2 = M1B + 80,
                         M2B = M2 + 4 * 5 * 256;
};

// out[t] += W tile t * x over the K steps [0, NQ) of a pack with NQL K steps at float offset BASE (the
// caller initialises out: bias rows from LDS, a table row, or zero); weights streamed PFP fragments ahead.
// Fragments go in tile pairs (t, t+1) with the K steps inside and the pair's two fragments' MFMAs
// interleaved, so no MFMA waits on the one before it (v_mfma_f32_16x16x4_f32: 32-cycle issue, 40-cycle
// dependent-accumulator latency); an odd last tile runs alone.  Each tile still accumulates its K steps
// in the same order (the results do not change).
constexpr int PFP = 4;     // weight-fragment ring depth (2, 4, 6 measured: 4 best)
// waves per SIMD walk_kernel is compiled for, and waves per workgroup (each wave owns its 16 slots and a
// 12.25 KB LDS stash, the workgroup one constant table; 3 waves per SIMD and 8-wave workgroups measured slower)
constexpr int WALK_WAVES = 2;
constexpr int WALK_WPB = 4;

template <int NTO, int NQ, int NQL, int BASE>
__device__ __forceinline__ void cgemm(__amdgpu_buffer_rsrc_t wr, const floatx4 (&x)[NQ], floatx4 (&o)[NTO]) {
    using O = PairOrder<NTO, NQ>;
    const int vo = lane_id() * 16;
    constexpr int N = NTO * NQ, D = PFP < N ? PFP : N;
    auto off = [](int i) { return BASE / 4 + (O::t(i) * NQL + O::q(i)) * 64; };
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

// Cross-phase weight prefetch: every GEMM phase of a pass starts with its first PFP fragments already in
// registers.  The previous phase loads them into its ring slots as they free up (its last PFP refills), so
// the L2 latency of a phase's first fragments overlaps the previous phase's MFMAs instead of stalling at
// every phase start; the pass's last GEMM prefetches the next pass's lin_event fragments.
static_assert(PFP == 4, "the phase hand-off carries 4 fragments (pair order: (t0,q0) (t1,q0) (t0,q1) (t1,q1))");
struct NextFr {
    int o[PFP];   // float4 offsets of the next phase's first PFP fragments (wave-uniform)
};
// fragment k < 4 of a cgemm in pair order, pack with NQL K steps at float4 offset base
template <int NQL>
__device__ __forceinline__ NextFr pair_first(int base) {
    return NextFr{{base, base + NQL * 64, base + 64, base + NQL * 64 + 64}};
}

// cgemm whose first PFP fragments come in `pre`; on return `pre` holds the next phase's first PFP fragments
// (nx), loaded into the ring slots of this GEMM's last PFP fragments
template <int NTO, int NQ, int NQL, int BASE>
__device__ __forceinline__ void cgemm_p(__amdgpu_buffer_rsrc_t wr, const floatx4 (&x)[NQ], floatx4 (&o)[NTO],
                                        float4 (&pre)[PFP], const NextFr &nx) {
    using O = PairOrder<NTO, NQ>;
    const int vo = lane_id() * 16;
    constexpr int N = NTO * NQ, D = PFP;
    static_assert(N >= D, "a phase shorter than the ring");
    auto off = [](int i) { return BASE / 4 + (O::t(i) * NQL + O::q(i)) * 64; };
    float4 buf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) buf[i] = pre[i];
    auto refill = [&](int i) {   // slot i % D: fragment i + D of this GEMM, else the next phase's
        if (i + D < N) buf[i % D] = wload(wr, vo, off(i + D));
        else buf[i % D] = wload(wr, vo, nx.o[i + D - N]);
    };
#pragma unroll
    for (int k = 0; k < O::NP * NQ; ++k) {
        const int i = 2 * k, t = O::t(i), q = O::q(i);
        const float4 w0 = buf[i % D];
        refill(i);
        const float4 w1 = buf[(i + 1) % D];
        refill(i + 1);
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
            refill(i);
            o[NTO - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, x[q].x, o[NTO - 1], 0, 0, 0);
            o[NTO - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, x[q].y, o[NTO - 1], 0, 0, 0);
            o[NTO - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, x[q].z, o[NTO - 1], 0, 0, 0);
            o[NTO - 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, x[q].w, o[NTO - 1], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int k = 0; k < D; ++k) pre[k] = buf[(N + k) % D];
}

// two column sets through the same weight fragments (one load feeds 8 MFMAs)
template <int NTO, int NQ, int BASE>
__device__ __forceinline__ void cgemm2(__amdgpu_buffer_rsrc_t wr, const floatx4 (&x)[NQ], const floatx4 (&y)[NQ],
                                       floatx4 (&o)[NTO], floatx4 (&p)[NTO]) {
    const int vo = lane_id() * 16;
    constexpr int N = NTO * NQ, D = PF < N ? PF : N;
    float4 buf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) buf[i] = wload(wr, vo, BASE / 4 + i * 64);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int t = i / NQ, q = i % NQ;
        const float4 w = buf[i % D];
        if (i + D < N) buf[i % D] = wload(wr, vo, BASE / 4 + (i + D) * 64);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, x[q].x, o[t], 0, 0, 0);
        p[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, y[q].x, p[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, x[q].y, o[t], 0, 0, 0);
        p[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, y[q].y, p[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, x[q].z, o[t], 0, 0, 0);
        p[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, y[q].z, p[t], 0, 0, 0);
        o[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, x[q].w, o[t], 0, 0, 0);
        p[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, y[q].w, p[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Per-workgroup LDS table of the small per-feature vectors the walk kernel reads: accumulator
// initialisers (biases, folded constant vectors, the category table), the last MLP row, and the time
// encoder's frequency and phase laid out on the event-feature axis k (zero outside the time block), so
// they are ds_reads (broadcast within a lane group; no VALU work), not L2 loads.  G1 and G1C hold the
// same bias (two copies: the two branches' accumulators are initialised by two reads, not a read and
// four register moves).
template <int NQE, int NTD>
struct WalkConsts {
    static constexpr int XW = 0, XP = XW + 16 * NQE, EV = XP + 16 * NQE, EVC = EV + 16 * NTD, DEVC = EVC + 16 * NTD,
                         G1 = DEVC + 16 * NTD, G1C = G1 + HID, V0 = G1C + HID, CP = V0 + 2 * HID,
                         U = CP + HID, M2 = U + 2 * HID, M3 = M2 + HID, TC = M3 + HID, M3B = TC + 13 * 80,
                         C0 = M3B + 1, SIZE = M3B + 4;
};

template <int NQE, int NTD, bool ZN = false>
__device__ __forceinline__ void load_consts(const EncW &P, float *cs) {
    using C = WalkConsts<NQE, NTD>;
    for (int i = threadIdx.x; i < C::SIZE; i += blockDim.x) {
        float v;
        if (i < C::EV) {
            const int k = i < C::XP ? i : i - C::XP, ti = k - P.de - 3;
            v = (ti >= 0 && ti < P.dn) ? (i < C::XP ? P.freq[ti] : P.phase[ti]) : 0.f;
        } else if (i < C::EVC) v = P.ev.b[i - C::EV];
        else if (i < C::DEVC) v = P.evc[i - C::EVC];
        else if (i < C::G1) v = P.devc[i - C::DEVC];
        else if (i < C::G1C) v = P.g1.b[i - C::G1];
        else if (i < C::V0) v = P.g1.b[i - C::G1C];
        else if (i < C::CP) v = ZN ? (i - C::V0 < HID ? P.v0z[i - C::V0] : 0.f) : P.v0[i - C::V0];
        else if (i < C::U) v = P.cp[i - C::CP];
        else if (i < C::M2) v = ZN ? (i - C::U < HID ? P.uz[i - C::U] : 0.f) : P.u[i - C::U];
        else if (i < C::M3) v = P.m2.b[i - C::M2];
        else if (i < C::TC) v = P.m3w[i - C::M3];
        else if (i < C::M3B) v = P.tc[i - C::TC];
        else if (i == C::M3B) v = P.m3b[0];
        else if (i == C::C0) v = P.c0[0];
        else v = 0.f;
        cs[i] = v;
    }
}

// this lane's 4 entries of tile t of an LDS vector
__device__ __forceinline__ float4 lds4(const float *v, int t) {
    return *reinterpret_cast<const float4 *>(v + 16 * t + 4 * ((threadIdx.x & 63) >> 4));
}
__device__ __forceinline__ floatx4 ldsx4(const float *v, int t) {
    const float4 b = lds4(v, t);
    return floatx4{b.x, b.y, b.z, b.w};
}

__device__ __forceinline__ floatx4 add4(const floatx4 &a, const float4 &b) {
    return floatx4{a[0] + b.x, a[1] + b.y, a[2] + b.z, a[3] + b.w};
}

__device__ __forceinline__ floatx4 relu_add4(const floatx4 &a, const float4 &b) {
    return floatx4{relu(a[0] + b.x), relu(a[1] + b.y), relu(a[2] + b.z), relu(a[3] + b.w)};
}

__device__ __forceinline__ floatx4 relu4(const floatx4 &a) {
    return floatx4{relu(a[0]), relu(a[1]), relu(a[2]), relu(a[3])};
}

struct WalkArgs {
    EncW P;
    int64_t n_slots;      // total hop-1 slots = n_event_groups * (W / M)
    int32_t W, M, BW;     // walks per event-group, walks per slot, walks per std group (B*W)
    const float *n_feat, *e_feat;
    const int32_t *node6, *eid3, *cat;
    const float *ts3, *cnt, *stdv;
    const double *cut;
    float *out;
    const float *etab;    // [n_ids][16*NTD] lin_event's edge-feature part + bias per edge id (Q0 > 0)
    uint32_t *ticket;     // the launch's unit counter (persistent waves; zeroed before the launch)
};

// Phase timing (debug builds only, -DTM_STAMPS; tools/stamps.py): s_memtime deltas of lane 0 per
// pass type accumulated for every 16th workgroup (sampled over the whole launch).
#ifdef TM_STAMPS
__device__ unsigned long long g_st[3][10];
__device__ unsigned long long g_live;   // waves inside the pass loop right now
#define TM_STAMP(k)                                 \
    do {                                            \
        __builtin_amdgcn_sched_barrier(0);          \
        T[k] = __builtin_amdgcn_s_memtime();        \
        __builtin_amdgcn_sched_barrier(0);          \
    } while (0)
#else
#define TM_STAMP(k) (void)T
#endif
// Wave timeline (debug builds only, -DTM_TRACE; tools/walk_trace.py): per wave of the last launch, s_memrealtime
// (100 MHz) at [0] entry, [1] after the constant table, [2..15] the end of each pass of its first two units,
// [16..27] the end of each of its first 12 units, [28] its unit count, [29] HW_ID | XCC_ID << 32
#ifdef TM_TRACE
__device__ unsigned long long g_tr[8192][32];
#endif

constexpr int EQ_MAX = 4;   // edge features span at most 4 K steps (de <= 64, checked on the host)
static_assert(EQ_MAX == 4, "load_ef holds 4 K steps");

// per-position scalars of one pass (walk row gw, position p): edge, its two endpoints, the time
// offset to position 2 (:326) and the three edge counts; loaded one pass ahead of their use
// raw loads, unconditional (an invalid column's gw is a valid row: coords() gives it group 0, slot 0), so no
// branch ends the block they are issued in and nothing waits for them there; the users apply v (invalid: zeros)
// and form dt = ts3[2] - ts3[p] a pass later
struct PosIn {
    int32_t e, ns, nt;
    float ta, tb, c0, c1, c2;
    bool v;
    __device__ __forceinline__ int32_t edge() const { return v ? e : 0; }
};

__device__ __forceinline__ PosIn load_pos(const WalkArgs &a, int64_t gw, int p, bool valid) {
    PosIn r;
    r.v = valid;
    r.e = a.eid3[gw * 3 + p];
    r.ns = a.node6[gw * 6 + 2 * p];
    r.nt = a.node6[gw * 6 + 2 * p + 1];
    r.ta = a.ts3[gw * 3 + p];
    r.tb = a.ts3[gw * 3 + 2];
    r.c0 = a.cnt[gw * 9 + p * 3 + 0];
    r.c1 = a.cnt[gw * 9 + p * 3 + 1];
    r.c2 = a.cnt[gw * 9 + p * 3 + 2];
    return r;
}

// edge-feature part of x: unconditional (clamped) loads, all in flight together
__device__ __forceinline__ void load_ef(const WalkArgs &a, int32_t e, float (&ef)[4][4]) {
    const int g = lane_id() >> 4, de = a.P.de;
    const float *erow = a.e_feat + (int64_t)e * de;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if ((de & 3) == 0 && 16 * q + 16 <= de) {         // whole K step inside the row: one float4
            const float4 v = *reinterpret_cast<const float4 *>(erow + 16 * q + 4 * g);
            ef[q][0] = v.x;
            ef[q][1] = v.y;
            ef[q][2] = v.z;
            ef[q][3] = v.w;
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = 16 * q + 4 * g + s;
                ef[q][s] = (16 * q < de) ? erow[k < de ? k : de - 1] : 0.f;
            }
        }
    }
}

// Element s of K step q of the event features x[k] = [E(e) | cnt | cos(dt * w + phi)] (:176-179,
// TimeEncode :45-59) for this lane's feature k = 16q + 4g + s, with the step's time-encoder frequency w
// and phase ph in registers.  PURE (a step holding only time features, known at compile time): the cos
// alone.  Otherwise the cos is evaluated unconditionally (the opaque asm keeps the compiler from wrapping
// the polynomial in an exec-mask branch, which serialised it against the MFMAs) and the count / edge
// lanes select their values.  Padding lanes (k >= kev) keep cos(0) = 1: lin_event's packed weights are
// zero there.  In table mode the edge lanes are 0 (their product comes from the table row).
template <bool ETAB, bool PURE>
__device__ __forceinline__ float gen_one(int q, int s, float w, float ph, const float (&ef)[EQ_MAX][4], int g,
                                         int de, float dt, float c0, float c1, float c2) {
    float c = time_cos(dt, w, ph);
    if constexpr (PURE) return c;
    const int k = 16 * q + 4 * g + s;
    const int qe = q < EQ_MAX ? q : 0;
    if (!ETAB && 16 * q + 16 <= de) return ef[qe][s];
    asm volatile("" : "+v"(c));
    float v = c;
    if (k < de + 3) v = (k == de) ? c0 : (k == de + 1) ? c1 : c2;
    if (k < de) v = ETAB ? 0.f : ef[qe][s];
    return v;
}

// streamed-edge-feature variant (EQ_MAX*16 < de): e4 = this lane's 4 edge features of K step q
template <int NQE, int NTD>
__device__ __forceinline__ floatx4 gen_x_s(int q, const float *cs, const float4 &e4, int g, int de, int kev, float dt,
                                           float c0, float c1, float c2) {
    using C = WalkConsts<NQE, NTD>;
    floatx4 xq;
    const float4 w4 = lds4(cs + C::XW, q), p4 = lds4(cs + C::XP, q);
    const float wv[4] = {w4.x, w4.y, w4.z, w4.w}, pv[4] = {p4.x, p4.y, p4.z, p4.w}, ev[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int k = 16 * q + 4 * g + s;
        float v;
        if (16 * q + 16 <= de) v = ev[s];
        else {
            v = (k < kev) ? time_cos(dt, wv[s], pv[s]) : 0.f;
            if (k < de + 3) v = (k == de) ? c0 : (k == de + 1) ? c1 : c2;
            if (k < de) v = ev[s];
        }
        xq[s] = v;
    }
    return xq;
}

// this lane's float4 of K step q of an edge-feature row (de % 4 == 0): clamped unconditional load,
// zero outside the row
__device__ __forceinline__ float4 ef_step(const float4 *erow4, int q, int g, int de) {
    const int i = 4 * q + g, n4 = de >> 2;
    const float4 v = erow4[i < n4 ? i : n4 - 1];
    return i < n4 ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

// table mode: this lane's 4 features of each of the 11 output tiles of edge e's table row (loaded a
// pass ahead; they initialise the next pass's lin_event accumulators)
#define ETAB_N(q0) ((q0) > 0 ? 11 : 1)
template <int Q0>
__device__ __forceinline__ void load_et(const WalkArgs &a, int32_t e, float4 (&et)[ETAB_N(Q0)]) {
    if constexpr (Q0 > 0) {
        const float4 *trow = reinterpret_cast<const float4 *>(a.etab + (int64_t)e * 176);
        const int g = lane_id() >> 4;
#pragma unroll
        for (int t = 0; t < 11; ++t) et[t] = trow[4 * t + g];
    }
}

// One walk position for the 16 columns of this wave -> H = [relu(g1 A + b) | relu(g1 B + b)] (8 tiles,
// B layout), event_gcn's hidden layer of both branches; the second MLP layer (g2) is folded into the
// layers that read F = [U_s | U_t] (FoldLay).
// lin_event runs K-outer ((q, t) fragment order): the next K step's 4 event features are generated one
// element per tile between this step's MFMAs.  Its accumulators start from the bias (LDS) or, in table
// mode, from the edge's table row (edge-feature product + bias; the slot pass adds the folded time steps).
// Both nodes' feature rows are requested before the K loop (their latency overlaps it) and consumed
// in its epilogue.  Tiles past dn in the last node tile hold a clamped duplicate; g1's packed weights are
// zero for those inputs, so they contribute nothing.
// SEF (streamed edge features, EQ_MAX*16 < de <= 176): ef holds K steps 0 and 1 (loaded during the
// previous pass); step q + 2's float4 is loaded while step q's MFMAs run.
template <int NQE, int NTD, bool SEF, int Q0, bool ZN, class Extra>
__device__ __forceinline__ void encode_position(const WalkArgs &a, __amdgpu_buffer_rsrc_t wr, const float *cs,
                                                const PosIn &pi, const float (&ef)[EQ_MAX][4],
                                                float4 (&et)[ETAB_N(Q0)], Extra &&extra, int p, floatx4 (&H)[8],
                                                float4 (&pre)[PFP], const NextFr &nx, unsigned long long (&T)[10]) {
    constexpr bool ETAB = Q0 > 0;
    static_assert(!(ETAB && SEF), "table mode replaces the streamed edge features");
    using C = WalkConsts<NQE, NTD>;
    using LY = WalkLay<NQE>;
    const EncW &P = a.P;
    const int g = lane_id() >> 4;
    const int de = P.de, dn = P.dn, kev = P.kev;
    const float dt = pi.v ? pi.tb - pi.ta : 0.f, c0 = pi.v ? pi.c0 : 0.f, c1 = pi.v ? pi.c1 : 0.f,
                c2 = pi.v ? pi.c2 : 0.f;
    const float4 *nrow_s = reinterpret_cast<const float4 *>(a.n_feat + (int64_t)(pi.v ? pi.ns : 0) * dn);
    const float4 *nrow_t = reinterpret_cast<const float4 *>(a.n_feat + (int64_t)(pi.v ? pi.nt : 0) * dn);
    floatx4 L[NTD];
    if constexpr (ETAB) {
#pragma unroll
        for (int t = 0; t < NTD; ++t) L[t] = floatx4{et[t].x, et[t].y, et[t].z, et[t].w};
        if (p == 2) {                                    // slot pass: + the folded time steps (wave-uniform)
#pragma unroll
            for (int t = 0; t < NTD; ++t) L[t] = add4(L[t], lds4(cs + C::DEVC, t));
        }
    } else {
        const float *bias = cs + (p == 2 ? C::EVC : C::EV);
#pragma unroll
        for (int t = 0; t < NTD; ++t) L[t] = ldsx4(bias, t);
    }
    TM_STAMP(1);
    constexpr int JN = 3;                                // node tiles in flight in event_gcn's K loop
    float4 rs[JN], rt[JN];
    auto nload = [&](int q) {
        const int f4 = (q < NTD - 1) ? 4 * q + g : min(4 * q + g, dn / 4 - 1);
        rs[q % JN] = nrow_s[f4];
        rt[q % JN] = nrow_t[f4];
    };
    {
        const int vo = lane_id() * 16;
        constexpr int nq = NQE;
        constexpr int N = NTD * (NQE - Q0), D = PFP;
        static_assert(D >= PFP && D <= N, "lin_event ring depth");
        constexpr int EVF4 = LY::EV / 4;
        // the first D fragments (EVF4 + ((i % NTD) * nq + Q0 + i / NTD) * 64) come in pre, requested during
        // the previous pass; the ring's last D refills request event_gcn's first K step (G1 tiles 0..3)
        float4 buf[D];
#pragma unroll
        for (int i = 0; i < D; ++i) buf[i] = i < PFP ? pre[i] : wload(wr, vo, EVF4 + ((i % NTD) * nq + Q0 + i / NTD) * 64);
        auto g1f = [](int k) { return LY::G1 / 4 + k * NTD * 64; };
        const int qend = p == 2 ? P.qt : NQE;            // slot pass: steps >= qt folded into evc / devc
        if constexpr (SEF) {
            const float4 *erow4 = reinterpret_cast<const float4 *>(a.e_feat + (int64_t)pi.edge() * de);
            float4 ring[2];
            ring[0] = make_float4(ef[0][0], ef[0][1], ef[0][2], ef[0][3]);
            ring[1] = make_float4(ef[1][0], ef[1][1], ef[1][2], ef[1][3]);
            floatx4 xq = gen_x_s<NQE, NTD>(0, cs, ring[0], g, de, kev, dt, c0, c1, c2);
#pragma unroll
            for (int q = 0; q < NQE; ++q) {
                if (q < qend) {                           // wave-uniform (a break would stop the unrolling)
                    floatx4 xn = xq;
                    float4 e2 = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (q + 2 < NQE && 16 * (q + 2) < de) e2 = ef_step(erow4, q + 2, g, de);
                    if (q + 1 < NQE) xn = gen_x_s<NQE, NTD>(q + 1, cs, ring[(q + 1) & 1], g, de, kev, dt, c0, c1, c2);
#pragma unroll
                    for (int t = 0; t < NTD; ++t) {
                        const int i = q * NTD + t;
                        const float4 w = buf[i % D];
                        if (i + D < N) buf[i % D] = wload(wr, vo, EVF4 + (((i + D) % NTD) * nq + (i + D) / NTD) * 64);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, xq.x, L[t], 0, 0, 0);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, xq.y, L[t], 0, 0, 0);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, xq.z, L[t], 0, 0, 0);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, xq.w, L[t], 0, 0, 0);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    ring[q & 1] = e2;
                    xq = xn;
                }
            }
        } else {
            const float *cw = cs + C::XW, *cp = cs + C::XP;
            floatx4 xq;
            {
                const float4 w4 = lds4(cw, Q0), p4 = lds4(cp, Q0);
                xq[0] = gen_one<ETAB, false>(Q0, 0, w4.x, p4.x, ef, g, de, dt, c0, c1, c2);
                xq[1] = gen_one<ETAB, false>(Q0, 1, w4.y, p4.y, ef, g, de, dt, c0, c1, c2);
                xq[2] = gen_one<ETAB, false>(Q0, 2, w4.z, p4.z, ef, g, de, dt, c0, c1, c2);
                xq[3] = gen_one<ETAB, false>(Q0, 3, w4.w, p4.w, ef, g, de, dt, c0, c1, c2);
            }
#pragma unroll
            for (int q = Q0; q < NQE; ++q) {
                if (q < qend) {                           // wave-uniform (a break would stop the unrolling)
                    // step q + 1's constants from LDS now (first use after tile 0's MFMAs)
                    float4 w4 = make_float4(0.f, 0.f, 0.f, 0.f), p4 = w4;
                    if (q + 1 < NQE) {
                        w4 = lds4(cw, q + 1);
                        p4 = lds4(cp, q + 1);
                    }
                    const float wq[4] = {w4.x, w4.y, w4.z, w4.w}, pq[4] = {p4.x, p4.y, p4.z, p4.w};
                    constexpr bool pure_next_ok = ETAB;   // table mode: steps >= Q0 + 2 hold only time features
                    floatx4 xn = xq;
                    auto gen = [&](int t) {
                        if (q + 1 < NQE && t < 4) {
                            if (pure_next_ok && q + 1 >= Q0 + 2)
                                xn[t] = gen_one<ETAB, true>(q + 1, t, wq[t], pq[t], ef, g, de, dt, c0, c1, c2);
                            else
                                xn[t] = gen_one<ETAB, false>(q + 1, t, wq[t], pq[t], ef, g, de, dt, c0, c1, c2);
                        }
                    };
                    auto wnext = [&](int i) {   // fragment i + D of the ring into slot i % D (past N: G1's)
                        if (i + D < N) buf[i % D] = wload(wr, vo, EVF4 + (((i + D) % NTD) * nq + Q0 + (i + D) / NTD) * 64);
                        else if (i + D - N < PFP) buf[i % D] = wload(wr, vo, g1f(i + D - N));
                    };
                    // tile pairs with interleaved MFMAs (no MFMA waits on its predecessor); an odd last tile alone
#pragma unroll
                    for (int t = 0; t + 1 < NTD; t += 2) {
                        const int i = (q - Q0) * NTD + t;
                        const float4 w0 = buf[i % D];
                        wnext(i);
                        const float4 w1 = buf[(i + 1) % D];
                        wnext(i + 1);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.x, xq.x, L[t], 0, 0, 0);
                        L[t + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.x, xq.x, L[t + 1], 0, 0, 0);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.y, xq.y, L[t], 0, 0, 0);
                        L[t + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.y, xq.y, L[t + 1], 0, 0, 0);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.z, xq.z, L[t], 0, 0, 0);
                        L[t + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.z, xq.z, L[t + 1], 0, 0, 0);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.w, xq.w, L[t], 0, 0, 0);
                        L[t + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.w, xq.w, L[t + 1], 0, 0, 0);
                        gen(t);
                        gen(t + 1);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    if constexpr (NTD % 2) {
                        constexpr int t = NTD - 1;
                        const int i = (q - Q0) * NTD + t;
                        const float4 w = buf[i % D];
                        wnext(i);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, xq.x, L[t], 0, 0, 0);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, xq.y, L[t], 0, 0, 0);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, xq.z, L[t], 0, 0, 0);
                        L[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, xq.w, L[t], 0, 0, 0);
                        gen(t);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    xq = xn;
                }
            }
        }
        // G1's first fragments: in the ring's slots after a full K loop; the slot pass (K loop cut at qt) and
        // the streamed-edge-feature loop request them now
        if (SEF || p == 2) {
#pragma unroll
            for (int k = 0; k < PFP; ++k) buf[(N + k) % D] = wload(wr, vo, g1f(k));
        }
#pragma unroll
        for (int k = 0; k < PFP; ++k) pre[k] = buf[(N + k) % D];
    }
    TM_STAMP(2);
    // event_gcn's first layer K-outer: K step q of A = x_s + relu(x_t + L), B = x_t + relu(x_s + L) (:93-96,
    // lin_event shared) is built from node-row tile q just before its MFMAs, the node tiles requested
    // JN - 1 steps ahead and the step's 4 weight fragments one step ahead (the two branches share them).
    // The node rows are never all live at once (and not during lin_event's K loop).  Each output tile
    // accumulates its K steps in the same order as cgemm2 (same results).
    // ZN (every node-feature row zero, tm_weights_set_node_zero): A and B are the same expression of L,
    // 0 + relu(0 + L), so both branches are bit-identical: one branch is computed (and no node row read)
    floatx4 Hs[4], Ht[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        Hs[t] = ldsx4(cs + C::G1, t);
        if constexpr (!ZN) Ht[t] = ldsx4(cs + C::G1C, t);
    }
    if constexpr (ZN) {
        // one branch: 16 MFMAs per K step, too few to hide a weight fragment requested one step ahead (stamps:
        // the phase ran at 69 % of the shared-pipe ideal), so the fragments come through a 3-deep ring, two
        // steps ahead; the next phase's first fragments are requested at step NTD - 2
        const int vo = lane_id() * 16;
        float4 wz[3][4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            wz[0][t] = pre[t];
            wz[1][t] = wload(wr, vo, LY::G1 / 4 + (t * NTD + 1) * 64);
        }
#pragma unroll
        for (int q = 0; q < NTD; ++q) {
            if (q + 2 < NTD) {
#pragma unroll
                for (int t = 0; t < 4; ++t) wz[(q + 2) % 3][t] = wload(wr, vo, LY::G1 / 4 + (t * NTD + q + 2) * 64);
            } else if (q + 2 == NTD) {
#pragma unroll
                for (int t = 0; t < 4; ++t) wz[(q + 2) % 3][t] = wload(wr, vo, nx.o[t]);
            }
            extra(q);                                    // the caller's loads placed at step q
            floatx4 A;
#pragma unroll
            for (int r = 0; r < 4; ++r) A[r] = 0.f + relu(0.f + L[q][r]);
            // the 4 tiles' chains interleaved; each tile accumulates its k values in the same order as below
#pragma unroll
            for (int t = 0; t < 4; ++t) Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wz[q % 3][t].x, A.x, Hs[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 4; ++t) Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wz[q % 3][t].y, A.y, Hs[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 4; ++t) Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wz[q % 3][t].z, A.z, Hs[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 4; ++t) Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wz[q % 3][t].w, A.w, Hs[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) pre[t] = wz[NTD % 3][t];
    } else {
        const int vo = lane_id() * 16;
        float4 wq[2][4];
        {
#pragma unroll
            for (int q = 0; q < JN - 1 && q < NTD; ++q) nload(q);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) wq[0][t] = pre[t];
#pragma unroll
        for (int q = 0; q < NTD; ++q) {
            if (q + JN - 1 < NTD) nload(q + JN - 1);
            if (q + 1 < NTD) {
#pragma unroll
                for (int t = 0; t < 4; ++t) wq[(q + 1) & 1][t] = wload(wr, vo, LY::G1 / 4 + (t * NTD + q + 1) * 64);
            } else {                                     // the last step: the next phase's first fragments
#pragma unroll
                for (int t = 0; t < 4; ++t) wq[(q + 1) & 1][t] = wload(wr, vo, nx.o[t]);
            }
            extra(q);                                    // the caller's loads placed at step q
            const float4 xs4 = rs[q % JN], xt4 = rt[q % JN];
            const float sv[4] = {xs4.x, xs4.y, xs4.z, xs4.w}, tv[4] = {xt4.x, xt4.y, xt4.z, xt4.w};
            floatx4 A, Bq;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float l = L[q][r];
                A[r] = sv[r] + relu(tv[r] + l);
                Bq[r] = tv[r] + relu(sv[r] + l);
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float4 w = wq[q & 1][t];
                Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, A.x, Hs[t], 0, 0, 0);
                Ht[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, Bq.x, Ht[t], 0, 0, 0);
                Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, A.y, Hs[t], 0, 0, 0);
                Ht[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, Bq.y, Ht[t], 0, 0, 0);
                Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, A.z, Hs[t], 0, 0, 0);
                Ht[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, Bq.z, Ht[t], 0, 0, 0);
                Hs[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, A.w, Hs[t], 0, 0, 0);
                Ht[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, Bq.w, Ht[t], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) pre[t] = wq[NTD & 1][t];
    }
    TM_STAMP(3);
    TM_STAMP(4);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        H[t] = relu4(Hs[t]);
        H[4 + t] = ZN ? H[t] : relu4(Ht[t]);
    }
    TM_STAMP(5);
}

// sum over the 4 lane groups sharing a column (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float col_sum(float v) {
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}

// per-walk scalars of the head, loaded at the start of the position-1 pass
// raw loads (see PosIn): the head applies v (invalid: cut 0, std 1, times 0, category 12) and the std's epsilon
struct HeadIn {
    double cu;
    float sd, t0, t1;
    int32_t c;
    bool v;
};

// per-wave LDS stash of a slot's position-2 results, read by its walks' position-0/1 passes
struct Stash {
    floatx4 V[8][64];     // kv H_2 + v0 (= G^T Wp): the attention score of position i is V . H_i + cw
    floatx4 P2[4][64];    // A1D H_2 + cp: attention.MLP.0's input part that does not depend on alpha
    float cw[64];         // u . H_2 + c0 (= Wp . beta)
};

// Attention head + final MLP for the 16 walks of this wave (explainer_new.py:789-846 and :121-125,
// :195-201) in the folded form: score_i = V . H_i + cw, alpha = softmax(score * time weight),
// hid = relu(P2 + alpha_0 R_0 + alpha_1 R_1) (R_i = A1G H_i; alpha_0 + alpha_1 = 1 carries a1 beta),
// M1 = relu(M1A2 hid + tc[cat]), M2 = relu(m2 M1 + b), imp = sigmoid(m3 . M2 + b).
template <int NQE, int NTD>
__device__ __forceinline__ void walk_head(const WalkArgs &a, __amdgpu_buffer_rsrc_t wr, const float *cs, int64_t gw,
                                          bool valid, const HeadIn &hi, const Stash &st, float s0, float s1,
                                          const floatx4 (&R0)[4], const floatx4 (&R1)[4], float4 (&pre)[PFP],
                                          const NextFr &nx_end) {
    using C = WalkConsts<NQE, NTD>;
    using LY = WalkLay<NQE>;
    const EncW &P = a.P;
    const int lane = threadIdx.x & 63, g = lane_id() >> 4;
    float tw0 = 1.f, tw1 = 1.f;                          // plain Attention (tg = 0): 0.7f + 0.3f == 1.0f exactly
    if (valid && P.tg) {
        const float cu = hi.v ? (float)hi.cu : 0.f, sd = hi.v ? hi.sd + 1e-6f : 1.f;
        tw0 = expf(-fabsf(cu - (hi.v ? hi.t0 : 0.f)) / sd);
        tw1 = expf(-fabsf(cu - (hi.v ? hi.t1 : 0.f)) / sd);
    }
    // scores * (1.0 - 0.3 + 0.3 * time_weight) (:835-836), softmax over the 2 targets
    s0 *= __fadd_rn(0.7f, __fmul_rn(0.3f, tw0));
    s1 *= __fadd_rn(0.7f, __fmul_rn(0.3f, tw1));
    const float mx = fmaxf(s0, s1), e0 = expf(s0 - mx), e1 = expf(s1 - mx), sum = e0 + e1;
    const float al0 = e0 / sum, al1 = e1 / sum;
    floatx4 X[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const floatx4 p2 = st.P2[t][lane];
#pragma unroll
        for (int r = 0; r < 4; ++r) X[t][r] = relu(p2[r] + (al0 * R0[t][r] + al1 * R1[t][r]));
    }
    // MLP.0 over [attention out | one-hot(cat)] (compute_catogory_feautres :308-315): the one-hot column and
    // the biases come in as the accumulators' initial value, row cat of tc (row 12 for a padding column)
    const int32_t c = (valid && hi.v && hi.c >= 0 && hi.c < 12) ? hi.c : 12;
    floatx4 M1[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const float4 b = *reinterpret_cast<const float4 *>(cs + C::TC + 80 * c + 16 * t + 4 * g);
        M1[t] = floatx4{b.x, b.y, b.z, b.w};
    }
    cgemm_p<5, 4, 4, FoldLay::M1A2>(wr, X, M1, pre, pair_first<5>(LY::M2 / 4));
#pragma unroll
    for (int t = 0; t < 5; ++t) M1[t] = relu4(M1[t]);
    floatx4 M2[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) M2[t] = ldsx4(cs + C::M2, t);
    cgemm_p<4, 5, 5, LY::M2>(wr, M1, M2, pre, nx_end);
    float z = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const float4 w3 = lds4(cs + C::M3, t);
        z += relu(M2[t][0]) * w3.x + relu(M2[t][1]) * w3.y + relu(M2[t][2]) * w3.z + relu(M2[t][3]) * w3.w;
    }
    z = col_sum(z) + cs[C::M3B];
    if (valid && g == 0) a.out[gw] = 1.f / (1.f + expf(-z));
}

// this column's V . H (the 4 lane groups' parts summed); ZN: VZ . U over the first 4 tiles
template <bool ZN = false>
__device__ __forceinline__ float score_dot(const Stash &st, const floatx4 (&H)[8]) {
    const int lane = threadIdx.x & 63;
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < (ZN ? 4 : 8); ++t) {
        const floatx4 v = st.V[t][lane];
#pragma unroll
        for (int r = 0; r < 4; ++r) s = __builtin_fmaf(v[r], H[t][r], s);
    }
    return col_sum(s) + st.cw[lane];
}

// SPLIT (small grids, e.g. one reference batch per call in the drop-in surface): a wave takes one walk m of
// its unit's 16 slots -- the slot pass, then that walk's positions 0 and 1 (3 passes instead of 1 + 2M) --
// so a unit's M walks run on M waves at once.  The slot pass is repeated by each of them (same values);
// the chip is far from full at these sizes, and the latency of a call is one wave's pass chain.
// (Running the three positions of an M == 1 unit on three waves at once, the stash and position 0's inputs
// crossing LDS behind workgroup barriers, measured no faster for the drop-in: with three side calls in flight
// the 3x waves no longer fit one round of residency -- profiles/r05_dropin_pp_ab.txt.)
template <int NQE, int NTD, bool SEF = false, int QE0 = 0, bool SPLIT = false, bool ZN = false>
__global__ void __launch_bounds__(64 * WALK_WPB, 4 * WALK_WAVES / WALK_WPB) walk_kernel(WalkArgs a) {
    using C = WalkConsts<NQE, NTD>;
    const EncW &P = a.P;
    const int lane = threadIdx.x & 63, col = lane & 15;
    const int32_t NS = a.W / a.M;
    const int64_t n_units = (a.n_slots + 15) / 16;
    // persistent waves (not SPLIT): the grid is one round of resident workgroups; a wave starts with unit = its
    // global wave id and takes each next unit from the launch's counter (a ticket offset by the grid's waves),
    // requested at the top of its current unit's last pass, where the next unit's scalars and table row are
    // requested (round 6; before, at the start of the current unit: a reserved unit then waited a whole unit time,
    // which widened the end-of-grid spread, tools/walk_trace.py).  Static striding (unit w, w + stride, ...) measured 1.3 % slower
    // than one unit per wave, dynamic tickets 1.4 % faster (profiles/r03_walk_xpf_ab.txt, r05_walk_ab.txt).
    constexpr bool PERSIST = !SPLIT;
    const int64_t ustride = PERSIST ? (int64_t)gridDim.x * (blockDim.x >> 6) : n_units;
    int64_t unit = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    auto ticket = [&]() -> int64_t {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(a.ticket, 1u);
        return ustride + (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)t);
    };
    int m0 = 0;                                         // SPLIT: this wave's walk within each slot
    if constexpr (SPLIT) {
        m0 = (int)(unit % a.M);
        unit /= a.M;
    }
    // this column's hop-1 slot of unit u: (group, event) row and slot within it
    auto coords = [&](int64_t u, bool &v, int64_t &eg_, int32_t &j_) {
        const int64_t gs = u * 16 + col;
        v = u < n_units && gs < a.n_slots;
        eg_ = v ? gs / NS : 0;
        j_ = v ? (int32_t)(gs % NS) : 0;
    };
    bool valid;
    int64_t eg;
    int32_t j;
    coords(unit, valid, eg, j);
    // LDS: per-wave stash of the slot's position-2 results (12.25 KB per wave), then the constant table
    __shared__ Stash stash[WALK_WPB];
    __shared__ float4 cs4[(C::SIZE + 3) / 4];
    float *cs = reinterpret_cast<float *>(cs4);
#ifdef TM_TRACE
    const int64_t trw = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    int trn = 0;
    const unsigned long long tr0 = __builtin_amdgcn_s_memrealtime();
#endif
    load_consts<NQE, NTD, ZN>(P, cs);
    __syncthreads();
#ifdef TM_TRACE
    if (lane == 0 && trw < 8192) {
        g_tr[trw][0] = tr0;
        g_tr[trw][1] = __builtin_amdgcn_s_memrealtime();
        g_tr[trw][28] = 0;
        g_tr[trw][29] = (unsigned)__builtin_amdgcn_s_getreg(63492) | ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(30740) << 32);
    }
#endif
    if (unit >= n_units) return;                        // whole wave idle (wave-uniform)
    Stash &st = stash[threadIdx.x >> 6];
    // every weight fragment off one buffer resource (WalkLay offsets from the folded region's base)
    const auto wr = wrsrc(P.kv.w);
    floatx4 R0[4];                                      // A1G H_0, carried to the position-1 pass
    float s0 = 0.f;
    const int n_pass = SPLIT ? 3 : 1 + 2 * a.M;
    PosIn cur = load_pos(a, eg * a.W + (int64_t)j * a.M, 2, valid);
    float ef[EQ_MAX][4] = {};
    float4 et[ETAB_N(QE0)];
    // lin_event's first PFP fragments (ring order: tile k % NTD, K step QE0 + k / NTD), carried pass to pass
    NextFr lin0;
#pragma unroll
    for (int k = 0; k < PFP; ++k) lin0.o[k] = WalkLay<NQE>::EV / 4 + ((k % NTD) * NQE + QE0 + k / NTD) * 64;
    float4 pre[PFP];
#pragma unroll
    for (int k = 0; k < PFP; ++k) pre[k] = wload(wr, lane_id() * 16, lin0.o[k]);
    if constexpr (QE0 == 0) load_ef(a, cur.edge(), ef);
    else load_et<QE0>(a, cur.edge(), et);
#ifdef TM_STAMPS
    const unsigned long long clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) atomicMax(&g_st[2][9], atomicAdd(&g_live, 1ull) + 1);   // waves resident at once (max)
#endif
#pragma nounroll
    for (;;) {
    // the next unit: a persistent wave takes its ticket at the top of its current unit's LAST pass (the next unit's
    // slot-pass scalars are requested inside that pass), so no wave holds a reserved unit for a whole unit time --
    // the waves' end times then spread over one unit's last pass plus one unit, not two units
    int64_t unext = unit + ustride;
    bool vn = false;
    int64_t egn = 0;
    int32_t jn = 0;
    if constexpr (!PERSIST) coords(unext, vn, egn, jn);
    // pass 0: position 2 once per slot (walk j*M carries it); then per walk m: position 0, position 1
#pragma nounroll
    for (int pass = 0; pass < n_pass; ++pass) {
        if (PERSIST && pass + 1 == n_pass) {
            unext = ticket();
            coords(unext, vn, egn, jn);
        }
        // remaining-work priority (s_setprio 3 -> 0 over the unit's passes): of the two waves sharing a SIMD's
        // MFMA pipe, the one with more of its unit left issues first, so a pair ends its units together; the
        // default oldest-first arbitration starves the younger wave (its units took 100-300 us at the 8-rank
        // share) and leaves its last unit running alone at the end of the grid (tools/walk_trace.py).  With the
        // late tickets: walk_kernel 0.872 -> 0.852 ms at 24 batches, 6.083 -> 6.038 ms at 192
        // (profiles/r06_walk_tail_ab.txt)
        if (PERSIST) {
            const int q = (pass * 4) / n_pass;
            if (q == 0) __builtin_amdgcn_s_setprio(3);
            else if (q == 1) __builtin_amdgcn_s_setprio(2);
            else if (q == 2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        const int m = SPLIT ? m0 : pass == 0 ? 0 : (pass - 1) >> 1;
        const int p = pass == 0 ? 2 : ((pass - 1) & 1);
        const int64_t gw = eg * a.W + (int64_t)j * a.M + m;
        HeadIn hi{0.0, 1.f, 0.f, 0.f, -1, false};
        auto load_hi = [&]() {                           // consumed by the head (p == 1); issued every pass, so
            hi.v = valid;                                // no branch holds the waits for them at the loads
            hi.cu = a.cut[eg];
            hi.sd = a.stdv[gw / a.BW];
            hi.t0 = a.ts3[gw * 3 + 0];
            hi.t1 = a.ts3[gw * 3 + 1];
            hi.c = a.cat[gw];
        };
        // next pass's scalars (after the last pass: the next unit's slot pass); its edge features / table
        // row once this pass's lin_event is done
        const bool last = pass + 1 == n_pass;
        const int pn = !last ? ((pass & 1) == 0 ? 0 : 1) : 2;
        const int64_t gwn = !last ? eg * a.W + (int64_t)j * a.M + (SPLIT ? m0 : pass >> 1) : egn * a.W + (int64_t)jn * a.M;
        PosIn nxt;
        // the next pass's scalars (and the head's inputs of a position-1 pass) are requested inside event_gcn's
        // K loop at its first step (its weights are requested a whole step ahead there), not at the top of the
        // pass where lin_event's weight refills waited behind them
        auto extra = [&](int q) {
            if (q == 0) {
                load_hi();
                nxt = load_pos(a, gwn, pn, !last ? valid : vn);
            }
        };
        floatx4 H[8];
        unsigned long long T[10];
        TM_STAMP(0);
        encode_position<NQE, NTD, SEF, QE0, ZN>(a, wr, cs, cur, ef, et, extra, p, H, pre,
                                            ZN ? pair_first<4>(p == 2 ? FoldLay::A1DZ / 4 : FoldLay::A1GZ / 4)
                                               : pair_first<8>(p == 2 ? FoldLay::A1D / 4 : FoldLay::A1G / 4), T);
        if constexpr (QE0 == 0) load_ef(a, nxt.edge(), ef);
        else load_et<QE0>(a, nxt.edge(), et);
        cur = nxt;
        TM_STAMP(6);
        // ZN: H = [U; U]: the layers reading H as their 64-column-folded forms on U (FoldLay KVZ ...)
        floatx4 Uv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) Uv[t] = H[t];
        if (ZN && p == 2) {
            floatx4 P2[4], V[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) P2[t] = ldsx4(cs + C::CP, t);
            cgemm_p<4, 4, 4, FoldLay::A1DZ>(wr, Uv, P2, pre, pair_first<4>(FoldLay::KVZ / 4));
#pragma unroll
            for (int t = 0; t < 4; ++t) V[t] = ldsx4(cs + C::V0, t);
            cgemm_p<4, 4, 4, FoldLay::KVZ>(wr, Uv, V, pre, lin0);
            TM_STAMP(7);
            float cw = 0.f;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float4 b = lds4(cs + C::U, t);
                cw = __builtin_fmaf(Uv[t][0], b.x, cw);
                cw = __builtin_fmaf(Uv[t][1], b.y, cw);
                cw = __builtin_fmaf(Uv[t][2], b.z, cw);
                cw = __builtin_fmaf(Uv[t][3], b.w, cw);
            }
            cw = col_sum(cw) + cs[C::C0];
#pragma unroll
            for (int t = 0; t < 4; ++t) st.V[t][lane] = V[t];
#pragma unroll
            for (int t = 0; t < 4; ++t) st.P2[t][lane] = P2[t];
            st.cw[lane] = cw;
        } else if (p == 2) {
            // P2 = A1D H_2 + cp; V = kv H_2 + v0 (= G^T Wp); cw = u . H_2 + c0 (= Wp . beta)
            floatx4 P2[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) P2[t] = ldsx4(cs + C::CP, t);
            cgemm_p<4, 8, 8, FoldLay::A1D>(wr, H, P2, pre, pair_first<8>(FoldLay::KV / 4));
            floatx4 V[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) V[t] = ldsx4(cs + C::V0, t);
            cgemm_p<8, 8, 8, FoldLay::KV>(wr, H, V, pre, lin0);
            TM_STAMP(7);
            float cw = 0.f;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const float4 b = lds4(cs + C::U, t);
                cw = __builtin_fmaf(H[t][0], b.x, cw);
                cw = __builtin_fmaf(H[t][1], b.y, cw);
                cw = __builtin_fmaf(H[t][2], b.z, cw);
                cw = __builtin_fmaf(H[t][3], b.w, cw);
            }
            cw = col_sum(cw) + cs[C::C0];
#pragma unroll
            for (int t = 0; t < 8; ++t) st.V[t][lane] = V[t];
#pragma unroll
            for (int t = 0; t < 4; ++t) st.P2[t][lane] = P2[t];
            st.cw[lane] = cw;
        }
        floatx4 R[4];
        float s = 0.f;
        if (p != 2) {
            // R = A1G H_p (attention.MLP.0 of W2's output for this position), score = V . H_p + cw
#pragma unroll
            for (int t = 0; t < 4; ++t) R[t] = floatx4{0.f, 0.f, 0.f, 0.f};
            if constexpr (ZN) cgemm_p<4, 4, 4, FoldLay::A1GZ>(wr, Uv, R, pre, p == 1 ? pair_first<4>(FoldLay::M1A2 / 4) : lin0);
            else cgemm_p<4, 8, 8, FoldLay::A1G>(wr, H, R, pre, p == 1 ? pair_first<4>(FoldLay::M1A2 / 4) : lin0);
            s = score_dot<ZN>(st, H);
            TM_STAMP(7);
            if (p == 0) {
#pragma unroll
                for (int t = 0; t < 4; ++t) R0[t] = R[t];
                s0 = s;
            }
        }
        if (p == 1) walk_head<NQE, NTD>(a, wr, cs, gw, valid, hi, st, s0, s, R0, R, pre, lin0);
        TM_STAMP(8);
#ifdef TM_TRACE
        if (lane == 0 && trw < 8192 && trn < 2 && pass < 7) g_tr[trw][2 + 7 * trn + pass] = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef TM_STAMPS
        if (lane == 0 && blockIdx.x % 16 == 5) {
            for (int k = 0; k < 8; ++k) atomicAdd(&g_st[p][k], T[k + 1] - T[k]);
            atomicAdd(&g_st[p][8], 1ull);
        }
#endif
    }
#ifdef TM_TRACE
    if (lane == 0 && trw < 8192) {
        if (trn < 12) g_tr[trw][16 + trn] = __builtin_amdgcn_s_memrealtime();
        g_tr[trw][28] = ++trn;
    }
#endif
    unit = unext;
    if (unit >= n_units) break;                         // wave-uniform: every wave leaves after its last unit
    valid = vn;
    eg = egn;
    j = jn;
    }
#ifdef TM_STAMPS
    // in-kernel clock: shader-clock ticks over 100 MHz real-time ticks of the wave's pass loop
    if (lane == 0 && blockIdx.x % 16 == 5) {
        atomicAdd(&g_st[0][9], __builtin_amdgcn_s_memtime() - clk_t0);
        atomicAdd(&g_st[1][9], __builtin_amdgcn_s_memrealtime() - clk_r0);
    }
    if (lane == 0) atomicAdd(&g_live, ~0ull);
#endif
}

// host: the live weight pointers are where WalkLay<nqe> puts them
static bool walk_layout_ok(const EncW &P, int nqe) {
    const float *base = reinterpret_cast<const float *>(P.kv.w);
    auto at = [&](const float4 *w, int off) { return reinterpret_cast<const float *>(w) == base + off; };
    const int ev = FoldLay::SIZE, g1 = ev + 11 * nqe * 256 + 176, m2 = g1 + 4 * 11 * 256 + 64 + 4 * 4 * 256 + 64 +
                                                                     2 * (8 * 8 * 256 + 128) + 4 * 8 * 256 + 64 +
                                                                     4 * 4 * 256 + 64 + 5 * 5 * 256 + 80;
    return at(P.ev.w, ev) && at(P.g1.w, g1) && at(P.m2.w, m2) && at(P.a1d.w, FoldLay::A1D) &&
           at(P.a1g.w, FoldLay::A1G) && at(P.m1a2.w, FoldLay::M1A2) && at(P.kvz.w, FoldLay::KVZ) &&
           at(P.a1dz.w, FoldLay::A1DZ) && at(P.a1gz.w, FoldLay::A1GZ) && P.g1.nt == 4 && P.g1.nq == 11 && P.m2.nt == 4 && P.m2.nq == 5 && P.ev.nt == 11 && P.ev.nq == nqe;
}

// ------------------------------------------------------------------ per-edge dependency gate table
// The dependency gate (:367-386) is a function of (E[e], t) only, and every record of an edge id
// carries the edge's single timestamp, so gf(e) = 0.5 + 0.5*sigmoid(depMLP([E[e] | cos(t_e*w+phi)]))
// is computed once per edge id per call instead of once per walk position.
__global__ void __launch_bounds__(256) gate_table_kernel(EncW P, int32_t n_ids, const double *__restrict__ ets,
                                                         const float *__restrict__ e_feat, float *__restrict__ gf) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int de = P.de, kdep = P.kdep, kd16 = r16(kdep), ldx = kd16 + 8, ldg = r16(P.h) + 8, ldg2 = r16(P.h / 2) + 8;
    float *X = smem, *G1 = X + TILE_ROWS * ldx, *G2 = G1 + TILE_ROWS * ldg;
    const int tid = threadIdx.x;
    const int32_t e0 = blockIdx.x * TILE_ROWS;
    for (int i = tid; i < TILE_ROWS * kd16; i += blockDim.x) {
        const int r = i / kd16, c = i % kd16;
        const int32_t e = e0 + r;
        float v = 0.f;
        if (e < n_ids) {
            if (c < de) v = e_feat[(int64_t)e * de + c];
            else if (c < kdep) v = time_cos((float)ets[e], P.freq[c - de], P.phase[c - de]);
        }
        X[r * ldx + c] = v;
    }
    __syncthreads();
    gemm<2>(X, ldx, P.d1, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) G1[erow(mt, r) * ldg + c] = relu(acc[r] + P.d1.b[c]);
    });
    __syncthreads();
    gemm<2>(G1, ldg, P.d2, [&](int mt, int nt, floatx4 acc) {
        const int c = ecol(nt);
        for (int r = 0; r < 4; ++r) G2[erow(mt, r) * ldg2 + c] = relu(acc[r] + P.d2.b[c]);
    });
    __syncthreads();
    const int r = tid >> 3, sub = tid & 7;
    const float s = gate_logit_lds(G2 + r * ldg2, P.d3w, sub, P.h / 2);
    if (sub == 0 && e0 + r < n_ids) {
        const float z = s + P.d3b[0];
        gf[e0 + r] = P.dep ? 0.5f + 0.5f * (1.f / (1.f + expf(-z))) : 1.f;
    }
}

// Register-resident gate table: one wave = 16 edge ids (MFMA columns), the gate MLP's weights as the
// A operand (walk_kernel's layout), X = [E[e] | cos(t_e w + phi)] generated straight into the B
// fragments, G1 -> G2 -> logit chained in registers.  NQ = K steps of X (de + dn rounded up / 16).
// NQX > 0: the same edge-feature fragments also give the walk kernel's edge table, etab[e] =
// lin_event.W[:, :de] . E[e] + lin_event.b (16 * 11 features; the walk kernel starts lin_event's
// accumulators from it), from lin_event's pack (NQL K steps): the first NQX K steps with the lanes past
// de zeroed.
// Per-position mode (row_eid != nullptr, tm_dropin_forward): column = walk position r of the call, its edge
// id row_eid[r] and raw time row_t[r] (:371) instead of edge id r and its timestamp; gf[r] = the position's
// gate factor (the same arithmetic as per edge id: the drop-in equals the pipeline bit for bit).
// List mode (list != nullptr, per-position mode only): column i takes position list[i] for i < *list_n (the
// gate-cache misses of tm_dropin_forward) and also stores (t, gate factor) in cache[edge id] (gate_cache_pack).
__device__ __forceinline__ unsigned long long gate_cache_pack(float t, float f) {
    return ((unsigned long long)__float_as_uint(t) << 32) | (unsigned long long)__float_as_uint(f);
}
// one wave's 16 columns i0 .. i0 + 15 (of n_ids; i0 < n_ids, wave-uniform)
template <int NQ, int NQX = 0, int NQL = 1>
__device__ __forceinline__ void gate_reg_cols(const EncW &P, int64_t i0, int32_t n_ids, const double *__restrict__ ets,
                                              const float *__restrict__ e_feat, float *__restrict__ gf,
                                              float *__restrict__ etab, const int32_t *__restrict__ row_eid,
                                              const float *__restrict__ row_t, const int32_t *list,
                                              unsigned long long *__restrict__ cache, int64_t n_cache) {
    const int lane = threadIdx.x & 63, col = lane & 15, g = lane_id() >> 4;
    const bool valid = i0 + col < n_ids;
    const int64_t e = !list ? i0 + col : valid ? (int64_t)list[i0 + col] : 0;
    const int64_t ec = !valid ? 0 : row_eid ? (int64_t)row_eid[e] : e;
    const int de = P.de, kdep = P.kdep;
    // no timestamps: edge table only (gf is null too)
    const float t = row_eid ? (valid ? row_t[e] : 0.f) : ets ? (float)ets[ec] : 0.f;
    const float *erow = e_feat + ec * de;
    floatx4 X[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if ((de & 3) == 0 && 16 * q + 16 <= de) {     // whole K step inside the edge-feature row
            const float4 v = *reinterpret_cast<const float4 *>(erow + 16 * q + 4 * g);
            X[q] = floatx4{v.x, v.y, v.z, v.w};
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = 16 * q + 4 * g + s;
                float v = 0.f;
                if (k < de) v = erow[k];
                else if (k < kdep) v = time_cos(t, P.freq[k - de], P.phase[k - de]);
                X[q][s] = v;
            }
        }
    }
    if constexpr (NQX > 0) {
        floatx4 XE[NQX], ET[11];
#pragma unroll
        for (int q = 0; q < NQX; ++q) {
#pragma unroll
            for (int s = 0; s < 4; ++s) XE[q][s] = (16 * q + 4 * g + s < de) ? X[q][s] : 0.f;
        }
        rgemm<11, NQX, NQL>(P.ev, XE, ET);
        if (valid) {
            float4 *row = reinterpret_cast<float4 *>(etab + e * 176);
#pragma unroll
            for (int t = 0; t < 11; ++t) {
                const float4 b = *reinterpret_cast<const float4 *>(P.ev.b + 16 * t + 4 * g);
                row[4 * t + g] = make_float4(ET[t][0] + b.x, ET[t][1] + b.y, ET[t][2] + b.z, ET[t][3] + b.w);
            }
        }
    }
    floatx4 G1[4];
    rgemm<4, NQ>(P.d1, X, G1);
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) G1[tt] = relu_add4(G1[tt], *reinterpret_cast<const float4 *>(P.d1.b + 16 * tt + 4 * g));
    floatx4 G2[2];
    rgemm<2, 4>(P.d2, G1, G2);
    // this lane group's part of the logit in gate_part's order (features 16t + 4g + r), then
    // (part0 + part1) + (part2 + part3) across the lane groups, exactly as gate_logit_lds sums it
    float z = 0.f;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
        const float4 b = *reinterpret_cast<const float4 *>(P.d2.b + 16 * tt + 4 * g);
        const float4 w3 = *reinterpret_cast<const float4 *>(P.d3w + 16 * tt + 4 * g);
        const float bb[4] = {b.x, b.y, b.z, b.w}, ww[4] = {w3.x, w3.y, w3.z, w3.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) z = __builtin_fmaf(relu(G2[tt][r] + bb[r]), ww[r], z);
    }
    z += __shfl_xor(z, 16);
    z += __shfl_xor(z, 32);
    z += P.d3b[0];
    if (gf && valid && g == 0) {
        const float f = P.dep ? 0.5f + 0.5f * (1.f / (1.f + expf(-z))) : 1.f;
        gf[e] = f;
        if (cache && ec >= 0 && ec < n_cache && __float_as_uint(t) != 0xFFFFFFFFu)
            __atomic_store_n(&cache[ec], gate_cache_pack(t, f), __ATOMIC_RELAXED);
    }
}

template <int NQ, int NQX = 0, int NQL = 1>
__global__ void __launch_bounds__(256) gate_reg_kernel(EncW P, int32_t n_ids, const double *__restrict__ ets,
                                                       const float *__restrict__ e_feat, float *__restrict__ gf,
                                                       float *__restrict__ etab = nullptr,
                                                       const int32_t *__restrict__ row_eid = nullptr,
                                                       const float *__restrict__ row_t = nullptr,
                                                       const int32_t *__restrict__ list = nullptr,
                                                       const uint32_t *__restrict__ list_n = nullptr,
                                                       unsigned long long *__restrict__ cache = nullptr,
                                                       int64_t n_cache = 0) {
    const int64_t i0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16;
    if (list) n_ids = (int32_t)*list_n;
    if (i0 >= n_ids) return;                             // wave-uniform
    gate_reg_cols<NQ, NQX, NQL>(P, i0, n_ids, ets, e_feat, gf, etab, row_eid, row_t, list, cache, n_cache);
}

// The drop-in's gate-factor cache (tm_dropin_gate_cache): per walk position, a hit on (edge id, exact fp32 time)
// gives the factor gate_reg_kernel computed for it; the misses go to a list (one atomic per wave) that the list
// mode of gate_reg_kernel computes and stores.  Runs in std_cut_kernel's workgroups 1.. (one launch fewer).  The factor is a function of (E[e], t) alone, so the result equals
// the uncached path's bit for bit.
__device__ __forceinline__ void gate_cache_lookup(int64_t i, const int32_t *__restrict__ eid, const float *__restrict__ ts,
                                                  const unsigned long long *__restrict__ cache, int64_t n_cache,
                                                  float *__restrict__ gf, int32_t *__restrict__ list,
                                                  uint32_t *__restrict__ list_n, int64_t n_pos) {
    const int lane = threadIdx.x & 63;
    bool miss = false;
    if (i < n_pos) {
        const int32_t e = eid[i];
        const uint32_t tb = __float_as_uint(ts[i]);
        miss = true;
        if (e >= 0 && e < n_cache && tb != 0xFFFFFFFFu) {
            const unsigned long long v = __atomic_load_n(&cache[e], __ATOMIC_RELAXED);
            if ((uint32_t)(v >> 32) == tb) {
                gf[i] = __uint_as_float((uint32_t)v);
                miss = false;
            }
        }
    }
    const unsigned long long m = __ballot(miss);
    if (m == 0) return;
    const int first = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(list_n, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl(base, first);
    if (miss) list[base + __popcll(m & ((1ull << lane) - 1))] = (int32_t)i;
}

// std_cut_kernel with the cache misses computed where they are found (tm_dropin_forward with the gate cache and the
// register gate): workgroups 1.. look up their 1024 walk positions, list the misses in LDS, and their 16 waves run
// gate_reg_kernel's list mode over that list (the same arithmetic: bit-identical factors, the cache filled the same
// way) -- one launch per side call instead of two.  Two workgroups missing the same (edge id, time) both compute
// it (same value); a hit on an entry another workgroup just stored is the same value too.
template <int NQ>
__global__ void __launch_bounds__(1024) std_cut_gate_kernel(int32_t B, int32_t W, CutArg c, const float *__restrict__ ts3,
                                                            double *__restrict__ cut_out, float *__restrict__ std_out,
                                                            int32_t do_std, GateLookup gl, EncW P,
                                                            const float *__restrict__ e_feat) {
    if (blockIdx.x == 0) {
        std_cut_body(B, W, c, ts3, cut_out, std_out, do_std, gl);
        return;
    }
    __shared__ int32_t miss[1024];
    __shared__ uint32_t n_miss;
    if (threadIdx.x == 0) n_miss = 0u;
    __syncthreads();
    gate_cache_lookup((int64_t)(blockIdx.x - 1) * blockDim.x + threadIdx.x, gl.eid, gl.ts, gl.cache, gl.n_cache, gl.gf,
                      miss, &n_miss, gl.n_pos);
    __syncthreads();
    const int32_t n = (int32_t)n_miss;
    for (int32_t i0 = (int32_t)(threadIdx.x >> 6) * 16; i0 < n; i0 += (int32_t)(blockDim.x >> 6) * 16)
        gate_reg_cols<NQ>(P, i0, n, nullptr, e_feat, gl.gf, nullptr, gl.eid, gl.ts, miss,
                          const_cast<unsigned long long *>(gl.cache), gl.n_cache);
}

// threads per (group, event) workgroup of explain_tab_kernel (its loops stride by blockDim.x): one wave
// (256 -> 64: 0.136 -> 0.110 ms per 19,200 x 3 rows at the metric config; a workgroup is a short chain of
// dependent loads and LDS atomics, so four times as many of them in flight per CU hide that latency)
constexpr int EXPLAIN_TPB = 64;   // one wave per (group, event); 128 / 256 threads measured within noise / slower
// retrieve_edge_imp_node with the gate table: per (group, event) the LDS hash keeps, per edge id,
// the max graphlet importance of the walks through it; edge_imp = that max * gf(e), which equals
// max_w(imp_w * gf(e)) bit for bit (rounding is monotone).
__global__ void __launch_bounds__(256) explain_tab_kernel(int32_t W, int32_t N, int32_t hbits, int32_t n_ids,
                                                          const float *__restrict__ gf,
                                                          const int32_t *__restrict__ eid3,
                                                          const float *__restrict__ imp,
                                                          const int32_t *__restrict__ sub1_node,
                                                          const int32_t *__restrict__ sub1_eid,
                                                          const int32_t *__restrict__ sub2_node,
                                                          const int32_t *__restrict__ sub2_eid, float *__restrict__ out1,
                                                          float *__restrict__ out2, int32_t *err) {
    extern __shared__ __attribute__((aligned(16))) int32_t hkey[];
    const int hsize = 1 << hbits;
    uint32_t *hval = reinterpret_cast<uint32_t *>(hkey + hsize);
    const int64_t ge = blockIdx.x;
    const int tid = threadIdx.x;
    for (int i = tid; i < hsize; i += blockDim.x) {
        hkey[i] = -1;
        hval[i] = 0u;
    }
    __syncthreads();
    const int32_t *e3 = eid3 + ge * (int64_t)W * 3;
    for (int r = tid; r < 3 * W; r += blockDim.x) {
        const int32_t key = e3[r];
        const float v = imp[ge * W + r / 3];
        uint32_t h = hash_eid(key) >> (32 - hbits);
        while (true) {
            const int32_t prev = atomicCAS(&hkey[h], -1, key);
            if (prev == -1 || prev == key) break;
            h = (h + 1) & (hsize - 1);
        }
        atomicMax(&hval[h], __float_as_uint(v));
    }
    __syncthreads();
    const int n1 = N, n2 = N * N;
    for (int i = tid; i < n1 + n2; i += blockDim.x) {
        const bool h1 = i < n1;
        const int64_t o = h1 ? ge * n1 + i : ge * n2 + (i - n1);
        const int32_t key = h1 ? sub1_eid[o] : sub2_eid[o];
        const int32_t nd = h1 ? sub1_node[o] : sub2_node[o];
        uint32_t h = hash_eid(key) >> (32 - hbits);
        float p = 0.f;
        while (true) {
            const int32_t k = hkey[h];
            if (k == key) {
                if (key < 0 || key >= n_ids) {
                    if (err) atomicCAS(err, 0, TM_E_ARG);
                } else {
                    p = __uint_as_float(hval[h]) * gf[key];
                }
                break;
            }
            if (k == -1) break;
            h = (h + 1) & (hsize - 1);
        }
        const float a = fmaxf(p * 10.f, 1.f), b = fmaxf((1.f - p) * 10.f, 1.f);
        const float v = nd == 0 ? 0.f : a / (a + b);
        if (h1) out1[o] = v;
        else out2[o] = v;
    }
}

// ------------------------------------------------------------------ weight packing
// packed[((nt*nq + q)*64 + l)*4 + s] = W[16nt + (l&15)][16q + 4(l>>4) + s]; all packs (and the slot
// pass's folded bias evc) are written by pack_all_weights (encoder_train.hip) in one launch.

}  // namespace tmk

using namespace tmk;


extern "C" int tm_weights_create(int32_t de, int32_t dn, int32_t h, int device, tm_weights **out) {
    return tm_weights_create_ex(de, dn, h, 1, device, out);
}

extern "C" int tm_weights_create_ex(int32_t de, int32_t dn, int32_t h, int32_t if_cat, int device, tm_weights **out) {
    if (!out || de <= 0 || dn <= 0 || h <= 0) return fail(TM_E_ARG, "tm_weights_create: bad arguments");
    if (h % 16 || h > 256)
        return fail(TM_E_UNSUPPORTED, "tm_weights_create: hid_dim must be a multiple of 16 up to 256");
    *out = nullptr;
    tm_weights *w = new tm_weights();
    w->device = device;
    w->de = de;
    w->dn = dn;
    w->h = h;
    EncW &P = w->P;
    P.de = de;
    P.dn = dn;
    P.kev = de + 3 + dn;
    P.kdep = de + dn;
    P.h = h;
    P.cat = if_cat ? 1 : 0;
    P.hm = if_cat ? h + 12 : h;
    const int h2 = 2 * h, hm = P.hm;
    struct L {
        Lin *lin;
        int wi, nout, k;
    } ls[] = {{&P.ev, 0, dn, P.kev}, {&P.g1, 2, h, dn},  {&P.g2, 4, h, h},   {&P.w1, 6, h2, h2},
              {&P.w2, 8, h2, h2},    {&P.a1, 10, h, h2}, {&P.a2, 12, h, h},  {&P.m1, 14, hm, hm},
              {&P.m2, 16, h, hm},    {&P.d1, 20, h, P.kdep}, {&P.d2, 22, h / 2, h}};
    // the folded packs of the fused walk kernel first (fixed size: their offsets and those of the layers
    // after them are compile-time constants of the kernel, WalkLay)
    size_t total = tmk::FoldLay::SIZE;
    std::vector<size_t> woff, boff;
    for (auto &l : ls) {
        l.lin->nt = r16(l.nout) / 16;
        l.lin->nq = r16(l.k) / 16;
        l.lin->nout = l.nout;
        l.lin->k = l.k;
        woff.push_back(total);
        total += (size_t)l.lin->nt * l.lin->nq * 256;
        boff.push_back(total);
        total += (size_t)l.lin->nt * 16;
        w->specs.push_back({l.lin, l.wi, l.nout, l.k});
    }
    const size_t m3w = total; total += r16(h);
    const size_t m3b = total; total += 4;
    const size_t d3w = total; total += r16(h / 2);
    const size_t d3b = total; total += 4;
    const size_t fq = total; total += r16(dn);
    const size_t ph = total; total += r16(dn);
    const size_t evc = total; total += r16(dn);
    const size_t devc = total; total += r16(dn);
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess || hipMalloc(&w->buf, total * sizeof(float)) != hipSuccess ||
        hipMemset(w->buf, 0, total * sizeof(float)) != hipSuccess) {
        (void)hipSetDevice(prev);
        delete w;
        return fail(TM_E_HIP, "tm_weights_create: allocation failed");
    }
    (void)hipSetDevice(prev);
    w->n_floats = total;
    for (size_t i = 0; i < w->specs.size(); ++i) {
        Lin *l = w->specs[i].lin;
        l->w = reinterpret_cast<const float4 *>(w->buf + woff[i]);
        l->b = w->buf + boff[i];
    }
    P.m3w = w->buf + m3w;
    P.m3b = w->buf + m3b;
    P.d3w = w->buf + d3w;
    P.d3b = w->buf + d3b;
    P.freq = w->buf + fq;
    P.phase = w->buf + ph;
    P.evc = w->buf + evc;
    P.devc = w->buf + devc;
    P.qt = (de + 3 + 15) / 16;
    {   // folded packs (tmk::FoldLay)
        using F = tmk::FoldLay;
        struct FL {
            Lin *lin;
            int off, nout, k;
        } fl[] = {{&P.kv, F::KV, h2, h2},     {&P.a1d, F::A1D, h, h2},   {&P.a1g, F::A1G, h, h2},
                  {&P.m1a2, F::M1A2, hm, h},  {&P.kvz, F::KVZ, h, h},    {&P.a1dz, F::A1DZ, h, h},
                  {&P.a1gz, F::A1GZ, h, h}};
        for (auto &f : fl) {
            f.lin->w = reinterpret_cast<const float4 *>(w->buf + f.off);
            f.lin->b = nullptr;
            f.lin->nout = f.nout;
            f.lin->k = f.k;
            f.lin->nt = r16(f.nout) / 16;
            f.lin->nq = r16(f.k) / 16;
        }
        P.v0 = w->buf + F::V0;
        P.u = w->buf + F::U;
        P.c0 = w->buf + F::C0;
        P.cp = w->buf + F::CP;
        P.tc = w->buf + F::TC;
        P.v0z = w->buf + F::V0Z;
        P.uz = w->buf + F::UZ;
        (void)hipGetDevice(&prev);
        const bool ok = hipSetDevice(device) == hipSuccess &&
                        hipMalloc(&w->fold64, sizeof(double) * F::S64_SIZE) == hipSuccess &&
                        hipMalloc(&w->fold32, sizeof(float) * F::S_SIZE) == hipSuccess;
        (void)hipSetDevice(prev);
        if (!ok) {
            tm_weights_free(w);
            return fail(TM_E_HIP, "tm_weights_create: allocation failed");
        }
    }
    if (int rc = train_packs_create(w)) {
        tm_weights_free(w);
        return rc;
    }
    tm_weights_bump(w);
    *out = w;
    return TM_OK;
}

static std::atomic<uint64_t> g_weights_stamp{0};
void tm_weights_bump(tm_weights *w) { w->version = g_weights_stamp.fetch_add(1, std::memory_order_relaxed) + 1; }

extern "C" uint64_t tm_weights_version(const tm_weights *w) { return w ? w->version : 0; }

extern "C" int tm_weights_set_node_zero(tm_weights *w, int32_t node_zero) {
    if (!w) return fail(TM_E_ARG, "tm_weights_set_node_zero: NULL weights");
    w->node_zero = node_zero ? 1 : 0;
    tm_weights_bump(w);
    return TM_OK;
}

extern "C" int tm_weights_variant(tm_weights *w, int32_t temporal_guidance, int32_t dependency_gate) {
    if (!w) return fail(TM_E_ARG, "tm_weights_variant: NULL weights");
    tm_weights_bump(w);
    w->P.tg = temporal_guidance ? 1 : 0;
    w->P.dep = dependency_gate ? 1 : 0;
    return TM_OK;
}

extern "C" int tm_weights_pack(tm_weights *w, const float *const *t, void *stream) {
    if (!w || !t) return fail(TM_E_ARG, "tm_weights_pack: bad arguments");
    for (int i = 0; i < TM_N_WEIGHTS; ++i)
        if (!t[i]) return fail(TM_E_ARG, "tm_weights_pack: NULL tensor " + std::to_string(i));
    hipStream_t s = S_(stream);
    tm_weights_bump(w);
    pack_all_weights(w, t, s);
    TM_CHECK_LAUNCH();
    return TM_OK;
}

extern "C" int tm_weights_free(tm_weights *w) {
    if (!w) return TM_OK;
    if (w->buf) (void)hipFree(w->buf);
    if (w->fold64) (void)hipFree(w->fold64);
    if (w->fold32) (void)hipFree(w->fold32);
    train_packs_free(w);
    delete w;
    return TM_OK;
}

extern "C" int64_t tm_encoder_workspace_bytes(const tm_weights *w, int64_t n_walks) {
    (void)w;
    return n_walks * 3 * 2 * (w ? w->h : HID) * (int64_t)sizeof(float) + (n_walks + 64) * (int64_t)sizeof(float) + 256;
}

static size_t gate_lds(const EncW &P) {
    return sizeof(float) * (TILE_ROWS * (r16(P.kdep) + 8) + TILE_ROWS * (r16(P.h) + 8) + TILE_ROWS * (r16(P.h / 2) + 8));
}

// lin_event's K steps before the first one holding a count or time feature (= de / 16), when the
// fused walk kernel has a table-mode instance for these dims (de = 32..47 with 11..14 K steps, as
// Enron's 32; de = 160..175 with 21..22, as BASELINE configs[4]'s 172), else 0
static int etab_q0(const EncW &P) {
    const int nqe = r16(P.kev) / 16, ntd = r16(P.dn) / 16, q0 = P.de / 16;
    if (P.h != HID || !P.cat) return 0;
    if (ntd != 11 || P.dn % 4 || P.ev.nt != 11 || P.ev.nq != nqe || P.d1.nt != 4 || P.d2.nq != 4 || P.d2.nt != 2)
        return 0;
    if (q0 == 2 && nqe >= 11 && nqe <= 14 && P.d1.nq == 13) return 2;
    if (q0 == 10 && (nqe == 21 || nqe == 22) && P.d1.nq == 22) return 10;
    return 0;
}

extern "C" int tm_edge_table_cols(const tm_weights *w) { return (w && etab_q0(w->P) > 0) ? 176 : 0; }

extern "C" int tm_edge_gate_table(const tm_weights *w, const tm_graph *g, const float *e_feat, float *out_gf,
                                  void *stream) {
    return tm_edge_tables(w, g, e_feat, out_gf, nullptr, stream);
}

// gate table (gf, needs the edge timestamps ets) and/or edge table (etab) over edge ids [0, n)
static int launch_edge_tables(const tm_weights *w, int32_t n, const double *ets, const float *e_feat, float *out_gf,
                              float *out_etab, void *stream) {
    const int q0 = etab_q0(w->P);
    if (out_etab && q0 == 0) return fail(TM_E_UNSUPPORTED, "tm_edge_tables: no edge table for these encoder dims");
    hipEvent_t pe = prof_begin(S_(stream));
    const int nq = w->P.d1.nq;
    const unsigned rblocks = (unsigned)((n + 63) / 64);
    if (out_etab) {   // one launch: gate table and edge table from the same edge-feature fragments
        const int nqe = w->P.ev.nq;
        if (q0 == 2 && nqe == 11) gate_reg_kernel<13, 3, 11><<<dim3(rblocks), 256, 0, S_(stream)>>>(w->P, n, ets, e_feat, out_gf, out_etab);
        else if (q0 == 2 && nqe == 12) gate_reg_kernel<13, 3, 12><<<dim3(rblocks), 256, 0, S_(stream)>>>(w->P, n, ets, e_feat, out_gf, out_etab);
        else if (q0 == 2 && nqe == 13) gate_reg_kernel<13, 3, 13><<<dim3(rblocks), 256, 0, S_(stream)>>>(w->P, n, ets, e_feat, out_gf, out_etab);
        else if (q0 == 2) gate_reg_kernel<13, 3, 14><<<dim3(rblocks), 256, 0, S_(stream)>>>(w->P, n, ets, e_feat, out_gf, out_etab);
        else if (nqe == 21) gate_reg_kernel<22, 11, 21><<<dim3(rblocks), 256, 0, S_(stream)>>>(w->P, n, ets, e_feat, out_gf, out_etab);
        else gate_reg_kernel<22, 11, 22><<<dim3(rblocks), 256, 0, S_(stream)>>>(w->P, n, ets, e_feat, out_gf, out_etab);
    } else if (w->P.d2.nq == 4 && w->P.d1.nt == 4 && w->P.d2.nt == 2) {   // hid_dim 64: register-resident path
        if (nq == 11) gate_reg_kernel<11><<<dim3(rblocks), 256, 0, S_(stream)>>>(w->P, n, ets, e_feat, out_gf);
        else if (nq == 12) gate_reg_kernel<12><<<dim3(rblocks), 256, 0, S_(stream)>>>(w->P, n, ets, e_feat, out_gf);
        else if (nq == 13) gate_reg_kernel<13><<<dim3(rblocks), 256, 0, S_(stream)>>>(w->P, n, ets, e_feat, out_gf);
        else if (nq == 22) gate_reg_kernel<22><<<dim3(rblocks), 256, 0, S_(stream)>>>(w->P, n, ets, e_feat, out_gf);
        else gate_table_kernel<<<dim3((n + TILE_ROWS - 1) / TILE_ROWS), 256, gate_lds(w->P), S_(stream)>>>(
            w->P, n, ets, e_feat, out_gf);
    } else {
        gate_table_kernel<<<dim3((n + TILE_ROWS - 1) / TILE_ROWS), 256, gate_lds(w->P), S_(stream)>>>(w->P, n, ets,
                                                                                                    e_feat, out_gf);
    }
    TM_CHECK_LAUNCH();
    prof_end("gate_table_kernel", S_(stream), pe);
    return TM_OK;
}

extern "C" int tm_edge_tables(const tm_weights *w, const tm_graph *g, const float *e_feat, float *out_gf,
                              float *out_etab, void *stream) {
    if (!w || !g || !e_feat || !out_gf) return fail(TM_E_ARG, "tm_edge_tables: bad arguments");
    if (!g->d.ts_unique)
        return fail(TM_E_UNSUPPORTED, "tm_edge_gate_table: an edge id carries several timestamps; use tm_edge_importance");
    return launch_edge_tables(w, g->d.max_eid + 1, g->d.ets, e_feat, out_gf, out_etab, stream);
}

extern "C" int tm_edge_feature_table(const tm_weights *w, const float *e_feat, int32_t n_ids, float *out_etab,
                                     void *stream) {
    if (!w || !e_feat || !out_etab || n_ids <= 0) return fail(TM_E_ARG, "tm_edge_feature_table: bad arguments");
    return launch_edge_tables(w, n_ids, nullptr, e_feat, nullptr, out_etab, stream);
}

extern "C" int tm_edge_importance_tab(const float *gf, int32_t n_ids, int32_t n_groups, int32_t B, int32_t W,
                                      int32_t N, const int32_t *eid3, const float *imp, const int32_t *sub1_node,
                                      const int32_t *sub1_eid, const int32_t *sub2_node, const int32_t *sub2_eid,
                                      float *out_h1, float *out_h2, int32_t *err_flag, void *stream) {
    if (n_groups < 0 || B < 0 || W <= 0 || N <= 0 || n_ids <= 0)
        return fail(TM_E_ARG, "tm_edge_importance_tab: bad arguments");
    const int64_t rows = (int64_t)n_groups * B;
    if (rows == 0) return TM_OK;
    if (!gf || !eid3 || !imp || !sub1_node || !sub1_eid || !sub2_node || !sub2_eid || !out_h1 || !out_h2)
        return fail(TM_E_ARG, "tm_edge_importance_tab: NULL pointer");
    int hbits = 6;
    while ((1 << hbits) < 2 * 3 * W) ++hbits;
    if (hbits > 14) return fail(TM_E_UNSUPPORTED, "tm_edge_importance_tab: too many walks per event");
    hipEvent_t pe = prof_begin(S_(stream));
    explain_tab_kernel<<<dim3((unsigned)rows), EXPLAIN_TPB, 2 * sizeof(int32_t) * (1u << hbits), S_(stream)>>>(
        W, N, hbits, n_ids, gf, eid3, imp, sub1_node, sub1_eid, sub2_node, sub2_eid, out_h1, out_h2, err_flag);
    TM_CHECK_LAUNCH();
    prof_end("explain_tab_kernel", S_(stream), pe);
    return TM_OK;
}

static size_t gcn_lds(const EncW &P) {
    const int xsz = std::max(TILE_ROWS * (r16(P.kev) + 8), 2 * TILE_ROWS * (r16(P.h) + 8));
    return sizeof(float) * (xsz + 2 * TILE_ROWS * (r16(P.dn) + 8));
}
static size_t head_lds(const EncW &P, int tr) { return sizeof(float) * (4 * tr * (2 * P.h + 8)); }
static void launch_gcn(const EncW &P, int node_zero, int64_t n_rows, size_t lds, const float *n_feat,
                       const float *e_feat, const int32_t *node6, const int32_t *eid3, const float *ts3, const float *cnt,
                       float *F, hipStream_t s) {
    const dim3 grid((unsigned)((n_rows + TILE_ROWS - 1) / TILE_ROWS));
    if (node_zero) gcn_kernel<true><<<grid, 256, lds, s>>>(P, n_rows, n_feat, e_feat, node6, eid3, ts3, cnt, F);
    else gcn_kernel<false><<<grid, 256, lds, s>>>(P, n_rows, n_feat, e_feat, node6, eid3, ts3, cnt, F);
}

// walks per head_kernel workgroup: 32 where the tiles fit the LDS, else 16
// 16 walks per head_kernel workgroup (35 KB of LDS at hid_dim 64, four per CU; 32-walk ones hold two per CU
// and measured 0-0.9 % slower per training step, profiles/r05_train_tiles_ab.txt)
static int head_tr(const EncW &) { return 16; }
static void launch_head(const EncW &P, int64_t n_walks, int64_t walks_per_group, int32_t W, const float *F,
                        const float *ts3, const double *cut, const int32_t *cat, const float *stdv, float *out,
                        const uint8_t *drop, float dscale, hipStream_t s) {
    const int tr = head_tr(P);
    if (tr == 32)
        head_kernel<32><<<dim3((unsigned)((n_walks + 31) / 32)), 256, head_lds(P, 32), s>>>(
            P, n_walks, walks_per_group, W, F, ts3, cut, cat, stdv, out, drop, dscale);
    else
        head_kernel<16><<<dim3((unsigned)((n_walks + 15) / 16)), 256, head_lds(P, 16), s>>>(
            P, n_walks, walks_per_group, W, F, ts3, cut, cat, stdv, out, drop, dscale);
}

// a grid of fewer units than this runs split (one wave per (unit, walk)): at most one round of resident
// waves either way (1024 SIMDs x 2 waves), so the call's latency is the shorter pass chain
constexpr int64_t WALK_SPLIT_UNITS = 512;

static bool walk_split(int64_t units, int32_t M) { return units * M <= 3 * WALK_SPLIT_UNITS && units < WALK_SPLIT_UNITS; }

// a.ticket zeroed on the stream before the launch unless walk_split (encoder_fwd_impl)
template <int NQE, bool SEF = false, int Q0 = 0, bool ZN = false>
static void launch_walk(const WalkArgs &a, unsigned blocks, hipStream_t s) {
    const int64_t units = (a.n_slots + 15) / 16;
    if (walk_split(units, a.M)) {
        const unsigned sb = (unsigned)((units * a.M + WALK_WPB - 1) / WALK_WPB);
        walk_kernel<NQE, 11, SEF, Q0, true, ZN><<<dim3(sb), 64 * WALK_WPB, 0, s>>>(a);
        return;
    }
    // one round of resident workgroups (occupancy x CUs of the current device), cached per instance
    static int cap[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
        if (cap[dev] == 0) {
            int per_cu = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, walk_kernel<NQE, 11, SEF, Q0, false, ZN>, 64 * WALK_WPB, 0) ==
                    hipSuccess &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && per_cu > 0 &&
                cus > 0)
                cap[dev] = per_cu * cus;
            else
                cap[dev] = -1;
        }
        if (cap[dev] > 0 && blocks > (unsigned)cap[dev]) blocks = (unsigned)cap[dev];
    }
    const int dbg = debug_opt(TM_DEBUG_WALK_BLOCKS);   // A/B of smaller persistent grids (tools/walk_grid_ab.sh)
    if (dbg > 0 && blocks > (unsigned)dbg) blocks = (unsigned)dbg;
    walk_kernel<NQE, 11, SEF, Q0, false, ZN><<<dim3(blocks), 64 * WALK_WPB, 0, s>>>(a);
}

extern "C" int tm_encoder_fwd(const tm_weights *w, const float *n_feat, const float *e_feat, int32_t n_groups,
                              int32_t B, int32_t W, int32_t M, const int32_t *node6, const int32_t *eid3,
                              const float *ts3, const int32_t *cat, const double *cut, const float *cnt,
                              void *workspace, float *out_imp, void *stream) {
    return tm_encoder_fwd_tab(w, n_feat, e_feat, nullptr, n_groups, B, W, M, node6, eid3, ts3, cat, cut, cnt,
                              workspace, out_imp, stream);
}

static int encoder_fwd_impl(const tm_weights *w, const float *n_feat, const float *e_feat, const float *etab,
                            int32_t n_groups, int32_t B, int32_t W, int32_t M, const int32_t *node6, const int32_t *eid3,
                            const float *ts3, const int32_t *cat, const double *cut, const float *cnt, void *workspace,
                            float *out_imp, void *stream, bool do_std);

extern "C" int tm_encoder_fwd_tab(const tm_weights *w, const float *n_feat, const float *e_feat, const float *etab,
                                  int32_t n_groups, int32_t B, int32_t W, int32_t M, const int32_t *node6,
                                  const int32_t *eid3, const float *ts3, const int32_t *cat, const double *cut,
                                  const float *cnt, void *workspace, float *out_imp, void *stream) {
    return encoder_fwd_impl(w, n_feat, e_feat, etab, n_groups, B, W, M, node6, eid3, ts3, cat, cut, cnt, workspace,
                            out_imp, stream, true);
}

// the encoder launches; do_std = false: the groups' std values are already in the workspace (std_cut_kernel)
static int encoder_fwd_impl(const tm_weights *w, const float *n_feat, const float *e_feat, const float *etab,
                            int32_t n_groups, int32_t B, int32_t W, int32_t M, const int32_t *node6, const int32_t *eid3,
                            const float *ts3, const int32_t *cat, const double *cut, const float *cnt, void *workspace,
                            float *out_imp, void *stream, bool do_std) {
    if (!w || n_groups < 0 || B < 0 || W < 0 || M <= 0) return fail(TM_E_ARG, "tm_encoder_fwd: bad arguments");
    if (W % M) return fail(TM_E_SHAPE, "tm_encoder_fwd: W must be a multiple of M (walks per hop-1 slot)");
    const int64_t n_walks = (int64_t)n_groups * B * W;
    if (n_walks == 0) return TM_OK;
    if (!n_feat || !e_feat || !node6 || !eid3 || !ts3 || !cat || !cut || !cnt || !workspace || !out_imp)
        return fail(TM_E_ARG, "tm_encoder_fwd: NULL pointer");
    const EncW &P = w->P;
    const size_t lds_g = gcn_lds(P);
    if (lds_g > 160 * 1024) return fail(TM_E_UNSUPPORTED, "tm_encoder_fwd: feature dims too large for LDS tile");
    hipStream_t s = S_(stream);
    float *F = reinterpret_cast<float *>(workspace);
    float *stdv = F + n_walks * 3 * 2 * P.h;
    hipEvent_t pe = nullptr;
    if (do_std) {
        pe = prof_begin(s);
        if (P.tg) std_kernel<<<dim3(n_groups), 1024, 0, s>>>(B, W, cut, ts3, stdv);
        TM_CHECK_LAUNCH();
        prof_end("std_kernel", s, pe);
    }
    if (etab && etab_q0(P) == 0) return fail(TM_E_UNSUPPORTED, "tm_encoder_fwd_tab: no edge table for these dims");
    const int nqe = r16(P.kev) / 16, ntd = r16(P.dn) / 16;
    const bool narrow = nqe >= 11 && nqe <= 14 && P.de <= 16 * EQ_MAX;
    // wide edge features (e.g. BASELINE configs[4]: de = dn = 172): streamed per K step
    const bool wide = (nqe == 21 || nqe == 22) && P.de > 16 * EQ_MAX && P.de % 4 == 0;
    if (ntd == 11 && P.dn % 4 == 0 && (narrow || wide) && P.h == HID && P.cat) {
        // fused register-resident path
        if (!walk_layout_ok(P, nqe)) return fail(TM_E_UNSUPPORTED, "tm_encoder_fwd: weight layout mismatch");
        const int64_t n_slots = n_walks / M;
        const int64_t units = (n_slots + 15) / 16;
        // the unit counter of a dynamic persistent launch lives in the workspace's F region (unused by this path)
        WalkArgs a{P, n_slots, W, M, B * W, n_feat, e_feat, node6, eid3, cat, ts3, cnt, stdv, cut, out_imp, etab,
                   reinterpret_cast<uint32_t *>(F)};
        const unsigned blocks = (unsigned)((units + WALK_WPB - 1) / WALK_WPB);
        const int q0 = etab ? etab_q0(P) : 0;
        if (!walk_split(units, M)) TM_HIP(hipMemsetAsync(a.ticket, 0, sizeof(uint32_t), s));
        pe = prof_begin(s);
        if (q0 == 2 && w->node_zero) {   // edge table, zero node features: one event_gcn branch (ZN)
            if (nqe == 11) launch_walk<11, false, 2, true>(a, blocks, s);
            else if (nqe == 12) launch_walk<12, false, 2, true>(a, blocks, s);
            else if (nqe == 13) launch_walk<13, false, 2, true>(a, blocks, s);
            else launch_walk<14, false, 2, true>(a, blocks, s);
        } else if (q0 == 2) {        // edge table: lin_event from K step 2
            if (nqe == 11) launch_walk<11, false, 2>(a, blocks, s);
            else if (nqe == 12) launch_walk<12, false, 2>(a, blocks, s);
            else if (nqe == 13) launch_walk<13, false, 2>(a, blocks, s);
            else launch_walk<14, false, 2>(a, blocks, s);
        } else if (q0 == 10) {   // edge table: lin_event from K step 10 (no streamed edge features)
            if (nqe == 21) launch_walk<21, false, 10>(a, blocks, s);
            else launch_walk<22, false, 10>(a, blocks, s);
        } else if (wide) {
            if (nqe == 21) launch_walk<21, true>(a, blocks, s);
            else launch_walk<22, true>(a, blocks, s);
        } else if (nqe == 11) launch_walk<11>(a, blocks, s);
        else if (nqe == 12) launch_walk<12>(a, blocks, s);
        else if (nqe == 13) launch_walk<13>(a, blocks, s);
        else launch_walk<14>(a, blocks, s);
        TM_CHECK_LAUNCH();
        prof_end("walk_kernel", s, pe);
        return TM_OK;
    }
    const int64_t n_rows = n_walks * 3;
    pe = prof_begin(s);
    launch_gcn(P, w->node_zero, n_rows, lds_g, n_feat, e_feat, node6, eid3, ts3, cnt, F, s);
    TM_CHECK_LAUNCH();
    prof_end("gcn_kernel", s, pe);
    pe = prof_begin(s);
    launch_head(P, n_walks, (int64_t)B * W, W, F, ts3, cut, cat, stdv, out_imp, nullptr, 1.f, s);
    TM_CHECK_LAUNCH();
    prof_end("head_kernel", s, pe);
    return TM_OK;
}

// Training forward (explainer_new.py:174-201 with dropout active): the LDS-tiled kernels, keeping
// F [n_walks*3, 2h] and the per-group std in `workspace` for tm_encoder_bwd.  drop nullable (eval).
extern "C" int tm_encoder_train_fwd(const tm_weights *w, const float *n_feat, const float *e_feat, int32_t n_groups,
                                    int32_t B, int32_t W, const int32_t *node6, const int32_t *eid3, const float *ts3,
                                    const int32_t *cat, const double *cut, const float *cnt, const uint8_t *drop,
                                    float drop_scale, void *workspace, float *out_imp, void *stream) {
    if (!w || n_groups < 0 || B < 0 || W < 0) return fail(TM_E_ARG, "tm_encoder_train_fwd: bad arguments");
    const int64_t n_walks = (int64_t)n_groups * B * W;
    if (n_walks == 0) return TM_OK;
    if (!n_feat || !e_feat || !node6 || !eid3 || !ts3 || !cat || !cut || !cnt || !workspace || !out_imp)
        return fail(TM_E_ARG, "tm_encoder_train_fwd: NULL pointer");
    const EncW &P = w->P;
    const size_t lds_g = gcn_lds(P);
    if (lds_g > 160 * 1024) return fail(TM_E_UNSUPPORTED, "tm_encoder_train_fwd: feature dims too large for LDS tile");
    hipStream_t s = S_(stream);
    float *F = reinterpret_cast<float *>(workspace);
    float *stdv = F + n_walks * 3 * 2 * P.h;
    hipEvent_t pe = prof_begin(s);
    if (P.tg) std_kernel<<<dim3(n_groups), 1024, 0, s>>>(B, W, cut, ts3, stdv);
    TM_CHECK_LAUNCH();
    prof_end("std_kernel", s, pe);
    const int64_t n_rows = n_walks * 3;
    pe = prof_begin(s);
    if (!launch_gcn_fwd_reg(P, w->node_zero, n_rows, n_feat, e_feat, node6, eid3, ts3, cnt, F, s))
        launch_gcn(P, w->node_zero, n_rows, lds_g, n_feat, e_feat, node6, eid3, ts3, cnt, F, s);
    TM_CHECK_LAUNCH();
    prof_end("gcn_kernel", s, pe);
    pe = prof_begin(s);
    launch_head(P, n_walks, (int64_t)B * W, W, F, ts3, cut, cat, stdv, out_imp, drop, drop_scale, s);
    TM_CHECK_LAUNCH();
    prof_end("head_kernel", s, pe);
    return TM_OK;
}

extern "C" int tm_edge_importance(const tm_weights *w, const float *e_feat, int32_t n_groups, int32_t B, int32_t W,
                                  int32_t N, const int32_t *eid3, const float *ts3, const float *imp,
                                  const int32_t *sub1_node, const int32_t *sub1_eid, const int32_t *sub2_node,
                                  const int32_t *sub2_eid, float *out_h1, float *out_h2, void *stream) {
    if (!w || n_groups < 0 || B < 0 || W <= 0 || N <= 0) return fail(TM_E_ARG, "tm_edge_importance: bad arguments");
    const int64_t rows = (int64_t)n_groups * B;
    if (rows == 0) return TM_OK;
    if (!e_feat || !eid3 || !ts3 || !imp || !sub1_node || !sub1_eid || !sub2_node || !sub2_eid || !out_h1 || !out_h2)
        return fail(TM_E_ARG, "tm_edge_importance: NULL pointer");
    int hbits = 6;
    while ((1 << hbits) < 2 * 3 * W) ++hbits;
    if (hbits > 14) return fail(TM_E_UNSUPPORTED, "tm_edge_importance: too many walks per event");
    const EncW &P = w->P;
    const size_t lds = gate_lds(P);
    const size_t hlds = 2 * sizeof(int32_t) * (1u << hbits);
    if (lds > 160 * 1024) return fail(TM_E_UNSUPPORTED, "tm_edge_importance: LDS budget exceeded");
    const int64_t n_pos = rows * 3 * W;
    float *wv = static_cast<float *>(scratch(sizeof(float) * (size_t)n_pos, S_(stream)));
    if (!wv) return fail(TM_E_HIP, "tm_edge_importance: scratch allocation failed");
    hipEvent_t pe = prof_begin(S_(stream));
    gate_pos_kernel<<<dim3((unsigned)((n_pos + TILE_ROWS - 1) / TILE_ROWS)), 256, lds, S_(stream)>>>(P, n_pos, W, e_feat,
                                                                                                   eid3, ts3, imp, wv);
    TM_CHECK_LAUNCH();
    explain_hash_kernel<<<dim3((unsigned)rows), 256, hlds, S_(stream)>>>(W, N, hbits, eid3, wv, nullptr, sub1_node,
                                                                        sub1_eid, sub2_node, sub2_eid, out_h1, out_h2);
    TM_CHECK_LAUNCH();
    prof_end("explain_kernel", S_(stream), pe);
    return TM_OK;
}

// ------------------------------------------------------------------ drop-in eval context
// The reference's eval loop calls TempME.forward once per side, then retrieve_explanation
// (temp_exp_main.py:446-453).  tm_dropin_forward is one such forward in ONE library call: the side
// stream (three, round robin) is ordered after the caller's stream, the cut times are staged through a
// device ring (sent as kernel arguments) (a repeated cut array -- the same ts_l_cut for the three sides -- is sent once), std +
// encoder run on the side stream from a per-stream workspace, the dependency-gate factor of every walk
// position (the part of retrieve_edge_imp_node that does not depend on graphlet_imp) follows on the
// same stream, and the caller's stream waits for it.  tm_edge_importance_gf then finishes
// retrieve_edge_imp_node from those factors.
// up to 256 cut times as a kernel argument: the host values travel with the launch (asynchronous, no
// host buffer to keep alive -- a small hipMemcpyAsync from host memory can block until the stream drains)
struct CutChunk {
    double v[256];
};

__global__ void put_cut_kernel(double *__restrict__ dst, int32_t n, CutChunk c) {
    if ((int)threadIdx.x < n) dst[threadIdx.x] = c.v[threadIdx.x];
}

struct tm_dropin {
    static constexpr int SIDES = 3, SLOTS = 64, SLOT_DOUBLES = 512;
    int device = 0;
    hipStream_t side[SIDES] = {};
    hipEvent_t ev_cur = nullptr, ev_side[SIDES] = {};
    bool prep_pending[SIDES] = {}, own[SIDES] = {};
    double *hcopy = nullptr, *dring = nullptr;   // host copies of the slots (memo) | device ring
    hipEvent_t copy_ev[SLOTS] = {}, read_ev[SLOTS][SIDES] = {};
    bool read_used[SLOTS][SIDES] = {};
    int slot_next = 0, last_slot = -1, last_n = 0, last_side = -1;
    void *ws[SIDES] = {};
    size_t ws_bytes[SIDES] = {};
    double *dcut[SIDES] = {};   // per side stream: the cut times its std_cut_kernel writes (stream-ordered reuse)
    // gate-factor cache (tm_dropin_gate_cache): (fp32 time bits << 32 | factor bits) per edge id, all ones = empty;
    // valid for the weights / version / edge-feature table it was filled with
    unsigned long long *gcache = nullptr;
    int64_t gcache_n = 0;
    const void *gkey_w = nullptr;
    uint64_t gkey_ver = 0;
    const float *gkey_ef = nullptr;
    int32_t *glist[SIDES] = {};   // per side: miss list [n_pos] and two miss counters after it (alternate calls)
    int64_t glist_n[SIDES] = {};
    int gpar[SIDES] = {};         // the counter this side's next call uses
};

extern "C" void tm_dropin_free(tm_dropin *d) {
    if (!d) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(d->device);
    for (int k = 0; k < tm_dropin::SIDES; ++k)
        if (d->side[k]) (void)hipStreamSynchronize(d->side[k]);
    if (d->gcache) (void)hipFree(d->gcache);
    for (int k = 0; k < tm_dropin::SIDES; ++k) {
        if (d->glist[k]) (void)hipFree(d->glist[k]);
        if (d->dcut[k]) (void)hipFree(d->dcut[k]);
        if (d->ws[k]) (void)hipFree(d->ws[k]);
        if (d->ev_side[k]) (void)hipEventDestroy(d->ev_side[k]);
        if (d->side[k] && d->own[k]) (void)hipStreamDestroy(d->side[k]);
    }
    for (int i = 0; i < tm_dropin::SLOTS; ++i) {
        if (d->copy_ev[i]) (void)hipEventDestroy(d->copy_ev[i]);
        for (int k = 0; k < tm_dropin::SIDES; ++k)
            if (d->read_ev[i][k]) (void)hipEventDestroy(d->read_ev[i][k]);
    }
    if (d->ev_cur) (void)hipEventDestroy(d->ev_cur);
    free(d->hcopy);
    if (d->dring) (void)hipFree(d->dring);
    (void)hipSetDevice(prev);
    delete d;
}

extern "C" int tm_dropin_gate_cache(tm_dropin *d, int64_t n_edge_rows) {
    if (!d || n_edge_rows < 0) return fail(TM_E_ARG, "tm_dropin_gate_cache: bad arguments");
    int prev = 0;
    (void)hipGetDevice(&prev);
    hipError_t e = hipSetDevice(d->device);
    for (int k = 0; k < tm_dropin::SIDES && e == hipSuccess; ++k)
        if (d->side[k]) e = hipStreamSynchronize(d->side[k]);
    if (e == hipSuccess && d->gcache) e = hipFree(d->gcache);
    d->gcache = nullptr;
    d->gcache_n = 0;
    d->gkey_w = nullptr;
    if (e == hipSuccess && n_edge_rows > 0) {
        e = hipMalloc(&d->gcache, sizeof(unsigned long long) * (size_t)n_edge_rows);
        if (e == hipSuccess) d->gcache_n = n_edge_rows;
    }
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return fail(TM_E_HIP, std::string("tm_dropin_gate_cache: ") + hipGetErrorString(e));
    return TM_OK;
}

// the caller rewrote the edge-feature table in place (same address): the next tm_dropin_forward with out_gfac
// empties the cache (a stamp of 0 matches no weight state)
extern "C" int tm_dropin_gate_cache_clear(tm_dropin *d) {
    if (!d) return fail(TM_E_ARG, "tm_dropin_gate_cache_clear: NULL context");
    d->gkey_ver = 0;
    return TM_OK;
}

extern "C" int tm_dropin_create(int32_t device, tm_dropin **out) {
    if (!out) return fail(TM_E_ARG, "tm_dropin_create: NULL out");
    *out = nullptr;
    int prev = 0;
    TM_HIP(hipGetDevice(&prev));
    TM_HIP(hipSetDevice(device));
    tm_dropin *d = new tm_dropin();
    d->device = device;
    bool ok = hipEventCreateWithFlags(&d->ev_cur, hipEventDisableTiming) == hipSuccess;
    for (int k = 0; ok && k < tm_dropin::SIDES; ++k)
        ok = (d->own[k] = hipStreamCreateWithFlags(&d->side[k], hipStreamNonBlocking) == hipSuccess) &&
             hipEventCreateWithFlags(&d->ev_side[k], hipEventDisableTiming) == hipSuccess;
    for (int i = 0; ok && i < tm_dropin::SLOTS; ++i) {
        ok = hipEventCreateWithFlags(&d->copy_ev[i], hipEventDisableTiming) == hipSuccess;
        for (int k = 0; ok && k < tm_dropin::SIDES; ++k)
            ok = hipEventCreateWithFlags(&d->read_ev[i][k], hipEventDisableTiming) == hipSuccess;
    }
    const size_t ring = sizeof(double) * tm_dropin::SLOTS * tm_dropin::SLOT_DOUBLES;
    d->hcopy = static_cast<double *>(malloc(ring));
    ok = ok && d->hcopy && hipMalloc(reinterpret_cast<void **>(&d->dring), ring) == hipSuccess;
    for (int k = 0; ok && k < tm_dropin::SIDES; ++k)
        ok = hipMalloc(reinterpret_cast<void **>(&d->dcut[k]), sizeof(double) * 256) == hipSuccess;
    (void)hipSetDevice(prev);
    if (!ok) {
        tm_dropin_free(d);
        return fail(TM_E_HIP, "tm_dropin_create: stream / event / buffer allocation failed");
    }
    *out = d;
    return TM_OK;
}

// side stream k from the caller (e.g. torch streams, so the caller's allocator can serve them); the
// context's own stream k is destroyed once idle
extern "C" int tm_dropin_set_stream(tm_dropin *d, int32_t k, void *stream) {
    if (!d || k < 0 || k >= tm_dropin::SIDES || !stream) return fail(TM_E_ARG, "tm_dropin_set_stream: bad arguments");
    if (d->own[k]) {
        TM_HIP(hipStreamSynchronize(d->side[k]));
        TM_HIP(hipStreamDestroy(d->side[k]));
        d->own[k] = false;
    }
    d->side[k] = S_(stream);
    d->prep_pending[k] = true;
    return TM_OK;
}

extern "C" int tm_dropin_forward(tm_dropin *d, int32_t k, int32_t sync, const tm_weights *w, const float *n_feat,
                                 const float *e_feat, const float *etab, int32_t B, int32_t W, const int32_t *node6,
                                 const int32_t *eid3, const float *ts3, const int32_t *cat, const double *cut_host,
                                 const double *cut_dev, const float *cnt, float *out_imp, float *out_gfac,
                                 void *stream) {
    if (!d || !w || B < 0 || W <= 0 || k < 0 || k >= tm_dropin::SIDES)
        return fail(TM_E_ARG, "tm_dropin_forward: bad arguments");
    if (B == 0) return TM_OK;
    if (!cut_host == !cut_dev) return fail(TM_E_ARG, "tm_dropin_forward: exactly one of cut_host / cut_dev");
    if (cut_host && B > tm_dropin::SLOT_DOUBLES) return fail(TM_E_UNSUPPORTED, "tm_dropin_forward: batch too large");
    hipStream_t cur = S_(stream);
    hipStream_t side = d->side[k];
    // gate-factor cache: new weights (or a repack: w->version is a process-wide stamp, so a freed and re-created
    // tm_weights at the same address never matches), another edge-feature table or tm_dropin_gate_cache_clear
    // empty it, on the caller's stream (ordered after every earlier side call) before every side stream's next use
    if (out_gfac && d->gcache && (d->gkey_w != w || d->gkey_ver != w->version || d->gkey_ef != e_feat)) {
        TM_HIP(hipMemsetAsync(d->gcache, 0xFF, sizeof(unsigned long long) * (size_t)d->gcache_n, cur));
        d->gkey_w = w;
        d->gkey_ver = w->version;
        d->gkey_ef = e_feat;
        sync = 1;
    }
    // sync: work on the caller's stream this call depends on (weights / tables repacked there, a device
    // cut tensor) -- every side stream waits for the caller's stream once, at its next use.  Otherwise
    // the side stream is not ordered after the caller's: it reads resident pack data and writes buffers
    // the caller allocated on the side stream itself.
    if (sync) {
        TM_HIP(hipEventRecord(d->ev_cur, cur));
        for (int j = 0; j < tm_dropin::SIDES; ++j) d->prep_pending[j] = true;
    }
    if (d->prep_pending[k]) {
        TM_HIP(hipStreamWaitEvent(side, d->ev_cur, 0));
        d->prep_pending[k] = false;
    }
    const double *cut = cut_dev;
    int slot = -1;
    const int64_t n_walks = (int64_t)B * W;
    const size_t need = (size_t)tm_encoder_workspace_bytes(w, n_walks);
    if (d->ws_bytes[k] < need) {
        TM_HIP(hipStreamSynchronize(side));
        if (d->ws[k]) TM_HIP(hipFree(d->ws[k]));
        d->ws[k] = nullptr;
        d->ws_bytes[k] = 0;
        TM_HIP(hipMalloc(&d->ws[k], need));
        d->ws_bytes[k] = need;
    }
    // the gate factors: hid_dim 64 has the register-resident gate (one wave per 16 positions, MFMA chain in
    // registers), cached per (edge id, time) when the drop-in has a cache; other dims the LDS-tiled gate
    const EncW &P = w->P;
    const int64_t n_pos = n_walks * 3;
    const int nq = P.d1.nq;
    const bool reg = out_gfac && P.dep && P.d2.nq == 4 && P.d1.nt == 4 && P.d2.nt == 2 && n_pos < INT32_MAX &&
                     (nq == 11 || nq == 12 || nq == 13 || nq == 22);
    GateLookup gl{};
    if (reg && d->gcache) {
        if (d->glist_n[k] < n_pos) {
            TM_HIP(hipStreamSynchronize(side));
            if (d->glist[k]) TM_HIP(hipFree(d->glist[k]));
            d->glist[k] = nullptr;
            d->glist_n[k] = 0;
            TM_HIP(hipMalloc(&d->glist[k], sizeof(int32_t) * ((size_t)n_pos + 2)));
            d->glist_n[k] = n_pos;
            TM_HIP(hipMemsetAsync(d->glist[k] + n_pos, 0, 2 * sizeof(uint32_t), side));
            d->gpar[k] = 0;
        }
        uint32_t *cnts = reinterpret_cast<uint32_t *>(d->glist[k] + d->glist_n[k]);
        gl = GateLookup{n_pos, d->gcache_n, eid3, ts3, d->gcache, out_gfac, d->glist[k], cnts + d->gpar[k],
                        cnts + (d->gpar[k] ^ 1)};
        d->gpar[k] ^= 1;
    }
    const unsigned lookup_blocks = gl.cnt ? (unsigned)((n_pos + 1023) / 1024) : 0u;
    // with the cache: the misses are computed by the lookup's own workgroups (std_cut_gate_kernel), no gate launch
    const bool fused_gate = gl.cnt != nullptr && (nq == 11 || nq == 12 || nq == 13);
    auto launch_std = [&](int32_t b_, const CutArg &c, double *cut_out, float *std_out, int32_t do_std) {
        const dim3 grid(1 + lookup_blocks);
        if (!fused_gate) std_cut_kernel<<<grid, 1024, 0, side>>>(b_, W, c, ts3, cut_out, std_out, do_std, gl);
        else if (nq == 11) std_cut_gate_kernel<11><<<grid, 1024, 0, side>>>(b_, W, c, ts3, cut_out, std_out, do_std, gl, P, e_feat);
        else if (nq == 12) std_cut_gate_kernel<12><<<grid, 1024, 0, side>>>(b_, W, c, ts3, cut_out, std_out, do_std, gl, P, e_feat);
        else std_cut_gate_kernel<13><<<grid, 1024, 0, side>>>(b_, W, c, ts3, cut_out, std_out, do_std, gl, P, e_feat);
    };
    bool std_done = false;
    if (cut_host && B <= 256) {
        // the cut times travel as the std launch's argument; std_cut_kernel writes them to this side's
        // buffer for the encoder (stream order keeps the buffer's previous readers ahead of it)
        CutArg c;
        memcpy(c.v, cut_host, sizeof(double) * (size_t)B);
        float *stdv = reinterpret_cast<float *>(d->ws[k]) + n_walks * 3 * 2 * w->P.h;
        hipEvent_t pe = prof_begin(side);
        launch_std(B, c, d->dcut[k], stdv, w->P.tg ? 1 : 0);
        TM_CHECK_LAUNCH();
        prof_end("std_kernel", side, pe);
        cut = d->dcut[k];
        std_done = true;
    } else if (cut_host) {
        const size_t bytes = sizeof(double) * (size_t)B;
        if (d->last_slot >= 0 && d->last_n == B &&
            memcmp(d->hcopy + (size_t)d->last_slot * tm_dropin::SLOT_DOUBLES, cut_host, bytes) == 0) {
            slot = d->last_slot;   // the previous side's cut array again: already on the device
            if (d->last_side != k) TM_HIP(hipStreamWaitEvent(side, d->copy_ev[slot], 0));
        } else {
            slot = d->slot_next;
            d->slot_next = (slot + 1) % tm_dropin::SLOTS;
            for (int j = 0; j < tm_dropin::SIDES; ++j)   // every kernel that read this slot's last contents done
                if (d->read_used[slot][j]) {
                    TM_HIP(hipEventSynchronize(d->read_ev[slot][j]));
                    d->read_used[slot][j] = false;
                }
            double *h = d->hcopy + (size_t)slot * tm_dropin::SLOT_DOUBLES;
            memcpy(h, cut_host, bytes);
            for (int32_t i0 = 0; i0 < B; i0 += 256) {
                CutChunk c;
                const int32_t n = std::min<int32_t>(256, B - i0);
                memcpy(c.v, cut_host + i0, sizeof(double) * (size_t)n);
                put_cut_kernel<<<1, 256, 0, side>>>(d->dring + (size_t)slot * tm_dropin::SLOT_DOUBLES + i0, n, c);
                TM_CHECK_LAUNCH();
            }
            TM_HIP(hipEventRecord(d->copy_ev[slot], side));
            d->last_slot = slot;
            d->last_n = B;
            d->last_side = k;
        }
        cut = d->dring + (size_t)slot * tm_dropin::SLOT_DOUBLES;
    }
    if (!std_done && gl.cnt) {   // no cut times in the launch argument: the lookup alone (workgroup 0 idle but the reset)
        CutArg c;
        launch_std(0, c, nullptr, nullptr, 0);
        TM_CHECK_LAUNCH();
    }
    int rc = encoder_fwd_impl(w, n_feat, e_feat, etab, 1, B, W, 1, node6, eid3, ts3, cat, cut, cnt, d->ws[k], out_imp,
                              side, !std_done);
    if (rc != TM_OK) return rc;
    if (out_gfac && !fused_gate) {
        const size_t lds = gate_lds(P);
        if (lds > 160 * 1024) return fail(TM_E_UNSUPPORTED, "tm_dropin_forward: LDS budget exceeded");
        hipEvent_t pe = prof_begin(side);
        const unsigned rblocks = (unsigned)((n_pos + 63) / 64);
        if (gl.cnt) {
            // cached: the hits have their factor (the lookup), the misses (listed) run the register gate and fill
            // the cache
#define TM_GATE_LIST(Q)                                                                                            \
    gate_reg_kernel<Q><<<dim3(rblocks), 256, 0, side>>>(P, (int32_t)n_pos, nullptr, e_feat, out_gfac, nullptr, eid3, \
                                                         ts3, gl.list, gl.cnt, d->gcache, d->gcache_n)
            if (nq == 11) TM_GATE_LIST(11);
            else if (nq == 12) TM_GATE_LIST(12);
            else if (nq == 13) TM_GATE_LIST(13);
            else TM_GATE_LIST(22);
#undef TM_GATE_LIST
        } else if (reg && nq == 11)
            gate_reg_kernel<11><<<dim3(rblocks), 256, 0, side>>>(P, (int32_t)n_pos, nullptr, e_feat, out_gfac, nullptr, eid3, ts3);
        else if (reg && nq == 12)
            gate_reg_kernel<12><<<dim3(rblocks), 256, 0, side>>>(P, (int32_t)n_pos, nullptr, e_feat, out_gfac, nullptr, eid3, ts3);
        else if (reg && nq == 13)
            gate_reg_kernel<13><<<dim3(rblocks), 256, 0, side>>>(P, (int32_t)n_pos, nullptr, e_feat, out_gfac, nullptr, eid3, ts3);
        else if (reg)
            gate_reg_kernel<22><<<dim3(rblocks), 256, 0, side>>>(P, (int32_t)n_pos, nullptr, e_feat, out_gfac, nullptr, eid3, ts3);
        else
            gate_pos_kernel<<<dim3((unsigned)((n_pos + TILE_ROWS - 1) / TILE_ROWS)), 256, lds, side>>>(
                P, n_pos, W, e_feat, eid3, ts3, nullptr, out_gfac);
        TM_CHECK_LAUNCH();
        prof_end("gate_pos_kernel", side, pe);
    }
    if (slot >= 0) {
        TM_HIP(hipEventRecord(d->read_ev[slot][k], side));
        d->read_used[slot][k] = true;
    }
    TM_HIP(hipEventRecord(d->ev_side[k], side));
    TM_HIP(hipStreamWaitEvent(cur, d->ev_side[k], 0));
    return TM_OK;
}

static int edge_importance_gf3(int32_t B, int32_t W, int32_t N, const float *gf0, const float *gf1, const float *gf2,
                               const int32_t *e0, const int32_t *e1, const int32_t *e2, const float *i0, const float *i1,
                               const float *i2, const int32_t *n10, const int32_t *n11, const int32_t *n12,
                               const int32_t *x10, const int32_t *x11, const int32_t *x12, const int32_t *n20,
                               const int32_t *n21, const int32_t *n22, const int32_t *x20, const int32_t *x21,
                               const int32_t *x22, float *out_h1, float *out_h2, float *keep_h1, float *keep_h2,
                               void *stream);

extern "C" int tm_edge_importance_gf3(int32_t B, int32_t W, int32_t N, const float *gf0, const float *gf1,
                                      const float *gf2, const int32_t *e0, const int32_t *e1, const int32_t *e2,
                                      const float *i0, const float *i1, const float *i2, const int32_t *n10,
                                      const int32_t *n11, const int32_t *n12, const int32_t *x10, const int32_t *x11,
                                      const int32_t *x12, const int32_t *n20, const int32_t *n21, const int32_t *n22,
                                      const int32_t *x20, const int32_t *x21, const int32_t *x22, float *out_h1,
                                      float *out_h2, void *stream) {
    return edge_importance_gf3(B, W, N, gf0, gf1, gf2, e0, e1, e2, i0, i1, i2, n10, n11, n12, x10, x11, x12, n20, n21,
                               n22, x20, x21, x22, out_h1, out_h2, nullptr, nullptr, stream);
}

extern "C" int tm_edge_importance_gf3_bern(int32_t B, int32_t W, int32_t N, const float *gf0, const float *gf1,
                                           const float *gf2, const int32_t *e0, const int32_t *e1, const int32_t *e2,
                                           const float *i0, const float *i1, const float *i2, const int32_t *n10,
                                           const int32_t *n11, const int32_t *n12, const int32_t *x10,
                                           const int32_t *x11, const int32_t *x12, const int32_t *n20,
                                           const int32_t *n21, const int32_t *n22, const int32_t *x20,
                                           const int32_t *x21, const int32_t *x22, float *out_p1, float *out_p2,
                                           float *keep_h1, float *keep_h2, void *stream) {
    if (!keep_h1 || !keep_h2) return fail(TM_E_ARG, "tm_edge_importance_gf3_bern: NULL keep output");
    return edge_importance_gf3(B, W, N, gf0, gf1, gf2, e0, e1, e2, i0, i1, i2, n10, n11, n12, x10, x11, x12, n20, n21,
                               n22, x20, x21, x22, out_p1, out_p2, keep_h1, keep_h2, stream);
}

static int edge_importance_gf3(int32_t B, int32_t W, int32_t N, const float *gf0, const float *gf1, const float *gf2,
                               const int32_t *e0, const int32_t *e1, const int32_t *e2, const float *i0, const float *i1,
                               const float *i2, const int32_t *n10, const int32_t *n11, const int32_t *n12,
                               const int32_t *x10, const int32_t *x11, const int32_t *x12, const int32_t *n20,
                               const int32_t *n21, const int32_t *n22, const int32_t *x20, const int32_t *x21,
                               const int32_t *x22, float *out_h1, float *out_h2, float *keep_h1, float *keep_h2,
                               void *stream) {
    if (B < 0 || W <= 0 || N <= 0) return fail(TM_E_ARG, "tm_edge_importance_gf3: bad arguments");
    if (B == 0) return TM_OK;
    ExplainSides a{{gf0, gf1, gf2}, {i0, i1, i2}, {e0, e1, e2}, {n10, n11, n12}, {x10, x11, x12}, {n20, n21, n22},
                   {x20, x21, x22}};
    for (int s = 0; s < 3; ++s)
        if (!a.gf[s] || !a.imp[s] || !a.eid3[s] || !a.s1n[s] || !a.s1e[s] || !a.s2n[s] || !a.s2e[s])
            return fail(TM_E_ARG, "tm_edge_importance_gf3: NULL pointer");
    if (!out_h1 || !out_h2) return fail(TM_E_ARG, "tm_edge_importance_gf3: NULL output");
    int hbits = 6;
    while ((1 << hbits) < 2 * 3 * W) ++hbits;
    if (hbits > 14) return fail(TM_E_UNSUPPORTED, "tm_edge_importance_gf3: too many walks per event");
    const size_t hlds = 2 * sizeof(int32_t) * (1u << hbits);
    hipEvent_t pe = prof_begin(S_(stream));
    explain_hash3_kernel<<<dim3((unsigned)(3 * B)), 256, hlds, S_(stream)>>>(a, B, W, N, hbits, out_h1, out_h2,
                                                                            keep_h1, keep_h2);
    TM_CHECK_LAUNCH();
    prof_end("explain_hash_kernel", S_(stream), pe);
    return TM_OK;
}

extern "C" int tm_edge_importance_gf(const float *gfac, int32_t n_groups, int32_t B, int32_t W, int32_t N,
                                     const int32_t *eid3, const float *imp, const int32_t *sub1_node,
                                     const int32_t *sub1_eid, const int32_t *sub2_node, const int32_t *sub2_eid,
                                     float *out_h1, float *out_h2, void *stream) {
    if (n_groups < 0 || B < 0 || W <= 0 || N <= 0) return fail(TM_E_ARG, "tm_edge_importance_gf: bad arguments");
    const int64_t rows = (int64_t)n_groups * B;
    if (rows == 0) return TM_OK;
    if (!gfac || !eid3 || !imp || !sub1_node || !sub1_eid || !sub2_node || !sub2_eid || !out_h1 || !out_h2)
        return fail(TM_E_ARG, "tm_edge_importance_gf: NULL pointer");
    int hbits = 6;
    while ((1 << hbits) < 2 * 3 * W) ++hbits;
    if (hbits > 14) return fail(TM_E_UNSUPPORTED, "tm_edge_importance_gf: too many walks per event");
    const size_t hlds = 2 * sizeof(int32_t) * (1u << hbits);
    hipEvent_t pe = prof_begin(S_(stream));
    explain_hash_kernel<<<dim3((unsigned)rows), 256, hlds, S_(stream)>>>(W, N, hbits, eid3, gfac, imp, sub1_node,
                                                                        sub1_eid, sub2_node, sub2_eid, out_h1, out_h2);
    TM_CHECK_LAUNCH();
    prof_end("explain_hash_kernel", S_(stream), pe);
    return TM_OK;
}

#ifdef TM_TRACE
extern "C" int tm_debug_trace(unsigned long long *host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(tmk::g_tr), sizeof(unsigned long long) * 8192 * 32, 0,
                                    hipMemcpyDeviceToHost);
}
#endif
#ifdef TM_STAMPS
extern "C" int tm_debug_stamps(unsigned long long *host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(tmk::g_st), sizeof(unsigned long long) * 30, 0,
                                    hipMemcpyDeviceToHost);
}
#endif
