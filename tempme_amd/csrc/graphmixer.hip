// Base-GraphMixer node embeddings with hop-1 explanation weights on gfx950 (the consumer of the
// explanation path for base_type == 'graphmixer': temp_exp_main.py feeds retrieve_explanation's
// hop-1 weights into GraphMixer.contrast).
//
// Reference (dharunm236/TempME, GraphM/graphmixer.py):
//   compute_node_temporal_embeddings :142-193  edge features (zeroed on padding neighbours unless
//                                              edge_attr is given), TimeEncoder of cut - t (zeroed on
//                                              padding), projection, MLPMixer x L, masked mean over the
//                                              tokens, softmax(valid ? 1 : -1e10) * ew neighbour mean
//   TimeEncoder                      :21-50    cos(Linear(1, d)(t))
//   MLPMixer / FeedForwardNet        :244-315  token mix (LayerNorm over tokens, N -> N/2 -> N, GELU),
//                                              channel mix (LayerNorm over channels, C -> 4C -> C), the
//                                              explanation weight on the input and both branch outputs
//
// One workgroup (4 waves) per row (root node): the row's N <= 32 neighbour tokens stay in LDS for the
// whole embedding, in ~50 KB at C = T = 172 so three workgroups share a CU (12 waves, the register
// budget set to match).  GEMMs (projection, channel FFN) on fp32 MFMA 16x16x4 with the activations as
// the A operand read from LDS (ds_read_b128: LDS layout swaps the (4 k-steps x 4 lane groups) inside
// every 16-wide K block so a lane's four K values are contiguous) and the weights as the B operand from
// fragments packed once per weight version (tm_gm_pack, one dwordx4 per lane per 16-K block); a wave
// takes the output tiles wave + 4i and runs them in one K loop (each A fragment read once for all of
// them, the next block's fragments in flight, ping-pong registers).  The projection input goes through
// LDS one K half at a time; the channel LayerNorm is applied to the first FFN GEMM's A fragments as they
// are read (no normalised copy of X); the 4C hidden features go through LDS in chunks of 192 (GELU in
// the first GEMM's epilogue) and the second GEMM accumulates across the chunks in registers.  Token
// mixing, LayerNorm statistics and the masked means are VALU / wave reductions.  The output layer and
// the MergeLayer score are plain [rows x 2C] GEMMs left to the library (tempme_amd/graphmixer.py).
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace tmk {

typedef float gmx4 __attribute__((ext_vector_type(4)));

constexpr int GM_MT = 32;      // tokens per row (two 16-row MFMA tiles)
constexpr int GM_HCH = 192;    // channel-FFN hidden features per LDS chunk (12 tiles: 3 per wave; 128: 2 % slower)
constexpr int GM_MAXL = 4;

struct GmArgs {
    int32_t R, N, C, T, D, L, HT, HC;
    const int32_t *node, *nid, *eid;
    const double *cut, *ts;
    const float *ew, *edge_attr, *n_feat, *e_feat, *time_w, *time_b;
    const float4 *proj_w;
    const float *proj_b;
    const float *const *lw;   // [L][12] device table (kept out of the scalar register file)
    float *x_mean, *node_out;
};

__host__ __device__ inline int32_t gm_r16(int32_t x) { return (x + 15) & ~15; }

// row `off` of the device layer table as a global-address-space table of global pointers: loads through
// generic pointers are FLAT loads, which also count on lgkmcnt (every later LDS wait waited for them)
__device__ __forceinline__ gptr<const gptr<const float>> gm_layer(const float *const *lw, int off) {
    return (gptr<const gptr<const float>>)(lw + off);
}

// LDS index of (token m, feature k) in a [32][P] image: inside each 16-wide K block the position of
// k = 16G + 4s + j is 16G + 4j + s, so lane group j's four K values of one MFMA block are one float4
__device__ __forceinline__ int gm_idx(int m, int k, int P) { return m * P + (k & ~15) + 4 * (k & 3) + ((k >> 2) & 3); }

// threadIdx.x laundered through an opaque asm: lane-dependent addresses computed from it cannot be hoisted
// out of the layer loop by LICM (hoisted, they stay live across every phase and cost the third wave)
__device__ __forceinline__ int gm_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

__device__ __forceinline__ float gm_gelu(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

// sum over the 64 lanes of a wave
__device__ __forceinline__ float gm_wsum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// The wave's output tiles nt0 + 4 i (i < ntw <= NTW) in one K loop: per K block the A fragments are read
// from LDS once for all of them (and, LN, normalised once: the channel LayerNorm (:300) applied as they
// are read, (x - mean_m) * rstd_m * w_k + b_k with the LN parameters in the image's permuted K order, so
// no normalised copy of X takes LDS), and the next block's weight fragments and A fragments are in
// flight during this block's NTW * NMT * 4 MFMAs.  acc accumulates (callers zero it).  Padding tokens
// (m >= N) only produce rows the caller discards; channels >= C have w = b = 0.
template <int NMT, int NTW, bool LN>
__device__ __forceinline__ void gm_gemm_mt(const float *X, int P, int GX, const float4 *Wp, int NT, int nt0, int ntw,
                                           int G0, int nG, gmx4 (&acc)[NTW][2], const float *lnw, const float *lnb,
                                           const float (&mr)[2], const float (&rr)[2]) {
    const int lane = gm_tid() & 63, m = lane & 15, j = lane >> 4;
    const size_t gs = (size_t)NT * 64;
    const float4 *wp = Wp + (size_t)nt0 * 64 + lane + (size_t)G0 * gs;
    const float *xr = X + m * P + 4 * j + 16 * (G0 - GX);
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    // block g's fragments: B of the wave's tiles, A of its token tiles, LN weight / bias of its K values
    auto load = [&](int g, float4 (&b)[NTW], float4 (&x)[NMT], float4 &lw, float4 &lb) {
#pragma unroll
        for (int i = 0; i < NTW; ++i) b[i] = i < ntw ? wp[i * 256 + (size_t)g * gs] : z4;
#pragma unroll
        for (int q = 0; q < NMT; ++q) x[q] = *reinterpret_cast<const float4 *>(xr + 16 * q * P + 16 * g);
        if (LN) {
            lw = *reinterpret_cast<const float4 *>(lnw + 16 * (G0 + g) + 4 * j);
            lb = *reinterpret_cast<const float4 *>(lnb + 16 * (G0 + g) + 4 * j);
        }
    };
    auto mma = [&](const float4 (&b)[NTW], const float4 (&x)[NMT], const float4 &lw, const float4 &lb) {
        float4 av[NMT];
#pragma unroll
        for (int q = 0; q < NMT; ++q) {
            av[q] = x[q];
            if (LN) {
                av[q].x = (x[q].x - mr[q]) * rr[q] * lw.x + lb.x;
                av[q].y = (x[q].y - mr[q]) * rr[q] * lw.y + lb.y;
                av[q].z = (x[q].z - mr[q]) * rr[q] * lw.z + lb.z;
                av[q].w = (x[q].w - mr[q]) * rr[q] * lw.w + lb.w;
            }
        }
#pragma unroll
        for (int i = 0; i < NTW; ++i) {
            if (i >= ntw) break;
#pragma unroll
            for (int q = 0; q < NMT; ++q) {
                acc[i][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q].x, b[i].x, acc[i][q], 0, 0, 0);
                acc[i][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q].y, b[i].y, acc[i][q], 0, 0, 0);
                acc[i][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q].z, b[i].z, acc[i][q], 0, 0, 0);
                acc[i][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q].w, b[i].w, acc[i][q], 0, 0, 0);
            }
        }
    };
    // ping-pong buffers (no register copies: a copy of a pending load would wait for it)
    float4 b0[NTW], b1[NTW], x0[NMT], x1[NMT], w0 = z4, w1 = z4, l0 = z4, l1 = z4;
    if (nG > 0) load(0, b0, x0, w0, l0);
    for (int g = 0; g < nG; g += 2) {
        if (g + 1 < nG) load(g + 1, b1, x1, w1, l1);
        mma(b0, x0, w0, l0);
        if (g + 1 >= nG) break;
        if (g + 2 < nG) load(g + 2, b0, x0, w0, l0);
        mma(b1, x1, w1, l1);
    }
}

// LDS plan (floats): X [32][XP] | U [ulen] | token mean, rstd [2][32] | LN weight, bias [2][C16] | ew_eff,
// valid [2][32].  U holds, in turn, the projection input one K half at a time ([32][16 KH + 4]), the token
// mixing's column statistics and the channel FFN's hidden chunk ([32][GM_HCH + 4]).  ~50 KB at C = T =
// 172: three workgroups (12 waves) per CU, the register budget set to match (amdgpu_waves_per_eu).
template <int NMT, int NTW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) gm_embed_kernel(GmArgs a) {
    extern __shared__ float gm_lds[];
    const int r = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int N = a.N, C = a.C, T = a.T, D = a.D;
    const int C16 = gm_r16(C), KG = gm_r16(C + T) / 16, KH = (KG + 1) / 2;
    const int XP = C16 + 4, HP = GM_HCH + 4, K0P = 16 * KH + 4;
    const int ulen = max(max(GM_MT * K0P, GM_MT * HP), 2 * C16);
    float *X = gm_lds, *U = X + GM_MT * XP;
    float *X0 = U, *H = U;
    float *tmean = U + ulen, *trstd = tmean + GM_MT, *lnw = trstd + GM_MT, *lnb = lnw + C16;
    float *sew = lnb + C16, *sval = sew + GM_MT;
    const bool has_ew = a.ew != nullptr;
    if (tid < GM_MT) {
        const bool v = tid < N && a.nid[(size_t)r * N + tid] != 0;
        sval[tid] = v ? 1.f : 0.f;
        // exp_src * mask (:154-155); without explanation weights the mixer multiplies by nothing (1.0)
        sew[tid] = tid < N ? (has_ew ? a.ew[(size_t)r * N + tid] * (v ? 1.f : 0.f) : 1.f) : 0.f;
    }
    __syncthreads();
    const int NT = C16 / 16, ntw = (NT - wave + 3) / 4;   // this wave's output tiles: wave + 4 i, i < ntw
    float mr[2] = {0.f, 0.f}, rr[2] = {0.f, 0.f};
    // ---- projection (:156-167): X = [E(e) | cos(dt w + b)] Wp^T + bp, K in two halves through U
    // (padding neighbours: time part zeroed, edge part too unless edge_attr is given)
    const double cut = a.cut[r];
    for (int h = 0; h < 2; ++h) {
        const int G0 = h * KH, nG = min(KH, KG - G0), W16 = 16 * nG;
        if (nG <= 0) break;
        for (int i = tid; i < GM_MT * W16; i += blockDim.x) {
            const int t = i / W16, k = 16 * G0 + (i - t * W16);
            float v = 0.f;
            if (t < N) {
                const bool valid = sval[t] != 0.f;
                if (k < C) {
                    if (a.edge_attr) v = a.edge_attr[((size_t)r * N + t) * C + k];
                    else if (valid) v = a.e_feat[(size_t)a.eid[(size_t)r * N + t] * C + k];
                } else if (k < C + T && valid) {
                    // Linear(1, d) on fp32 dt: one rounding of dt * w + b (what the reference's CPU addmm gives)
                    const float dt = (float)(cut - a.ts[(size_t)r * N + t]);
                    const float arg = (float)((double)dt * (double)a.time_w[k - C] + (double)a.time_b[k - C]);
                    v = cos_rd(arg);   // branch-free fp64-reduced cos (common.h), |err| <= 1.7e-7
                }
            }
            X0[gm_idx(t, k - 16 * G0, K0P)] = v;
        }
        __syncthreads();
        {
            gmx4 acc[NTW][2];
#pragma unroll
            for (int i = 0; i < NTW; ++i) acc[i][0] = acc[i][1] = gmx4{0.f, 0.f, 0.f, 0.f};
            gm_gemm_mt<NMT, NTW, false>(X0, K0P, G0, a.proj_w, NT, wave, ntw, G0, nG, acc, nullptr, nullptr, mr, rr);
#pragma unroll
            for (int i = 0; i < NTW; ++i) {
                if (i >= ntw) break;
                const int n = 16 * (wave + 4 * i) + (lane & 15);
                const float bv = n < C ? a.proj_b[n] : 0.f;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int t = 16 * mt + 4 * (lane >> 4) + e;
                        const int ix = gm_idx(t, n, XP);
                        const bool in = mt < NMT && n < C && t < N;
                        // first half stored, second half (+ bias) added: the same two-part sum for every element
                        if (h == 0) X[ix] = in ? acc[i][mt][e] : 0.f;
                        else if (in) X[ix] = X[ix] + acc[i][mt][e] + bv;
                    }
            }
        }
        __syncthreads();
    }
    if (KG == 1) {   // one K half only: the bias is still owed
        for (int i = tid; i < GM_MT * C16; i += blockDim.x) {
            const int t = i / C16, n = i - t * C16;
            if (t < N && n < C) X[gm_idx(t, n, XP)] += a.proj_b[n];
        }
        __syncthreads();
    }
    for (int l = 0; l < a.L; ++l) {
        const auto w = gm_layer(a.lw, 12 * l);
        // ---- token mixing (:289-297).  Per channel c: H = gelu(W1 LN_t(X[:, c] * ew) + b1), Y = W2 H + b2,
        // X[:, c] = (Y + ... ) * ew + X[:, c] * ew -- two tiny GEMMs per 16-channel tile on MFMA: W1 (HT x N) as
        // the A operand against the normalised column (B, K = tokens), then W2 (N x HT) against H, whose
        // K order is permuted (step s, lane group g <-> hidden unit 4g + s) so H stays in the registers the
        // first MFMA left it in.  Column statistics first, one thread per channel.
        float *cm = U, *cr = U + C16;
        for (int c = tid; c < C; c += blockDim.x) {
            float sm = 0.f;
            for (int t = 0; t < N; ++t) sm += X[gm_idx(t, c, XP)] * sew[t];
            const float mean = sm / (float)N;
            float q = 0.f;
            for (int t = 0; t < N; ++t) {
                const float d = X[gm_idx(t, c, XP)] * sew[t] - mean;
                q += d * d;
            }
            cm[c] = mean;
            cr[c] = 1.f / sqrtf(q / (float)N + 1e-5f);
        }
        // channel LayerNorm parameters in the image's permuted K order (read as float4 by gm_gemm_mt)
        for (int k = tid; k < C16; k += blockDim.x) {
            const int p = (k & ~15) + 4 * (k & 3) + ((k >> 2) & 3);
            lnw[p] = k < C ? w[6][k] : 0.f;
            lnb[p] = k < C ? w[7][k] : 0.f;
        }
        __syncthreads();
        {
            const int ln = gm_tid() & 63, g = ln >> 4, li = ln & 15, HT = a.HT;
            float a1[2][4], a2[2][4], lg[2][4], lb[2][4], b2v[2][4], b1v[4];
#pragma unroll
            for (int G = 0; G < 2; ++G)
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) {
                    const int t = 16 * G + 4 * s2 + g;          // step-2 K index of this lane
                    a1[G][s2] = (li < HT && t < N) ? w[2][li * N + t] : 0.f;
                    lg[G][s2] = t < N ? w[0][t] : 0.f;
                    lb[G][s2] = t < N ? w[1][t] : 0.f;
                    const int tt = 16 * G + li, j = 4 * g + s2;   // step-3 A: W2[t][j], K permuted
                    a2[G][s2] = (tt < N && j < HT) ? w[4][tt * HT + j] : 0.f;
                    const int tr = 16 * G + 4 * g + s2;         // step-3 D row of this lane's element s2
                    b2v[G][s2] = tr < N ? w[5][tr] : 0.f;
                }
#pragma unroll
            for (int i = 0; i < 4; ++i) b1v[i] = 4 * g + i < HT ? w[3][4 * g + i] : 0.f;
            for (int nt = wave; nt < NT; nt += 4) {
                const int c = 16 * nt + li;
                const bool cv = c < C;
                const float mean = cv ? cm[c] : 0.f, rstd = cv ? cr[c] : 0.f;
                gmx4 hacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int G = 0; G < 2; ++G)
#pragma unroll
                    for (int s2 = 0; s2 < 4; ++s2) {
                        const int t = 16 * G + 4 * s2 + g;
                        const float xn = (cv && t < N) ? (X[gm_idx(t, c, XP)] * sew[t] - mean) * rstd * lg[G][s2] + lb[G][s2] : 0.f;
                        hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[G][s2], xn, hacc, 0, 0, 0);
                    }
                float h[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) h[i] = 4 * g + i < HT ? gm_gelu(hacc[i] + b1v[i]) : 0.f;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    gmx4 y = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int s2 = 0; s2 < 4; ++s2) y = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[mt][s2], h[s2], y, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int t = 16 * mt + 4 * g + i;
                        if (cv && t < N) {
                            const int ix = gm_idx(t, c, XP);
                            X[ix] = (y[i] + b2v[mt][i]) * sew[t] + X[ix] * sew[t];
                        }
                    }
                }
            }
        }
        __syncthreads();
        // ---- channel LayerNorm statistics (:300), one wave per token; applied inside the first FFN GEMM
        for (int t = wave; t < GM_MT; t += 4) {
            float mean = 0.f, rstd = 0.f;
            if (t < N) {
                float s = 0.f, q = 0.f;
                for (int c = lane; c < C; c += 64) s += X[gm_idx(t, c, XP)];
                mean = gm_wsum(s) / (float)C;
                for (int c = lane; c < C; c += 64) {
                    const float d = X[gm_idx(t, c, XP)] - mean;
                    q += d * d;
                }
                rstd = 1.f / sqrtf(gm_wsum(q) / (float)C + 1e-5f);
            }
            if (lane == 0) {
                tmean[t] = mean;
                trstd[t] = rstd;
            }
        }
        __syncthreads();
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            mr[mt] = tmean[16 * mt + (lane & 15)];
            rr[mt] = trstd[16 * mt + (lane & 15)];
        }
        // ---- channel FFN (:302-305): hidden chunks of GM_HCH through LDS (GELU in the first GEMM's epilogue)
        const int NH = gm_r16(a.HC) / 16;
        const float4 *W1 = (const float4 *)(w[8]), *W2 = (const float4 *)(w[10]);
        // every chunk's first GEMM normalises the layer's input X, so the second GEMM accumulates its
        // output tiles in registers across the chunks and X is updated once, after them
        gmx4 acc2[NTW][2];
#pragma unroll
        for (int i = 0; i < NTW; ++i) acc2[i][0] = acc2[i][1] = gmx4{0.f, 0.f, 0.f, 0.f};
        for (int h0 = 0; h0 < NH; h0 += GM_HCH / 16) {
            const int nh = min(GM_HCH / 16, NH - h0), nw1 = (nh - wave + 3) / 4;
            {
                gmx4 acc[GM_HCH / 64][2];
#pragma unroll
                for (int i = 0; i < GM_HCH / 64; ++i) acc[i][0] = acc[i][1] = gmx4{0.f, 0.f, 0.f, 0.f};
                gm_gemm_mt<NMT, GM_HCH / 64, true>(X, XP, 0, W1, NH, h0 + wave, nw1, 0, C16 / 16, acc, lnw, lnb, mr, rr);
#pragma unroll
                for (int i = 0; i < GM_HCH / 64; ++i) {
                    if (i >= nw1) break;
                    const int ht = wave + 4 * i, n = 16 * (h0 + ht) + (lane & 15);
                    const float bv = n < a.HC ? w[9][n] : 0.f;
#pragma unroll
                    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int t = 16 * mt + 4 * (lane >> 4) + e;
                            H[gm_idx(t, 16 * ht + (lane & 15), HP)] = (mt < NMT && n < a.HC) ? gm_gelu(acc[i][mt][e] + bv) : 0.f;
                        }
                }
            }
            __syncthreads();
            gm_gemm_mt<NMT, NTW, false>(H, HP, h0, W2, NT, wave, ntw, h0, nh, acc2, nullptr, nullptr, mr, rr);
            __syncthreads();
        }
        // X = (Y + b2) * ew + X (:305, the explanation weight on the branch output)
#pragma unroll
        for (int i = 0; i < NTW; ++i) {
            const int nt = wave + 4 * i;
            if (nt >= NT) break;
            const int n = 16 * nt + (lane & 15);
            const float bv = n < C ? w[11][n] : 0.f;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int t = 16 * mt + 4 * (lane >> 4) + e;
                    if (mt < NMT && t < N && n < C) {
                        const int ix = gm_idx(t, n, XP);
                        X[ix] = (acc2[i][mt][e] + bv) * sew[t] + X[ix];
                    }
                }
        }
        __syncthreads();
    }
    // ---- masked mean over the tokens (:176-178) and the neighbour-feature mean (:181-189)
    for (int c = tid; c < C; c += blockDim.x) {
        float s = 0.f;
        for (int t = 0; t < N; ++t) s += X[gm_idx(t, c, XP)] * sval[t] * (has_ew ? sew[t] : 1.f);
        a.x_mean[(size_t)r * C + c] = s / (float)N;
    }
    float nvalid = 0.f;
    for (int t = 0; t < N; ++t) nvalid += sval[t];
    for (int d = tid; d < D; d += blockDim.x) {
        float s = 0.f;
        for (int t = 0; t < N; ++t) {
            // softmax(valid ? 1 : -1e10) over the row: 1 / n_valid on valid neighbours (exp(-1e10 - 1) == 0),
            // 1 / N everywhere when none is valid
            float sc = nvalid > 0.f ? sval[t] / nvalid : 1.f / (float)N;
            if (has_ew) sc *= sew[t];
            s += a.n_feat[(size_t)a.nid[(size_t)r * N + t] * D + d] * sc;
        }
        a.node_out[(size_t)r * D + d] = s / (float)N + a.n_feat[(size_t)a.node[r] * D + d];
    }
}

// W [n_out][k] row-major -> B-operand fragments: packed[(G * NT + nt) * 64 + lane][s] =
// W[16 nt + (lane & 15)][16 G + 4 s + (lane >> 4)] (zero outside W)
__global__ void gm_pack_kernel(const float *__restrict__ w, int32_t n_out, int32_t k, float *__restrict__ out) {
    const int32_t NT = gm_r16(n_out) / 16, KG = gm_r16(k) / 16;
    const int64_t total = (int64_t)KG * NT * 64 * 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int s = (int)(i & 3), lane = (int)((i >> 2) & 63);
        const int64_t f = i >> 8;
        const int nt = (int)(f % NT), G = (int)(f / NT);
        const int n = 16 * nt + (lane & 15), kk = 16 * G + 4 * s + (lane >> 4);
        out[i] = (n < n_out && kk < k) ? w[(int64_t)n * k + kk] : 0.f;
    }
}

// ================================================================== register-resident form (gm_fused_kernel)
//
// The walk kernel's orientation (encoder.hip): weights are the MFMA A operand (16 output features per
// tile), a wave's 16 tokens are the B operand's columns, lane l holding features 16q + 4(l>>4) + {0..3}
// of token l & 15 -- so the D tile of one GEMM is the B fragment of K tile q of the next and a token
// tile's whole channel FFN, C -> 4C -> C, runs in registers: per pair of hidden tiles the first GEMM
// (two interleaved accumulators over the C / 16 K tiles of the LayerNorm-ed input), GELU on the
// accumulators, then the second GEMM accumulates the pair into the C / 16 output tiles.  No LDS in the
// FFN, no hidden chunks, no barriers inside a layer's channel mix.  Weight fragments stream from L2
// GF_PF ahead in one ring across the pair loop (the fragments of a pair: 4 C/16, a multiple of GF_PF).
// LDS holds the X image [token][channel] (row stride 16 NC + 4) for what crosses tokens: the token
// mixing (both token tiles of a row) and the residual; the projection input's edge-feature rows are
// staged in the same image first (coalesced row loads), the time features computed in the K loop.
constexpr int GF_PF = 4;

// W [n_out][k] row-major -> A-operand fragments, tiles rounded up to multiples of n_mult / k_mult:
// packed[((t * KT + q) * 64 + lane) * 4 + s] = W[16 t + (lane & 15)][16 q + 4 (lane >> 4) + s] (zero outside W)
__global__ void gm_pack_a_kernel(const float *__restrict__ w, int32_t n_out, int32_t k, int32_t KT, int64_t total,
                                 float *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int s = (int)(i & 3), lane = (int)((i >> 2) & 63);
        const int64_t f = i >> 8;
        const int q = (int)(f % KT), t = (int)(f / KT);
        const int n = 16 * t + (lane & 15), kk = 16 * q + 4 * (lane >> 4) + s;
        out[i] = (n < n_out && kk < k) ? w[(int64_t)n * k + kk] : 0.f;
    }
}

// a pointer read from the device layer table is wave-uniform, but the compiler cannot prove it (the
// table is ordinary global memory): without this, a buffer resource built from it sits in VGPRs and every
// buffer load becomes a readfirstlane waterfall loop
template <class P>
__device__ __forceinline__ const float *gf_uniform(P p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<const float *>(((uint64_t)hi << 32) | lo);
}

// the same as a global-address-space pointer, for plain loads (a generic pointer makes them FLAT loads,
// which count on lgkmcnt too: the next LDS wait would also wait for them)
template <class P>
__device__ __forceinline__ gptr<const float> gf_uniform_g(P p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (gptr<const float>)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t gf_rsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, 0x7fffffff, 0x00020000);
}

// one 1-KB fragment: lane offset vo (VGPR), fragment byte offset so (wave-uniform, SGPR)
__device__ __forceinline__ float4 gf_frag(__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
}

__device__ __forceinline__ gmx4 gf_mfma4(const float4 &a, const float4 &b, gmx4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
    return c;
}

// a [n] fp32 vector (n % 4 == 0) as a buffer resource: a float4 at byte offset 16 i (i < n / 4) is
// one buffer load, and any float4 at or beyond n reads zero (the hardware range check on the
// offset incl. the immediate) -- no clamped index, no select, no branch, no 64-bit address per lane
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gf_vrsrc(const float *v, int n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(v), (short)0, n * 4, 0x00020000);
}
__device__ __forceinline__ float4 gf_vload(__amdgpu_buffer_rsrc_t r, int byte_off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

// A wave's place in the workgroup, recomputed at the start of every phase from the laundered thread id
// (gm_tid): values derived once at kernel entry are loop-invariant to the compiler, which then hoists
// every lane mask and LDS address of the layer loop out of it and holds them across all phases.
template <int NC, int NTT>
struct GfIds {
    static constexpr int RPW = 4 / NTT, XS = 16 * NC + 4, C16 = 16 * NC;
    int lane, m, j, tt, rl, tok;
    float *Xr, *Xw, *sew, *sval;
    __device__ __forceinline__ GfIds() {
        extern __shared__ float gm_lds[];
        const int t = gm_tid(), wave = t >> 6;
        lane = t & 63;
        m = lane & 15;
        j = lane >> 4;
        rl = wave / NTT;
        tt = wave % NTT;
        tok = 16 * tt + m;
        Xr = gm_lds + rl * NTT * 16 * XS;                   // the row's image: token t at Xr + t * XS
        Xw = Xr + tt * 16 * XS;                             // this wave's 16 tokens
        sew = gm_lds + 64 * XS + rl * 64;
        sval = sew + 32;
    }
};

// NC = channel tiles (C <= 16 NC), NTT = token tiles per row (N <= 16 NTT).  A workgroup of 4 waves takes
// 4 / NTT rows, one wave per (row, token tile).  LDS plan (floats): X image [4 waves][16 tokens][XS] |
// per row: ew_eff, valid [2][32].
template <int NC, int NTT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NC <= 13 ? 3 : 2))) gm_fused_kernel(GmArgs a) {
    typedef GfIds<NC, NTT> Ids;
    constexpr int RPW = Ids::RPW, XS = Ids::XS;
    extern __shared__ float gm_lds[];
    const int R = a.R, N = a.N, C = a.C, T = a.T;
    const bool has_ew = a.ew != nullptr;
    {
        const int tid = gm_tid();
        if (tid < RPW * 32) {
            const int rl2 = tid >> 5, t = tid & 31, r2 = min((int)blockIdx.x * RPW + rl2, R - 1);
            float *se = gm_lds + 64 * XS + rl2 * 64;
            const bool v = t < N && a.nid[(size_t)r2 * N + t] != 0;
            se[32 + t] = v ? 1.f : 0.f;
            // exp_src * mask (:154-155); without explanation weights the mixer multiplies by nothing (1.0)
            se[t] = t < N ? (has_ew ? a.ew[(size_t)r2 * N + t] * (v ? 1.f : 0.f) : 1.f) : 0.f;
        }
    }
    // ---- projection input: the wave's 16 edge-feature rows into its image (padding neighbours zeroed
    // unless edge_attr is given), one coalesced row load per token
    {
        const Ids I;
        const int rr = min((int)blockIdx.x * RPW + I.rl, R - 1);
        const size_t rowN = (size_t)rr * N;
        const int nf4 = C >> 2;
#pragma unroll 4
        for (int mm = 0; mm < 16; ++mm) {
            const int t = 16 * I.tt + mm, tc = min(t, N - 1);
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (I.lane < nf4) {
                if (a.edge_attr) {
                    v = reinterpret_cast<const float4 *>(a.edge_attr + (rowN + tc) * C)[I.lane];
                    if (t >= N) v = make_float4(0.f, 0.f, 0.f, 0.f);
                } else {
                    const bool ok = t < N && a.nid[rowN + tc] != 0;
                    v = reinterpret_cast<const float4 *>(a.e_feat + (size_t)a.eid[rowN + tc] * C)[I.lane];
                    if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                *reinterpret_cast<float4 *>(I.Xw + mm * XS + 4 * I.lane) = v;
            }
        }
    }
    __syncthreads();
    // ---- projection (:156-167): X = [E(e) | cos(dt w + b)] Wp^T + bp over K tiles padded to a multiple
    // of 4 (zero fragments); B fragment of K tile q: edge features from the image, time features computed
    {
        const Ids I;
        const int m = I.m, j = I.j, vo = I.lane * 16;
        const int rr = min((int)blockIdx.x * RPW + I.rl, R - 1), tokc = min(I.tok, N - 1);
        const size_t rowN = (size_t)rr * N;
        const bool tv = I.tok < N && a.nid[rowN + tokc] != 0;
        const float dt = (float)(a.cut[rr] - a.ts[rowN + tokc]);
        // KP = the pack's K tiles per output tile (tm_gm_pack_a k_mult 4: the fragment pitch); the loop runs
        // QG K tiles per iteration up to KL.  The ring slot of fragment f is f % GF_PF in every iteration, so an
        // iteration's QG * NC fragments must be a multiple of GF_PF: QG = 4 (pairs of K tiles, which stop at the
        // K tiles C + T needs, broke that for odd NC: profiles/r05_gm_fused_ab.txt)
        constexpr int QG = 4;
        static_assert((QG * NC) % GF_PF == 0, "ring slots repeat per iteration");
        const int KP = ((C + T + 63) / 64) * 4;
        const int KL = ((C + T + 16 * QG - 1) / (16 * QG)) * QG;
        const auto wr = gf_rsrc(a.proj_w);
        const auto rtw = gf_vrsrc(a.time_w, T), rtb = gf_vrsrc(a.time_b, T), rb = gf_vrsrc(a.proj_b, C);
        gmx4 y[NC];
#pragma unroll
        for (int o = 0; o < NC; ++o) {
            const float4 b = gf_vload(rb, 64 * o + 16 * j);
            y[o] = gmx4{b.x, b.y, b.z, b.w};
        }
        // fragment (o, q) at ((o * KP + q) * 64 + lane) * 16 B; the ring walks q-major, o-minor
        float4 ring[GF_PF];
#pragma unroll
        for (int i = 0; i < GF_PF; ++i) ring[i] = gf_frag(wr, vo, ((i % NC) * KP + i / NC) * 1024);
        for (int q0 = 0; q0 < KL; q0 += QG) {
            // iteration bases opaque per iteration: loop strength reduction would otherwise keep every
            // fragment's offset as its own SGPR induction variable
            int qb = q0 * 1024, qn = min(q0 + QG, KL - QG) * 1024;
            asm volatile("" : "+s"(qb), "+s"(qn));
#pragma unroll
            for (int dq = 0; dq < QG; ++dq) {
                const int k0 = 16 * (q0 + dq) + 4 * j;
                float4 bx;
                if (k0 < C) {
                    bx = *reinterpret_cast<const float4 *>(I.Xw + m * XS + k0);
                } else {
                    // Linear(1, d) on fp32 dt: one rounding of dt * w + b (the reference's CPU addmm); k >= T
                    // reads w = b = 0 and is zeroed
                    const int kt = k0 - C;
                    const float4 fw = gf_vload(rtw, 4 * kt), fb = gf_vload(rtb, 4 * kt);
                    const bool on = tv && kt < T;
                    auto te = [&](float fr, float ph) {
                        return on ? cos_rd((float)((double)dt * (double)fr + (double)ph)) : 0.f;
                    };
                    bx = make_float4(te(fw.x, fb.x), te(fw.y, fb.y), te(fw.z, fb.z), te(fw.w, fb.w));
                }
#pragma unroll
                for (int o = 0; o < NC; ++o) {
                    const int f = dq * NC + o, fn = f + GF_PF;   // this fragment, the one issued into its slot
                    const float4 w = ring[f % GF_PF];
                    const int dn = fn / NC, on = fn % NC;        // K tile q0 + dn (dn < QG) or the next iteration's
                    ring[f % GF_PF] = dn < QG ? gf_frag(wr, vo, qb + (on * KP + dn) * 1024)
                                              : gf_frag(wr, vo, qn + (on * KP + dn - QG) * 1024);
                    y[o] = gf_mfma4(w, bx, y[o]);
                }
            }
        }
        // X = projection, zero on padding tokens and channels (the image keeps them zero from here on)
#pragma unroll
        for (int o = 0; o < NC; ++o) {
            const bool in = I.tok < N && 16 * o + 4 * j < C;
            *reinterpret_cast<float4 *>(I.Xw + m * XS + 16 * o + 4 * j) =
                in ? make_float4(y[o][0], y[o][1], y[o][2], y[o][3]) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __syncthreads();
    const int NH2 = ((a.HC + 31) / 32) * 2;   // hidden tiles, rounded up to pairs (zero fragments)
    for (int l = 0; l < a.L; ++l) {
        const auto w = gm_layer(a.lw, 12 * l);
        // ---- token mixing (:289-297): per 16-channel tile, the token LayerNorm's column statistics of
        // X * ew in registers (a lane holds 4 NTT of the column's tokens; the 4 lane groups combine by two
        // shuffles), then W1 (HT x N) against the normalised column and W2 (N x HT) against H on MFMA (H's
        // K order permuted so it stays in the registers the first MFMA left it in).  A wave's channel tiles
        // are its own, so no barrier separates the statistics from the mixing.
        {
            const Ids I;
            const int g = I.j, li = I.m, HT = a.HT;
            const auto tw0 = gf_uniform_g(w[0]), tw1 = gf_uniform_g(w[1]), tw2 = gf_uniform_g(w[2]),
                       tw3 = gf_uniform_g(w[3]), tw4 = gf_uniform_g(w[4]), tw5 = gf_uniform_g(w[5]);
            float a1[NTT][4], a2[NTT][4], lg[NTT][4], lb[NTT][4], b2v[NTT][4], b1v[4];
#pragma unroll
            for (int G = 0; G < NTT; ++G)
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) {
                    const int t = 16 * G + 4 * s2 + g;
                    a1[G][s2] = (li < HT && t < N) ? tw2[li * N + t] : 0.f;
                    lg[G][s2] = t < N ? tw0[t] : 0.f;
                    lb[G][s2] = t < N ? tw1[t] : 0.f;
                    const int tt2 = 16 * G + li, jj = 4 * g + s2;
                    a2[G][s2] = (tt2 < N && jj < HT) ? tw4[tt2 * HT + jj] : 0.f;
                    const int tr = 16 * G + 4 * g + s2;
                    b2v[G][s2] = tr < N ? tw5[tr] : 0.f;
                }
#pragma unroll
            for (int i = 0; i < 4; ++i) b1v[i] = 4 * g + i < HT ? tw3[4 * g + i] : 0.f;
            // two of the wave's channel tiles per iteration: two independent MFMA / shuffle chains in flight
            // (the same operations per tile, so the same results; one tile per iteration measured 1 % slower,
            // profiles/r05_gm_fused_ab.txt).  Branch-free: the image's rows past N and
            // columns past C hold zeros (the projection wrote them), lg / lb are zero past N, so loads and xn
            // need no select; the token mask of the variance is a float in a VGPR (a compare per element would
            // hold a lane mask in SGPRs); writes keep the lane's channel test (padding columns stay zero).
            float tmk[NTT][4];
#pragma unroll
            for (int G = 0; G < NTT; ++G)
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) {
                    float m = 16 * G + 4 * s2 + g < N ? 1.f : 0.f;
                    asm volatile("" : "+v"(m));
                    tmk[G][s2] = m;
                }
            for (int nt0 = I.tt; nt0 < NC; nt0 += 2 * NTT) {
                float v[2][NTT][4], mean[2], rstd[2];
                int c[2];
                bool cv[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int ntu = min(nt0 + u * NTT, NC - 1);
                    c[u] = 16 * ntu + li;
                    cv[u] = nt0 + u * NTT < NC && c[u] < C;
                    float sm = 0.f;
#pragma unroll
                    for (int G = 0; G < NTT; ++G)
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2) {
                            const int t = 16 * G + 4 * s2 + g;
                            v[u][G][s2] = I.Xr[t * XS + c[u]] * I.sew[t];
                            sm += v[u][G][s2];
                        }
                    mean[u] = sm;
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    float sm = mean[u];
                    sm += __shfl_xor(sm, 16);
                    sm += __shfl_xor(sm, 32);
                    mean[u] = sm / (float)N;
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    float q = 0.f;
#pragma unroll
                    for (int G = 0; G < NTT; ++G)
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2) {
                            const float d = (v[u][G][s2] - mean[u]) * tmk[G][s2];
                            q += d * d;
                        }
                    rstd[u] = q;
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    float q = rstd[u];
                    q += __shfl_xor(q, 16);
                    q += __shfl_xor(q, 32);
                    rstd[u] = 1.f / sqrtf(q / (float)N + 1e-5f);
                }
                gmx4 hacc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
                for (int G = 0; G < NTT; ++G)
#pragma unroll
                    for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            const float xn = (v[u][G][s2] - mean[u]) * rstd[u] * lg[G][s2] + lb[G][s2];
                            hacc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[G][s2], xn, hacc[u], 0, 0, 0);
                        }
                float h[2][4];
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int i = 0; i < 4; ++i) h[u][i] = 4 * g + i < HT ? gm_gelu(hacc[u][i] + b1v[i]) : 0.f;
#pragma unroll
                for (int mt = 0; mt < NTT; ++mt) {
                    gmx4 yy[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
                    for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
                        for (int u = 0; u < 2; ++u)
                            yy[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[mt][s2], h[u][s2], yy[u], 0, 0, 0);
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        if (!cv[u]) continue;
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int t = 16 * mt + 4 * g + i;
                            const int ix = t * XS + c[u];
                            I.Xr[ix] = (yy[u][i] + b2v[mt][i]) * I.sew[t] + I.Xr[ix] * I.sew[t];
                        }
                    }
                }
            }
        }
        __syncthreads();
        // ---- channel mixing (:300-305): the wave's token tile from the image; channel LayerNorm per
        // token (column) in registers, then the FFN with the hidden features in registers
        {
            const Ids I;
            const int m = I.m, j = I.j, vo = I.lane * 16;
            gmx4 xn[NC], y[NC];
            {
                float4 xv[NC];
                float s = 0.f;
#pragma unroll
                for (int q = 0; q < NC; ++q) {
                    xv[q] = *reinterpret_cast<const float4 *>(I.Xw + m * XS + 16 * q + 4 * j);
                    s += (xv[q].x + xv[q].y) + (xv[q].z + xv[q].w);
                }
                s += __shfl_xor(s, 16);
                s += __shfl_xor(s, 32);
                const float mean = s / (float)C;
                float v = 0.f;
#pragma unroll
                for (int q = 0; q < NC; ++q) {
                    const bool in = 16 * q + 4 * j < C;
                    const float d0 = xv[q].x - mean, d1 = xv[q].y - mean, d2 = xv[q].z - mean, d3 = xv[q].w - mean;
                    v += in ? (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3) : 0.f;
                }
                v += __shfl_xor(v, 16);
                v += __shfl_xor(v, 32);
                const float rstd = 1.f / sqrtf(v / (float)C + 1e-5f);
                const auto rw = gf_vrsrc(gf_uniform(w[6]), C), rb = gf_vrsrc(gf_uniform(w[7]), C);
#pragma unroll
                for (int q = 0; q < NC; ++q) {
                    const float4 lw = gf_vload(rw, 64 * q + 16 * j), lbv = gf_vload(rb, 64 * q + 16 * j);
                    xn[q] = gmx4{(xv[q].x - mean) * rstd * lw.x + lbv.x, (xv[q].y - mean) * rstd * lw.y + lbv.y,
                                 (xv[q].z - mean) * rstd * lw.z + lbv.z, (xv[q].w - mean) * rstd * lw.w + lbv.w};
                }
            }
            {
                const auto rb = gf_vrsrc(gf_uniform(w[11]), C);
#pragma unroll
                for (int o = 0; o < NC; ++o) {
                    const float4 b = gf_vload(rb, 64 * o + 16 * j);
                    y[o] = gmx4{b.x, b.y, b.z, b.w};
                }
            }
            const auto r1 = gf_rsrc(gf_uniform(w[8])), r2 = gf_rsrc(gf_uniform(w[10]));
            const auto rb1 = gf_vrsrc(gf_uniform(w[9]), a.HC);
            const int NP = NH2 / 2;
            // pair p's fragment f (compile-time) at the pair's base offset (opaque per pair, as in the
            // projection) + a constant.  f < 2 NC: W1 tile 2p + (f & 1), K tile f >> 1 (pack [HC tiles][NC]);
            // else g = f - 2 NC: W2 tile g >> 1, K tile 2p + (g & 1) (pack [NC][NH2])
            auto issue = [&](int f, int pb1, int pb2) -> float4 {
                if (f < 2 * NC) return gf_frag(r1, vo, pb1 + (((f & 1) * NC + (f >> 1)) * 64) * 16);
                const int g = f - 2 * NC;
                return gf_frag(r2, vo, pb2 + (((g >> 1) * NH2 + (g & 1)) * 64) * 16);
            };
            constexpr int F = 4 * NC;
            float4 ring[GF_PF];
#pragma unroll
            for (int i = 0; i < GF_PF; ++i) ring[i] = issue(i, 0, 0);
            for (int p = 0; p < NP; ++p) {
                int pb1 = p * 2 * NC * 1024, pb2 = p * 2 * 1024;
                int nb1 = min(p + 1, NP - 1) * 2 * NC * 1024, nb2 = min(p + 1, NP - 1) * 2 * 1024;
                asm volatile("" : "+s"(pb1), "+s"(pb2), "+s"(nb1), "+s"(nb2));
                const float4 c0 = gf_vload(rb1, 128 * p + 16 * j), c1 = gf_vload(rb1, 128 * p + 64 + 16 * j);
                gmx4 h0 = {c0.x, c0.y, c0.z, c0.w}, h1 = {c1.x, c1.y, c1.z, c1.w};
#pragma unroll
                for (int q = 0; q < NC; ++q) {
                    const int f = 2 * q;
                    const float4 w0 = ring[f % GF_PF];
                    ring[f % GF_PF] = f + GF_PF < F ? issue(f + GF_PF, pb1, pb2) : issue(f + GF_PF - F, nb1, nb2);
                    const float4 w1 = ring[(f + 1) % GF_PF];
                    ring[(f + 1) % GF_PF] = f + 1 + GF_PF < F ? issue(f + 1 + GF_PF, pb1, pb2) : issue(f + 1 + GF_PF - F, nb1, nb2);
                    h0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.x, xn[q][0], h0, 0, 0, 0);
                    h1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.x, xn[q][0], h1, 0, 0, 0);
                    h0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.y, xn[q][1], h0, 0, 0, 0);
                    h1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.y, xn[q][1], h1, 0, 0, 0);
                    h0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.z, xn[q][2], h0, 0, 0, 0);
                    h1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.z, xn[q][2], h1, 0, 0, 0);
                    h0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w0.w, xn[q][3], h0, 0, 0, 0);
                    h1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.w, xn[q][3], h1, 0, 0, 0);
                }
                // GELU (:303); padding hidden units have zero weights and bias, gelu(0) = 0
                const float4 g0 = make_float4(gm_gelu(h0[0]), gm_gelu(h0[1]), gm_gelu(h0[2]), gm_gelu(h0[3]));
                const float4 g1 = make_float4(gm_gelu(h1[0]), gm_gelu(h1[1]), gm_gelu(h1[2]), gm_gelu(h1[3]));
#pragma unroll
                for (int o = 0; o < NC; ++o) {
                    const int f = 2 * NC + 2 * o;
                    const float4 w0 = ring[f % GF_PF];
                    ring[f % GF_PF] = f + GF_PF < F ? issue(f + GF_PF, pb1, pb2) : issue(f + GF_PF - F, nb1, nb2);
                    const float4 w1 = ring[(f + 1) % GF_PF];
                    ring[(f + 1) % GF_PF] = f + 1 + GF_PF < F ? issue(f + 1 + GF_PF, pb1, pb2) : issue(f + 1 + GF_PF - F, nb1, nb2);
                    y[o] = gf_mfma4(w0, g0, y[o]);
                    y[o] = gf_mfma4(w1, g1, y[o]);
                }
            }
            // X = (Y + b2) * ew + X (:305, the explanation weight on the branch output)
            const float e = I.sew[min(I.tok, 31)];
#pragma unroll
            for (int o = 0; o < NC; ++o) {
                float *px = I.Xw + m * XS + 16 * o + 4 * j;
                const float4 xo = *reinterpret_cast<const float4 *>(px);
                const bool in = I.tok < N && 16 * o + 4 * j < C;
                *reinterpret_cast<float4 *>(px) =
                    in ? make_float4(y[o][0] * e + xo.x, y[o][1] * e + xo.y, y[o][2] * e + xo.z, y[o][3] * e + xo.w)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        __syncthreads();
    }
    // ---- masked mean over the tokens (:176-178) and the neighbour-feature mean (:181-189), the row's
    // NTT waves over channels / node features
    const Ids I;
    const int r = blockIdx.x * RPW + I.rl;
    if (r < R) {
        const int D = a.D;
        for (int c = I.tt * 64 + I.lane; c < C; c += 64 * NTT) {
            float s = 0.f;
            for (int t = 0; t < N; ++t) s += I.Xr[t * XS + c] * I.sval[t] * (has_ew ? I.sew[t] : 1.f);
            a.x_mean[(size_t)r * C + c] = s / (float)N;
        }
        float nvalid = 0.f;
        for (int t = 0; t < N; ++t) nvalid += I.sval[t];
        for (int d = I.tt * 64 + I.lane; d < D; d += 64 * NTT) {
            float s = 0.f;
            for (int t = 0; t < N; ++t) {
                float sc = nvalid > 0.f ? I.sval[t] / nvalid : 1.f / (float)N;
                if (has_ew) sc *= I.sew[t];
                s += a.n_feat[(size_t)a.nid[(size_t)r * N + t] * D + d] * sc;
            }
            a.node_out[(size_t)r * D + d] = s / (float)N + a.n_feat[(size_t)a.node[r] * D + d];
        }
    }
}


// ================================================================== backward: d explanation weights
//
// The explainer's training signal through a frozen base GraphMixer (temp_exp_main.py:614-632 with
// base_type == 'graphmixer'): d ew [R, N] from d x_mean [R, C] and d node_out [R, D].  One workgroup per
// row, the LDS-tiled layout of gm_embed_kernel.  The row's forward runs first, keeping every mixer's
// input image XL[l]; then per layer, last first, with G = d(layer output) in LDS:
//   out1 = (Y_tok + b) * ew + X * ew      recomputed per channel (thread per channel, VALU, N <= 32 tokens)
//   channel branch, per hidden chunk: Z2 = W1 LN(out1) + b1 (MFMA, LN applied to the A fragments), H = gelu(Z2)
//     -> Y_ch += W2 H (for the ew term), dG2 = (G ew) W2 (MFMA on the transposed pack), dZ2 = dG2 gelu'(Z2),
//     dV += dZ2 W1 (MFMA on the transposed pack, the chunk's K slice)
//   d ew_t += sum_c G (Y_ch + b2);  G <- G + LN_backward(dV)          (= d out1)
//   token branch per channel: d ew_t += sum_c G (Y_tok + b) + da X, da = G + LN_tok_backward(FFN_tok_backward(G ew)),
//     G <- da * ew                                                     (= d layer input)
// Per-token sums over channels go through an LDS image and one wave per token (fixed order, deterministic).
struct GmBwd {
    const float *d_xm, *d_no;   // [R][C], [R][D]
    float *d_ew;                // [R][N]
    const float *const *lw;     // [L][14]: tm_gm_embed's 12 (B-operand packs) + ffn.3^T, ffn.0^T packs
};
constexpr int GMB_LW = 14;

__device__ __forceinline__ float gm_gelu_d(float x) {
    return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.3989422804014327f * expf(-0.5f * x * x);
}

// token LayerNorm / FFN weights of one layer, staged in LDS
struct GmTokW {
    float *lg, *lb, *w1, *b1, *w2, *b2;
};
constexpr int GMB_TW = 2 * GM_MT + 2 * (GM_MT / 2) * GM_MT + GM_MT / 2 + GM_MT;   // its LDS floats

// LDS plan (floats): XL [L][32][XP] | X/G [32][XP] | O1 [32][XP] | DY [32][XP] | U [ulen] (projection
// input halves, hidden chunks) | token-FFN weights [GMB_TW] | tmean, trstd, sew, sval, dsew [5][32] |
// lnw, lnb [2][C16].  ~147 KB at C = T = 172 with 2 layers: one workgroup per CU.
static __host__ __device__ inline int gmb_ulen(int C, int T) {
    const int KG = gm_r16(C + T) / 16, K0P = 16 * ((KG + 1) / 2) + 4, HP = GM_HCH + 4;
    return GM_MT * K0P > GM_MT * HP ? GM_MT * K0P : GM_MT * HP;
}
static __host__ __device__ inline size_t gmb_lds_floats(int C, int T, int L) {
    const int XP = gm_r16(C) + 4;
    return (size_t)(L + 3) * GM_MT * XP + gmb_ulen(C, T) + GMB_TW + 5 * GM_MT + 2 * gm_r16(C);
}

// sum over c < C of the LDS image V[t][c], one wave per token (nw waves), added to out[t]
__device__ __forceinline__ void gmb_token_sums(const float *V, int XP, int N, int C, int nw, float *out) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int t = wave; t < N; t += nw) {
        float s = 0.f;
        for (int c = lane; c < C; c += 64) s += V[gm_idx(t, c, XP)];
        s = gm_wsum(s);
        if (lane == 0) out[t] += s;
    }
}

// Token mixing on MFMA (gm_fused_kernel's formulation), one wave per 16-channel tile nt: lane (li = lane & 15,
// g = lane >> 4) is channel c = 16 nt + li.  K operands hold tokens 16 G + 4 s2 + g (G < NMT) or hidden features
// 4 g + s2; MFMA outputs hold hidden features 4 g + i or tokens 16 mt + 4 g + i.  The weight fragments are read
// from the layer's LDS copy (w1 [HT][N], w2 [N][HT]) where they are used (held across the tile loop, they spill):
//   z1 = W1 xn: W1[li][t];  y = W2 h: W2[16 mt + li][4 g + s2];  dh = W2^T dy: W2[t][li];
//   dxn = W1^T dz1: W1[4 g + s2][16 mt + li]
struct GmbTokF {
    const GmTokW &tw;
    int N, HT, li, g;
    __device__ __forceinline__ float a1(int t) const { return (li < HT && t < N) ? tw.w1[li * N + t] : 0.f; }
    __device__ __forceinline__ float a2(int tr, int jj) const { return (tr < N && jj < HT) ? tw.w2[tr * HT + jj] : 0.f; }
    __device__ __forceinline__ float a2t(int t) const { return (li < HT && t < N) ? tw.w2[t * HT + li] : 0.f; }
    __device__ __forceinline__ float a1t(int tr, int jj) const { return (jj < HT && tr < N) ? tw.w1[jj * N + tr] : 0.f; }
    __device__ __forceinline__ float b1(int i) const { return 4 * g + i < HT ? tw.b1[4 * g + i] : 0.f; }
};

// one channel tile's token LayerNorm (statistics over the N tokens by two shuffles) and FFN: hacc = z1 - b1 at
// hidden 4 g + i, h = gelu(z1), y at tokens 16 mt + 4 g + i (b2 included)
template <int NMT>
__device__ __forceinline__ void gmb_tok_mfma(const GmbTokF &f, const float *S, const float *sew, int XP, int N,
                                             int HT, int c, bool cv, int g, float &mean, float &rstd, gmx4 &hacc,
                                             float (&h)[4], float (&y)[NMT][4]) {
    float v[NMT][4], sm = 0.f;
#pragma unroll
    for (int G = 0; G < NMT; ++G)
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            const int t = 16 * G + 4 * s2 + g;
            v[G][s2] = (cv && t < N) ? S[gm_idx(t, c, XP)] * sew[t] : 0.f;
            sm += v[G][s2];
        }
    sm += __shfl_xor(sm, 16);
    sm += __shfl_xor(sm, 32);
    mean = sm / (float)N;
    float q = 0.f;
#pragma unroll
    for (int G = 0; G < NMT; ++G)
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            const float d = v[G][s2] - mean;
            q += 16 * G + 4 * s2 + g < N ? d * d : 0.f;
        }
    q += __shfl_xor(q, 16);
    q += __shfl_xor(q, 32);
    rstd = 1.f / sqrtf(q / (float)N + 1e-5f);
    hacc = gmx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int G = 0; G < NMT; ++G)
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            const int t = 16 * G + 4 * s2 + g;
            const float xn = (cv && t < N) ? (v[G][s2] - mean) * rstd * f.tw.lg[t] + f.tw.lb[t] : 0.f;
            hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a1(t), xn, hacc, 0, 0, 0);
        }
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = 4 * g + i < HT ? gm_gelu(hacc[i] + f.b1(i)) : 0.f;
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) {
        gmx4 yy = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
            yy = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a2(16 * mt + f.li, 4 * g + s2), h[s2], yy, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int t = 16 * mt + 4 * g + i;
            y[mt][i] = yy[i] + (t < N ? f.tw.b2[t] : 0.f);
        }
    }
}

// TS8 with NMT == 2 (N > 16): 8 waves, wave = 4 mh + wq runs token tile mh of output tiles wq + 4i in every
// GEMM (the workgroup's 147 KB of LDS allows one per CU: 8 waves give each SIMD two); otherwise 4 waves.
template <int NMT, int NTW, bool TS8>
__global__ void __launch_bounds__(NMT == 2 && TS8 ? 512 : 256) gm_bwd_kernel(GmArgs a, GmBwd b) {
    extern __shared__ float gm_lds[];
    constexpr bool TS = NMT == 2 && TS8;
    // GMT: token tiles per wave in the GEMMs; WT: token tiles per wave in the epilogues (the 4-wave form writes
    // both tiles, zeros past NMT, as before the 8-wave form existed)
    constexpr int NWV = TS ? 8 : 4, GMT = TS ? 1 : NMT, WT = TS ? 1 : 2;
    const int r = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wq = TS ? (wave & 3) : wave, mh = TS ? (wave >> 2) : 0;
    const int N = a.N, C = a.C, T = a.T, D = a.D, L = a.L, HT = a.HT;
    const int C16 = gm_r16(C), KG = gm_r16(C + T) / 16, KH = (KG + 1) / 2;
    const int XP = C16 + 4, HP = GM_HCH + 4, K0P = 16 * KH + 4, IMG = GM_MT * XP;
    float *XL = gm_lds, *X = XL + L * IMG, *G = X, *O1 = X + IMG, *DY = O1 + IMG, *U = DY + IMG;
    float *TW = U + gmb_ulen(C, T);
    float *tmean = TW + GMB_TW, *trstd = tmean + GM_MT, *sew = trstd + GM_MT, *sval = sew + GM_MT;
    float *dsew = sval + GM_MT, *lnw = dsew + GM_MT, *lnb = lnw + C16;
    float *X0 = U, *H = U;
    if (tid < GM_MT) {
        const bool v = tid < N && a.nid[(size_t)r * N + tid] != 0;
        sval[tid] = v ? 1.f : 0.f;
        sew[tid] = tid < N ? a.ew[(size_t)r * N + tid] * (v ? 1.f : 0.f) : 0.f;
        dsew[tid] = 0.f;
    }
    __syncthreads();
    const int NT = C16 / 16, ntw = (NT - wq + 3) / 4;
    const int NH = gm_r16(a.HC) / 16;
    float mr[2] = {0.f, 0.f}, rr[2] = {0.f, 0.f};
    // ---- forward: projection (as gm_embed_kernel)
    const double cut = a.cut[r];
    for (int h = 0; h < 2; ++h) {
        const int G0 = h * KH, nG = min(KH, KG - G0), W16 = 16 * nG;
        if (nG <= 0) break;
        for (int i = tid; i < GM_MT * W16; i += blockDim.x) {
            const int t = i / W16, k = 16 * G0 + (i - t * W16);
            float v = 0.f;
            if (t < N) {
                const bool valid = sval[t] != 0.f;
                if (k < C) {
                    if (a.edge_attr) v = a.edge_attr[((size_t)r * N + t) * C + k];
                    else if (valid) v = a.e_feat[(size_t)a.eid[(size_t)r * N + t] * C + k];
                } else if (k < C + T && valid) {
                    const float dt = (float)(cut - a.ts[(size_t)r * N + t]);
                    const float arg = (float)((double)dt * (double)a.time_w[k - C] + (double)a.time_b[k - C]);
                    v = cos_rd(arg);
                }
            }
            X0[gm_idx(t, k - 16 * G0, K0P)] = v;
        }
        __syncthreads();
        {
            gmx4 acc[NTW][2];
#pragma unroll
            for (int i = 0; i < NTW; ++i) acc[i][0] = acc[i][1] = gmx4{0.f, 0.f, 0.f, 0.f};
            gm_gemm_mt<GMT, NTW, false>(X0 + 16 * mh * K0P, K0P, G0, a.proj_w, NT, wq, ntw, G0, nG, acc, nullptr,
                                            nullptr, mr, rr);
#pragma unroll
            for (int i = 0; i < NTW; ++i) {
                if (i >= ntw) break;
                const int n = 16 * (wq + 4 * i) + (lane & 15);
                const float bv = n < C ? a.proj_b[n] : 0.f;
#pragma unroll
                for (int q = 0; q < WT; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int mt = mh + q, t = 16 * mt + 4 * (lane >> 4) + e;
                        const int ix = gm_idx(t, n, XP);
                        const bool in = mt < NMT && n < C && t < N;
                        if (h == 0) X[ix] = in ? acc[i][q][e] : 0.f;
                        else if (in) X[ix] = X[ix] + acc[i][q][e] + bv;
                    }
            }
        }
        __syncthreads();
    }
    if (KG == 1) {
        for (int i = tid; i < GM_MT * C16; i += blockDim.x) {
            const int t = i / C16, n = i - t * C16;
            if (t < N && n < C) X[gm_idx(t, n, XP)] += a.proj_b[n];
        }
        __syncthreads();
    }
    // stage layer l's token LayerNorm / FFN weights into TW; channel LN parameters (permuted K order) into
    // lnw / lnb
    auto stage_layer = [&](int l) -> GmTokW {
        const auto w = gm_layer(b.lw, GMB_LW * l);
        GmTokW tw{TW, TW + GM_MT, TW + 2 * GM_MT, TW + 2 * GM_MT + (GM_MT / 2) * GM_MT,
                  TW + 2 * GM_MT + (GM_MT / 2) * GM_MT + GM_MT / 2, TW + 2 * GM_MT + GM_MT * GM_MT + GM_MT / 2};
        for (int i = tid; i < N; i += blockDim.x) {
            tw.lg[i] = w[0][i];
            tw.lb[i] = w[1][i];
            tw.b2[i] = w[5][i];
        }
        for (int i = tid; i < HT * N; i += blockDim.x) {
            tw.w1[i] = w[2][i];
            tw.w2[i] = w[4][i];
        }
        for (int i = tid; i < HT; i += blockDim.x) tw.b1[i] = w[3][i];
        for (int k = tid; k < C16; k += blockDim.x) {
            const int pk = (k & ~15) + 4 * (k & 3) + ((k >> 2) & 3);
            lnw[pk] = k < C ? w[6][k] : 0.f;
            lnb[pk] = k < C ? w[7][k] : 0.f;
        }
        return tw;
    };
    // token mixing of one channel c from image S into image Dst: Dst = (y) * ew + S * ew (thread per channel)
    // (MFMA, one wave per 16-channel tile; S == Dst allowed: a lane rewrites only its own channel's tokens after
    // the wave has read them)
    auto token_mix = [&](const GmTokW &tw, const float *S, float *Dst) {
        const int tl = gm_tid(), li = tl & 15, g = (tl >> 4) & 3;   // laundered: no lane address hoisted out
        const GmbTokF f{tw, N, HT, li, g};
        for (int nt = tl >> 6; nt < NT; nt += NWV) {
            const int c = 16 * nt + li;
            const bool cv = c < C;
            float mean, rstd, h[4], y[NMT][4];
            gmx4 hacc;
            gmb_tok_mfma<NMT>(f, S, sew, XP, N, HT, c, cv, g, mean, rstd, hacc, h, y);
#pragma unroll
            for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int t = 16 * mt + 4 * g + i;
                    if (cv && t < N) {
                        const int ix = gm_idx(t, c, XP);
                        Dst[ix] = y[mt][i] * sew[t] + S[ix] * sew[t];
                    }
                }
        }
    };
    // channel LayerNorm statistics of image S (one wave per token) into tmean / trstd, then this lane's rows
    auto chan_stats = [&](const float *S) {
        for (int t = wave; t < GM_MT; t += NWV) {
            float mean = 0.f, rstd = 0.f;
            if (t < N) {
                float s = 0.f, q = 0.f;
                for (int c = lane; c < C; c += 64) s += S[gm_idx(t, c, XP)];
                mean = gm_wsum(s) / (float)C;
                for (int c = lane; c < C; c += 64) {
                    const float d = S[gm_idx(t, c, XP)] - mean;
                    q += d * d;
                }
                rstd = 1.f / sqrtf(gm_wsum(q) / (float)C + 1e-5f);
            }
            if (lane == 0) {
                tmean[t] = mean;
                trstd[t] = rstd;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < WT; ++q) {
            mr[q] = tmean[16 * (mh + q) + (lane & 15)];
            rr[q] = trstd[16 * (mh + q) + (lane & 15)];
        }
    };
    // ---- forward through the mixers, keeping each layer's input
    for (int l = 0; l < L; ++l) {
        const auto w = gm_layer(b.lw, GMB_LW * l);
        for (int i = tid; i < IMG; i += blockDim.x) XL[l * IMG + i] = X[i];
        const GmTokW tw = stage_layer(l);
        __syncthreads();
        token_mix(tw, X, X);
        __syncthreads();
        chan_stats(X);
        const float4 *W1 = (const float4 *)(w[8]), *W2 = (const float4 *)(w[10]);
        gmx4 acc2[NTW][2];
#pragma unroll
        for (int i = 0; i < NTW; ++i) acc2[i][0] = acc2[i][1] = gmx4{0.f, 0.f, 0.f, 0.f};
        for (int h0 = 0; h0 < NH; h0 += GM_HCH / 16) {
            const int nh = min(GM_HCH / 16, NH - h0), nw1 = (nh - wq + 3) / 4;
            gmx4 acc[GM_HCH / 64][2];
#pragma unroll
            for (int i = 0; i < GM_HCH / 64; ++i) acc[i][0] = acc[i][1] = gmx4{0.f, 0.f, 0.f, 0.f};
            gm_gemm_mt<GMT, GM_HCH / 64, true>(X + 16 * mh * XP, XP, 0, W1, NH, h0 + wq, nw1, 0, C16 / 16, acc, lnw, lnb,
                                               mr, rr);
#pragma unroll
            for (int i = 0; i < GM_HCH / 64; ++i) {
                if (i >= nw1) break;
                const int ht = wq + 4 * i, n = 16 * (h0 + ht) + (lane & 15);
                const float bv = n < a.HC ? w[9][n] : 0.f;
#pragma unroll
                for (int q = 0; q < WT; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int mt = mh + q, t = 16 * mt + 4 * (lane >> 4) + e;
                        H[gm_idx(t, 16 * ht + (lane & 15), HP)] = (mt < NMT && n < a.HC) ? gm_gelu(acc[i][q][e] + bv) : 0.f;
                    }
            }
            __syncthreads();
            gm_gemm_mt<GMT, NTW, false>(H + 16 * mh * HP, HP, h0, W2, NT, wq, ntw, h0, nh, acc2, nullptr, nullptr, mr, rr);
            __syncthreads();
        }
#pragma unroll
        for (int i = 0; i < NTW; ++i) {
            const int nt = wq + 4 * i;
            if (nt >= NT) break;
            const int n = 16 * nt + (lane & 15);
            const float bv = n < C ? w[11][n] : 0.f;
#pragma unroll
            for (int q = 0; q < WT; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int mt = mh + q, t = 16 * mt + 4 * (lane >> 4) + e;
                    if (mt < NMT && t < N && n < C) {
                        const int ix = gm_idx(t, n, XP);
                        X[ix] = (acc2[i][q][e] + bv) * sew[t] + X[ix];
                    }
                }
        }
        __syncthreads();
    }
    // ---- d of the masked token mean (:176-178) and the neighbour-feature mean (:181-189)
    float nvalid = 0.f;
    for (int t = 0; t < N; ++t) nvalid += sval[t];
    const float *dxm = b.d_xm + (size_t)r * C;
    // DY <- dxm_c X[t][c] sval_t / N (per-token sums give the x_mean part of d sew); G <- dxm_c sval_t sew_t / N
    for (int i = tid; i < GM_MT * C16; i += blockDim.x) {
        const int t = i / C16, c = i - t * C16;
        const int ix = gm_idx(t, c, XP);
        const bool in = t < N && c < C;
        const float g = in ? dxm[c] : 0.f;
        DY[ix] = in ? g * X[ix] * sval[t] / (float)N : 0.f;
        G[ix] = in ? g * sval[t] * sew[t] / (float)N : 0.f;
    }
    __syncthreads();
    gmb_token_sums(DY, XP, N, C, NWV, dsew);
    {   // node_out: d sew_t += sum_d dno_d n_feat[nid_t][d] sc_t / N, one wave per token
        const float *dno = b.d_no + (size_t)r * D;
        for (int t = wave; t < N; t += NWV) {
            const float sc = nvalid > 0.f ? sval[t] / nvalid : 1.f / (float)N;
            const float *nf = a.n_feat + (size_t)a.nid[(size_t)r * N + t] * D;
            float s = 0.f;
            for (int d = lane; d < D; d += 64) s += dno[d] * nf[d];
            s = gm_wsum(s);
            if (lane == 0) dsew[t] += s * sc / (float)N;
        }
    }
    __syncthreads();
    // ---- the mixers backwards
    for (int l = L - 1; l >= 0; --l) {
        const auto w = gm_layer(b.lw, GMB_LW * l);
        const float *XI = XL + l * IMG;
        const GmTokW tw = stage_layer(l);
        // out1's padding (tokens >= N, channels >= C) must read as 0: the channel FFN's A fragments and its
        // LayerNorm (weight 0 there) multiply whatever the LDS holds
        for (int i = tid; i < IMG; i += blockDim.x) O1[i] = 0.f;
        __syncthreads();
        token_mix(tw, XI, O1);                                    // out1
        // DY = G ew (d channel-FFN output)
        for (int i = tid; i < GM_MT * C16; i += blockDim.x) {
            const int t = i / C16, c = i - t * C16;
            const int ix = gm_idx(t, c, XP);
            DY[ix] = (t < N && c < C) ? G[ix] * sew[t] : 0.f;
        }
        __syncthreads();
        chan_stats(O1);
        const float4 *W1 = (const float4 *)(w[8]), *W2 = (const float4 *)(w[10]);
        const float4 *W2T = (const float4 *)(w[12]), *W1T = (const float4 *)(w[13]);
        gmx4 acc2[NTW][2], accv[NTW][2];
#pragma unroll
        for (int i = 0; i < NTW; ++i) acc2[i][0] = acc2[i][1] = accv[i][0] = accv[i][1] = gmx4{0.f, 0.f, 0.f, 0.f};
        for (int h0 = 0; h0 < NH; h0 += GM_HCH / 16) {
            const int nh = min(GM_HCH / 16, NH - h0), nw1 = (nh - wq + 3) / 4;
            gmx4 acc[GM_HCH / 64][2], accd[GM_HCH / 64][2];
#pragma unroll
            for (int i = 0; i < GM_HCH / 64; ++i)
                acc[i][0] = acc[i][1] = accd[i][0] = accd[i][1] = gmx4{0.f, 0.f, 0.f, 0.f};
            gm_gemm_mt<GMT, GM_HCH / 64, true>(O1 + 16 * mh * XP, XP, 0, W1, NH, h0 + wq, nw1, 0, C16 / 16, acc, lnw, lnb,
                                               mr, rr);
            gm_gemm_mt<GMT, GM_HCH / 64, false>(DY + 16 * mh * XP, XP, 0, W2T, NH, h0 + wq, nw1, 0, C16 / 16, accd,
                                                nullptr, nullptr, mr, rr);
            // H = gelu(Z2) for Y_ch; dZ2 = dG2 gelu'(Z2) kept in accd for the second pass through U
#pragma unroll
            for (int i = 0; i < GM_HCH / 64; ++i) {
                if (i >= nw1) break;
                const int ht = wq + 4 * i, n = 16 * (h0 + ht) + (lane & 15);
                const float bv = n < a.HC ? w[9][n] : 0.f;
#pragma unroll
                for (int q = 0; q < WT; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int mt = mh + q, t = 16 * mt + 4 * (lane >> 4) + e;
                        const bool in = mt < NMT && n < a.HC;
                        const float z = acc[i][q][e] + bv;
                        H[gm_idx(t, 16 * ht + (lane & 15), HP)] = in ? gm_gelu(z) : 0.f;
                        accd[i][q][e] = in ? accd[i][q][e] * gm_gelu_d(z) : 0.f;
                    }
            }
            __syncthreads();
            gm_gemm_mt<GMT, NTW, false>(H + 16 * mh * HP, HP, h0, W2, NT, wq, ntw, h0, nh, acc2, nullptr, nullptr, mr, rr);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < GM_HCH / 64; ++i) {
                if (i >= nw1) break;
                const int ht = wq + 4 * i;
#pragma unroll
                for (int q = 0; q < WT; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int t = 16 * (mh + q) + 4 * (lane >> 4) + e;
                        H[gm_idx(t, 16 * ht + (lane & 15), HP)] = accd[i][q][e];
                    }
            }
            __syncthreads();
            gm_gemm_mt<GMT, NTW, false>(H + 16 * mh * HP, HP, h0, W1T, NT, wq, ntw, h0, nh, accv, nullptr, nullptr, mr,
                                        rr);
            __syncthreads();
        }
        // d sew_t += sum_c G (Y_ch + b2)
#pragma unroll
        for (int i = 0; i < NTW; ++i) {
            const int nt = wq + 4 * i;
            if (nt >= NT) break;
            const int n = 16 * nt + (lane & 15);
            const float bv = n < C ? w[11][n] : 0.f;
#pragma unroll
            for (int q = 0; q < WT; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int mt = mh + q, t = 16 * mt + 4 * (lane >> 4) + e;
                    const int ix = gm_idx(t, n, XP);
                    DY[ix] = (mt < NMT && t < N && n < C) ? G[ix] * (acc2[i][q][e] + bv) : 0.f;
                }
        }
        __syncthreads();
        gmb_token_sums(DY, XP, N, C, NWV, dsew);
        __syncthreads();
        // channel LayerNorm backward: DY = dV * ln weight; G += rstd (DY - mean_c DY - xhat mean_c(DY xhat))
#pragma unroll
        for (int i = 0; i < NTW; ++i) {
            const int nt = wq + 4 * i;
            if (nt >= NT) break;
            const int n = 16 * nt + (lane & 15);
            const float gw = n < C ? w[6][n] : 0.f;
#pragma unroll
            for (int q = 0; q < WT; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int mt = mh + q, t = 16 * mt + 4 * (lane >> 4) + e;
                    DY[gm_idx(t, n, XP)] = (mt < NMT && t < N && n < C) ? accv[i][q][e] * gw : 0.f;
                }
        }
        __syncthreads();
        for (int t = wave; t < N; t += NWV) {
            const float mean = tmean[t], rstd = trstd[t];
            float s1 = 0.f, s2 = 0.f;
            for (int c = lane; c < C; c += 64) {
                const int ix = gm_idx(t, c, XP);
                const float dv = DY[ix], xh = (O1[ix] - mean) * rstd;
                s1 += dv;
                s2 += dv * xh;
            }
            s1 = gm_wsum(s1) / (float)C;
            s2 = gm_wsum(s2) / (float)C;
            for (int c = lane; c < C; c += 64) {
                const int ix = gm_idx(t, c, XP);
                const float xh = (O1[ix] - mean) * rstd;
                G[ix] += rstd * (DY[ix] - s1 - xh * s2);
            }
        }
        __syncthreads();
        // token branch on MFMA, one wave per 16-channel tile: G = d out1 -> d layer input; DY = the channel's
        // terms of d sew.  dy = G ew, dh = W2^T dy, dz1 = dh gelu'(z1), dxn = W1^T dz1, then the LayerNorm-over-
        // tokens backward (sums over tokens by two shuffles)
        {
            const int tl = gm_tid(), li = tl & 15, g = (tl >> 4) & 3;
            const GmbTokF f{tw, N, HT, li, g};
            for (int nt = tl >> 6; nt < NT; nt += NWV) {
                const int c = 16 * nt + li;
                const bool cv = c < C;
                float mean, rstd, h[4], y[NMT][4];
                gmx4 hacc;
                gmb_tok_mfma<NMT>(f, XI, sew, XP, N, HT, c, cv, g, mean, rstd, hacc, h, y);
                gmx4 dh = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kb = 0; kb < NMT; ++kb)
#pragma unroll
                    for (int s2 = 0; s2 < 4; ++s2) {
                        const int t = 16 * kb + 4 * s2 + g;
                        const float dy = (cv && t < N) ? G[gm_idx(t, c, XP)] * sew[t] : 0.f;
                        dh = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a2t(t), dy, dh, 0, 0, 0);
                    }
                float dz[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) dz[i] = 4 * g + i < HT ? dh[i] * gm_gelu_d(hacc[i] + f.b1(i)) : 0.f;
                float dtg[NMT][4], xh[NMT][4], s1 = 0.f, s2v = 0.f;
#pragma unroll
                for (int mt = 0; mt < NMT; ++mt) {
                    gmx4 dx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int s2 = 0; s2 < 4; ++s2)
                        dx = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a1t(16 * mt + li, 4 * g + s2), dz[s2], dx, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int t = 16 * mt + 4 * g + i;
                        const bool in = cv && t < N;
                        dtg[mt][i] = in ? dx[i] * tw.lg[t] : 0.f;
                        xh[mt][i] = in ? (XI[gm_idx(t, c, XP)] * sew[t] - mean) * rstd : 0.f;
                        s1 += dtg[mt][i];
                        s2v += dtg[mt][i] * xh[mt][i];
                    }
                }
                s1 += __shfl_xor(s1, 16);
                s1 += __shfl_xor(s1, 32);
                s2v += __shfl_xor(s2v, 16);
                s2v += __shfl_xor(s2v, 32);
                s1 /= (float)N;
                s2v /= (float)N;
#pragma unroll
                for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int t = 16 * mt + 4 * g + i;
                        if (cv && t < N) {
                            const int ix = gm_idx(t, c, XP);
                            const float gv = G[ix];
                            const float da = gv + rstd * (dtg[mt][i] - s1 - xh[mt][i] * s2v);
                            DY[ix] = gv * y[mt][i] + da * XI[ix];
                            G[ix] = da * sew[t];
                        }
                    }
            }
        }
        __syncthreads();
        gmb_token_sums(DY, XP, N, C, NWV, dsew);
        __syncthreads();
    }
    if (tid < N) b.d_ew[(size_t)r * N + tid] = dsew[tid] * sval[tid];
}

}  // namespace tmk

using namespace tmk;

static inline size_t gm_lds_bytes(int32_t C, int32_t T) {
    const size_t C16 = gm_r16(C), XP = C16 + 4, KG = gm_r16(C + T) / 16, K0P = 16 * ((KG + 1) / 2) + 4, HP = GM_HCH + 4;
    const size_t ulen = std::max(std::max(GM_MT * K0P, GM_MT * HP), 2 * C16);
    return sizeof(float) * (GM_MT * XP + ulen + 2 * GM_MT + 2 * C16 + 2 * GM_MT);
}

extern "C" int64_t tm_gm_packed_floats(int32_t n_out, int32_t k) {
    if (n_out <= 0 || k <= 0) return 0;
    return (int64_t)(gm_r16(n_out) / 16) * (gm_r16(k) / 16) * 256;
}

extern "C" int tm_gm_pack(const float *w, int32_t n_out, int32_t k, float *packed, void *stream) {
    if (!w || !packed || n_out <= 0 || k <= 0) return fail(TM_E_ARG, "tm_gm_pack: bad arguments");
    const int64_t total = tm_gm_packed_floats(n_out, k);
    const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
    gm_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w, n_out, k, packed);
    TM_CHECK_LAUNCH();
    return TM_OK;
}

static inline int64_t gm_pack_a_tiles(int32_t n, int32_t mult) { return (int64_t)((gm_r16(n) / 16 + mult - 1) / mult) * mult; }

extern "C" int64_t tm_gm_packed_a_floats(int32_t n_out, int32_t k, int32_t n_mult, int32_t k_mult) {
    if (n_out <= 0 || k <= 0 || n_mult <= 0 || k_mult <= 0) return 0;
    return gm_pack_a_tiles(n_out, n_mult) * gm_pack_a_tiles(k, k_mult) * 256;
}

extern "C" int tm_gm_pack_a(const float *w, int32_t n_out, int32_t k, int32_t n_mult, int32_t k_mult, float *packed,
                            void *stream) {
    if (!w || !packed || n_out <= 0 || k <= 0 || n_mult <= 0 || k_mult <= 0) return fail(TM_E_ARG, "tm_gm_pack_a: bad arguments");
    const int64_t total = tm_gm_packed_a_floats(n_out, k, n_mult, k_mult);
    const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
    gm_pack_a_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w, n_out, k, (int32_t)gm_pack_a_tiles(k, k_mult), total, packed);
    TM_CHECK_LAUNCH();
    return TM_OK;
}

static inline size_t gm_fused_lds_bytes(int32_t C, int32_t N) {
    const size_t NC = gm_r16(C) / 16, XS = 16 * NC + 4, RPW = N > 16 ? 2 : 4;
    return sizeof(float) * (64 * XS + RPW * 64);
}

// the register-resident kernel's instances: channel tiles NC = C / 16 rounded up
#define GM_FUSED_NC(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)

extern "C" int tm_gm_fused_ok(int32_t N, int32_t C, int32_t T, int32_t HC) {
    return N > 0 && N <= GM_MT && C >= 4 && C <= 256 && C % 4 == 0 && T >= 4 && T % 4 == 0 && HC >= 4 && HC % 4 == 0 &&
           gm_fused_lds_bytes(C, N) <= 80 * 1024;
}

extern "C" int tm_gm_embed(const tm_gm_embed_args *p, void *stream) {
    if (!p) return fail(TM_E_ARG, "tm_gm_embed: NULL arguments");
    const tm_gm_embed_args &q = *p;
    if (q.R < 0 || q.N <= 0 || q.C <= 0 || q.T < 0 || q.D <= 0 || q.L < 0 || q.HT < 0 || q.HC <= 0)
        return fail(TM_E_ARG, "tm_gm_embed: bad dimensions");
    if (q.N > GM_MT || q.HT > GM_MT / 2 || q.L > GM_MAXL || q.C > 256)
        return fail(TM_E_UNSUPPORTED, "tm_gm_embed: needs num_tokens <= 32, token hidden <= 16, <= 4 layers, "
                                      "channels <= 256");
    if (q.R == 0) return TM_OK;
    if (!q.node || !q.nid || !q.cut || !q.ts || !q.n_feat || (!q.e_feat && !q.edge_attr) || (q.T && (!q.time_w || !q.time_b)) ||
        !q.proj_w || !q.proj_b || !q.x_mean || !q.node_out || (!q.eid && !q.edge_attr))
        return fail(TM_E_ARG, "tm_gm_embed: NULL pointer");
    GmArgs a{};
    a.R = q.R; a.N = q.N; a.C = q.C; a.T = q.T; a.D = q.D; a.L = q.L; a.HT = q.HT; a.HC = q.HC;
    a.node = q.node; a.nid = q.nid; a.eid = q.eid; a.cut = q.cut; a.ts = q.ts; a.ew = q.ew; a.edge_attr = q.edge_attr;
    a.n_feat = q.n_feat; a.e_feat = q.e_feat; a.time_w = q.time_w; a.time_b = q.time_b;
    a.proj_w = reinterpret_cast<const float4 *>(q.proj_w);
    a.proj_b = q.proj_b;
    if (q.L > 0 && !q.layer_table) return fail(TM_E_ARG, "tm_gm_embed: NULL layer table");
    a.lw = q.layer_table;
    a.x_mean = q.x_mean;
    a.node_out = q.node_out;
    if (tm_gm_fused_ok(q.N, q.C, q.T, q.HC)) {
        // packs by tm_gm_pack_a: proj_w (1, 4), channel ffn.0 (2, 1), ffn.3 (1, 2)
        const size_t lds = gm_fused_lds_bytes(q.C, q.N);
        const int nc = gm_r16(q.C) / 16, rpw = q.N > 16 ? 2 : 4;
        const unsigned grid = (unsigned)((q.R + rpw - 1) / rpw);
        hipEvent_t pe = prof_begin((hipStream_t)stream);
        auto launch = [&](auto kern) -> int {
            TM_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            kern<<<grid, 256, lds, (hipStream_t)stream>>>(a);
            return TM_OK;
        };
        int rc = TM_E_UNSUPPORTED;
#define GM_CASE(X)                                                                                  \
        if (nc == X) rc = q.N > 16 ? launch(gm_fused_kernel<X, 2>) : launch(gm_fused_kernel<X, 1>);
        GM_FUSED_NC(GM_CASE)
#undef GM_CASE
        if (rc != TM_OK) return rc == TM_E_UNSUPPORTED ? fail(rc, "tm_gm_embed: no kernel instance") : rc;
        TM_CHECK_LAUNCH();
        prof_end("gm_fused_kernel", (hipStream_t)stream, pe);
        return TM_OK;
    }
    const size_t lds = gm_lds_bytes(q.C, q.T);
    if (lds > 160 * 1024) return fail(TM_E_UNSUPPORTED, "tm_gm_embed: edge + time dims too large for LDS");
    hipEvent_t pe = prof_begin((hipStream_t)stream);
    // output tiles per wave in the channel FFN's second GEMM (accumulated across the hidden chunks)
    const bool t3 = gm_r16(q.C) / 16 <= 12;
    auto launch = [&](auto kern) -> int {
        TM_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        kern<<<q.R, 256, lds, (hipStream_t)stream>>>(a);
        return TM_OK;
    };
    int rc;
    if (q.N > 16) rc = t3 ? launch(gm_embed_kernel<2, 3>) : launch(gm_embed_kernel<2, 4>);
    else rc = t3 ? launch(gm_embed_kernel<1, 3>) : launch(gm_embed_kernel<1, 4>);
    if (rc != TM_OK) return rc;
    TM_CHECK_LAUNCH();
    prof_end("gm_embed_kernel", (hipStream_t)stream, pe);
    return TM_OK;
}

extern "C" int tm_gm_embed_bwd_ok(int32_t N, int32_t C, int32_t T, int32_t L, int32_t HT) {
    return N > 0 && N <= GM_MT && HT >= 0 && HT <= GM_MT / 2 && L >= 0 && L <= GM_MAXL && C > 0 && C <= 256 && T >= 0 &&
           sizeof(float) * gmb_lds_floats(C, T, L) <= 160 * 1024;
}

extern "C" int tm_gm_embed_bwd(const tm_gm_embed_args *p, const float *d_x_mean, const float *d_node_out, float *d_ew,
                               void *stream) {
    if (!p) return fail(TM_E_ARG, "tm_gm_embed_bwd: NULL arguments");
    const tm_gm_embed_args &q = *p;
    if (q.R < 0 || q.N <= 0 || q.C <= 0 || q.T < 0 || q.D <= 0 || q.L < 0 || q.HT < 0 || q.HC <= 0)
        return fail(TM_E_ARG, "tm_gm_embed_bwd: bad dimensions");
    if (q.N > GM_MT || q.HT > GM_MT / 2 || q.L > GM_MAXL || q.C > 256)
        return fail(TM_E_UNSUPPORTED, "tm_gm_embed_bwd: needs num_tokens <= 32, token hidden <= 16, <= 4 layers, "
                                      "channels <= 256");
    if (q.R == 0) return TM_OK;
    if (!q.node || !q.nid || !q.cut || !q.ts || !q.n_feat || (!q.e_feat && !q.edge_attr) || (q.T && (!q.time_w || !q.time_b)) ||
        !q.proj_w || !q.proj_b || (!q.eid && !q.edge_attr) || !q.ew || !d_x_mean || !d_node_out || !d_ew ||
        (q.L > 0 && !q.layer_table))
        return fail(TM_E_ARG, "tm_gm_embed_bwd: NULL pointer");
    const size_t lds = sizeof(float) * gmb_lds_floats(q.C, q.T, q.L);
    if (lds > 160 * 1024) return fail(TM_E_UNSUPPORTED, "tm_gm_embed_bwd: dims too large for the LDS tile");
    GmArgs a{};
    a.R = q.R; a.N = q.N; a.C = q.C; a.T = q.T; a.D = q.D; a.L = q.L; a.HT = q.HT; a.HC = q.HC;
    a.node = q.node; a.nid = q.nid; a.eid = q.eid; a.cut = q.cut; a.ts = q.ts; a.ew = q.ew; a.edge_attr = q.edge_attr;
    a.n_feat = q.n_feat; a.e_feat = q.e_feat; a.time_w = q.time_w; a.time_b = q.time_b;
    a.proj_w = reinterpret_cast<const float4 *>(q.proj_w);
    a.proj_b = q.proj_b;
    GmBwd b{d_x_mean, d_node_out, d_ew, q.layer_table};
    hipEvent_t pe = prof_begin((hipStream_t)stream);
    const bool t3 = gm_r16(q.C) / 16 <= 12;
    // more than 16 neighbours: two token tiles, one per wave of the 8-wave form (two waves per SIMD instead of one:
    // 7.85 -> 7.12 ms per 1,800 rows at configs[4] shapes, round 5; the 4-wave form is tools/patches/gm_variants.patch)
    auto launch = [&](auto kern, int threads) -> int {
        TM_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        kern<<<q.R, threads, lds, (hipStream_t)stream>>>(a, b);
        return TM_OK;
    };
    int rc;
    if (q.N > 16) rc = t3 ? launch(gm_bwd_kernel<2, 3, true>, 512) : launch(gm_bwd_kernel<2, 4, true>, 512);
    else rc = t3 ? launch(gm_bwd_kernel<1, 3, false>, 256) : launch(gm_bwd_kernel<1, 4, false>, 256);
    if (rc != TM_OK) return rc;
    TM_CHECK_LAUNCH();
    prof_end("gm_bwd_kernel", (hipStream_t)stream, pe);
    return TM_OK;
}
