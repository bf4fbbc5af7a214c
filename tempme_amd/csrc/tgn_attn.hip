// Base-TGN temporal attention with explanation weights on gfx950 (the consumer of the explanation
// path: temp_exp_main.py:614-616 feeds retrieve_explanation's output into TGN.contrast).
//
// Reference (dharunm236/TempME, TGN/modules/embedding_module.py):
//   embedding_update_layer :356-393  per layer: source rows, their n_ngh neighbours, mask = node==0,
//                                    explanation weight row = layer's slice of explain_weights
//   TemporalAttentionLayer :181-216  query = [src feature | cos(b)], key = value = [ngh feature |
//                                    edge feature | cos(dt*w+b)], mask .repeat(n_head,1,1) (:211-212)
//   MultiHeadAttention     :52-86    q/k/v projections (no bias), explain_weight .repeat (:74-75)
//   ScaledDotProductAttention :16-32 bmm / temperature, masked_fill(-1e10), softmax, * explain weight,
//                                    bmm with v
//
// What runs here is the per-neighbour part of one layer.  With W_q,h / W_k,h / W_v,h the head-h
// row blocks of w_qs / w_ks / w_vs, the score (W_q,h q).(W_k,h k_j) equals qf_h . k_j with
// qf_h = W_k,h^T W_q,h q, and sum_j a_j W_v,h k_j equals W_v,h (sum_j a_j k_j).  So the caller
// projects each SOURCE row once (qf, then fc*W_v on the result) and this kernel only touches raw
// keys: it builds key[r,j] on the fly from the feature tables (never materialised), scores it
// against every head, and accumulates the weighted raw keys with an online softmax.  The
// reference's per-neighbour 2*H*d_key^2 MACs (the bulk of its FLOPs) are gone; what is left is
// gather-bound (one key row per neighbour).
//
// Mapping: one 64-lane wave per source row, all heads; key element c = lane + 64*i lives in
// register i of that lane (KPL = ceil(d_key/64) registers), so every feature-table row is read with
// consecutive lanes on consecutive floats.
#include "common.h"

namespace tmk {

constexpr int ATT_MAXH = 4;
constexpr int ATT_WAVES = 4;

__device__ __forceinline__ float wave_sum(float v) {
    // butterfly: every lane ends with the same value (a+b == b+a)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// per-lane constants of the key layout
template <int KPL>
struct KeyLane {
    int seg[KPL];     // 0 node feature, 1 edge feature, 2 time feature, 3 padding
    int off[KPL];     // column inside the segment
    float tw[KPL], tb[KPL];
};

template <int KPL>
__device__ __forceinline__ KeyLane<KPL> key_lane(const tm_tgn_attn &a, int lane) {
    KeyLane<KPL> L;
    const int dn = a.d_node, de = a.d_edge, dk = a.d_node + a.d_edge + a.d_time;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
        const int c = lane + 64 * i;
        L.seg[i] = c < dn ? 0 : c < dn + de ? 1 : c < dk ? 2 : 3;
        L.off[i] = L.seg[i] == 0 ? c : L.seg[i] == 1 ? c - dn : L.seg[i] == 2 ? c - dn - de : 0;
        L.tw[i] = L.seg[i] == 2 ? a.time_w[L.off[i]] : 0.f;
        L.tb[i] = L.seg[i] == 2 ? a.time_b[L.off[i]] : 0.f;
    }
    return L;
}

// key[slot] -> k[] (this lane's elements).  TimeEncode is Linear(1, d) then cos
// (embedding_module.py:108-112): torch's CPU addmm rounds t*w+b once, i.e. an fma.
template <int KPL>
__device__ __forceinline__ void build_key(const tm_tgn_attn &a, const KeyLane<KPL> &L, int64_t slot, float k[KPL]) {
    const float *nrow, *erow;
    if (a.node_idx) {
        int32_t id = a.node_idx[slot];
        if ((uint32_t)id >= (uint32_t)a.node_rows) {
            if (a.err_flag) *a.err_flag = TM_E_ARG;
            id = 0;
        }
        nrow = a.node_tab + (int64_t)id * a.d_node;
    } else {
        nrow = a.node_tab + slot * a.d_node;
    }
    if (a.edge_idx) {
        int32_t id = a.edge_idx[slot];
        if ((uint32_t)id >= (uint32_t)a.edge_rows) {
            if (a.err_flag) *a.err_flag = TM_E_ARG;
            id = 0;
        }
        erow = a.edge_tab + (int64_t)id * a.d_edge;
    } else {
        erow = a.edge_tab + slot * a.d_edge;
    }
    const float t = a.dt[slot];
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
        float v = 0.f;
        if (L.seg[i] == 0) v = nrow[L.off[i]];
        else if (L.seg[i] == 1) v = erow[L.off[i]];
        else if (L.seg[i] == 2) v = cos_rd(__builtin_fmaf(t, L.tw[i], L.tb[i]));
        k[i] = v;
    }
}

__device__ __forceinline__ int64_t pair_row(const tm_tgn_attn &a, int64_t r, int h) {
    if (!a.head_major_rows) return r;
    const int64_t seg = a.seg_rows > 0 ? a.seg_rows : a.rows;
    const int64_t base = r - r % seg;
    return base + ((r - base) * a.n_head + h) % seg;
}

template <int KPL>
__global__ void __launch_bounds__(64 * ATT_WAVES) tgn_attn_fwd_kernel(tm_tgn_attn a, float *__restrict__ z,
                                                                      float *__restrict__ stats) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * ATT_WAVES + (threadIdx.x >> 6);
    if (r >= a.rows) return;
    const int H = a.n_head, N = a.n_ngh, dk = a.d_node + a.d_edge + a.d_time;
    const KeyLane<KPL> L = key_lane<KPL>(a, lane);
    float q[ATT_MAXH][KPL], acc[ATT_MAXH][KPL], m[ATT_MAXH], l[ATT_MAXH];
    int64_t mr[ATT_MAXH];
#pragma unroll
    for (int h = 0; h < ATT_MAXH; ++h) {
        m[h] = -__builtin_inff();
        l[h] = 0.f;
        mr[h] = h < H ? pair_row(a, r, h) : 0;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
            const int c = lane + 64 * i;
            q[h][i] = (h < H && c < dk) ? a.qf[(r * H + h) * dk + c] : 0.f;
            acc[h][i] = 0.f;
        }
    }
    for (int j = 0; j < N; ++j) {
        float k[KPL];
        build_key<KPL>(a, L, r * N + j, k);
#pragma unroll
        for (int h = 0; h < ATT_MAXH; ++h) {
            if (h < H) {
                float p = 0.f;
#pragma unroll
                for (int i = 0; i < KPL; ++i) p = __builtin_fmaf(q[h][i], k[i], p);
                float s = wave_sum(p) / a.temperature;
                const int64_t ms = mr[h] * N + j;
                if (a.mask_node[ms] == 0) s = -1e10f;
                const float e = a.ew ? a.ew[ms] : 1.f;
                const float mn = fmaxf(m[h], s);
                const float sc = expf(m[h] - mn), w = expf(s - mn);
                l[h] = l[h] * sc + w;
                const float we = w * e;
#pragma unroll
                for (int i = 0; i < KPL; ++i) acc[h][i] = __builtin_fmaf(we, k[i], acc[h][i] * sc);
                m[h] = mn;
            }
        }
    }
#pragma unroll
    for (int h = 0; h < ATT_MAXH; ++h) {
        if (h < H) {
            const float inv = 1.f / l[h];
#pragma unroll
            for (int i = 0; i < KPL; ++i) {
                const int c = lane + 64 * i;
                if (c < dk) z[(r * H + h) * dk + c] = acc[h][i] * inv;
            }
            if (lane == 0) {
                stats[(r * H + h) * 2] = m[h];
                stats[(r * H + h) * 2 + 1] = l[h];
            }
        }
    }
}

// The same forward with the row's neighbours split over the workgroup's ATT_WAVES waves (wave w takes
// j = w, w + 4, ...), each running its own online softmax; the partial states (max, normaliser,
// weighted key sum) merge through LDS in wave order.  A row's neighbours are independent gathers, so
// four waves keep four of them in flight where one wave walked the chain alone; the 300-row root
// layer of a bs=100 contrast had only 300 waves for 1,024 SIMDs.
template <int KPL, int HM>
__global__ void __launch_bounds__(64 * ATT_WAVES) tgn_attn_fwd_split_kernel(tm_tgn_attn a, float *__restrict__ z,
                                                                            float *__restrict__ stats) {
    __shared__ float s_acc[ATT_WAVES][HM][KPL][64], s_m[ATT_WAVES][HM], s_l[ATT_WAVES][HM];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t r = blockIdx.x;
    const int H = a.n_head, N = a.n_ngh, dk = a.d_node + a.d_edge + a.d_time;
    const KeyLane<KPL> L = key_lane<KPL>(a, lane);
    float q[HM][KPL], acc[HM][KPL], m[HM], l[HM];
    int64_t mr[HM];
#pragma unroll
    for (int h = 0; h < HM; ++h) {
        m[h] = -__builtin_inff();
        l[h] = 0.f;
        mr[h] = h < H ? pair_row(a, r, h) : 0;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
            const int c = lane + 64 * i;
            q[h][i] = (h < H && c < dk) ? a.qf[(r * H + h) * dk + c] : 0.f;
            acc[h][i] = 0.f;
        }
    }
    for (int j = wv; j < N; j += ATT_WAVES) {
        float k[KPL];
        build_key<KPL>(a, L, r * N + j, k);
#pragma unroll
        for (int h = 0; h < HM; ++h) {
            if (h < H) {
                float p = 0.f;
#pragma unroll
                for (int i = 0; i < KPL; ++i) p = __builtin_fmaf(q[h][i], k[i], p);
                float s = wave_sum(p) / a.temperature;
                const int64_t ms = mr[h] * N + j;
                if (a.mask_node[ms] == 0) s = -1e10f;
                const float e = a.ew ? a.ew[ms] : 1.f;
                const float mn = fmaxf(m[h], s);
                const float sc = expf(m[h] - mn), w = expf(s - mn);
                l[h] = l[h] * sc + w;
                const float we = w * e;
#pragma unroll
                for (int i = 0; i < KPL; ++i) acc[h][i] = __builtin_fmaf(we, k[i], acc[h][i] * sc);
                m[h] = mn;
            }
        }
    }
#pragma unroll
    for (int h = 0; h < HM; ++h) {
#pragma unroll
        for (int i = 0; i < KPL; ++i) s_acc[wv][h][i][lane] = acc[h][i];
        if (lane == 0) {
            s_m[wv][h] = m[h];
            s_l[wv][h] = l[h];
        }
    }
    __syncthreads();
    if (wv != 0) return;
#pragma unroll
    for (int h = 0; h < HM; ++h) {
        if (h >= H) continue;
        float M = s_m[0][h];
#pragma unroll
        for (int w = 1; w < ATT_WAVES; ++w) M = fmaxf(M, s_m[w][h]);
        float Ls = 0.f, sc[ATT_WAVES];
#pragma unroll
        for (int w = 0; w < ATT_WAVES; ++w) {
            sc[w] = s_l[w][h] > 0.f ? expf(s_m[w][h] - M) : 0.f;   // a wave with no neighbour adds nothing
            Ls += s_l[w][h] * sc[w];
        }
        const float inv = 1.f / Ls;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
            float v = 0.f;
#pragma unroll
            for (int w = 0; w < ATT_WAVES; ++w) v = __builtin_fmaf(s_acc[w][h][i][lane], sc[w], v);
            const int c = lane + 64 * i;
            if (c < dk) z[(r * H + h) * dk + c] = v * inv;
        }
        if (lane == 0) {
            stats[(r * H + h) * 2] = M;
            stats[(r * H + h) * 2 + 1] = Ls;
        }
    }
}

// Backward of z[r,h] = sum_j p_j e_j k_j, p = softmax(s), s_j = qf_h.k_j / T (masked: constant):
//   c_j = gz_h.k_j;  d e_j += p_j c_j;  S_h = sum_j p_j e_j c_j;  ds_j = p_j (e_j c_j - S_h) (0 if masked)
//   d k_j = sum_h p_j e_j gz_h + (ds_j / T) qf_h        (node-feature columns only are written)
// Pass 1 rebuilds every key (scores and c_j); pass 2 needs only the per-(j,h) scalars kept in LDS.
template <int KPL, bool DNODE, int HM>
__global__ void __launch_bounds__(64 * ATT_WAVES) tgn_attn_bwd_kernel(tm_tgn_attn a, const float *__restrict__ stats,
                                                                      const float *__restrict__ gz,
                                                                      float *__restrict__ d_parts,
                                                                      float *__restrict__ d_node) {
    extern __shared__ float sh[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t r = (int64_t)blockIdx.x * ATT_WAVES + wave;
    if (r >= a.rows) return;
    const int H = a.n_head, N = a.n_ngh, dk = a.d_node + a.d_edge + a.d_time;
    float *pe_s = sh + (size_t)wave * 3 * N * HM;  // [N][MAXH] p*e
    float *ds_s = pe_s + N * HM;                   // [N][MAXH] p (0 if masked)
    float *ec_s = ds_s + N * HM;                   // [N][MAXH] e*c
    const KeyLane<KPL> L = key_lane<KPL>(a, lane);
    float q[HM][KPL], g[HM][KPL], m[HM], il[HM], S[HM];
    int64_t mr[HM];
#pragma unroll
    for (int h = 0; h < HM; ++h) {
        S[h] = 0.f;
        mr[h] = h < H ? pair_row(a, r, h) : 0;
        m[h] = h < H ? stats[(r * H + h) * 2] : 0.f;
        il[h] = h < H ? 1.f / stats[(r * H + h) * 2 + 1] : 0.f;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
            const int c = lane + 64 * i;
            const bool ok = h < H && c < dk;
            q[h][i] = ok ? a.qf[(r * H + h) * dk + c] : 0.f;
            g[h][i] = ok ? gz[(r * H + h) * dk + c] : 0.f;
        }
    }
    for (int j = 0; j < N; ++j) {
        float k[KPL];
        build_key<KPL>(a, L, r * N + j, k);
#pragma unroll
        for (int h = 0; h < HM; ++h) {
            if (h < H) {
                float ps = 0.f, pc = 0.f;
#pragma unroll
                for (int i = 0; i < KPL; ++i) {
                    ps = __builtin_fmaf(q[h][i], k[i], ps);
                    pc = __builtin_fmaf(g[h][i], k[i], pc);
                }
                float s = wave_sum(ps) / a.temperature;
                const float c = wave_sum(pc);
                const int64_t ms = mr[h] * N + j;
                const bool masked = a.mask_node[ms] == 0;
                if (masked) s = -1e10f;
                const float e = a.ew ? a.ew[ms] : 1.f;
                const float p = expf(s - m[h]) * il[h];
                S[h] = __builtin_fmaf(p * e, c, S[h]);
                if (lane == 0) {
                    d_parts[(r * H + h) * N + j] = p * c;
                    if (DNODE) {
                        pe_s[j * HM + h] = p * e;
                        ds_s[j * HM + h] = masked ? 0.f : p;
                        ec_s[j * HM + h] = e * c;
                    }
                }
            }
        }
    }
    if (!DNODE) return;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float invT = 1.f / a.temperature;
    for (int j = 0; j < N; ++j) {
        float dkv[KPL];
#pragma unroll
        for (int i = 0; i < KPL; ++i) dkv[i] = 0.f;
#pragma unroll
        for (int h = 0; h < HM; ++h) {
            if (h < H) {
                const float pe = pe_s[j * HM + h];
                const float ds = ds_s[j * HM + h] * (ec_s[j * HM + h] - S[h]) * invT;
#pragma unroll
                for (int i = 0; i < KPL; ++i) dkv[i] = __builtin_fmaf(pe, g[h][i], __builtin_fmaf(ds, q[h][i], dkv[i]));
            }
        }
        float *dst = d_node + (r * N + j) * (int64_t)a.d_node;
#pragma unroll
        for (int i = 0; i < KPL; ++i)
            if (L.seg[i] == 0) dst[L.off[i]] = dkv[i];
    }
}

}  // namespace tmk

using namespace tmk;

static int check_attn(const tm_tgn_attn *a, const char *who) {
    if (!a) return fail(TM_E_ARG, std::string(who) + ": NULL descriptor");
    if (a->rows < 0 || a->n_ngh <= 0 || a->n_head < 1 || a->n_head > ATT_MAXH || a->d_node <= 0 || a->d_edge < 0 ||
        a->d_time < 0 || !(a->temperature > 0.f))
        return fail(TM_E_ARG, std::string(who) + ": bad sizes");
    const int dk = a->d_node + a->d_edge + a->d_time;
    if (dk > 64 * 8) return fail(TM_E_UNSUPPORTED, std::string(who) + ": d_key > 512");
    if (a->rows == 0) return TM_OK;
    if (!a->node_tab || (a->d_edge && !a->edge_tab) || !a->dt || (a->d_time && (!a->time_w || !a->time_b)) ||
        !a->mask_node || !a->qf)
        return fail(TM_E_ARG, std::string(who) + ": NULL pointer");
    if (a->seg_rows < 0 || (a->seg_rows > 0 && a->rows % a->seg_rows))
        return fail(TM_E_SHAPE, std::string(who) + ": rows must be a multiple of seg_rows");
    if ((a->node_idx && a->node_rows <= 0) || (a->edge_idx && a->edge_rows <= 0))
        return fail(TM_E_ARG, std::string(who) + ": empty feature table");
    return TM_OK;
}

template <int KPL>
static void launch_fwd(const tm_tgn_attn &a, float *z, float *stats, hipStream_t s) {
    if (a.n_ngh >= ATT_WAVES) {   // one row per workgroup, its neighbours over the waves
        // the heads' register arrays sized for at most 2 heads where that covers them (TGN's default n_heads):
        // 143 -> 96 VGPRs, 3 -> 5 waves per SIMD, 0.075 -> 0.055 ms per launch (round 5, profiles/r05_tgn_attn_ab.txt)
        if (a.n_head <= 2) tgn_attn_fwd_split_kernel<KPL, 2><<<dim3((unsigned)a.rows), 64 * ATT_WAVES, 0, s>>>(a, z, stats);
        else tgn_attn_fwd_split_kernel<KPL, ATT_MAXH><<<dim3((unsigned)a.rows), 64 * ATT_WAVES, 0, s>>>(a, z, stats);
        return;
    }
    const unsigned blocks = (unsigned)((a.rows + ATT_WAVES - 1) / ATT_WAVES);
    tgn_attn_fwd_kernel<KPL><<<dim3(blocks), 64 * ATT_WAVES, 0, s>>>(a, z, stats);
}

template <int KPL>
static void launch_bwd(const tm_tgn_attn &a, const float *stats, const float *gz, float *dp, float *dn, hipStream_t s) {
    const unsigned blocks = (unsigned)((a.rows + ATT_WAVES - 1) / ATT_WAVES);
    // the per-wave (p e, p, e c) rows are [n_ngh][HM]: LDS sized for the instance launched, so the 2-head form
    // does not reserve (and lose occupancy to) 4 heads' worth
    const int hm = a.n_head <= 2 ? 2 : ATT_MAXH;
    const size_t lds = dn ? sizeof(float) * 3 * a.n_ngh * hm * ATT_WAVES : 0;
    // the heads' register arrays sized for at most 2 heads where that covers them (as the forward)
    if (a.n_head <= 2) {
        if (dn) tgn_attn_bwd_kernel<KPL, true, 2><<<dim3(blocks), 64 * ATT_WAVES, lds, s>>>(a, stats, gz, dp, dn);
        else tgn_attn_bwd_kernel<KPL, false, 2><<<dim3(blocks), 64 * ATT_WAVES, 0, s>>>(a, stats, gz, dp, dn);
    } else {
        if (dn) tgn_attn_bwd_kernel<KPL, true, ATT_MAXH><<<dim3(blocks), 64 * ATT_WAVES, lds, s>>>(a, stats, gz, dp, dn);
        else tgn_attn_bwd_kernel<KPL, false, ATT_MAXH><<<dim3(blocks), 64 * ATT_WAVES, 0, s>>>(a, stats, gz, dp, dn);
    }
}

#define TM_KPL_DISPATCH(KPLV, CALL) \
    switch (KPLV) {                 \
        case 1: CALL(1); break;     \
        case 2: CALL(2); break;     \
        case 3: CALL(3); break;     \
        case 4: CALL(4); break;     \
        case 5: CALL(5); break;     \
        case 6: CALL(6); break;     \
        case 7: CALL(7); break;     \
        default: CALL(8); break;    \
    }

extern "C" int tm_tgn_attn_fwd(const tm_tgn_attn *a, float *z, float *stats, void *stream) {
    int rc = check_attn(a, "tm_tgn_attn_fwd");
    if (rc != TM_OK || a->rows == 0) return rc;
    if (!z || !stats) return fail(TM_E_ARG, "tm_tgn_attn_fwd: NULL output");
    hipStream_t s = (hipStream_t)stream;
    const int kpl = (a->d_node + a->d_edge + a->d_time + 63) / 64;
    hipEvent_t pe = prof_begin(s);
#define TM_FWD(K) launch_fwd<K>(*a, z, stats, s)
    TM_KPL_DISPATCH(kpl, TM_FWD)
#undef TM_FWD
    TM_CHECK_LAUNCH();
    prof_end("tgn_attn_fwd_kernel", s, pe);
    return TM_OK;
}

extern "C" int tm_tgn_attn_bwd(const tm_tgn_attn *a, const float *stats, const float *gz, float *d_ew_parts,
                               float *d_node, void *stream) {
    int rc = check_attn(a, "tm_tgn_attn_bwd");
    if (rc != TM_OK || a->rows == 0) return rc;
    if (!stats || !gz || !d_ew_parts) return fail(TM_E_ARG, "tm_tgn_attn_bwd: NULL pointer");
    if (d_node && a->node_idx) return fail(TM_E_ARG, "tm_tgn_attn_bwd: d_node needs a dense node table");
    if ((size_t)3 * a->n_ngh * ATT_MAXH * ATT_WAVES * sizeof(float) > 64 * 1024)
        return fail(TM_E_UNSUPPORTED, "tm_tgn_attn_bwd: n_ngh too large");
    hipStream_t s = (hipStream_t)stream;
    const int kpl = (a->d_node + a->d_edge + a->d_time + 63) / 64;
    hipEvent_t pe = prof_begin(s);
#define TM_BWD(K) launch_bwd<K>(*a, stats, gz, d_ew_parts, d_node, s)
    TM_KPL_DISPATCH(kpl, TM_BWD)
#undef TM_BWD
    TM_CHECK_LAUNCH();
    prof_end("tgn_attn_bwd_kernel", s, pe);
    return TM_OK;
}
