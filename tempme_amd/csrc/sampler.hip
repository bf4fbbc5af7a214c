// Temporal k-hop sampling, temporal-walk motif enumeration and motif bookkeeping on gfx950.
//
// Reference (dharunm236/TempME):
//   k-hop:  utils/graph.py:103-146 (find_before), :197-231 (get_temporal_neighbor), :233-262 (find_k_hop)
//   walks:  utils/graph.py:149-194 (find_before_walk), :265-306 (find_k_walks), :308-333 (get_next_step),
//           :335-476 (get_final_step)
//   motif:  processed/data_preprocess.py:148-214 (marginal), :327-343 (new_edge_info);
//           utils/null_model.py:75-121 (statistic); utils/batch_loader.py:39-42 (RandEdgeSampler.sample)
//
// Layout: adjacency records are 16-byte {ngh, eid, ts(f64)} so every sampled slot is one
// dwordx4 gather; e_idx -> position is an O(1) per-edge table (EdgeEnds); the filtered
// step-3 candidate sets of get_final_step are counted and indexed through a per-node
// (neighbor, position)-sorted pair index with binary searches instead of O(deg) scans.
#include <cstdlib>

#include "common.h"




namespace tmk {

// output stores are plain (write-back) stores: streamed non-temporal stores measured slower (events_kernel
// 0.170 -> 0.175 ms, the k-hop kernel's in-row scattered outputs 2.4x slower)
#define TM_ST(dst, v) ((dst) = (v))

constexpr int kMaxN = 64;   // n_degree supported by the sampling kernels (reference: 20..60)
constexpr int kMaxM = 8;    // walks per hop-1 slot (reference: 3, null model 1)

__device__ __forceinline__ void set_err(int32_t *err, int32_t code) {
    if (err) atomicCAS(err, 0, code);
}

// cut length of find_before (graph.py:103-146); time path or e_idx path
__device__ __forceinline__ int32_t find_before_len(const DevGraph &g, int32_t u, bool time_path, double cut,
                                                   int32_t e, int32_t *err) {
    if (u < 0 || u >= g.n_nodes) {
        set_err(err, TM_E_ARG);
        return 0;
    }
    if (time_path) return bisect_ts(g, u, cut);
    if (!(u > 0)) return 0;
    int32_t l = edge_len(g, u, e);
    if (l < 0) {
        set_err(err, TM_E_EDGE_NOT_IN_LIST);
        return 0;
    }
    return l;
}

// bisect_left over node u's timestamps by the whole wave (all 64 lanes call it, the result is
// uniform): each round tests 64 evenly spaced records and keeps the gap holding the answer, so a
// list of up to 4096 records costs two dependent loads instead of twelve.
__device__ int32_t bisect_ts_wave(const DevGraph &g, int32_t u, double x) {
    const int32_t s = g.off[u], lane = threadIdx.x & 63;
    int32_t lo = 0, hi = g.off[u + 1] - s;
    while (hi - lo > 64) {
        const int32_t stride = (hi - lo + 63) / 64, q = lo + lane * stride;
        const bool lt = q < hi && g.tsd[s + q] < x;
        const int32_t c = __popcll(__ballot(lt));        // sorted: the samples below x are a prefix
        const int32_t nlo = c > 0 ? lo + (c - 1) * stride + 1 : lo;
        hi = min(hi, lo + c * stride);
        lo = nlo;
    }
    const int32_t q = lo + lane;
    const bool lt = q < hi && g.tsd[s + q] < x;
    return lo + __popcll(__ballot(lt));
}

// rank-th smallest position of the union of two sorted, disjoint position lists
__device__ __forceinline__ int32_t kth_of_two(const int32_t *p1, int32_t n1, const int32_t *p2, int32_t n2, int32_t r) {
    int32_t lo = max(0, r + 1 - n2), hi = min(n1, r + 1);
    while (lo < hi) {
        int32_t mid = (lo + hi) >> 1, j = r + 1 - mid;
        if (j == 0 || p1[mid] > p2[j - 1]) hi = mid;
        else lo = mid + 1;
    }
    int32_t i = lo, j = r + 1 - lo;
    int32_t a = i > 0 ? p1[i - 1] : -1, b = j > 0 ? p2[j - 1] : -1;
    return a > b ? a : b;
}

// K (node, neighbour) block lookups in lockstep (u < 0: empty block): base and size of each block
template <int K>
__device__ __forceinline__ void pair_blocks(const DevGraph &g, const int32_t (&u)[K], const int32_t (&x)[K],
                                            int32_t (&base)[K], int32_t (&n)[K]) {
    uint32_t h[K];
    bool live[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        live[k] = u[k] >= 0;
        h[k] = pblk_hash(u[k], x[k]) & g.pblk_mask;
        base[k] = n[k] = 0;
    }
    while (true) {
        bool any = false;
#pragma unroll
        for (int k = 0; k < K; ++k) any |= live[k];
        if (!any) break;
        PairBlk b[K];
#pragma unroll
        for (int k = 0; k < K; ++k) b[k] = live[k] ? g.pblk[h[k]] : PairBlk{-1, 0, 0, 0};   // no access when done
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (!live[k]) continue;
            if (b[k].u == u[k] && b[k].x == x[k]) {
                base[k] = b[k].base;
                n[k] = b[k].n;
                live[k] = false;
            } else if (b[k].u == -1) {
                live[k] = false;
            } else {
                h[k] = (h[k] + 1) & g.pblk_mask;
            }
        }
    }
}

// K lower bounds "number of the block's positions < p" in lockstep, each down the block's search
// tree (common.h): one F-key node per level; live[k] false: 0
template <int K>
__device__ __forceinline__ void blk_lb_multi(const DevGraph &g, const int32_t (&base)[K], const int32_t (&n)[K],
                                             const int32_t (&p)[K], const bool (&live)[K], int32_t (&res)[K]) {
    constexpr int NQ = kBlkFan / 4;      // quads per node
    int32_t h[K], l[K], off[K], j[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        h[k] = blk_levels(n[k]);
        l[k] = live[k] && n[k] > 0 ? h[k] : -1;
        off[k] = base[k];
        j[k] = 0;
        res[k] = 0;
    }
    while (true) {
        bool any = false;
#pragma unroll
        for (int k = 0; k < K; ++k) any |= l[k] >= 0;
        if (!any) break;
        int4 v[K][NQ];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            // a block of <= F keys holds ceil(n/4) quads; every tree node F/4
            const int32_t nq = h[k] == 0 ? (n[k] + 3) >> 2 : NQ;
            const int4 *q = reinterpret_cast<const int4 *>(g.ppos + off[k] + kBlkFan * j[k]);
#pragma unroll
            for (int t = 0; t < NQ; ++t)
                v[k][t] = (l[k] >= 0 && t < nq) ? q[t] : make_int4(INT32_MAX, INT32_MAX, INT32_MAX, INT32_MAX);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (l[k] < 0) continue;
            int32_t c = 0;
#pragma unroll
            for (int t = 0; t < NQ; ++t)
                c += (v[k][t].x < p[k]) + (v[k][t].y < p[k]) + (v[k][t].z < p[k]) + (v[k][t].w < p[k]);
            if (l[k] == 0) {
                res[k] = kBlkFan * j[k] + c;
                l[k] = -1;
            } else if (l[k] == h[k] && c == 0) {
                res[k] = 0;
                l[k] = -1;
            } else {
                off[k] += blk_level_len(n[k], l[k], h[k]);
                j[k] = kBlkFan * j[k] + c - 1;
                --l[k];
            }
        }
    }
}

// one lower bound down a block's search tree
__device__ __forceinline__ int32_t blk_lb(const DevGraph &g, int32_t base, int32_t n, int32_t p) {
    const int32_t b[1] = {base}, nn[1] = {n}, pp[1] = {p};
    const bool live[1] = {true};
    int32_t r[1];
    blk_lb_multi<1>(g, b, nn, pp, live, r);
    return r[0];
}

// phase stamps inside final_step (debug builds only, -DTM_STAMPS): s_memtime into T[k] at wave-uniform points
#ifdef TM_STAMPS
#define TM_FS(k)                                            \
    do {                                                    \
        if (T) {                                            \
            __builtin_amdgcn_sched_barrier(0);              \
            T[k] = __builtin_amdgcn_s_memtime();            \
            __builtin_amdgcn_sched_barrier(0);              \
        }                                                   \
    } while (0)
#else
#define TM_FS(k) (void)T
#endif

struct Step3 {
    int32_t src, ngh, eid;
    float ts;
    int32_t code, t;
};

// get_final_step for one walk (graph.py:353-474), incl. quirks:
//  * case order A (src1==src2 && tgt1!=tgt2) / B (tgt1==src2 && src1!=tgt2) / C (else)
//  * nodeedge2idx[..].get(e2) of None slices the WHOLE list (future leak)
//  * node 0 is padding (cut 0) even when it is a real node
// pos2 / rank2: the step-2 record's position in src2's list and its rank in its (src2, tgt2) block (-1:
// none).  In the filtered cases the a-side node is src2 and a2 = tgt2, so when the cut of e2 is the
// record's own position (no tie group moved it) the count of a2-entries before the cut is rank2.
__device__ Step3 final_step(const DevGraph &g, Key key, uint32_t ev, uint32_t w, int32_t src1, int32_t tgt1,
                            int32_t src2, int32_t tgt2, int32_t e2, int32_t pos2, int32_t rank2,
                            unsigned long long *T = nullptr) {
    int32_t code, a_node, a1 = 0, a2 = 0, b_node, bf = 0;
    bool filt;
    if (src1 == src2 && tgt1 != tgt2) {
        code = 2; a_node = src1; a1 = tgt1; a2 = tgt2; b_node = tgt2; bf = tgt1; filt = true;
    } else if (tgt1 == src2 && src1 != tgt2) {
        code = 3; a_node = tgt1; a1 = src1; a2 = tgt2; b_node = tgt2; bf = src1; filt = true;
    } else {
        code = 1; a_node = tgt1; b_node = tgt2; filt = false;
    }
    // everything the cut lengths and the record offsets need, loaded together up front:
    // final_len (graph.py:357, :366): node 0 / out of range -> 0; e2 not in the node's dict -> whole list
    const bool va = a_node > 0 && a_node < g.n_nodes, vb = b_node > 0 && b_node < g.n_nodes;
    const EdgeEnds x2 = (e2 >= 0 && e2 <= g.max_eid) ? g.ends[e2] : EdgeEnds{-1, 0, -1, 0};
    const int2 oa = va ? g.span[a_node] : make_int2(0, 0), ob = vb ? g.span[b_node] : make_int2(0, 0);
    const int32_t oa0 = oa.x, oa1 = oa.y, ob0 = ob.x, ob1 = ob.y;
    int32_t ca = !va ? 0 : x2.node_a == a_node ? x2.len_a : x2.node_b == a_node ? x2.len_b : oa1 - oa0;
    int32_t cb = !vb ? 0 : x2.node_a == b_node ? x2.len_a : x2.node_b == b_node ? x2.len_b : ob1 - ob0;
    if (g.strict) {   // strict_temporal: the None lookup cuts at e2's own time instead of leaking the future
        const double t2 = (e2 >= 0 && e2 <= g.max_eid) ? g.ets[e2] : 0.0;
        if (va && x2.node_a != a_node && x2.node_b != a_node) ca = bisect_ts(g, a_node, t2);
        if (vb && x2.node_a != b_node && x2.node_b != b_node) cb = bisect_ts(g, b_node, t2);
    }
    int32_t na, nb, k1 = 0, n1 = 0, k2 = 0, n2 = 0, kb = 0;
    TM_FS(8);
    if (filt) {
        // filtered counts: the (node, neighbour) block of each of the three neighbours from the block
        // table, then the entries before the cut inside each block down its search tree; the lookups
        // and the searches each run in lockstep
        const bool sa = ca > 0, sb = cb > 0;
        const int32_t us[3] = {sa ? a_node : -1, sa ? a_node : -1, sb ? b_node : -1}, xs[3] = {a1, a2, bf};
        int32_t bs[3], bn[3], cnt[3];
        pair_blocks<3>(g, us, xs, bs, bn);
        const bool r2 = pos2 >= 0 && ca == pos2;
        cnt[0] = blk_lb(g, bs[0], bn[0], ca);
        cnt[2] = blk_lb(g, bs[2], bn[2], cb);
        cnt[1] = r2 ? 0 : blk_lb(g, bs[1], bn[1], ca);   // a tie group moved e2's cut off its own record
        n1 = cnt[0];
        n2 = r2 ? (sa ? rank2 : 0) : cnt[1];
        nb = cnt[2];
        k1 = bs[0] + blk_keys_off(bn[0]);
        k2 = bs[1] + blk_keys_off(bn[1]);
        kb = bs[2] + blk_keys_off(bn[2]);
        na = n1 + n2;
    } else {
        na = ca;
        nb = cb;
    }
    TM_FS(9);
    Step3 o{0, 0, 0, 0.f, code, 0};
    if (na + nb == 0) {
        TM_FS(10);
        TM_FS(11);
        return o;
    }
    const int32_t r = draw(key, TM_STAGE_STEP3, ev, w, 0, (uint32_t)(na + nb));
    int32_t ent;
    if (r < na) {
        o.src = a_node;
        int32_t pos = filt ? kth_of_two(g.ppos + k1, n1, g.ppos + k2, n2, r) : r;
        ent = oa0 + pos;
    } else {
        o.src = b_node;
        int32_t rr = r - na;
        int32_t pos = filt ? g.ppos[kb + rr] : rr;
        ent = ob0 + pos;
    }
    TM_FS(10);
    const Rec rc = g.rec[ent];
    o.ngh = rc.ngh;
    o.eid = rc.eid;
    o.ts = rc.ts;
    int32_t t;
    const int32_t s = o.src, n = o.ngh;
    if (code == 2) {
        t = (s == src1 && n == tgt1) ? 1 : (s == src1 && n == tgt2) ? 2 : (s == tgt1 && n == tgt2) ? 3 : 0;
    } else if (code == 3) {
        t = (s == tgt1 && n == src1) ? 1 : (s == tgt1 && n == tgt2) ? 3 : (s == tgt2 && n == src1) ? 2 : 0;
    } else {
        t = (s == src1 && n != tgt1) ? 3 : (s == tgt1 && n != src1) ? 2 : (s == src1 && n == tgt1) ? 1
            : (s == tgt1 && n == src1) ? 1 : 0;
    }
    o.t = t;
    TM_FS(11);
    return o;
}

// anony [1, code, t] -> category id (marginal order, data_preprocess.py:171-178) or null key-1
__device__ __forceinline__ int32_t cat_of(int32_t code, int32_t t, int null_order) {
    if (t < 0 || t > 3) return -1;
    // packed 4-bit tables indexed by t
    const uint32_t cat2 = 0x2103, cat3 = 0x5647, cat1 = 0x89AB;      // t=0..3 -> {3,0,1,2} {7,4,6,5} {11,10,9,8}
    const uint32_t nul2 = 0x2310, nul3 = 0x6754, nul1 = 0xBA98;      // {0,1,3,2} {4,5,7,6} {8,9,10,11}
    uint32_t tab = null_order ? (code == 2 ? nul2 : code == 3 ? nul3 : code == 1 ? nul1 : 0xFFFF)
                              : (code == 2 ? cat2 : code == 3 ? cat3 : code == 1 ? cat1 : 0xFFFF);
    uint32_t v = (tab >> (4 * t)) & 0xF;
    return v == 0xF ? -1 : (int32_t)v;
}

// step 2 of one walk: the m-th smallest of the M draws over the concatenated candidates
// [root's prefix before e1 | v1's prefix before e1] (graph.py:323-332).
struct Step2 {
    int32_t src, ngh, eid;
    float ts;
    int32_t pos, rank;    // the record's position in src's list and its (src, ngh) block rank; -1: none
};

// candidate cut lengths and record offsets of step 2 for one hop-1 slot (shared by its M walks):
// walk_len (graph.py:171-176) of root u and of v1 from one EdgeEnds load
struct Step2Cuts {
    int32_t cu, cv, ou, ov;
};

__device__ __forceinline__ Step2Cuts step2_cuts(const DevGraph &g, int32_t u, int32_t v1, int32_t e1) {
    const bool vu = u > 0 && u < g.n_nodes, vv = v1 > 0 && v1 < g.n_nodes;
    const EdgeEnds x1 = (e1 >= 0 && e1 <= g.max_eid) ? g.ends[e1] : EdgeEnds{-1, 0, -1, 0};
    const int32_t lu = x1.node_a == u ? x1.len_a : x1.node_b == u ? x1.len_b : -1;
    const int32_t lv = x1.node_a == v1 ? x1.len_a : x1.node_b == v1 ? x1.len_b : -1;
    return Step2Cuts{(vu && lu > 0) ? lu : 0, (vv && lv > 0) ? lv : 0, vu ? g.off[u] : 0, vv ? g.off[v1] : 0};
}

// MC > 0: M is the compile-time constant MC (3 for the walks, 1 for the null model) and the rank of
// each draw is MC x MC compares; MC = 0: any M <= kMaxM, padded to kMaxM.
template <int MC = 0>
__device__ __forceinline__ Step2 next_step(const DevGraph &g, Key key, uint32_t ev, uint32_t slot, int32_t M,
                                           int32_t m, int32_t u, int32_t v1, const Step2Cuts &sc) {
    constexpr int MX = MC > 0 ? MC : kMaxM;
    if (MC > 0) M = MC;
    Step2 o{0, 0, 0, 0.f, -1, -1};
    const int32_t cu = sc.cu, cv = sc.cv, ou = sc.ou, ov = sc.ov, tot = cu + cv;
    if (tot == 0) return o;
    uint32_t dv[MX];
    const uint4 b0 = draw_block(key, TM_STAGE_STEP2, ev, slot, 0);          // draws 0..3 of the slot
    const uint4 b1 = (MX > 4 && M > 4) ? draw_block(key, TM_STAGE_STEP2, ev, slot, 1) : b0;
    const uint32_t words[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int k = 0; k < MX; ++k) dv[k] = k < M ? (uint32_t)scale_draw(words[k], tot) : 0xFFFFFFFFu;
    uint32_t sel = 0;
#pragma unroll
    for (int k = 0; k < MX; ++k) {
        int32_t rank = 0;
#pragma unroll
        for (int i = 0; i < MX; ++i) rank += (dv[i] < dv[k]) || (i < k && dv[i] == dv[k]);
        if (k < M && rank == m) sel = dv[k];
    }
    const int32_t x = (int32_t)sel;
    int32_t ent;
    if (x < cu) {
        o.src = u;
        o.pos = x;
        ent = ou + x;
    } else {
        o.src = v1;
        o.pos = x - cu;
        ent = ov + (x - cu);
    }
    const Rec rc = g.rec[ent];
    o.ngh = rc.ngh;
    o.eid = rc.eid;
    o.ts = rc.ts;
    o.rank = rc.brank;
    return o;
}

// ------------------------------------------------------------------ k-hop: one Philox block per thread
// A workgroup takes R = 256 / NB rows (NB = ceil(N/4) Philox blocks per row).  Each thread computes
// ONE Philox block = 4 consecutive draws of its row (the contract's counter (row, j>>2), word j&3),
// so a wave covers 256 draws instead of 64 lanes x 1; the row's cut length and record offset are
// looked up once per row, the draws go to LDS, and each thread ranks its 4 draws against the row
// (np.sort order, ties by draw index) and gathers their records.
__global__ void __launch_bounds__(256) khop_kernel(DevGraph g, Key key, uint32_t stage, int32_t N, int64_t rows,
                                                   int64_t rows_per_event, const int32_t *__restrict__ root,
                                                   const double *__restrict__ cut, const int32_t *__restrict__ eidx,
                                                   int time_path, const uint32_t *__restrict__ event_ids,
                                                   int32_t *__restrict__ on, int32_t *__restrict__ oe,
                                                   float *__restrict__ ot, int32_t *err) {
    extern __shared__ uint32_t kh_lds[];
    const int32_t NB = (N + 3) >> 2, R = 256 / NB;
    int32_t *rc = reinterpret_cast<int32_t *>(kh_lds), *ro = rc + R;   // per row: cut length, record offset
    uint32_t *dd = kh_lds + 2 * R;                                     // [R][N] draws
    const int64_t r0 = (int64_t)blockIdx.x * R;
    const int tid = threadIdx.x;
    if (tid < R) {
        const int64_t r = r0 + tid;
        int32_t c = 0, o = 0;
        if (r < rows) {
            const int32_t u = root[r];
            c = find_before_len(g, u, time_path, time_path ? cut[r] : 0.0, time_path ? 0 : eidx[r], err);
            o = (c > 0) ? g.off[u] : 0;
        }
        rc[tid] = c;
        ro[tid] = o;
    }
    __syncthreads();
    const int32_t lr = tid / NB, kb = tid % NB;
    const int64_t r = r0 + lr;
    const bool act = lr < R && r < rows;
    uint32_t d[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    int32_t c = 0;
    if (act) {
        c = rc[lr];
        if (c > 0) {
            const uint4 b = draw_block(key, stage, event_ids[r / rows_per_event], (uint32_t)(r % rows_per_event), kb);
            d[0] = scale_draw(b.x, c);
            d[1] = scale_draw(b.y, c);
            d[2] = scale_draw(b.z, c);
            d[3] = scale_draw(b.w, c);
        }
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if (4 * kb + w < N) dd[lr * N + 4 * kb + w] = d[w];
    }
    __syncthreads();
    if (!act) return;
    int32_t rank[4] = {0, 0, 0, 0};
    if (c > 0)
        for (int32_t i = 0; i < N; ++i) {
            const uint32_t di = dd[lr * N + i];
#pragma unroll
            for (int w = 0; w < 4; ++w) rank[w] += (di < d[w]) || (i < 4 * kb + w && di == d[w]);
        }
    Rec rec[4];
#pragma unroll
    for (int w = 0; w < 4; ++w)
        rec[w] = (c > 0 && 4 * kb + w < N) ? g.rec[ro[lr] + (int32_t)d[w]] : Rec{0, 0, 0.f, 0};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int32_t k = 4 * kb + w;
        if (k >= N) break;
        const int64_t o = r * N + (c > 0 ? rank[w] : k);
        on[o] = rec[w].ngh;
        oe[o] = rec[w].eid;
        ot[o] = rec[w].ts;
    }
}

// ------------------------------------------------------------------ walks: one thread per walk
// ------------------------------------------------------------------ 2-hop fused: hop 1 and hop 2 in one launch
// find_k_hop(2, ...) as the reference calls it: a workgroup takes EPB roots, samples their hop-1 rows
// (kept in LDS), looks up the hop-2 rows' cut lengths and offsets once per row, then draws, ranks and
// gathers the EPB*N hop-2 rows -- one launch, and no hop-1 -> hop-2 round trip through HBM.
// Same Philox-block-per-thread scheme as khop_kernel.
// roots per workgroup: ~three hop-2 Philox blocks per thread (8 roots at N=20): each workgroup is a
// chain of dependent lookups with barriers between the levels, and more rows per level keep more
// gathers in flight per barrier (A/B at N=20: 2 / 4 / 8 / 16 roots -> 48 / 51 / 52 / 51 % of HBM)
__host__ __device__ inline int32_t khop2_epb(int32_t N) {
    const int32_t e = 3200 / (N * N);
    return e < 1 ? 1 : e > 8 ? 8 : e;
}

__host__ __device__ inline size_t khop2_lds_bytes(int32_t N) {
    const size_t epb = khop2_epb(N), rows2 = epb * N;
    return sizeof(int32_t) * (3 * epb + epb * N + 3 * rows2 + 2 * rows2 + rows2 * N);
}

// one level: record gathers of thread (row lr, block kb)'s 4 draws and their ranks among the row's N
// draws in dd; results staged in LDS at (row, rank) so the workgroup writes its output range coalesced

template <bool kStage, bool keyed>
__device__ __forceinline__ void khop_emit(const DevGraph &g, int32_t N, const uint32_t *dd, int32_t lr, int32_t kb,
                                          const uint32_t (&d)[4], int32_t c, int32_t o, int32_t *sn, int32_t *se,
                                          float *st) {
    // record gathers first (independent of the ranks), then the rank loop under their latency
    Rec rec[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) rec[w] = (c > 0 && 4 * kb + w < N) ? g.rec[o + (int32_t)d[w]] : Rec{0, 0, 0.f, 0};
    int32_t rank[4] = {0, 0, 0, 0};
    if (keyed && c > 0) {
        // dd holds (draw << 6 | index): unique keys, so the np.sort rank (ties by index) is one compare
        uint32_t my[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) my[w] = (d[w] << 6) | (uint32_t)(4 * kb + w);
        const uint4 *row = reinterpret_cast<const uint4 *>(dd + lr * N);
        if ((N & 3) == 0) {
            for (int32_t i4 = 0; i4 < (N >> 2); ++i4) {
                const uint4 q = row[i4];
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    rank[w] += (q.x < my[w]) + (q.y < my[w]) + (q.z < my[w]) + (q.w < my[w]);
            }
        } else {
            for (int32_t i = 0; i < N; ++i) {
                const uint32_t q = dd[lr * N + i];
#pragma unroll
                for (int w = 0; w < 4; ++w) rank[w] += q < my[w];
            }
        }
    } else if (!keyed && c > 0) {
        if ((N & 3) == 0) {                              // row start 16-B aligned: 4 draws per LDS read
            const uint4 *row = reinterpret_cast<const uint4 *>(dd + lr * N);
            for (int32_t i4 = 0; i4 < (N >> 2); ++i4) {
                const uint4 q = row[i4];
                const uint32_t qv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int32_t i = 4 * i4 + v;
#pragma unroll
                    for (int w = 0; w < 4; ++w) rank[w] += (qv[v] < d[w]) || (i < 4 * kb + w && qv[v] == d[w]);
                }
            }
        } else {
            for (int32_t i = 0; i < N; ++i) {
                const uint32_t di = dd[lr * N + i];
#pragma unroll
                for (int w = 0; w < 4; ++w) rank[w] += (di < d[w]) || (i < 4 * kb + w && di == d[w]);
            }
        }
    }
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int32_t k = 4 * kb + w;
        if (k >= N) break;
        // kStage: (row, rank) in LDS; else sn/se/st already point at this row's output
        const int32_t slot = (kStage ? lr * N : 0) + (c > 0 ? rank[w] : k);
        sn[slot] = rec[w].ngh;
        se[slot] = rec[w].eid;
        st[slot] = rec[w].ts;
    }
}

// ranks of thread (row lr, block kb)'s 4 draws d among the row's N draws in dd (np.sort order, ties by
// index); rank stays k for an empty row
template <bool keyed>
__device__ __forceinline__ void khop_ranks(int32_t N, const uint32_t *dd, int32_t lr, int32_t kb,
                                           const uint32_t (&d)[4], int32_t c, int32_t (&rank)[4]) {
#pragma unroll
    for (int w = 0; w < 4; ++w) rank[w] = c > 0 ? 0 : 4 * kb + w;
    if (keyed && c > 0) {
        // dd holds (draw << 6 | index): unique keys, so the np.sort rank (ties by index) is one compare
        uint32_t my[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) my[w] = (d[w] << 6) | (uint32_t)(4 * kb + w);
        const uint4 *row = reinterpret_cast<const uint4 *>(dd + lr * N);
        if ((N & 3) == 0) {
            for (int32_t i4 = 0; i4 < (N >> 2); ++i4) {
                const uint4 q = row[i4];
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    rank[w] += (q.x < my[w]) + (q.y < my[w]) + (q.z < my[w]) + (q.w < my[w]);
            }
        } else {
            for (int32_t i = 0; i < N; ++i) {
                const uint32_t q = dd[lr * N + i];
#pragma unroll
                for (int w = 0; w < 4; ++w) rank[w] += q < my[w];
            }
        }
    } else if (!keyed && c > 0) {
        if ((N & 3) == 0) {                              // row start 16-B aligned: 4 draws per LDS read
            const uint4 *row = reinterpret_cast<const uint4 *>(dd + lr * N);
            for (int32_t i4 = 0; i4 < (N >> 2); ++i4) {
                const uint4 q = row[i4];
                const uint32_t qv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int32_t i = 4 * i4 + v;
#pragma unroll
                    for (int w = 0; w < 4; ++w) rank[w] += (qv[v] < d[w]) || (i < 4 * kb + w && qv[v] == d[w]);
                }
            }
        } else {
            for (int32_t i = 0; i < N; ++i) {
                const uint32_t di = dd[lr * N + i];
#pragma unroll
                for (int w = 0; w < 4; ++w) rank[w] += (di < d[w]) || (i < 4 * kb + w && di == d[w]);
            }
        }
    }
}

template <bool keyed>
__global__ void __launch_bounds__(256) khop2_kernel(DevGraph g, Key key, int32_t N, int32_t B,
                                                    const int32_t *__restrict__ root, const double *__restrict__ cut,
                                                    const int32_t *__restrict__ eidx,
                                                    const uint32_t *__restrict__ event_ids, int32_t *__restrict__ on,
                                                    int32_t *__restrict__ oe, float *__restrict__ ot, int32_t *err) {
    extern __shared__ uint32_t k2_lds[];
    const int32_t EPB = khop2_epb(N), NB = (N + 3) >> 2, R2 = EPB * N;
    // draw rows first so each row starts 16-B aligned when N % 4 == 0 (uint4 reads in khop_emit)
    uint32_t *d2 = k2_lds, *d1 = d2 + R2 * N;
    int32_t *h1n = reinterpret_cast<int32_t *>(d1 + EPB * N), *h1e = h1n + R2, *c2 = h1e + R2, *o2 = c2 + R2;
    float *h1t = reinterpret_cast<float *>(o2 + R2);
    int32_t *c1 = reinterpret_cast<int32_t *>(h1t + R2), *o1 = c1 + EPB;
    uint32_t *ev1 = reinterpret_cast<uint32_t *>(o1 + EPB);
    const int32_t e0 = blockIdx.x * EPB, ne = min(EPB, B - e0), tid = threadIdx.x;
    const bool time_path = eidx == nullptr;
    // output pointers in VGPRs (scalar file pressure, see events_kernel), global address space
    const auto gon = TM_OUTP(on);
    const auto goe = TM_OUTP(oe);
    const auto got = TM_OUTP(ot);
    // hop-1 rows
    if (tid < ne) {
        const int32_t u = root[e0 + tid];
        const int32_t c = find_before_len(g, u, time_path, time_path ? cut[e0 + tid] : 0.0,
                                          time_path ? 0 : eidx[e0 + tid], err);
        c1[tid] = c;
        o1[tid] = (u >= 0 && u < g.n_nodes) ? g.off[u] : 0;   // issued alongside the cut lookup
        ev1[tid] = event_ids[e0 + tid];
    }
    __syncthreads();
    if (tid < ne * NB) {
        const int32_t lr = tid / NB, kb = tid % NB, c = c1[lr];
        uint32_t d[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        if (c > 0) {
            const uint4 b = draw_block(key, 1, ev1[lr], 0, kb);
            d[0] = scale_draw(b.x, c);
            d[1] = scale_draw(b.y, c);
            d[2] = scale_draw(b.z, c);
            d[3] = scale_draw(b.w, c);
        }
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if (4 * kb + w < N) d1[lr * N + 4 * kb + w] = keyed ? (d[w] << 6) | (uint32_t)(4 * kb + w) : d[w];
    }
    __syncthreads();
    if (tid < ne * NB) {
        const int32_t lr = tid / NB, kb = tid % NB;
        uint32_t d[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t v = 4 * kb + w < N ? d1[lr * N + 4 * kb + w] : 0xFFFFFFFFu;
            d[w] = keyed ? v >> 6 : v;
        }
        khop_emit<true, keyed>(g, N, d1, lr, kb, d, c1[lr], o1[lr], h1n, h1e, h1t);
    }
    __syncthreads();
    for (int32_t x = tid; x < ne * N; x += blockDim.x) {                 // hop-1 rows, coalesced
        const int64_t o = (int64_t)e0 * N + x;
        gon[o] = h1n[x];
        goe[o] = h1e[x];
        got[o] = h1t[x];
    }
    // hop-2 rows (e_idx path, graph.py:247-250): cut length and record offset once per row
    for (int32_t x = tid; x < ne * N; x += blockDim.x) {
        const int32_t v = h1n[x];
        c2[x] = find_before_len(g, v, false, 0.0, h1e[x], err);
        o2[x] = (v >= 0 && v < g.n_nodes) ? g.off[v] : 0;
    }
    __syncthreads();
    for (int32_t x = tid; x < ne * N * NB; x += blockDim.x) {
        const int32_t lr = x / NB, kb = x % NB, c = c2[lr];
        uint32_t d[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        if (c > 0) {
            const uint4 b = draw_block(key, 2, ev1[lr / N], (uint32_t)(lr % N), kb);
            d[0] = scale_draw(b.x, c);
            d[1] = scale_draw(b.y, c);
            d[2] = scale_draw(b.z, c);
            d[3] = scale_draw(b.w, c);
        }
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if (4 * kb + w < N) d2[lr * N + 4 * kb + w] = keyed ? (d[w] << 6) | (uint32_t)(4 * kb + w) : d[w];
    }
    __syncthreads();
    const int64_t base2 = (int64_t)B * N + (int64_t)e0 * N * N;
    // ranks (np.sort order) of each row's draws, whole rows per pass so a pass can rewrite its rows in
    // slot order as record indices (-1: empty row -> zeros) once every thread of the pass has ranked
    const int32_t RP = (int32_t)blockDim.x / NB, rows2 = ne * N;
    for (int32_t r0 = 0; r0 < rows2; r0 += RP) {
        const int32_t lr = r0 + tid / NB, kb = tid % NB;
        const bool act = tid < RP * NB && lr < rows2;
        int32_t rank[4] = {0, 1, 2, 3}, c = 0;
        uint32_t d[4] = {0, 0, 0, 0};
        if (act) {
            c = c2[lr];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t v = 4 * kb + w < N ? d2[lr * N + 4 * kb + w] : 0xFFFFFFFFu;
                d[w] = keyed ? v >> 6 : v;
            }
            khop_ranks<keyed>(N, d2, lr, kb, d, c, rank);
        }
        __syncthreads();
        if (act) {
            const int32_t o = o2[lr];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const int32_t k = 4 * kb + w;
                if (k < N) d2[lr * N + (c > 0 ? rank[w] : k)] = c > 0 ? (uint32_t)(o + (int32_t)d[w]) : 0xFFFFFFFFu;
            }
        }
    }
    __syncthreads();
    // gathers in output order: every store instruction writes one contiguous run per array
    const int32_t tot = rows2 * N;
    for (int32_t q0 = tid; q0 < tot; q0 += 4 * (int32_t)blockDim.x) {
        Rec rc[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int32_t q = q0 + k * (int32_t)blockDim.x;
            const int32_t ix = q < tot ? (int32_t)d2[q] : -1;
            rc[k] = ix >= 0 ? g.rec[ix] : Rec{0, 0, 0.f, 0};
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int32_t q = q0 + k * (int32_t)blockDim.x;
            if (q >= tot) break;
            gon[base2 + q] = rc[k].ngh;
            goe[base2 + q] = rc[k].eid;
            got[base2 + q] = rc[k].ts;
        }
    }
}

__global__ void __launch_bounds__(256) walks_kernel(DevGraph g, Key key, int32_t N, int32_t M, int64_t n_walks,
                                                    const int32_t *__restrict__ root, const int32_t *__restrict__ h1n,
                                                    const int32_t *__restrict__ h1e, const float *__restrict__ h1t,
                                                    const uint32_t *__restrict__ event_ids, int32_t *__restrict__ node6,
                                                    int32_t *__restrict__ eid3, float *__restrict__ ts3,
                                                    int32_t *__restrict__ anony3, int32_t *__restrict__ cat) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_walks) return;
    const int32_t W = N * M;
    const int64_t b = i / W;
    const int32_t w = (int32_t)(i % W), j = w / M, m = w % M;
    const uint32_t ev = event_ids[b];
    const int32_t u = root[b], v1 = h1n[b * N + j], e1 = h1e[b * N + j];
    const float t1 = h1t[b * N + j];
    const Step2 s2 = next_step(g, key, ev, j, M, m, u, v1, step2_cuts(g, u, v1, e1));
    const Step3 s3 = final_step(g, key, ev, w, u, v1, s2.src, s2.ngh, s2.eid, s2.pos, s2.rank);
    int32_t *nd = node6 + i * 6;
    nd[0] = s3.src; nd[1] = s3.ngh; nd[2] = s2.src; nd[3] = s2.ngh; nd[4] = u; nd[5] = v1;
    eid3[i * 3 + 0] = s3.eid; eid3[i * 3 + 1] = s2.eid; eid3[i * 3 + 2] = e1;
    ts3[i * 3 + 0] = s3.ts; ts3[i * 3 + 1] = s2.ts; ts3[i * 3 + 2] = t1;
    if (anony3) {
        anony3[i * 3 + 0] = 1; anony3[i * 3 + 1] = s3.code; anony3[i * 3 + 2] = s3.t;
    }
    if (cat) cat[i] = cat_of(s3.code, s3.t, 0);
}

__global__ void neg_kernel(Key key, const int32_t *__restrict__ list, uint32_t n_list,
                           const uint32_t *__restrict__ event_ids, int32_t n, uint32_t j, int32_t *__restrict__ out) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = list[draw(key, TM_STAGE_NEG, event_ids[i], 0, j, n_list)];
}

// one Philox word per position: sort keys of the keyed permutation (utils/null_model.py:23)
__global__ void perm_keys_kernel(Key key, int64_t n, uint32_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = philox_word((uint32_t)i, key.tagbase | TM_STAGE_PERM, 0, 0, key.k0, key.k1, 0);
}

__global__ void __launch_bounds__(256) hist_kernel(const int32_t *__restrict__ anony3, int64_t n, int null_order,
                                                   int32_t *__restrict__ cat, uint32_t *__restrict__ bins_out) {
    __shared__ unsigned int bins[12];
    if (threadIdx.x < 12) bins[threadIdx.x] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t c = cat_of(anony3[i * 3 + 1], anony3[i * 3 + 2], null_order);
        if (cat) cat[i] = c;
        if (c >= 0) atomicAdd(&bins[c], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 12) bins_out[blockIdx.x * 12 + threadIdx.x] = bins[threadIdx.x];   // hist_reduce_kernel
}

// new_edge_info for one group of W walks (eids staged in LDS): thread w counts, for each of its
// 3 ids, the walks holding that id in column q.  Every thread reads the same walk w2 at a time
// (LDS broadcast), so a walk costs 3 reads and 9 compares instead of 9 reads per (w, p).
__device__ __forceinline__ void edge_counts_group(const int32_t *e_lds, int32_t W, float *out) {
    for (int32_t w0 = 0; w0 < W; w0 += blockDim.x) {
        const int32_t w = w0 + threadIdx.x;
        int32_t x[3], c[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
        for (int p = 0; p < 3; ++p) x[p] = w < W ? e_lds[w * 3 + p] : 0;
#pragma unroll 4
        for (int32_t w2 = 0; w2 < W; ++w2) {
            const int32_t y0 = e_lds[w2 * 3 + 0], y1 = e_lds[w2 * 3 + 1], y2 = e_lds[w2 * 3 + 2];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                c[p][0] += x[p] == y0;
                c[p][1] += x[p] == y1;
                c[p][2] += x[p] == y2;
            }
        }
        if (w < W)
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int q = 0; q < 3; ++q) out[(w * 3 + p) * 3 + q] = (float)c[p][q];
    }
}

__global__ void __launch_bounds__(256) edge_counts_kernel(const int32_t *__restrict__ eid3, int32_t W,
                                                          float *__restrict__ out) {
    extern __shared__ int32_t e_lds[];
    const int64_t base = (int64_t)blockIdx.x * W * 3;
    for (int32_t i = threadIdx.x; i < W * 3; i += blockDim.x) e_lds[i] = eid3[base + i];
    __syncthreads();
    edge_counts_group(e_lds, W, out + base * 3);
}

// ------------------------------------------------------------------ fused per-(event, side) sampler
// One wave per (event, side): hop 1 -> hop 2 -> step 2 -> step 3 -> category -> edge counts,
// intermediates in LDS sized to N and M.  The walk steps are chains of dependent L2 lookups (cut
// lengths, pair-index binary searches, record gathers), so the kernel is latency-bound: a single-wave
// workgroup with ~3 KB of LDS (N=20) lets 32 (event, side)s run per CU, where a 256-thread workgroup
// with N=64-sized arrays allowed 6 and left 3 of its 4 waves idle in the walk phase.  Side 0/1: root = src/dst, e_idx path (data_preprocess.py:114,
// :118); side 2: root = negative dst, time path (:122).
struct EventArgs {
    DevGraph g;
    uint64_t seed;
    uint32_t split;
    int32_t N, M, E;
    const int32_t *src, *dst, *eidx;
    const double *ts;
    const uint32_t *event_ids;
    const int32_t *dst_list;
    uint32_t n_dst;
    int32_t *dst_fake;
    int32_t *sub1_node, *sub1_eid;
    float *sub1_ts;
    int32_t *sub2_node, *sub2_eid;
    float *sub2_ts;
    int32_t *node6, *eid3;
    float *ts3;
    int32_t *cat;
    float *cnt;
    unsigned long long *hist;
    uint32_t *bins_out;     // [3 * E][12] per-(event, side) motif bins, reduced by hist_reduce_kernel
    int32_t *err;
};

// hist[k] += sum over the n_groups rows of bins[row][k].  252 threads (21 per category) stride over
// the flat array by a multiple of 12, so each thread always sums one category; one atomic per
// category per workgroup.
constexpr int kReduceThreads = 252;

__global__ void __launch_bounds__(kReduceThreads) hist_reduce_kernel(const uint32_t *__restrict__ bins,
                                                                     int64_t n_groups,
                                                                     unsigned long long *__restrict__ hist) {
    __shared__ unsigned long long red[kReduceThreads];
    unsigned long long acc = 0;
    const int64_t n = n_groups * 12;
    for (int64_t i = (int64_t)blockIdx.x * kReduceThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kReduceThreads)
        acc += bins[i];
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < 12) {
        unsigned long long t = 0;
        for (int j = threadIdx.x; j < kReduceThreads; j += 12) t += red[j];
        if (t) atomicAdd(&hist[threadIdx.x], t);
    }
}

static inline unsigned reduce_blocks(int64_t n_groups) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(64, (n_groups * 12 + 4095) / 4096));
}

// new_edge_info's counts through an LDS hash table (one wave per group): the distinct edge ids of a
// group are at most N (hop-1 column) + 2W, so a table of >= 1.75x that many slots keeps linear probing
// short.  Each slot holds the id and its three per-column counts packed 10 bits each (W <= 512).
__host__ __device__ inline int32_t ecnt_slots(int32_t N, int32_t W) {
    int32_t s = 64;
    while (s * 4 < 7 * (N + 2 * W)) s *= 2;
    return s;
}
__device__ __forceinline__ uint32_t ecnt_hash(int32_t x, uint32_t mask) { return ((uint32_t)x * 2654435761u >> 7) & mask; }

// count column q of id x (ids >= 0; empty slot = -1)
__device__ __forceinline__ void ecnt_insert(int32_t *keys, uint32_t *cnts, uint32_t mask, int32_t x, int q) {
    uint32_t h = ecnt_hash(x, mask);
    while (true) {
        const int32_t prev = atomicCAS(&keys[h], -1, x);
        if (prev == -1 || prev == x) break;
        h = (h + 1) & mask;
    }
    atomicAdd(&cnts[h], 1u << (10 * q));
}
__device__ __forceinline__ uint32_t ecnt_lookup(const int32_t *keys, const uint32_t *cnts, uint32_t mask, int32_t x) {
    uint32_t h = ecnt_hash(x, mask);
    while (keys[h] != x) h = (h + 1) & mask;
    return cnts[h];
}

// LDS of one (event, side): hop-1 row, hop-2 draws (reused as the edge-count table once hop 2 is
// done), hop-2 cut lengths, walk edge ids, histogram, step-2 cuts, hop-2 record indices in slot order
__host__ __device__ inline size_t events_d2_bytes(int32_t N, int32_t M) {
    const size_t d2 = sizeof(uint32_t) * (size_t)N * N, tab = sizeof(int32_t) * 2 * (size_t)ecnt_slots(N, N * M);
    return d2 > tab ? d2 : tab;
}
__host__ __device__ inline size_t events_lds_bytes(int32_t N, int32_t M) {
    return sizeof(int32_t) * ((size_t)3 * N + 2 * N + (size_t)N * M * 3 + 12) + events_d2_bytes(N, M) +
           sizeof(Step2Cuts) * (size_t)N + sizeof(int32_t) * (size_t)N * N;
}

// Phase timing (debug builds only, -DTM_STAMPS): s_memtime deltas of lane 0 for events 2000..3999
#ifdef TM_STAMPS
__device__ unsigned long long g_est[16];
#define TM_EST(k)                                   \
    do {                                            \
        __builtin_amdgcn_sched_barrier(0);          \
        T[k] = __builtin_amdgcn_s_memtime();        \
        __builtin_amdgcn_sched_barrier(0);          \
    } while (0)
#else
#define TM_EST(k) (void)T
#endif

// NC > 0: n_degree is the compile-time constant NC (the reference's default 20): the row / column splits of
// the draw and rank loops are constant divisions and their trip counts known (SQ_INSTS_VALU per wave, see
// profiles/r06_pmc_events_summary.json); NC = 0: any N <= kMaxN.  MC > 0 likewise fixes M.
template <bool keyed, int MC, int NC = 0>
__global__ void __launch_bounds__(64) events_kernel(EventArgs a) {
    unsigned long long T[12];
    TM_EST(0);
    extern __shared__ int32_t ev_lds[];
    const int32_t N = NC > 0 ? NC : a.N, M = MC > 0 ? MC : a.M, W = N * M;
    int32_t *h1n = ev_lds, *h1e = h1n + N;
    float *h1t = reinterpret_cast<float *>(h1e + N);
    uint32_t *d2 = reinterpret_cast<uint32_t *>(h1e + 2 * N);
    int32_t *c2 = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(d2) + events_d2_bytes(N, M)), *o2 = c2 + N,
            *weid = o2 + N;
    unsigned int *bins = reinterpret_cast<unsigned int *>(weid + W * 3);
    Step2Cuts *s2c = reinterpret_cast<Step2Cuts *>(bins + 12);
    int32_t *sidx = reinterpret_cast<int32_t *>(s2c + N);
    const DevGraph &g = a.g;
    // output pointers live in VGPRs (vptr): kept as uniform SGPR pairs next to the graph and input
    // pointers they overflow the scalar file and spill through v_readlane in every phase
    // (global address space: TM_OUTP)
    const auto o_dst_fake = TM_OUTP(a.dst_fake), o_sub1_node = TM_OUTP(a.sub1_node), o_sub1_eid = TM_OUTP(a.sub1_eid),
               o_sub2_node = TM_OUTP(a.sub2_node), o_sub2_eid = TM_OUTP(a.sub2_eid), o_node6 = TM_OUTP(a.node6),
               o_eid3 = TM_OUTP(a.eid3), o_cat = TM_OUTP(a.cat);
    const auto o_sub1_ts = TM_OUTP(a.sub1_ts), o_sub2_ts = TM_OUTP(a.sub2_ts), o_ts3 = TM_OUTP(a.ts3),
               o_cnt = TM_OUTP(a.cnt);
    const auto o_bins = TM_OUTP(a.bins_out);
    const int32_t e = blockIdx.x, s = blockIdx.y, tid = threadIdx.x;
    const uint32_t ev = a.event_ids[e];
    const Key key = make_key(a.seed, a.split, (uint32_t)(s + 1));
    if (tid < 12) bins[tid] = 0;
    // ---- root
    int32_t u;
    if (s == 0) u = a.src[e];
    else if (s == 1) u = a.dst[e];
    else u = a.dst_list[draw(make_key(a.seed, a.split, TM_SIDE_NONE), TM_STAGE_NEG, ev, 0, 1, a.n_dst)];
    if (s == 2 && tid == 0) o_dst_fake[e] = u;
    const int64_t se = (int64_t)s * a.E + e;
    // ---- hop 1 (one row, N draws), lanes of wave 0
    if (tid < 64) {
        int32_t c;
        if (s == 2 && u >= 0 && u < g.n_nodes) c = bisect_ts_wave(g, u, a.ts[e]);   // time path, whole wave
        else c = find_before_len(g, u, s == 2, a.ts[e], a.eidx ? a.eidx[e] : 0, tid == 0 ? a.err : nullptr);
        uint32_t d = 0xFFFFFFFFu;
        if (c > 0 && tid < N) d = (uint32_t)draw(key, 1, ev, 0, tid, c);
        // rank among the row's N draws (np.sort order, ties by index): lane k's draw read into a scalar
        // register (v_readlane, k is wave-uniform) instead of a ds_bpermute round trip per k
        const uint32_t dkey = keyed ? (d << 6) | (uint32_t)tid : d;   // unique keys: one compare
        int32_t rank = 0;
        for (int k = 0; k < N; ++k) {
            const uint32_t dk = (uint32_t)__builtin_amdgcn_readlane((int)dkey, k);
            rank += keyed ? (dk < dkey) : ((dk < d) || (k < tid && dk == d));
        }
        if (tid < N) {
            int32_t n_ = 0, e_ = 0;
            float t_ = 0.f;
            int32_t slot = tid;
            if (c > 0) {
                const Rec rc = g.rec[g.off[u] + (int32_t)d];
                n_ = rc.ngh; e_ = rc.eid; t_ = rc.ts; slot = rank;
            }
            h1n[slot] = n_; h1e[slot] = e_; h1t[slot] = t_;
            TM_ST(o_sub1_node[se * N + slot], n_);
            TM_ST(o_sub1_eid[se * N + slot], e_);
            TM_ST(o_sub1_ts[se * N + slot], t_);
        }
    }
    __syncthreads();
    TM_EST(1);
    // ---- hop 2 (N rows x N draws; e_idx path, graph.py:247-250)
    if (tid < N) {
        c2[tid] = find_before_len(g, h1n[tid], false, 0.0, h1e[tid], a.err);
        const int32_t v = h1n[tid];
        o2[tid] = (v >= 0 && v < g.n_nodes) ? g.off[v] : 0;   // record offset of the hop-2 row's node
        s2c[tid] = step2_cuts(g, u, v, h1e[tid]);            // step 2 of the slot's M walks
    }
    __syncthreads();
    TM_EST(2);
    // one Philox block per 4 draws of a row
    const int32_t NB = (N + 3) >> 2;
    for (int32_t x = tid; x < N * NB; x += blockDim.x) {
        const int32_t j = x / NB, kb = x % NB, c = c2[j];
        const uint4 b = draw_block(key, 2, ev, j, kb);
        const uint32_t wv[4] = {b.x, b.y, b.z, b.w};
        uint32_t o4[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int32_t k = 4 * kb + w;
            // keyed: (draw << 6 | index), unique, so the np.sort rank is one compare (see khop2_kernel)
            const uint32_t dv = (uint32_t)scale_draw(wv[w], c);
            o4[w] = c > 0 ? (keyed ? (dv << 6) | (uint32_t)k : dv) : 0xFFFFFFFFu;
        }
        if ((N & 3) == 0) {          // one 16-B store per lane (4-B stores at a 16-B lane stride: 4-way bank conflicts)
            *reinterpret_cast<uint4 *>(d2 + j * N + 4 * kb) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
        } else {
#pragma unroll
            for (int w = 0; w < 4; ++w)
                if (4 * kb + w < N) d2[j * N + 4 * kb + w] = o4[w];
        }
    }
    __syncthreads();
    // ranks (np.sort order) of 4 rows' draws per lane per round into slot order: sidx[row * N + rank] =
    // record index (-1: empty row -> zeros)
    constexpr int HB = 4;
    for (int32_t x0 = 0; x0 < N * N; x0 += HB * 64) {
        int32_t jr[HB], kr[HB], rank[HB];
        uint32_t dr[HB];
#pragma unroll
        for (int u = 0; u < HB; ++u) {
            const int32_t x = x0 + u * 64 + tid;
            jr[u] = x < N * N ? x / N : 0;
            kr[u] = x % N;
            dr[u] = x < N * N ? d2[x] : 0u;
            rank[u] = 0;
        }
        if (NC > 0 && (NC & 3) == 0) {
            // rows of a multiple of 4 draws are 16-B aligned: 4 columns per b128 read, one read per row in flight
            // (unrolling the column loop spends VGPRs the kernel's occupancy needs)
#pragma unroll 1
            for (int32_t i = 0; i < N; i += 4)
#pragma unroll
                for (int u = 0; u < HB; ++u) {
                    const uint4 q = *reinterpret_cast<const uint4 *>(d2 + jr[u] * N + i);
                    const uint32_t dq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        if (keyed) rank[u] += dq[t] < dr[u];
                        else rank[u] += (dq[t] < dr[u]) || (i + t < kr[u] && dq[t] == dr[u]);
                    }
                }
        } else {
            // the 4 rows' comparisons interleaved, 4 columns per iteration: 16 LDS reads in flight
#pragma unroll 4
            for (int32_t i = 0; i < N; ++i)
#pragma unroll
                for (int u = 0; u < HB; ++u) {
                    const uint32_t di = d2[jr[u] * N + i];
                    if (keyed) rank[u] += di < dr[u];
                    else rank[u] += (di < dr[u]) || (i < kr[u] && di == dr[u]);
                }
        }
#pragma unroll
        for (int u = 0; u < HB; ++u) {
            const int32_t x = x0 + u * 64 + tid;
            if (x >= N * N) continue;
            const int32_t c = c2[jr[u]];
            const bool ok = c > 0 && g.n_entries > 0;
            sidx[c > 0 ? jr[u] * N + rank[u] : x] = ok ? o2[jr[u]] + (int32_t)(keyed ? dr[u] >> 6 : dr[u]) : -1;
        }
    }
    __syncthreads();
    // gathers in output order, 4 in flight per lane: each store instruction writes one contiguous run per
    // array (stores scattered inside the rows cost the k-hop kernel a third of its time)
    for (int32_t q0 = tid; q0 < N * N; q0 += 4 * 64) {
        Rec rc[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int32_t q = q0 + 64 * k;
            const int32_t ix = q < N * N ? sidx[q] : -1;
            rc[k] = ix >= 0 ? g.rec[ix] : Rec{0, 0, 0.f, 0};
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int32_t q = q0 + 64 * k;
            if (q >= N * N) break;
            const int64_t o = se * N * N + q;
            o_sub2_node[o] = rc[k].ngh;
            o_sub2_eid[o] = rc[k].eid;
            o_sub2_ts[o] = rc[k].ts;
        }
    }
    TM_EST(3);
    // hop 2 is done with the draws: their LDS becomes the edge-count table
    const uint32_t tmask = (uint32_t)ecnt_slots(N, W) - 1;
    int32_t *tkeys = reinterpret_cast<int32_t *>(d2);
    uint32_t *tcnt = reinterpret_cast<uint32_t *>(tkeys + tmask + 1);
    __syncthreads();
    for (int32_t i = tid; i <= (int32_t)tmask; i += blockDim.x) {
        tkeys[i] = -1;
        tcnt[i] = 0;
    }
    __syncthreads();
    // ---- steps 2 + 3, one thread per walk; each walk's three ids counted into the table
    for (int32_t w = tid; w < W; w += blockDim.x) {
        const int32_t j = w / M, m = w % M;
        const int32_t v1 = h1n[j], e1 = h1e[j];
        const Step2 s2 = next_step<MC>(g, key, ev, j, M, m, u, v1, s2c[j]);
        TM_EST(6);
#ifdef TM_STAMPS
        const Step3 s3 = final_step(g, key, ev, w, u, v1, s2.src, s2.ngh, s2.eid, s2.pos, s2.rank, T);
#else
        const Step3 s3 = final_step(g, key, ev, w, u, v1, s2.src, s2.ngh, s2.eid, s2.pos, s2.rank);
#endif
        TM_EST(7);
        const int64_t o = se * W + w;
        const auto nd = o_node6 + o * 6;
        // per-lane row stores (24 / 12 B per walk); staging them in LDS for contiguous runs measured
        // slower (0.170 -> 0.178 ms: the extra LDS costs resident workgroups)
        TM_ST(nd[0], s3.src); TM_ST(nd[1], s3.ngh); TM_ST(nd[2], s2.src); TM_ST(nd[3], s2.ngh); TM_ST(nd[4], u); TM_ST(nd[5], v1);
        TM_ST(o_eid3[o * 3 + 0], s3.eid); TM_ST(o_eid3[o * 3 + 1], s2.eid); TM_ST(o_eid3[o * 3 + 2], e1);
        TM_ST(o_ts3[o * 3 + 0], s3.ts); TM_ST(o_ts3[o * 3 + 1], s2.ts); TM_ST(o_ts3[o * 3 + 2], h1t[j]);
        const int32_t c = cat_of(s3.code, s3.t, 0);
        TM_ST(o_cat[o], c);
        {   // histogram by wave ballots: one lane adds each category's count (LDS atomics from 60 lanes into
            // 12 words serialised on bank conflicts)
            const int lead = __ffsll((unsigned long long)__ballot(1)) - 1;
#pragma unroll
            for (int k = 0; k < 12; ++k) {
                const int nk = __popcll(__ballot(c == k));
                if (tid == lead && nk) bins[k] += (unsigned)nk;
            }
        }
        // walk ids column-major (p * W + w): 4-B lane stride, conflict-free
        weid[w] = s3.eid; weid[W + w] = s2.eid; weid[2 * W + w] = e1;
        ecnt_insert(tkeys, tcnt, tmask, s3.eid, 0);
        ecnt_insert(tkeys, tcnt, tmask, s2.eid, 1);
        ecnt_insert(tkeys, tcnt, tmask, e1, 2);
    }
    __syncthreads();
    TM_EST(4);
    // new_edge_info (data_preprocess.py:327-343): count of walk w's id p in column q
    const auto oc = o_cnt + se * W * 9;
    for (int32_t w = tid; w < W; w += blockDim.x) {
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const uint32_t c = ecnt_lookup(tkeys, tcnt, tmask, weid[p * W + w]);
#pragma unroll
            for (int q = 0; q < 3; ++q) TM_ST(oc[(w * 3 + p) * 3 + q], (float)((c >> (10 * q)) & 1023u));
        }
    }
    TM_EST(5);
#ifdef TM_STAMPS
    if (tid == 0 && e >= 2000 && e < 4000) {
        for (int k = 0; k < 5; ++k) atomicAdd(&g_est[k], T[k + 1] - T[k]);
        // inside steps 2 + 3: next_step (from the hop-2 end, incl. the table clear), final_step's loads, its
        // filtered counts, its draw + k-th selection, its record load, then stores / histogram / table inserts
        atomicAdd(&g_est[5], T[6] - T[3]);
        atomicAdd(&g_est[6], T[8] - T[6]);
        atomicAdd(&g_est[8], T[9] - T[8]);
        atomicAdd(&g_est[9], T[10] - T[9]);
        atomicAdd(&g_est[10], T[11] - T[10]);
        atomicAdd(&g_est[11], T[7] - T[11]);
        atomicAdd(&g_est[12], T[4] - T[7]);
        atomicAdd(&g_est[15], 1ull);
    }
#endif
    // per-(event, side) bins, summed by hist_reduce_kernel: 12 same-address device-scope atomics from
    // each of the 3E workgroups serialized on one line and cost the kernel 40 % of its time
    if (tid < 12) o_bins[se * 12 + tid] = bins[tid];
}

}  // namespace tmk

using namespace tmk;

static inline hipStream_t S(void *s) { return (hipStream_t)s; }

// keyed one-compare ranks need draw << 6 to fit 32 bits: draws are < n_entries.  tm_debug_set(
// TM_DEBUG_FORCE_UNKEYED, 1) (tests) selects the two-compare kernels on any graph.
static inline bool use_keyed(const tm_graph *g) {
    return g->d.n_entries < ((int64_t)1 << 26) && !debug_opt(TM_DEBUG_FORCE_UNKEYED);
}

extern "C" int tm_sample_khop(const tm_graph *g, tm_rng rng, int32_t k, int32_t N, int32_t B, const int32_t *root,
                              const double *cut, const int32_t *eidx, const uint32_t *event_ids, int32_t *out_node,
                              int32_t *out_eid, float *out_ts, int32_t *err_flag, void *stream) {
    if (!g || k < 0 || B < 0 || N <= 0) return fail(TM_E_ARG, "tm_sample_khop: bad arguments");
    if (N > kMaxN) return fail(TM_E_UNSUPPORTED, "tm_sample_khop: num_neighbors > 64");
    if (k == 0 || B == 0) return TM_OK;
    if (!root || !event_ids || !out_node || !out_eid || !out_ts || (!eidx && !cut))
        return fail(TM_E_ARG, "tm_sample_khop: NULL pointer");
    const Key key = make_key(rng.seed, rng.split, rng.side);
    hipEvent_t pe = prof_begin(S(stream));
    if (k == 2) {
        const int32_t epb = khop2_epb(N);
        // a draw is < its row's cut <= n_entries: below 2^26 it packs with its index into one sort key
        const dim3 grid((unsigned)((B + epb - 1) / epb));
        if (use_keyed(g))
            khop2_kernel<true><<<grid, 256, khop2_lds_bytes(N), S(stream)>>>(g->d, key, N, B, root, cut, eidx, event_ids,
                                                                              out_node, out_eid, out_ts, err_flag);
        else
            khop2_kernel<false><<<grid, 256, khop2_lds_bytes(N), S(stream)>>>(g->d, key, N, B, root, cut, eidx,
                                                                               event_ids, out_node, out_eid, out_ts,
                                                                               err_flag);
        TM_CHECK_LAUNCH();
        prof_end("khop_kernel", S(stream), pe);
        return TM_OK;
    }
    int64_t rows = B, rpe = 1, off = 0;
    const int32_t *rn = root, *re = eidx;
    for (int32_t h = 1; h <= k; ++h) {
        const bool tp = (h == 1 && eidx == nullptr);
        int32_t *on = out_node + off, *oe = out_eid + off;
        float *ot = out_ts + off;
        const int32_t NB = (N + 3) / 4, R = 256 / NB;
        const dim3 grid((unsigned)((rows + R - 1) / R));
        const size_t lds = sizeof(uint32_t) * ((size_t)2 * R + (size_t)R * N);
        khop_kernel<<<grid, 256, lds, S(stream)>>>(g->d, key, (uint32_t)h, N, rows, rpe, rn, cut, re, tp ? 1 : 0,
                                                   event_ids, on, oe, ot, err_flag);
        TM_CHECK_LAUNCH();
        rn = on;
        re = oe;
        off += rows * N;
        rows *= N;
        rpe *= N;
        if (rows > ((int64_t)1 << 40)) return fail(TM_E_UNSUPPORTED, "tm_sample_khop: too many rows");
    }
    prof_end("khop_kernel", S(stream), pe);   // all hops of one call
    return TM_OK;
}

extern "C" int tm_sample_walks(const tm_graph *g, tm_rng rng, int32_t N, int32_t M, int32_t B, const int32_t *root,
                               const int32_t *h1_node, const int32_t *h1_eid, const float *h1_ts,
                               const uint32_t *event_ids, int32_t *out_node6, int32_t *out_eid3, float *out_ts3,
                               int32_t *out_anony3, int32_t *out_cat, void *stream) {
    if (!g || N <= 0 || M <= 0 || B < 0) return fail(TM_E_ARG, "tm_sample_walks: bad arguments");
    if (M > kMaxM) return fail(TM_E_UNSUPPORTED, "tm_sample_walks: num_neighbors (walks per slot) > 8");
    if (B == 0) return TM_OK;
    if (!root || !h1_node || !h1_eid || !h1_ts || !event_ids || !out_node6 || !out_eid3 || !out_ts3)
        return fail(TM_E_ARG, "tm_sample_walks: NULL pointer");
    const int64_t n = (int64_t)B * N * M;
    walks_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, S(stream)>>>(
        g->d, make_key(rng.seed, rng.split, rng.side), N, M, n, root, h1_node, h1_eid, h1_ts, event_ids, out_node6,
        out_eid3, out_ts3, out_anony3, out_cat);
    TM_CHECK_LAUNCH();
    return TM_OK;
}

extern "C" int tm_neg_sample(tm_rng rng, const int32_t *list, int64_t n_list, const uint32_t *event_ids, int32_t n,
                             int32_t j, int32_t *out, void *stream) {
    if (n < 0 || n_list <= 0 || n_list > UINT32_MAX || j < 0) return fail(TM_E_ARG, "tm_neg_sample: bad arguments");
    if (n == 0) return TM_OK;
    if (!list || !event_ids || !out) return fail(TM_E_ARG, "tm_neg_sample: NULL pointer");
    neg_kernel<<<dim3((n + 255) / 256), 256, 0, S(stream)>>>(make_key(rng.seed, rng.split, TM_SIDE_NONE), list,
                                                             (uint32_t)n_list, event_ids, n, (uint32_t)j, out);
    TM_CHECK_LAUNCH();
    return TM_OK;
}

extern "C" int tm_perm_keys(uint64_t seed, uint32_t split, int64_t n, uint32_t *out_keys, void *stream) {
    if (n < 0) return fail(TM_E_ARG, "tm_perm_keys: bad arguments");
    if (n == 0) return TM_OK;
    if (!out_keys) return fail(TM_E_ARG, "tm_perm_keys: NULL pointer");
    perm_keys_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, S(stream)>>>(make_key(seed, split, TM_SIDE_NONE), n,
                                                                             out_keys);
    TM_CHECK_LAUNCH();
    return TM_OK;
}

extern "C" int tm_motif_hist(const int32_t *anony3, int64_t n, int32_t null_order, int32_t *out_cat,
                             unsigned long long *hist12, void *stream) {
    if (n < 0 || !hist12) return fail(TM_E_ARG, "tm_motif_hist: bad arguments");
    if (n == 0) return TM_OK;
    if (!anony3) return fail(TM_E_ARG, "tm_motif_hist: NULL anony");
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 2048);
    uint32_t *bins = static_cast<uint32_t *>(scratch(sizeof(uint32_t) * 12 * (size_t)blocks, S(stream)));
    if (!bins) return fail(TM_E_HIP, "tm_motif_hist: scratch allocation failed");
    hist_kernel<<<dim3((unsigned)blocks), 256, 0, S(stream)>>>(anony3, n, null_order, out_cat, bins);
    TM_CHECK_LAUNCH();
    hist_reduce_kernel<<<dim3(reduce_blocks(blocks)), kReduceThreads, 0, S(stream)>>>(bins, blocks, hist12);
    TM_CHECK_LAUNCH();
    return TM_OK;
}

extern "C" int tm_edge_counts(const int32_t *eid3, int32_t n_groups, int32_t W, float *out_cnt, void *stream) {
    if (n_groups < 0 || W <= 0 || W > 8192) return fail(TM_E_ARG, "tm_edge_counts: bad arguments");
    if (n_groups == 0) return TM_OK;
    if (!eid3 || !out_cnt) return fail(TM_E_ARG, "tm_edge_counts: NULL pointer");
    edge_counts_kernel<<<dim3(n_groups), 256, sizeof(int32_t) * W * 3, S(stream)>>>(eid3, W, out_cnt);
    TM_CHECK_LAUNCH();
    return TM_OK;
}

extern "C" int tm_sample_events(const tm_graph *g, uint64_t seed, uint32_t split, int32_t N, int32_t M,
                                int32_t n_events, const int32_t *src, const int32_t *dst, const double *ts,
                                const int32_t *eidx, const uint32_t *event_ids, const int32_t *dst_list,
                                int64_t n_dst, int32_t *dst_fake, int32_t *sub1_node, int32_t *sub1_eid,
                                float *sub1_ts, int32_t *sub2_node, int32_t *sub2_eid, float *sub2_ts,
                                int32_t *node6, int32_t *eid3, float *ts3, int32_t *cat, float *cnt,
                                unsigned long long *hist12, int32_t *err_flag, void *stream) {
    if (!g || N <= 0 || M <= 0 || n_events < 0 || n_dst <= 0 || n_dst > UINT32_MAX)
        return fail(TM_E_ARG, "tm_sample_events: bad arguments");
    if (N > kMaxN || M > kMaxM) return fail(TM_E_UNSUPPORTED, "tm_sample_events: N > 64 or M > 8");
    if (n_events == 0) return TM_OK;
    if (n_events > 65535 * 1024) return fail(TM_E_UNSUPPORTED, "tm_sample_events: too many events per launch");
    if (!src || !dst || !ts || !eidx || !event_ids || !dst_list || !dst_fake || !sub1_node || !sub1_eid ||
        !sub1_ts || !sub2_node || !sub2_eid || !sub2_ts || !node6 || !eid3 || !ts3 || !cat || !cnt || !hist12)
        return fail(TM_E_ARG, "tm_sample_events: NULL pointer");
    uint32_t *bins = static_cast<uint32_t *>(scratch(sizeof(uint32_t) * 12 * 3 * (size_t)n_events, S(stream)));
    if (!bins) return fail(TM_E_HIP, "tm_sample_events: scratch allocation failed");
    EventArgs a{g->d,     seed,     split,     N,         M,        n_events, src,  dst,   eidx, ts,     event_ids,
                dst_list, (uint32_t)n_dst, dst_fake, sub1_node, sub1_eid, sub1_ts, sub2_node, sub2_eid, sub2_ts,
                node6,    eid3,     ts3,       cat,       cnt,      hist12,   bins,     err_flag};
    hipEvent_t pe = prof_begin(S(stream));
    const size_t lds = events_lds_bytes(N, M);
    const dim3 grid(n_events, 3);
    const bool kd = use_keyed(g);
    if (M == 3 && N == 20) {
        if (kd) events_kernel<true, 3, 20><<<grid, 64, lds, S(stream)>>>(a);
        else events_kernel<false, 3, 20><<<grid, 64, lds, S(stream)>>>(a);
    } else if (M == 1 && N == 20) {
        if (kd) events_kernel<true, 1, 20><<<grid, 64, lds, S(stream)>>>(a);
        else events_kernel<false, 1, 20><<<grid, 64, lds, S(stream)>>>(a);
    } else if (M == 3) {
        if (kd) events_kernel<true, 3><<<grid, 64, lds, S(stream)>>>(a);
        else events_kernel<false, 3><<<grid, 64, lds, S(stream)>>>(a);
    } else if (M == 1) {
        if (kd) events_kernel<true, 1><<<grid, 64, lds, S(stream)>>>(a);
        else events_kernel<false, 1><<<grid, 64, lds, S(stream)>>>(a);
    } else {
        if (kd) events_kernel<true, 0><<<grid, 64, lds, S(stream)>>>(a);
        else events_kernel<false, 0><<<grid, 64, lds, S(stream)>>>(a);
    }
    TM_CHECK_LAUNCH();
    prof_end("events_kernel", S(stream), pe);
    pe = prof_begin(S(stream));
    hist_reduce_kernel<<<dim3(reduce_blocks(3 * (int64_t)n_events)), kReduceThreads, 0, S(stream)>>>(
        bins, 3 * (int64_t)n_events, hist12);
    TM_CHECK_LAUNCH();
    prof_end("hist_reduce_kernel", S(stream), pe);
    return TM_OK;
}

#ifdef TM_STAMPS
extern "C" int tm_debug_event_stamps(unsigned long long *host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(tmk::g_est), sizeof(unsigned long long) * 16, 0,
                                    hipMemcpyDeviceToHost);
}
#endif
