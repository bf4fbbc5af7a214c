// Temporal CSR build on the device from raw edge rows (utils/graph.py:13-101 and the
// adj_list construction of temp_exp_main.py:135-144).  tm_graph_build_edges runs this path; the
// adjacency-list entry (tm_graph_build) keeps the host builder (graph.cpp).
//
//   entries     row i -> entries 2i = (src; dst, e, t) and 2i+1 = (dst; src, e, t): the reference's
//               append order (src's list first, a self-loop twice in its node's list)
//   per node    stable radix sorts (rocPRIM) by the ts key, then by the owner: each node's list in
//               ts order with ties in append order == Python's stable sorted() (graph.py:48)
//   get_ts2idx  per entry: tie group [g0, g1) from a max-scan of group heads; a finished group's j-th
//               member ends at i - j (graph.py:93-99), the trailing group is never adjusted, and a
//               self-loop's two adjacent copies share one dict value (last index minus both copies' j)
//   e_idx table owner a = the smaller endpoint (first in node order), b = the larger
//   blocks      stable sorts by neighbour then owner give the (node, neighbour, position) order:
//               block heads, per-entry block rank, block regions (exclusive scan of their tree
//               lengths), keys, fence levels, and the (node, neighbour) hash table (64-bit CAS inserts)
// Rows whose edge id appears more than once fall back to the host builder (the device dict logic
// assumes one row per edge id).
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <vector>

#include "common.h"

namespace tmk {
namespace gdev {

constexpr int TB = 256;

inline unsigned grid(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + TB - 1) / TB, 1 << 16)); }

#define GS_LOOP(i, n) for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

// order-preserving 64-bit key of a double (-0.0 == 0.0, as Python compares them)
__device__ __forceinline__ uint64_t ts_key(double t) {
    if (t == 0.0) t = 0.0;
    const uint64_t b = (uint64_t)__double_as_longlong(t);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__global__ void k_entries(int64_t n_edges, int32_t V, int32_t max_eid, const int64_t *src, const int64_t *dst,
                          const int64_t *eidx, const double *ts, uint64_t *key, int32_t *idx, int32_t *own, int32_t *ngh,
                          int32_t *eid, double *tv, int32_t *ecount, int32_t *err) {
    GS_LOOP(i, n_edges) {
        const int64_t s = src[i], d = dst[i], e = eidx[i];
        if (s < 0 || s >= V || d < 0 || d >= V || e < 0 || e > max_eid) {
            atomicOr(err, 1);
            continue;
        }
        const uint64_t k = ts_key(ts[i]);
        const int64_t a = 2 * i, b = 2 * i + 1;
        key[a] = key[b] = k;
        idx[a] = (int32_t)a;
        idx[b] = (int32_t)b;
        own[a] = (int32_t)s;
        ngh[a] = (int32_t)d;
        own[b] = (int32_t)d;
        ngh[b] = (int32_t)s;
        eid[a] = eid[b] = (int32_t)e;
        tv[a] = tv[b] = ts[i];
        if (atomicAdd(&ecount[e], 1) > 0) atomicOr(err, 2);   // edge id on more than one row
    }
}

__global__ void k_gather_key(int64_t n, const int32_t *perm, const int32_t *src, int32_t *out) {
    GS_LOOP(k, n) out[k] = src[perm[k]];
}

__global__ void k_sorted(int64_t n, const int32_t *perm, const int32_t *own, const int32_t *ngh, const int32_t *eid,
                         const double *tv, int32_t *o_own, int32_t *o_ngh, int32_t *o_eid, double *o_ts, int32_t *cnt) {
    GS_LOOP(p, n) {
        const int32_t q = perm[p];
        o_own[p] = own[q];
        o_ngh[p] = ngh[q];
        o_eid[p] = eid[q];
        o_ts[p] = tv[q];
        atomicAdd(&cnt[own[q]], 1);
    }
}

// tie-group heads: p itself where a group starts, 0 elsewhere (max-scanned into g0)
__global__ void k_group_heads(int64_t n, const int32_t *own, const double *ts, const int32_t *off, int32_t *h) {
    GS_LOOP(p, n) {
        const bool head = p == off[own[p]] || !(ts[p] == ts[p - 1]);
        h[p] = head ? (int32_t)p : 0;
    }
}

__global__ void k_group_ends(int64_t n, const int32_t *own, const double *ts, const int32_t *off, const int32_t *g0,
                             int32_t *gend) {
    GS_LOOP(p, n) {
        const bool tail = p + 1 == off[own[p] + 1] || !(ts[p + 1] == ts[p]);
        if (tail) gend[g0[p]] = (int32_t)p + 1;
    }
}

__global__ void k_fill_ends(int64_t n, EdgeEnds *ends) {
    GS_LOOP(i, n) ends[i] = EdgeEnds{-1, 0, -1, 0};
}

// strict_temporal slice lengths: every record of the owner strictly earlier than the edge's own time
__global__ void k_strict_ends(int64_t n, DevGraph g, EdgeEnds *ends) {
    GS_LOOP(i, n) {
        EdgeEnds x = g.ends[i];
        const double t = g.ets[i];
        if (x.node_a >= 0) x.len_a = bisect_ts(g, x.node_a, t);
        if (x.node_b >= 0) x.len_b = bisect_ts(g, x.node_b, t);
        ends[i] = x;
    }
}

__global__ void k_fill_i32(int64_t n, int32_t *a, int32_t v) {
    GS_LOOP(i, n) a[i] = v;
}

__global__ void k_dict(int64_t n, const int32_t *own, const int32_t *ngh, const int32_t *eid, const double *ts,
                       const int32_t *off, const int32_t *g0, const int32_t *gend, int32_t *dict, EdgeEnds *ends, Rec *rec,
                       double *ets) {
    GS_LOOP(p, n) {
        const int32_t u = own[p], x = ngh[p], e = eid[p], s = off[u], d = off[u + 1] - s;
        const int32_t i = (int32_t)p - s, g = g0[p], j = (int32_t)p - g;
        const bool trailing = gend[g] == off[u + 1];
        int32_t v;
        if (x != u) {
            v = i - (trailing ? 0 : j);
        } else {
            // a self-loop's two copies are adjacent (consecutive appends, equal ts): both in one tie group
            const int32_t p0 = (p > s && eid[p - 1] == e && ngh[p - 1] == u) ? (int32_t)p - 1 : (int32_t)p;
            const int32_t j0 = p0 - g;
            v = (p0 + 1 - s) - (trailing ? 0 : 2 * j0 + 1);
        }
        dict[p] = v;
        const int32_t len = v < 0 ? max(0, d + v) : v;   // Python slice with a negative stop
        const int32_t a = x == u ? u : min(u, x);
        if (u == a) {
            ends[e].node_a = u;
            ends[e].len_a = len;
        } else {
            ends[e].node_b = u;
            ends[e].len_b = len;
        }
        rec[p] = Rec{x, e, (float)ts[p], 0};
        ets[e] = ts[p];
    }
}

// blocks in (owner, neighbour, position) order: k -> entry q = bperm[k]
__global__ void k_block_heads(int64_t n, const int32_t *bperm, const int32_t *own, const int32_t *ngh, int32_t *hpos,
                              int32_t *hflag) {
    GS_LOOP(k, n) {
        const int32_t q = bperm[k];
        bool head = k == 0;
        if (!head) {
            const int32_t r = bperm[k - 1];
            head = own[q] != own[r] || ngh[q] != ngh[r];
        }
        hpos[k] = head ? (int32_t)k : 0;
        hflag[k] = head ? 1 : 0;
    }
}

__global__ void k_block_info(int64_t n, const int32_t *bperm, const int32_t *own, const int32_t *ngh,
                             const int32_t *bstart, const int32_t *bincl, int32_t *bn, int32_t *bu, int32_t *bx,
                             int32_t *bs, Rec *rec) {
    GS_LOOP(k, n) {
        const int32_t q = bperm[k], b = bincl[k] - 1;
        rec[q].brank = (int32_t)k - bstart[k];
        const bool tail = k + 1 == n || bincl[k + 1] != bincl[k];
        if (tail) {
            bn[b] = (int32_t)k + 1 - bstart[k];
            bu[b] = own[q];
            bx[b] = ngh[q];
            bs[b] = bstart[k];
        }
    }
}

__global__ void k_region_len(int64_t nb, const int32_t *bn, int32_t *rl) {
    GS_LOOP(b, nb) rl[b] = blk_region_len(bn[b]);
}

__global__ void k_keys(int64_t n, const int32_t *bperm, const int32_t *own, const int32_t *off, const int32_t *bincl,
                       const int32_t *bs, const int32_t *bn, const int32_t *rbase, int32_t *ppos) {
    GS_LOOP(k, n) {
        const int32_t q = bperm[k], b = bincl[k] - 1;
        ppos[rbase[b] + blk_keys_off(bn[b]) + ((int32_t)k - bs[b])] = q - off[own[q]];
    }
}

// fence levels of the blocks with more than F keys, bottom-up: L_l[t] = L_(l-1)[F t]
__global__ void k_fences(int64_t nb, const int32_t *bn, const int32_t *rbase, int32_t *ppos) {
    GS_LOOP(b, nb) {
        const int32_t n = bn[b];
        if (n <= kBlkFan) continue;
        const int32_t h = blk_levels(n), base = rbase[b];
        int32_t lo = blk_keys_off(n);
        const int32_t *lower = ppos + base + lo;
        for (int32_t l = 1; l <= h; ++l) {
            lo -= blk_level_len(n, l, h);
            int32_t *lev = ppos + base + lo;
            const int32_t cnt = (int32_t)(((int64_t)n + ((int64_t)1 << (kBlkLog * l)) - 1) >> (kBlkLog * l));
            for (int32_t t = 0; t < cnt; ++t) lev[t] = lower[kBlkFan * t];
            lower = lev;
        }
    }
}

__global__ void k_pblk_fill(int64_t cap, PairBlk *t) {
    GS_LOOP(i, cap) t[i] = PairBlk{-1, 0, 0, 0};
}

__global__ void k_pblk_insert(int64_t nb, const int32_t *bu, const int32_t *bx, const int32_t *rbase, const int32_t *bn,
                              PairBlk *t, uint32_t mask) {
    GS_LOOP(b, nb) {
        const unsigned long long key = (unsigned long long)(uint32_t)bu[b] | (unsigned long long)(uint32_t)bx[b] << 32;
        uint32_t h = pblk_hash(bu[b], bx[b]) & mask;
        for (;;) {
            unsigned long long *slot = reinterpret_cast<unsigned long long *>(&t[h]);
            if (atomicCAS(slot, 0xFFFFFFFFull, key) == 0xFFFFFFFFull) {
                t[h].base = rbase[b];
                t[h].n = bn[b];
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

__global__ void k_span(int32_t V, const int32_t *off, int2 *span) {
    GS_LOOP(u, V) span[u] = make_int2(off[u], off[u + 1]);
}

// device scratch with its size, freed with the builder
struct Buf {
    std::vector<void *> ptrs;
    hipError_t e = hipSuccess;
    template <class T>
    T *get(int64_t n) {
        void *p = nullptr;
        if (e == hipSuccess) e = hipMalloc(&p, sizeof(T) * (size_t)std::max<int64_t>(n, 1));
        if (e == hipSuccess) ptrs.push_back(p);
        return static_cast<T *>(p);
    }
    ~Buf() {
        for (void *p : ptrs) (void)hipFree(p);
    }
};

template <class K, class VIn, class Vt>
hipError_t sort_pairs(Buf &buf, const K *kin, K *kout, VIn vin, Vt *vout, int64_t n, hipStream_t s) {
    size_t bytes = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, bytes, kin, kout, vin, vout, (size_t)n, 0, 8 * sizeof(K), s);
    if (e != hipSuccess) return e;
    void *tmp = buf.get<char>((int64_t)bytes);
    if (buf.e != hipSuccess) return buf.e;
    return rocprim::radix_sort_pairs(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0, 8 * sizeof(K), s);
}

template <class Op>
hipError_t incl_scan(Buf &buf, const int32_t *in, int32_t *out, int64_t n, Op op, hipStream_t s) {
    size_t bytes = 0;
    hipError_t e = rocprim::inclusive_scan(nullptr, bytes, in, out, (size_t)n, op, s);
    if (e != hipSuccess) return e;
    void *tmp = buf.get<char>((int64_t)bytes);
    if (buf.e != hipSuccess) return buf.e;
    return rocprim::inclusive_scan(tmp, bytes, in, out, (size_t)n, op, s);
}

hipError_t excl_sum(Buf &buf, const int32_t *in, int32_t *out, int64_t n, hipStream_t s) {
    size_t bytes = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, bytes, in, out, 0, (size_t)n, rocprim::plus<int32_t>(), s);
    if (e != hipSuccess) return e;
    void *tmp = buf.get<char>((int64_t)bytes);
    if (buf.e != hipSuccess) return buf.e;
    return rocprim::exclusive_scan(tmp, bytes, in, out, 0, (size_t)n, rocprim::plus<int32_t>(), s);
}

}  // namespace gdev
}  // namespace tmk

using namespace tmk;
using namespace tmk::gdev;

// 0: built; 1: rows need the host builder (an edge id on several rows); < 0: error
int tm_graph_build_edges_device(int32_t V, int64_t n_edges, const int64_t *src, const int64_t *dst, const int64_t *eidx,
                                const double *ts, int device, tm_graph **out) {
    // an empty edge set: nothing to sort or scan on the device (zero-size grids, no last block element
    // to read back); the host builder makes the empty graph
    if (n_edges <= 0) return 1;
    int32_t max_eid = 0;
    for (int64_t i = 0; i < n_edges; ++i) max_eid = (int32_t)std::max<int64_t>(max_eid, std::min<int64_t>(eidx[i], INT32_MAX));
    const int64_t n = 2 * n_edges, nn = std::max<int64_t>(n, 1);
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) prev = 0;
    if (hipSetDevice(device) != hipSuccess) return fail(TM_E_HIP, "tm_graph_build_edges: hipSetDevice failed");
    hipStream_t s = nullptr;
    int rc = TM_OK;
    tm_graph *g = nullptr;
    {
        Buf t;   // temporaries
        int64_t *d_src = t.get<int64_t>(n_edges), *d_dst = t.get<int64_t>(n_edges), *d_eidx = t.get<int64_t>(n_edges);
        double *d_ts = t.get<double>(n_edges);
        uint64_t *key = t.get<uint64_t>(nn), *key2 = t.get<uint64_t>(nn);
        int32_t *idx = t.get<int32_t>(nn), *perm1 = t.get<int32_t>(nn), *perm = t.get<int32_t>(nn);
        int32_t *own = t.get<int32_t>(nn), *ngh = t.get<int32_t>(nn), *eid = t.get<int32_t>(nn);
        double *tv = t.get<double>(nn);
        int32_t *okey = t.get<int32_t>(nn), *okey2 = t.get<int32_t>(nn);
        int32_t *s_own = t.get<int32_t>(nn), *cnt = t.get<int32_t>((int64_t)V + 1);
        int32_t *hpos = t.get<int32_t>(nn), *g0 = t.get<int32_t>(nn), *gend = t.get<int32_t>(nn);
        int32_t *ecount = t.get<int32_t>((int64_t)max_eid + 1), *err = t.get<int32_t>(1);
        int32_t *bperm1 = t.get<int32_t>(nn), *bperm = t.get<int32_t>(nn), *hflag = t.get<int32_t>(nn),
                *bstart = t.get<int32_t>(nn), *bincl = t.get<int32_t>(nn);
        if (t.e != hipSuccess) {
            (void)hipSetDevice(prev);
            return fail(TM_E_HIP, std::string("tm_graph_build_edges: ") + hipGetErrorString(t.e));
        }
        g = new tm_graph();
        g->device = device;
        hipError_t e = hipSuccess;
        e = e ? e : hipMalloc(&g->d_off, sizeof(int32_t) * (V + 1));
        e = e ? e : hipMalloc(&g->d_span, sizeof(int2) * V);
        e = e ? e : hipMalloc(&g->d_rec, sizeof(Rec) * nn);
        e = e ? e : hipMalloc(&g->d_tsd, sizeof(double) * nn);
        e = e ? e : hipMalloc(&g->d_ends, sizeof(EdgeEnds) * ((size_t)max_eid + 1));
        e = e ? e : hipMalloc(&g->d_ets, sizeof(double) * ((size_t)max_eid + 1));
        e = e ? e : hipMalloc(&g->d_hngh, sizeof(int32_t) * nn);
        e = e ? e : hipMalloc(&g->d_heid, sizeof(int32_t) * nn);
        e = e ? e : hipMalloc(&g->d_dict, sizeof(int32_t) * nn);
        e = e ? e : hipMemcpyAsync(d_src, src, sizeof(int64_t) * n_edges, hipMemcpyHostToDevice, s);
        e = e ? e : hipMemcpyAsync(d_dst, dst, sizeof(int64_t) * n_edges, hipMemcpyHostToDevice, s);
        e = e ? e : hipMemcpyAsync(d_eidx, eidx, sizeof(int64_t) * n_edges, hipMemcpyHostToDevice, s);
        e = e ? e : hipMemcpyAsync(d_ts, ts, sizeof(double) * n_edges, hipMemcpyHostToDevice, s);
        e = e ? e : hipMemsetAsync(ecount, 0, sizeof(int32_t) * ((size_t)max_eid + 1), s);
        e = e ? e : hipMemsetAsync(err, 0, sizeof(int32_t), s);
        e = e ? e : hipMemsetAsync(cnt, 0, sizeof(int32_t) * (V + 1), s);
        e = e ? e : hipMemsetAsync(g->d_ets, 0, sizeof(double) * ((size_t)max_eid + 1), s);
        if (e == hipSuccess) {
            k_entries<<<grid(n_edges), TB, 0, s>>>(n_edges, V, max_eid, d_src, d_dst, d_eidx, d_ts, key, idx, own, ngh,
                                                   eid, tv, ecount, err);
            k_fill_ends<<<grid((int64_t)max_eid + 1), TB, 0, s>>>((int64_t)max_eid + 1, g->d_ends);
            e = hipGetLastError();
        }
        int32_t herr = 0;
        e = e ? e : hipMemcpyAsync(&herr, err, sizeof(int32_t), hipMemcpyDeviceToHost, s);
        e = e ? e : hipStreamSynchronize(s);
        if (e == hipSuccess && herr) {
            rc = (herr & 1) ? fail(TM_E_ARG, "tm_graph_build_edges: node or edge id out of range") : 1;
        } else if (e == hipSuccess) {
            // (owner, ts, append order): stable sort by the ts key, then by the owner
            e = sort_pairs(t, key, key2, idx, perm1, n, s);
            if (e == hipSuccess) k_gather_key<<<grid(n), TB, 0, s>>>(n, perm1, own, okey);
            e = e ? e : sort_pairs(t, okey, okey2, perm1, perm, n, s);
            double *h_ts = g->d_tsd;
            if (e == hipSuccess)
                k_sorted<<<grid(n), TB, 0, s>>>(n, perm, own, ngh, eid, tv, s_own, g->d_hngh, g->d_heid, h_ts, cnt);
            e = e ? e : excl_sum(t, cnt, g->d_off, (int64_t)V + 1, s);
            if (e == hipSuccess) {
                k_group_heads<<<grid(n), TB, 0, s>>>(n, s_own, h_ts, g->d_off, hpos);
                e = hipGetLastError();
            }
            e = e ? e : incl_scan(t, hpos, g0, n, rocprim::maximum<int32_t>(), s);
            if (e == hipSuccess) {
                k_group_ends<<<grid(n), TB, 0, s>>>(n, s_own, h_ts, g->d_off, g0, gend);
                k_dict<<<grid(n), TB, 0, s>>>(n, s_own, g->d_hngh, g->d_heid, h_ts, g->d_off, g0, gend, g->d_dict,
                                              g->d_ends, g->d_rec, g->d_ets);
                k_span<<<grid(V), TB, 0, s>>>(V, g->d_off, g->d_span);
                e = hipGetLastError();
            }
            // blocks: the node-sorted positions 0..n-1 in (owner, neighbour, position) order -- stable sorts by
            // the neighbour, then by the owner
            if (e == hipSuccess) {
                rocprim::counting_iterator<int32_t> iota(0);
                e = sort_pairs(t, g->d_hngh, okey2, iota, bperm1, n, s);
            }
            if (e == hipSuccess) k_gather_key<<<grid(n), TB, 0, s>>>(n, bperm1, s_own, okey);
            e = e ? e : sort_pairs(t, okey, okey2, bperm1, bperm, n, s);
            if (e == hipSuccess) {
                k_block_heads<<<grid(n), TB, 0, s>>>(n, bperm, s_own, g->d_hngh, hpos, hflag);
                e = hipGetLastError();
            }
            e = e ? e : incl_scan(t, hpos, bstart, n, rocprim::maximum<int32_t>(), s);
            e = e ? e : incl_scan(t, hflag, bincl, n, rocprim::plus<int32_t>(), s);
            int32_t nb = 0;
            if (n > 0) {
                e = e ? e : hipMemcpyAsync(&nb, bincl + (n - 1), sizeof(int32_t), hipMemcpyDeviceToHost, s);
                e = e ? e : hipStreamSynchronize(s);
            }
            int32_t *bn = t.get<int32_t>(nb), *bu = t.get<int32_t>(nb), *bx = t.get<int32_t>(nb), *bs = t.get<int32_t>(nb),
                    *rl = t.get<int32_t>(nb), *rbase = t.get<int32_t>(nb);
            e = e ? e : t.e;
            if (e == hipSuccess && n > 0) {
                k_block_info<<<grid(n), TB, 0, s>>>(n, bperm, s_own, g->d_hngh, bstart, bincl, bn, bu, bx, bs, g->d_rec);
                k_region_len<<<grid(nb), TB, 0, s>>>(nb, bn, rl);
                e = hipGetLastError();
            }
            e = e ? e : (nb > 0 ? excl_sum(t, rl, rbase, nb, s) : hipSuccess);
            int32_t last_base = 0, last_len = 0;
            if (nb > 0) {
                e = e ? e : hipMemcpyAsync(&last_base, rbase + (nb - 1), sizeof(int32_t), hipMemcpyDeviceToHost, s);
                e = e ? e : hipMemcpyAsync(&last_len, rl + (nb - 1), sizeof(int32_t), hipMemcpyDeviceToHost, s);
                e = e ? e : hipStreamSynchronize(s);
            }
            const int64_t n_ppos = std::max<int64_t>((int64_t)last_base + last_len, 16);
            uint32_t cap = 16;
            while ((int64_t)cap < 2 * (int64_t)nb) cap <<= 1;
            e = e ? e : hipMalloc(&g->d_ppos, sizeof(int32_t) * n_ppos);
            e = e ? e : hipMalloc(&g->d_pblk, sizeof(PairBlk) * cap);
            if (e == hipSuccess) {
                k_fill_i32<<<grid(n_ppos), TB, 0, s>>>(n_ppos, g->d_ppos, INT32_MAX);
                k_pblk_fill<<<grid(cap), TB, 0, s>>>(cap, g->d_pblk);
                if (nb > 0) {
                    k_keys<<<grid(n), TB, 0, s>>>(n, bperm, s_own, g->d_off, bincl, bs, bn, rbase, g->d_ppos);
                    k_fences<<<grid(nb), TB, 0, s>>>(nb, bn, rbase, g->d_ppos);
                    k_pblk_insert<<<grid(nb), TB, 0, s>>>(nb, bu, bx, rbase, bn, g->d_pblk, cap - 1);
                }
                e = hipGetLastError();
            }
            e = e ? e : hipStreamSynchronize(s);
            if (e == hipSuccess) {
                g->d = DevGraph{V,         max_eid,   n,         g->d_off, g->d_span, g->d_rec, g->d_tsd,
                                g->d_ends, g->d_ppos, g->d_ets, 1,        g->d_pblk, cap - 1};
                g->dev_built = 1;
            }
        }
        if (e != hipSuccess) rc = fail(TM_E_HIP, std::string("tm_graph_build_edges: ") + hipGetErrorString(e));
    }
    (void)hipSetDevice(prev);
    if (rc != TM_OK) {
        tm_graph_free(g);
        return rc;
    }
    *out = g;
    return TM_OK;
}

// A strict_temporal view of g (SURVEY §7 opt-in; the reference has no such mode): the same device CSR,
// timestamps, block trees and pair table, with its own e_idx -> slice-length table holding
// bisect_left(ts_u, t(e)) instead of get_ts2idx's trailing-tie values (utils/graph.py:77-101), and the
// strict flag that makes get_final_step cut a None lookup at t(e2) (graph.py:357/:366).  The view shares
// the parent's buffers: free it (tm_graph_free) before the parent.
extern "C" int tm_graph_strict_view(const tm_graph *g, tm_graph **out) {
    using namespace tmk;
    using namespace tmk::gdev;
    if (!g || !out) return fail(TM_E_ARG, "tm_graph_strict_view: bad arguments");
    *out = nullptr;
    if (g->parent) g = g->parent;
    if (!g->d.ts_unique)
        return fail(TM_E_UNSUPPORTED, "tm_graph_strict_view: an edge id carries more than one timestamp");
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) prev = 0;
    hipError_t e = hipSetDevice(g->device);
    tm_graph *v = new tm_graph();
    v->device = g->device;
    v->parent = g;
    const int64_t n = (int64_t)g->d.max_eid + 1;
    e = e ? e : hipMalloc(&v->d_ends, sizeof(EdgeEnds) * n);
    if (e == hipSuccess) {
        k_strict_ends<<<grid(n), TB, 0, 0>>>(n, g->d, v->d_ends);
        e = hipGetLastError();
    }
    e = e ? e : hipDeviceSynchronize();
    (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        tm_graph_free(v);
        return fail(TM_E_HIP, std::string("tm_graph_strict_view: ") + hipGetErrorString(e));
    }
    v->d = g->d;
    v->d.ends = v->d_ends;
    v->d.strict = 1;
    *out = v;
    return TM_OK;
}
