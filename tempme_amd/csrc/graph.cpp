// Temporal CSR build (host, multi-threaded) + upload.  Replaces NeighborFinder.__init__ /
// init_off_set / get_ts2idx (utils/graph.py:13-101) and temp_exp_main.py:135-144's adjacency
// build.  Runs once per split; the hot path only reads the device arrays built here.
//
// Work split: every node's list is independent (sort by ts, get_ts2idx, (neighbour, position)
// blocks, their search trees), so nodes are dealt to threads in chunks; the e_idx table keeps the
// reference's node order (owner a = the first node holding the edge) in one sequential pass, and
// the block hash table is filled with 64-bit compare-and-swap inserts.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <numeric>
#include <sched.h>
#include <thread>
#include <vector>

#include "common.h"

namespace tmk {
static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
int fail(int code, const std::string &msg) {
    set_error(msg);
    return code;
}
}  // namespace tmk

using namespace tmk;

extern "C" const char *tm_last_error(void) { return tmk::g_last_error.c_str(); }
extern "C" int tm_version(void) { return 3; }

namespace tmk {
static std::atomic<int> g_debug[TM_DEBUG_N_OPTS];
static std::atomic<int> g_host_threads{0};
int debug_opt(int opt) { return opt > 0 && opt < TM_DEBUG_N_OPTS ? g_debug[opt].load(std::memory_order_relaxed) : 0; }
}  // namespace tmk

extern "C" int tm_debug_set(int32_t opt, int32_t value) {
    if (opt <= 0 || opt >= TM_DEBUG_N_OPTS) return fail(TM_E_ARG, "tm_debug_set: unknown option");
    g_debug[opt].store(value, std::memory_order_relaxed);
    return TM_OK;
}

extern "C" int tm_set_host_threads(int32_t n) {
    if (n < 0) return fail(TM_E_ARG, "tm_set_host_threads: negative");
    g_host_threads.store(n, std::memory_order_relaxed);
    return TM_OK;
}

namespace {

// threads for the host build: tm_set_host_threads (the Python loader passes the process's CPU share), else the
// CPUs this process may run on, at most 64
int build_threads() {
    const int n = g_host_threads.load(std::memory_order_relaxed);
    if (n > 0) return std::min(64, n);
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) return std::max(1, std::min(64, CPU_COUNT(&cs)));
    return (int)std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
}

// f(thread, begin, end) over [0, n) in chunks of `grain`, dealt dynamically; returns the thread count
template <class F>
int parallel_for(int64_t n, int64_t grain, F f) {
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(build_threads(), (n + grain - 1) / std::max<int64_t>(grain, 1)));
    std::atomic<int64_t> next{0};
    auto work = [&](int t) {
        for (;;) {
            const int64_t b = next.fetch_add(grain);
            if (b >= n) return;
            f(t, b, std::min(n, b + grain));
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &t : th) t.join();
    return nt;
}

struct Timer {
    bool on = debug_opt(TM_DEBUG_GRAPH_TIMING) != 0;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void lap(const char *what) {
        if (!on) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "tm_graph_build %-14s %8.2f ms\n", what,
                     std::chrono::duration<double, std::milli>(t1 - t0).count());
        t0 = t1;
    }
};

}  // namespace

static void free_graph(tm_graph *g) {
    if (!g) return;
    if (g->d_off) (void)hipFree(g->d_off);
    if (g->d_span) (void)hipFree(g->d_span);
    if (g->d_rec) (void)hipFree(g->d_rec);
    if (g->d_tsd) (void)hipFree(g->d_tsd);
    if (g->d_ends) (void)hipFree(g->d_ends);
    if (g->d_ppos) (void)hipFree(g->d_ppos);
    if (g->d_ets) (void)hipFree(g->d_ets);
    if (g->d_pblk) (void)hipFree(g->d_pblk);
    if (g->d_hngh) (void)hipFree(g->d_hngh);
    if (g->d_heid) (void)hipFree(g->d_heid);
    if (g->d_dict) (void)hipFree(g->d_dict);
    delete[] g->h_off;
    delete[] g->h_ngh;
    delete[] g->h_eid;
    delete[] g->h_dict;
    delete[] g->h_ts;
    delete g;
}

extern "C" int tm_graph_build(int32_t n_nodes, const int64_t *in_off, const int32_t *ngh, const int32_t *eid,
                              const double *ts, int device, tm_graph **out) {
    if (!out || !in_off || n_nodes <= 0) return fail(TM_E_ARG, "tm_graph_build: bad arguments");
    *out = nullptr;
    Timer tm;
    const int64_t n = in_off[n_nodes];
    if (in_off[0] != 0 || n < 0) return fail(TM_E_ARG, "tm_graph_build: in_off must start at 0");
    if (n > 0 && (!ngh || !eid || !ts)) return fail(TM_E_ARG, "tm_graph_build: NULL entry arrays");
    if (n >= INT32_MAX / 2) return fail(TM_E_UNSUPPORTED, "tm_graph_build: more than 2^30-1 adjacency entries");
    for (int32_t u = 0; u < n_nodes; ++u)
        if (in_off[u + 1] < in_off[u]) return fail(TM_E_ARG, "tm_graph_build: in_off not monotone");
    // range checks and the largest edge id, in parallel chunks
    std::atomic<int32_t> max_eid_a{0}, bad{0};
    parallel_for(n, 1 << 16, [&](int, int64_t b, int64_t e) {
        int32_t m = 0, bd = 0;
        for (int64_t i = b; i < e; ++i) {
            if (ngh[i] < 0 || ngh[i] >= n_nodes) bd |= 1;
            if (eid[i] < 0) bd |= 2;
            m = std::max(m, eid[i]);
        }
        int32_t cur = max_eid_a.load();
        while (m > cur && !max_eid_a.compare_exchange_weak(cur, m)) {
        }
        if (bd) bad.fetch_or(bd);
    });
    if (bad.load() & 1) return fail(TM_E_ARG, "tm_graph_build: neighbor id out of range");
    if (bad.load() & 2) return fail(TM_E_ARG, "tm_graph_build: negative edge id");
    const int32_t max_eid = max_eid_a.load();

    tm_graph *g = new tm_graph();
    g->device = device;
    g->h_off = new int64_t[n_nodes + 1];
    const int64_t nn = std::max<int64_t>(n, 1);
    g->h_ngh = new int32_t[nn];
    g->h_eid = new int32_t[nn];
    g->h_dict = new int32_t[nn];
    g->h_ts = new double[nn];
    std::unique_ptr<Rec[]> rec(new Rec[nn]);          // every entry written by the node pass
    std::vector<int32_t> off32(n_nodes + 1);
    for (int32_t u = 0; u <= n_nodes; ++u) {
        g->h_off[u] = in_off[u];
        off32[u] = (int32_t)in_off[u];
    }
    // timestamp of each edge id (its first record's) and whether all its records agree: the first
    // record by an atomic min over entry indices, then a parallel compare
    std::unique_ptr<std::atomic<int64_t>[]> first(new std::atomic<int64_t>[(size_t)max_eid + 1]);
    parallel_for((int64_t)max_eid + 1, 1 << 16, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) first[i].store(INT64_MAX, std::memory_order_relaxed);
    });
    parallel_for(n, 1 << 16, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
            std::atomic<int64_t> &f = first[eid[i]];
            int64_t cur = f.load(std::memory_order_relaxed);
            while (i < cur && !f.compare_exchange_weak(cur, i, std::memory_order_relaxed)) {
            }
        }
    });
    std::vector<double> ets((size_t)max_eid + 1);
    parallel_for((int64_t)max_eid + 1, 1 << 16, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
            const int64_t f = first[i].load(std::memory_order_relaxed);
            ets[i] = f == INT64_MAX ? 0.0 : ts[f];
        }
    });
    std::atomic<int32_t> ts_diff{0};
    parallel_for(n, 1 << 16, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i)
            if (!(ets[eid[i]] == ts[i])) {
                ts_diff.store(1);
                return;
            }
    });
    const int32_t ts_unique = ts_diff.load() ? 0 : 1;
    tm.lap("validate");

    // ---- per node: stable sort by ts, get_ts2idx, (neighbour, position) blocks and ranks
    std::unique_ptr<int64_t[]> pair_key(new int64_t[nn]);     // per entry after the sort: ngh << 32 | position
    std::vector<int32_t> nblk(n_nodes + 1, 0), plen(n_nodes + 1, 0);
    // per-thread scratch: the dense dict (every slot read is written first in the same list) and the
    // sort / tie buffers
    struct Scratch {
        std::unique_ptr<int32_t[]> dval;
        std::vector<int64_t> idx;
        std::vector<int32_t> tie;
    };
    std::vector<Scratch> scr(build_threads());
    parallel_for(n_nodes, 16, [&](int t_, int64_t b, int64_t e) {
        Scratch &sc = scr[t_];
        if (!sc.dval) sc.dval.reset(new int32_t[(size_t)max_eid + 1]);
        int32_t *dval = sc.dval.get();
        std::vector<int64_t> &idx = sc.idx;
        std::vector<int32_t> &tie = sc.tie;
        for (int64_t u = b; u < e; ++u) {
            const int64_t s = in_off[u], d = in_off[u + 1] - s;
            // neighbors sorted by time, ties kept in insertion order (graph.py:48: sorted() is stable)
            bool sorted = true;
            for (int64_t i = 1; i < d && sorted; ++i) sorted = !(ts[s + i] < ts[s + i - 1]);
            if (sorted) {
                std::copy(ngh + s, ngh + s + d, g->h_ngh + s);
                std::copy(eid + s, eid + s + d, g->h_eid + s);
                std::copy(ts + s, ts + s + d, g->h_ts + s);
            } else {
                idx.resize(d);
                std::iota(idx.begin(), idx.end(), s);
                std::stable_sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) { return ts[x] < ts[y]; });
                for (int64_t i = 0; i < d; ++i) {
                    g->h_ngh[s + i] = ngh[idx[i]];
                    g->h_eid[s + i] = eid[idx[i]];
                    g->h_ts[s + i] = ts[idx[i]];
                }
            }
            // get_ts2idx (graph.py:77-101), literally: overwrite, then subtract j inside each
            // finished tie group; the trailing group is never adjusted.
            tie.clear();
            double last_ts = -1.0;
            int32_t last_e = -1;
            for (int64_t i = 0; i < d; ++i) {
                const int32_t ei = g->h_eid[s + i];
                const double t = g->h_ts[s + i];
                dval[ei] = (int32_t)i;
                if (t == last_ts) {
                    if (tie.empty()) tie.push_back(last_e);
                    tie.push_back(ei);
                }
                if (!(t == last_ts) && !tie.empty()) {
                    for (size_t j = 0; j < tie.size(); ++j) dval[tie[j]] -= (int32_t)j;
                    tie.clear();
                }
                last_ts = t;
                last_e = ei;
            }
            for (int64_t i = 0; i < d; ++i) {
                g->h_dict[s + i] = dval[g->h_eid[s + i]];
                pair_key[s + i] = (int64_t)g->h_ngh[s + i] << 32 | (int64_t)i;
            }
            std::sort(pair_key.get() + s, pair_key.get() + s + d);
            int32_t blocks = 0, len = 0;
            for (int64_t i = 0; i < d;) {
                int64_t j = i + 1;
                while (j < d && (pair_key[s + j] >> 32) == (pair_key[s + i] >> 32)) ++j;
                const int32_t bn = (int32_t)(j - i);
                for (int64_t k = i; k < j; ++k) {
                    const int32_t p = (int32_t)(pair_key[s + k] & 0xFFFFFFFF);
                    rec[s + p] = Rec{g->h_ngh[s + p], g->h_eid[s + p], (float)g->h_ts[s + p], (int32_t)(k - i)};
                }
                if (bn > kBlkFan) len = (len + kBlkFan - 1) & ~(kBlkFan - 1);     // node-aligned tree
                len += blk_region_len(bn);
                ++blocks;
                i = j;
            }
            nblk[u] = blocks;
            plen[u] = (len + 15) & ~15;                   // node regions 64-B aligned
        }
    });
    tm.lap("nodes");

    // ---- block trees
    std::vector<int64_t> boff(n_nodes + 1, 0), poff(n_nodes + 1, 0);
    for (int32_t u = 0; u < n_nodes; ++u) {
        boff[u + 1] = boff[u] + nblk[u];
        poff[u + 1] = poff[u] + plen[u];
    }
    const int64_t n_blocks = boff[n_nodes], n_ppos = std::max<int64_t>(poff[n_nodes], 16);
    if (n_ppos >= INT32_MAX) {
        free_graph(g);
        return fail(TM_E_UNSUPPORTED, "tm_graph_build: block trees exceed 2^31 entries");
    }
    std::unique_ptr<int32_t[]> ppos(new int32_t[n_ppos]);
    parallel_for(n_ppos, 1 << 18, [&](int, int64_t b, int64_t e) { std::fill(ppos.get() + b, ppos.get() + e, INT32_MAX); });
    std::unique_ptr<PairBlk[]> blist(new PairBlk[std::max<int64_t>(n_blocks, 1)]);
    parallel_for(n_nodes, 16, [&](int, int64_t b, int64_t e) {
        for (int64_t u = b; u < e; ++u) {
            const int64_t s = in_off[u], d = in_off[u + 1] - s;
            int64_t bi = boff[u];
            int32_t len = 0;
            for (int64_t i = 0; i < d;) {
                int64_t j = i + 1;
                while (j < d && (pair_key[s + j] >> 32) == (pair_key[s + i] >> 32)) ++j;
                const int32_t bn = (int32_t)(j - i);
                if (bn > kBlkFan) len = (len + kBlkFan - 1) & ~(kBlkFan - 1);
                const int64_t base = poff[u] + len;
                int32_t *keys = ppos.get() + base + blk_keys_off(bn);
                for (int64_t k = i; k < j; ++k) keys[k - i] = (int32_t)(pair_key[s + k] & 0xFFFFFFFF);
                if (bn > kBlkFan) {   // fence levels, bottom-up: L_l[t] = L_(l-1)[F t]
                    const int32_t h = blk_levels(bn);
                    int32_t *lower = keys;
                    int64_t lo_off = blk_keys_off(bn);
                    for (int32_t l = 1; l <= h; ++l) {
                        lo_off -= blk_level_len(bn, l, h);
                        int32_t *lev = ppos.get() + base + lo_off;
                        const int32_t cnt =
                            (int32_t)(((int64_t)bn + ((int64_t)1 << (kBlkLog * l)) - 1) >> (kBlkLog * l));
                        for (int32_t t = 0; t < cnt; ++t) lev[t] = lower[kBlkFan * t];
                        lower = lev;
                    }
                }
                blist[bi++] = PairBlk{(int32_t)u, (int32_t)(pair_key[s + i] >> 32), (int32_t)base, bn};
                len += blk_region_len(bn);
                i = j;
            }
        }
    });
    tm.lap("trees");

    // ---- (node, neighbour) -> block hash table, load factor <= 1/2
    uint32_t cap = 16;
    while ((int64_t)cap < 2 * n_blocks) cap <<= 1;
    std::unique_ptr<PairBlk[]> pblk(new PairBlk[cap]);
    parallel_for(cap, 1 << 18, [&](int, int64_t b, int64_t e) {
        std::fill(pblk.get() + b, pblk.get() + e, PairBlk{-1, 0, 0, 0});
    });
    parallel_for(n_blocks, 4096, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
            const PairBlk &x = blist[i];
            const uint64_t key = (uint64_t)(uint32_t)x.u | (uint64_t)(uint32_t)x.x << 32;
            const uint64_t empty = (uint64_t)0xFFFFFFFFu;
            uint32_t h = pblk_hash(x.u, x.x) & (cap - 1);
            for (;;) {
                uint64_t *slot = reinterpret_cast<uint64_t *>(&pblk[h]);
                uint64_t expect = empty;
                if (__atomic_compare_exchange_n(slot, &expect, key, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
                    pblk[h].base = x.base;
                    pblk[h].n = x.n;
                    break;
                }
                h = (h + 1) & (cap - 1);
            }
        }
    });
    tm.lap("block table");

    // ---- e_idx -> (owner, slice length): owner a = the first node (in node order) holding the edge, b the
    // second (graph.py's dict per node); more than two owners is unsupported.  Owners by atomic min/max,
    // then every entry writes its owner's slice length (the same value for every entry of one list).
    std::vector<EdgeEnds> ends((size_t)max_eid + 1);
    std::unique_ptr<std::atomic<int32_t>[]> amin(new std::atomic<int32_t>[(size_t)max_eid + 1]),
        amax(new std::atomic<int32_t>[(size_t)max_eid + 1]);
    parallel_for((int64_t)max_eid + 1, 1 << 16, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
            amin[i].store(INT32_MAX, std::memory_order_relaxed);
            amax[i].store(-1, std::memory_order_relaxed);
        }
    });
    parallel_for(n_nodes, 64, [&](int, int64_t b, int64_t e) {
        for (int64_t u = b; u < e; ++u)
            for (int64_t i = in_off[u]; i < in_off[u + 1]; ++i) {
                const int32_t x = g->h_eid[i];
                int32_t c = amin[x].load(std::memory_order_relaxed);
                while ((int32_t)u < c && !amin[x].compare_exchange_weak(c, (int32_t)u, std::memory_order_relaxed)) {
                }
                c = amax[x].load(std::memory_order_relaxed);
                while ((int32_t)u > c && !amax[x].compare_exchange_weak(c, (int32_t)u, std::memory_order_relaxed)) {
                }
            }
    });
    std::atomic<int64_t> third{-1};
    parallel_for(n_nodes, 64, [&](int, int64_t b, int64_t e) {
        for (int64_t u = b; u < e; ++u) {
            const int64_t s0 = in_off[u], d = in_off[u + 1] - s0;
            for (int64_t i = s0; i < s0 + d; ++i) {
                const int32_t x = g->h_eid[i];
                const int32_t a = amin[x].load(std::memory_order_relaxed), bb = amax[x].load(std::memory_order_relaxed);
                int32_t v = g->h_dict[i];
                if (v < 0) v = (int32_t)std::max<int64_t>(0, d + v);  // Python slice with a negative stop
                if (u == a) {
                    ends[x].node_a = a;
                    ends[x].len_a = v;
                } else if (u == bb) {
                    ends[x].node_b = bb;
                    ends[x].len_b = v;
                } else {
                    third.store(x);
                }
            }
        }
    });
    if (third.load() >= 0) {
        free_graph(g);
        return fail(TM_E_UNSUPPORTED, "tm_graph_build: edge id " + std::to_string(third.load()) +
                                          " appears in the lists of more than two nodes");
    }
    parallel_for((int64_t)max_eid + 1, 1 << 16, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
            const int32_t a = amin[i].load(std::memory_order_relaxed), bb = amax[i].load(std::memory_order_relaxed);
            if (a == INT32_MAX) ends[i] = EdgeEnds{-1, 0, -1, 0};
            else if (a == bb) ends[i].node_b = -1, ends[i].len_b = 0;
        }
    });
    tm.lap("edge ends");

    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) prev = 0;
    if (hipSetDevice(device) != hipSuccess) {
        free_graph(g);
        return fail(TM_E_HIP, "tm_graph_build: hipSetDevice failed");
    }
    hipError_t e = hipSuccess;
    e = e ? e : hipMalloc(&g->d_off, sizeof(int32_t) * (n_nodes + 1));
    e = e ? e : hipMalloc(&g->d_span, sizeof(int2) * n_nodes);
    e = e ? e : hipMalloc(&g->d_rec, sizeof(Rec) * nn);
    e = e ? e : hipMalloc(&g->d_tsd, sizeof(double) * nn);
    e = e ? e : hipMalloc(&g->d_ends, sizeof(EdgeEnds) * ends.size());
    e = e ? e : hipMalloc(&g->d_ppos, sizeof(int32_t) * n_ppos);
    e = e ? e : hipMalloc(&g->d_ets, sizeof(double) * ets.size());
    e = e ? e : hipMalloc(&g->d_pblk, sizeof(PairBlk) * cap);
    e = e ? e : hipMemcpy(g->d_pblk, pblk.get(), sizeof(PairBlk) * cap, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(g->d_ets, ets.data(), sizeof(double) * ets.size(), hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(g->d_off, off32.data(), sizeof(int32_t) * (n_nodes + 1), hipMemcpyHostToDevice);
    {
        std::vector<int2> span(n_nodes);
        for (int32_t u = 0; u < n_nodes; ++u) span[u] = make_int2(off32[u], off32[u + 1]);
        e = e ? e : hipMemcpy(g->d_span, span.data(), sizeof(int2) * n_nodes, hipMemcpyHostToDevice);
    }
    e = e ? e : hipMemcpy(g->d_rec, rec.get(), sizeof(Rec) * nn, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(g->d_tsd, g->h_ts, sizeof(double) * nn, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(g->d_ends, ends.data(), sizeof(EdgeEnds) * ends.size(), hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(g->d_ppos, ppos.get(), sizeof(int32_t) * n_ppos, hipMemcpyHostToDevice);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        free_graph(g);
        return fail(TM_E_HIP, std::string("tm_graph_build: ") + hipGetErrorString(e));
    }
    tm.lap("upload");
    g->d = DevGraph{n_nodes,   max_eid,   n,        g->d_off,  g->d_span, g->d_rec,
                    g->d_tsd,  g->d_ends, g->d_ppos, g->d_ets, ts_unique, g->d_pblk, cap - 1};
    *out = g;
    return TM_OK;
}

// temp_exp_main.py:135-144 on raw edge rows: for every row (dst, e, t) is appended to src's list,
// then (src, e, t) to dst's; owner-major by a counting sort (stable, so each list keeps the rows'
// order), then tm_graph_build.
int tm_graph_build_edges_device(int32_t V, int64_t n_edges, const int64_t *src, const int64_t *dst, const int64_t *eidx,
                                const double *ts, int device, tm_graph **out);

extern "C" int tm_graph_build_edges(int32_t n_nodes, int64_t n_edges, const int64_t *src, const int64_t *dst,
                                    const int64_t *eidx, const double *ts, int device, tm_graph **out) {
    if (!out || n_nodes <= 0 || n_edges < 0) return fail(TM_E_ARG, "tm_graph_build_edges: bad arguments");
    if (n_edges > 0 && (!src || !dst || !eidx || !ts)) return fail(TM_E_ARG, "tm_graph_build_edges: NULL arrays");
    if (2 * n_edges >= INT32_MAX / 2) return fail(TM_E_UNSUPPORTED, "tm_graph_build_edges: too many edges");
    *out = nullptr;
    // the device builder (graph_dev.hip); the host builder below for rows that repeat an edge id, or on
    // request (tm_debug_set(TM_DEBUG_HOST_BUILD, 1): the tests that compare the two builders)
    if (!debug_opt(TM_DEBUG_HOST_BUILD)) {
        Timer tmd;
        const int rc = tm_graph_build_edges_device(n_nodes, n_edges, src, dst, eidx, ts, device, out);
        tmd.lap("device build");
        if (rc != 1) return rc;
    }
    Timer tm;
    // per-chunk node counts, then each chunk scatters its rows in order (stable)
    const int T = std::max(1, (int)std::min<int64_t>(build_threads(), (n_edges + 65535) / 65536));
    const int64_t chunk = (n_edges + T - 1) / T;
    std::vector<std::vector<int32_t>> cnt(T);
    std::atomic<int> bad{0};
    parallel_for(T, 1, [&](int, int64_t tb, int64_t te) {
        for (int64_t t = tb; t < te; ++t) {
            std::vector<int32_t> &c = cnt[t];
            c.assign((size_t)n_nodes, 0);
            for (int64_t i = t * chunk; i < std::min(n_edges, (t + 1) * chunk); ++i) {
                if (src[i] < 0 || src[i] >= n_nodes || dst[i] < 0 || dst[i] >= n_nodes) {
                    bad.store(1);
                    return;
                }
                if (eidx[i] < 0 || eidx[i] > INT32_MAX) {
                    bad.store(2);
                    return;
                }
                ++c[src[i]];
                ++c[dst[i]];
            }
        }
    });
    if (bad.load() == 1) return fail(TM_E_ARG, "tm_graph_build_edges: node id out of range");
    if (bad.load() == 2) return fail(TM_E_ARG, "tm_graph_build_edges: edge id out of range");
    std::vector<int64_t> off((size_t)n_nodes + 1, 0);
    for (int32_t u = 0; u < n_nodes; ++u) {
        int64_t acc = off[u];
        for (int t = 0; t < T; ++t) {       // chunk t's first slot of node u
            const int32_t c = cnt[t][u];
            cnt[t][u] = (int32_t)(acc - off[u]);
            acc += c;
        }
        off[u + 1] = acc;
    }
    const int64_t n = 2 * n_edges, nn = std::max<int64_t>(n, 1);
    std::unique_ptr<int32_t[]> ngh(new int32_t[nn]), eid(new int32_t[nn]);
    std::unique_ptr<double[]> t(new double[nn]);
    parallel_for(T, 1, [&](int, int64_t tb, int64_t te) {
        for (int64_t c = tb; c < te; ++c) {
            std::vector<int32_t> &pos = cnt[c];
            for (int64_t i = c * chunk; i < std::min(n_edges, (c + 1) * chunk); ++i) {
                int64_t p = off[src[i]] + pos[src[i]]++;
                ngh[p] = (int32_t)dst[i];
                eid[p] = (int32_t)eidx[i];
                t[p] = ts[i];
                p = off[dst[i]] + pos[dst[i]]++;
                ngh[p] = (int32_t)src[i];
                eid[p] = (int32_t)eidx[i];
                t[p] = ts[i];
            }
        }
    });
    tm.lap("edge rows");
    return tm_graph_build(n_nodes, off.data(), ngh.get(), eid.get(), t.get(), device, out);
}

extern "C" int tm_graph_free(tm_graph *g) {
    free_graph(g);
    return TM_OK;
}

extern "C" int tm_graph_info(const tm_graph *g, int32_t *n_nodes, int64_t *n_entries, int32_t *max_eid) {
    if (!g) return fail(TM_E_ARG, "tm_graph_info: NULL graph");
    if (n_nodes) *n_nodes = g->d.n_nodes;
    if (n_entries) *n_entries = g->d.n_entries;
    if (max_eid) *max_eid = g->d.max_eid;
    return TM_OK;
}

extern "C" int tm_graph_export(const tm_graph *gc, int64_t *off, int32_t *ngh, int32_t *eid, double *ts,
                               int32_t *dict_val) {
    if (!gc) return fail(TM_E_ARG, "tm_graph_export: NULL graph");
    if (gc->parent) return tm_graph_export(gc->parent, off, ngh, eid, ts, dict_val);
    tm_graph *g = const_cast<tm_graph *>(gc);
    const int64_t n = g->d.n_entries;
    if (g->dev_built) {   // host copies of a device-built graph, made once (the first export publishes them)
        static std::mutex export_mu;
        std::lock_guard<std::mutex> lock(export_mu);
        if (!g->h_off) {
            const int32_t V = g->d.n_nodes;
            const int64_t nn = std::max<int64_t>(n, 1);
            std::vector<int32_t> off32(V + 1);
            std::unique_ptr<int64_t[]> h_off(new int64_t[V + 1]);
            std::unique_ptr<int32_t[]> h_ngh(new int32_t[nn]), h_eid(new int32_t[nn]), h_dict(new int32_t[nn]);
            std::unique_ptr<double[]> h_ts(new double[nn]);
            int prev = 0;
            if (hipGetDevice(&prev) != hipSuccess) prev = 0;
            hipError_t e = hipSetDevice(g->device);
            e = e ? e : hipMemcpy(off32.data(), g->d_off, sizeof(int32_t) * (V + 1), hipMemcpyDeviceToHost);
            e = e ? e : hipMemcpy(h_ngh.get(), g->d_hngh, sizeof(int32_t) * nn, hipMemcpyDeviceToHost);
            e = e ? e : hipMemcpy(h_eid.get(), g->d_heid, sizeof(int32_t) * nn, hipMemcpyDeviceToHost);
            e = e ? e : hipMemcpy(h_dict.get(), g->d_dict, sizeof(int32_t) * nn, hipMemcpyDeviceToHost);
            e = e ? e : hipMemcpy(h_ts.get(), g->d_tsd, sizeof(double) * nn, hipMemcpyDeviceToHost);
            (void)hipSetDevice(prev);
            // nothing is published unless every copy succeeded (a failed export leaves no partial state)
            if (e != hipSuccess) return fail(TM_E_HIP, std::string("tm_graph_export: ") + hipGetErrorString(e));
            for (int32_t u = 0; u <= V; ++u) h_off[u] = off32[u];
            g->h_ngh = h_ngh.release();
            g->h_eid = h_eid.release();
            g->h_dict = h_dict.release();
            g->h_ts = h_ts.release();
            g->h_off = h_off.release();
        }
    }
    if (off) std::copy(g->h_off, g->h_off + g->d.n_nodes + 1, off);
    if (ngh) std::copy(g->h_ngh, g->h_ngh + n, ngh);
    if (eid) std::copy(g->h_eid, g->h_eid + n, eid);
    if (ts) std::copy(g->h_ts, g->h_ts + n, ts);
    if (dict_val) std::copy(g->h_dict, g->h_dict + n, dict_val);
    return TM_OK;
}
