// Temporal CSR build (host) + upload.  Replaces NeighborFinder.__init__ / init_off_set /
// get_ts2idx (utils/graph.py:13-101).  Runs once per split; the hot path only reads the
// device arrays built here.
#include <algorithm>
#include <numeric>
#include <unordered_map>
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
extern "C" int tm_version(void) { return 1; }

static void free_graph(tm_graph *g) {
    if (!g) return;
    if (g->d_off) (void)hipFree(g->d_off);
    if (g->d_rec) (void)hipFree(g->d_rec);
    if (g->d_ends) (void)hipFree(g->d_ends);
    if (g->d_pair) (void)hipFree(g->d_pair);
    if (g->d_ets) (void)hipFree(g->d_ets);
    if (g->d_pblk) (void)hipFree(g->d_pblk);
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
    const int64_t n = in_off[n_nodes];
    if (in_off[0] != 0 || n < 0) return fail(TM_E_ARG, "tm_graph_build: in_off must start at 0");
    if (n > 0 && (!ngh || !eid || !ts)) return fail(TM_E_ARG, "tm_graph_build: NULL entry arrays");
    if (n >= INT32_MAX) return fail(TM_E_UNSUPPORTED, "tm_graph_build: more than 2^31-1 adjacency entries");
    int32_t max_eid = 0;
    for (int32_t u = 0; u < n_nodes; ++u)
        if (in_off[u + 1] < in_off[u]) return fail(TM_E_ARG, "tm_graph_build: in_off not monotone");
    for (int64_t i = 0; i < n; ++i) {
        if (ngh[i] < 0 || ngh[i] >= n_nodes) return fail(TM_E_ARG, "tm_graph_build: neighbor id out of range");
        if (eid[i] < 0) return fail(TM_E_ARG, "tm_graph_build: negative edge id");
        max_eid = std::max(max_eid, eid[i]);
    }

    tm_graph *g = new tm_graph();
    g->device = device;
    g->h_off = new int64_t[n_nodes + 1];
    const int64_t nn = std::max<int64_t>(n, 1);
    g->h_ngh = new int32_t[nn];
    g->h_eid = new int32_t[nn];
    g->h_dict = new int32_t[nn];
    g->h_ts = new double[nn];
    std::vector<Rec> rec(nn);
    std::vector<Pair> pair(nn);
    std::vector<EdgeEnds> ends((size_t)max_eid + 1, EdgeEnds{-1, 0, -1, 0});
    std::vector<int32_t> off32(n_nodes + 1);
    std::vector<double> ets((size_t)max_eid + 1, 0.0);
    std::vector<char> seen((size_t)max_eid + 1, 0);
    int32_t ts_unique = 1;
    for (int64_t i = 0; i < n; ++i) {
        if (!seen[eid[i]]) {
            seen[eid[i]] = 1;
            ets[eid[i]] = ts[i];
        } else if (!(ets[eid[i]] == ts[i])) {
            ts_unique = 0;
        }
    }

    std::vector<int64_t> idx;
    std::unordered_map<int32_t, int32_t> dict;
    std::vector<int32_t> tie;
    for (int32_t u = 0; u < n_nodes; ++u) {
        const int64_t s = in_off[u], d = in_off[u + 1] - s;
        g->h_off[u] = s;
        off32[u] = (int32_t)s;
        // neighbors sorted by time, ties kept in insertion order (graph.py:48: sorted() is stable)
        idx.resize(d);
        std::iota(idx.begin(), idx.end(), s);
        std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return ts[a] < ts[b]; });
        for (int64_t i = 0; i < d; ++i) {
            g->h_ngh[s + i] = ngh[idx[i]];
            g->h_eid[s + i] = eid[idx[i]];
            g->h_ts[s + i] = ts[idx[i]];
        }
        // get_ts2idx (graph.py:77-101), literally: overwrite, then subtract j inside each
        // finished tie group; the trailing group is never adjusted.
        dict.clear();
        tie.clear();
        double last_ts = -1.0;
        int32_t last_e = -1;
        for (int64_t i = 0; i < d; ++i) {
            const int32_t e = g->h_eid[s + i];
            const double t = g->h_ts[s + i];
            dict[e] = (int32_t)i;
            if (t == last_ts) {
                if (tie.empty()) {
                    tie.push_back(last_e);
                    tie.push_back(e);
                } else {
                    tie.push_back(e);
                }
            }
            if (!(t == last_ts) && !tie.empty()) {
                for (size_t j = 0; j < tie.size(); ++j) dict[tie[j]] -= (int32_t)j;
                tie.clear();
            }
            last_ts = t;
            last_e = e;
        }
        for (int64_t i = 0; i < d; ++i) {
            g->h_dict[s + i] = dict[g->h_eid[s + i]];
            rec[s + i] = Rec{g->h_ngh[s + i], g->h_eid[s + i], g->h_ts[s + i]};
            pair[s + i] = Pair{g->h_ngh[s + i], (int32_t)i};
        }
        std::sort(pair.begin() + s, pair.begin() + s + d,
                  [](const Pair &a, const Pair &b) { return a.ngh < b.ngh || (a.ngh == b.ngh && a.pos < b.pos); });
        for (auto &kv : dict) {
            int32_t v = kv.second;
            if (v < 0) v = (int32_t)std::max<int64_t>(0, d + v);  // Python slice with a negative stop
            EdgeEnds &x = ends[kv.first];
            if (x.node_a == -1 || x.node_a == u) {
                x.node_a = u;
                x.len_a = v;
            } else if (x.node_b == -1 || x.node_b == u) {
                x.node_b = u;
                x.len_b = v;
            } else {
                free_graph(g);
                return fail(TM_E_UNSUPPORTED, "tm_graph_build: edge id " + std::to_string(kv.first) +
                                                  " appears in the lists of more than two nodes");
            }
        }
    }
    g->h_off[n_nodes] = n;
    off32[n_nodes] = (int32_t)n;

    // (node, neighbour) block table over the pair index, load factor <= 1/2
    int64_t n_blocks = 0;
    for (int32_t u = 0; u < n_nodes; ++u)
        for (int64_t i = off32[u]; i < off32[u + 1]; ++i) n_blocks += (i == off32[u] || pair[i].ngh != pair[i - 1].ngh);
    uint32_t cap = 16;
    while ((int64_t)cap < 2 * n_blocks) cap <<= 1;
    std::vector<PairBlk> pblk(cap, PairBlk{-1, 0, 0, 0});
    for (int32_t u = 0; u < n_nodes; ++u)
        for (int64_t i = off32[u]; i < off32[u + 1];) {
            int64_t j = i + 1;
            while (j < off32[u + 1] && pair[j].ngh == pair[i].ngh) ++j;
            uint32_t h = pblk_hash(u, pair[i].ngh) & (cap - 1);
            while (pblk[h].u != -1) h = (h + 1) & (cap - 1);
            pblk[h] = PairBlk{u, pair[i].ngh, (int32_t)i, (int32_t)j};
            i = j;
        }

    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) prev = 0;
    if (hipSetDevice(device) != hipSuccess) {
        free_graph(g);
        return fail(TM_E_HIP, "tm_graph_build: hipSetDevice failed");
    }
    hipError_t e = hipSuccess;
    e = e ? e : hipMalloc(&g->d_off, sizeof(int32_t) * (n_nodes + 1));
    e = e ? e : hipMalloc(&g->d_rec, sizeof(Rec) * nn);
    e = e ? e : hipMalloc(&g->d_ends, sizeof(EdgeEnds) * ends.size());
    e = e ? e : hipMalloc(&g->d_pair, sizeof(Pair) * nn);
    e = e ? e : hipMalloc(&g->d_ets, sizeof(double) * ets.size());
    e = e ? e : hipMalloc(&g->d_pblk, sizeof(PairBlk) * cap);
    e = e ? e : hipMemcpy(g->d_pblk, pblk.data(), sizeof(PairBlk) * cap, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(g->d_ets, ets.data(), sizeof(double) * ets.size(), hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(g->d_off, off32.data(), sizeof(int32_t) * (n_nodes + 1), hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(g->d_rec, rec.data(), sizeof(Rec) * nn, hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(g->d_ends, ends.data(), sizeof(EdgeEnds) * ends.size(), hipMemcpyHostToDevice);
    e = e ? e : hipMemcpy(g->d_pair, pair.data(), sizeof(Pair) * nn, hipMemcpyHostToDevice);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        free_graph(g);
        return fail(TM_E_HIP, std::string("tm_graph_build: ") + hipGetErrorString(e));
    }
    g->d = DevGraph{n_nodes, max_eid, n, g->d_off, g->d_rec, g->d_ends, g->d_pair, g->d_ets, ts_unique, g->d_pblk,
                    cap - 1};
    *out = g;
    return TM_OK;
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

extern "C" int tm_graph_export(const tm_graph *g, int64_t *off, int32_t *ngh, int32_t *eid, double *ts,
                               int32_t *dict_val) {
    if (!g) return fail(TM_E_ARG, "tm_graph_export: NULL graph");
    const int64_t n = g->d.n_entries;
    if (off) std::copy(g->h_off, g->h_off + g->d.n_nodes + 1, off);
    if (ngh) std::copy(g->h_ngh, g->h_ngh + n, ngh);
    if (eid) std::copy(g->h_eid, g->h_eid + n, eid);
    if (ts) std::copy(g->h_ts, g->h_ts + n, ts);
    if (dict_val) std::copy(g->h_dict, g->h_dict + n, dict_val);
    return TM_OK;
}
