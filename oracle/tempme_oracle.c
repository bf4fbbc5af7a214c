/* TEST INFRASTRUCTURE ONLY -- CPU oracle for the TempME explanation hot path.
 *
 * A literal, single-threaded (optionally OpenMP-over-events) plain-C
 * restatement of the reference's sampling and motif bookkeeping.  It is the
 * checker the HIP kernels are compared against and the "port" CPU baseline of
 * bench.py.  It is NOT linked into, loaded by or called from the product
 * package tempme_amd.  Pinned against the tests/golden fixtures (vectors produced by the
 * reference itself, see tests/golden/make_goldens.py).
 *
 * Reference functions restated (dharunm236/TempME @ /root/reference):
 *   or_graph_build        utils/graph.py:33-66  (init_off_set: per-node stable sort by ts)
 *                         utils/graph.py:77-101 (get_ts2idx: e_idx -> position dict, tie quirk)
 *   or_find_before        utils/graph.py:103-146 + :511-530 (bisect_left_adapt)
 *   or_khop               utils/graph.py:197-262 (get_temporal_neighbor, find_k_hop)
 *   or_walks              utils/graph.py:149-194, :265-476 (find_before_walk, find_k_walks,
 *                         get_next_step, get_final_step incl. the [:None] leak quirk)
 *   or_cat / or_hist      processed/data_preprocess.py:148-214 (marginal), utils/null_model.py:75-121
 *   or_edge_counts        processed/data_preprocess.py:327-343 (new_edge_info)
 *   or_neg_sample         utils/batch_loader.py:32-42 (RandEdgeSampler.sample)
 * RNG: the keyed Philox4x32-10 contract of oracle/philox.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ Philox */
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1; c[3] = (uint32_t)p0; c[0] = n0; c[2] = n2;
    }
}

typedef struct { uint64_t seed; uint32_t split, side; } or_rng;

static uint32_t draw_u32(or_rng g, uint32_t stage, uint32_t event, uint32_t row, uint32_t j) {
    uint32_t c[4] = {event, (g.split << 16) | (g.side << 8) | stage, row, j >> 2};
    philox(c, (uint32_t)g.seed, (uint32_t)(g.seed >> 32));
    return c[j & 3];
}

static int64_t draw(or_rng g, uint32_t stage, uint32_t event, uint32_t row, uint32_t j, int64_t high) {
    return (int64_t)(((uint64_t)draw_u32(g, stage, event, row, j) * (uint64_t)high) >> 32);
}

uint32_t or_draw_u32(uint64_t seed, uint32_t split, uint32_t side, uint32_t stage,
                     uint32_t event, uint32_t row, uint32_t j) {
    or_rng g = {seed, split, side};
    return draw_u32(g, stage, event, row, j);
}

/* ------------------------------------------------------------------ graph */
typedef struct {
    int32_t n_nodes;
    int64_t n_entries;
    int64_t *off;              /* [V+1] */
    int32_t *ngh, *eid;        /* [n_entries], per-node sorted by ts (stable) */
    double *ts;
    int64_t *doff;             /* per-node dict: [V+1] offsets into dkey/dval */
    int32_t *dkey, *dval;      /* sorted unique eids of the node, final dict value */
    int strict;                /* strict_temporal: see or_graph_set_strict */
    int32_t max_eid;
    double *ets;               /* [max_eid+1] timestamp of each edge id (strict mode only) */
} or_graph;

typedef struct { double ts; int64_t ord; int32_t ngh, eid; } ent_t;

static int cmp_ent(const void *a, const void *b) {
    const ent_t *x = a, *y = b;
    if (x->ts < y->ts) return -1;
    if (x->ts > y->ts) return 1;
    return (x->ord > y->ord) - (x->ord < y->ord);   /* stable: insertion order */
}

static int cmp_i32(const void *a, const void *b) {
    int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return (x > y) - (x < y);
}

static int64_t dict_find(const or_graph *g, int32_t u, int32_t e) {
    int64_t lo = g->doff[u], hi = g->doff[u + 1];
    while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        if (g->dkey[mid] < e) lo = mid + 1; else hi = mid;
    }
    if (lo < g->doff[u + 1] && g->dkey[lo] == e) return lo;
    return -1;
}

/* adjacency lists in insertion order: entries [in_off[u], in_off[u+1]) belong to u */
or_graph *or_graph_build(int32_t n_nodes, const int64_t *in_off, const int32_t *ngh,
                         const int32_t *eid, const double *ts) {
    or_graph *g = calloc(1, sizeof(or_graph));
    int64_t n = in_off[n_nodes];
    g->n_nodes = n_nodes; g->n_entries = n;
    g->off = malloc(sizeof(int64_t) * (n_nodes + 1));
    g->ngh = malloc(sizeof(int32_t) * (n ? n : 1));
    g->eid = malloc(sizeof(int32_t) * (n ? n : 1));
    g->ts = malloc(sizeof(double) * (n ? n : 1));
    g->doff = malloc(sizeof(int64_t) * (n_nodes + 1));
    g->dkey = malloc(sizeof(int32_t) * (n ? n : 1));
    g->dval = malloc(sizeof(int32_t) * (n ? n : 1));
    ent_t *tmp = malloc(sizeof(ent_t) * (n ? n : 1));
    int64_t dpos = 0;
    for (int32_t u = 0; u < n_nodes; ++u) {
        int64_t s = in_off[u], e = in_off[u + 1], d = e - s;
        g->off[u] = s;
        for (int64_t i = 0; i < d; ++i) {
            tmp[i].ts = ts[s + i]; tmp[i].ord = i; tmp[i].ngh = ngh[s + i]; tmp[i].eid = eid[s + i];
        }
        qsort(tmp, d, sizeof(ent_t), cmp_ent);
        for (int64_t i = 0; i < d; ++i) {
            g->ngh[s + i] = tmp[i].ngh; g->eid[s + i] = tmp[i].eid; g->ts[s + i] = tmp[i].ts;
        }
        /* unique sorted keys */
        g->doff[u] = dpos;
        for (int64_t i = 0; i < d; ++i) g->dkey[dpos + i] = g->eid[s + i];
        qsort(g->dkey + dpos, d, sizeof(int32_t), cmp_i32);
        int64_t m = 0;
        for (int64_t i = 0; i < d; ++i)
            if (m == 0 || g->dkey[dpos + m - 1] != g->dkey[dpos + i]) g->dkey[dpos + m++] = g->dkey[dpos + i];
        g->doff[u + 1] = dpos + m;
        /* simulate get_ts2idx (graph.py:77-101) literally */
        int32_t *tie = malloc(sizeof(int32_t) * (d + 2));
        int64_t ntie = 0;
        double last_ts = -1.0;
        int32_t last_e = -1;
        for (int64_t i = 0; i < d; ++i) {
            int32_t ei = g->eid[s + i];
            double ti = g->ts[s + i];
            g->dval[dict_find(g, u, ei)] = (int32_t)i;
            if (ti == last_ts) {
                if (ntie == 0) { tie[0] = last_e; tie[1] = ei; ntie = 2; }
                else tie[ntie++] = ei;
            }
            if (!(ti == last_ts) && ntie > 0) {
                for (int64_t j = 0; j < ntie; ++j) g->dval[dict_find(g, u, tie[j])] -= (int32_t)j;
                ntie = 0;
            }
            last_ts = ti; last_e = ei;
        }
        free(tie);
        dpos += m;
    }
    g->off[n_nodes] = n;
    free(tmp);
    return g;
}

void or_graph_free(or_graph *g) {
    if (!g) return;
    free(g->off); free(g->ngh); free(g->eid); free(g->ts); free(g->doff); free(g->dkey); free(g->dval);
    free(g->ets);
    free(g);
}

void or_graph_export(const or_graph *g, int64_t *off, int32_t *ngh, int32_t *eid, double *ts) {
    memcpy(off, g->off, sizeof(int64_t) * (g->n_nodes + 1));
    memcpy(ngh, g->ngh, sizeof(int32_t) * g->n_entries);
    memcpy(eid, g->eid, sizeof(int32_t) * g->n_entries);
    memcpy(ts, g->ts, sizeof(double) * g->n_entries);
}

static int64_t bisect_left(const double *a, int64_t n, double x) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        if (a[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* strict_temporal mode (SURVEY §7 opt-in; not in the reference): the slice of node u's list before edge e
 * is every record strictly earlier than e's own timestamp, bisect_left(ts_u, t(e)), instead of
 * get_ts2idx's trailing-tie value (graph.py:77-101); and a get_final_step lookup of an edge the node does
 * not hold (graph.py:357/:366 .get -> None -> the whole list, a future leak) is cut at t(e) too.
 * Requires one timestamp per edge id; returns -1 otherwise (nothing changed). */
int or_graph_set_strict(or_graph *g, int strict) {
    if (!strict) { g->strict = 0; return 0; }
    int32_t mx = 0;
    for (int64_t i = 0; i < g->n_entries; ++i) if (g->eid[i] > mx) mx = g->eid[i];
    double *ets = malloc(sizeof(double) * ((size_t)mx + 1));
    char *seen = calloc((size_t)mx + 1, 1);
    for (int64_t i = 0; i < g->n_entries; ++i) {
        int32_t e = g->eid[i];
        if (e < 0) continue;
        if (seen[e] && ets[e] != g->ts[i]) { free(ets); free(seen); return -1; }
        ets[e] = g->ts[i]; seen[e] = 1;
    }
    for (int32_t e = 0; e <= mx; ++e) if (!seen[e]) ets[e] = 0.0;
    free(seen);
    free(g->ets);
    g->ets = ets; g->max_eid = mx; g->strict = 1;
    return 0;
}

static double edge_ts(const or_graph *g, int32_t e) {
    return (e >= 0 && e <= g->max_eid) ? g->ets[e] : 0.0;
}

/* raw nodeedge2idx[u][e]; *found = 0 for None */
int32_t or_dict_raw(const or_graph *g, int32_t u, int32_t e, int32_t *found) {
    int64_t p = (u < 0 || u >= g->n_nodes) ? -1 : dict_find(g, u, e);
    *found = p >= 0;
    return p < 0 ? 0 : g->dval[p];
}

/* length of neighbors[:nodeedge2idx[u].get(e)], or -1 for None.  A dict value
 * can go negative (a self-loop inside a tie group is decremented twice,
 * graph.py:94-97); Python slicing then keeps deg + value entries. */
int32_t or_lookup(const or_graph *g, int32_t u, int32_t e) {
    int32_t found, v = or_dict_raw(g, u, e, &found);
    if (!found) return -1;
    if (g->strict) return (int32_t)bisect_left(g->ts + g->off[u], g->off[u + 1] - g->off[u], edge_ts(g, e));
    if (v < 0) {
        int64_t d = g->off[u + 1] - g->off[u] + v;
        v = d > 0 ? (int32_t)d : 0;
    }
    return v;
}

/* find_before (graph.py:103-146): returns cut length, or -1 (IndexError). */
int64_t or_find_before(const or_graph *g, int32_t u, double cut, int32_t e, int use_e) {
    int64_t s = g->off[u], d = g->off[u + 1] - s;
    if (!use_e) return bisect_left(g->ts + s, d, cut);
    if (!(u > 0)) return 0;
    int32_t p = or_lookup(g, u, e);
    return p < 0 ? -1 : p;
}

static int cmp_i64(const void *a, const void *b) {
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

/* find_k_hop (graph.py:233-262) for B target rows.  hop h outputs [B * N^h]
 * written at out_*[h] (row-major [B, N^h]).  Event of hop-h row r is
 * event_ids[r / N^(h-1)], row-in-event r % N^(h-1), stage h.
 * eidx == NULL -> hop 1 uses the time path.  Returns 0 or -1 (IndexError). */
int or_khop(const or_graph *g, or_rng rng, int32_t k, int32_t N, int32_t B, const int32_t *root,
            const double *cut, const int32_t *eidx, const uint32_t *event_ids,
            int32_t **out_node, int32_t **out_eid, float **out_ts) {
    int64_t rows = B, rpe = 1;
    int64_t *idx = malloc(sizeof(int64_t) * (N > 0 ? N : 1));
    const int32_t *rn = root, *re = eidx;
    const float *rt = NULL;
    int err = 0;
    for (int32_t h = 1; h <= k; ++h) {
        int32_t *on = out_node[h - 1], *oe = out_eid[h - 1];
        float *ot = out_ts[h - 1];
        for (int64_t r = 0; r < rows; ++r) {
            int32_t u = rn[r];
            int64_t c;
            if (h == 1) c = or_find_before(g, u, cut[r], re ? re[r] : 0, re != NULL);
            else c = or_find_before(g, u, (double)rt[r], re[r], 1);
            if (c < 0) { err = -1; c = 0; }
            for (int32_t j = 0; j < N; ++j) { on[r * N + j] = 0; oe[r * N + j] = 0; ot[r * N + j] = 0.f; }
            if (c == 0) continue;
            uint32_t ev = event_ids[r / rpe], rw = (uint32_t)(r % rpe);
            for (int32_t j = 0; j < N; ++j) idx[j] = draw(rng, (uint32_t)h, ev, rw, (uint32_t)j, c);
            qsort(idx, N, sizeof(int64_t), cmp_i64);
            int64_t s = g->off[u];
            for (int32_t j = 0; j < N; ++j) {
                on[r * N + j] = g->ngh[s + idx[j]];
                oe[r * N + j] = g->eid[s + idx[j]];
                ot[r * N + j] = (float)g->ts[s + idx[j]];
            }
        }
        rn = on; re = oe; rt = ot;
        rows *= N; rpe *= N;
    }
    free(idx);
    return err;
}

/* cut for get_final_step: nodeedge2idx[u].get(e) if u > 0 else 0, None -> whole list */
static int64_t final_cut(const or_graph *g, int32_t u, int32_t e) {
    if (!(u > 0)) return 0;
    int32_t p = or_lookup(g, u, e);
    if (p < 0 && g->strict) return bisect_left(g->ts + g->off[u], g->off[u + 1] - g->off[u], edge_ts(g, e));
    return p < 0 ? (g->off[u + 1] - g->off[u]) : p;
}

/* find_k_walks (graph.py:265-306) incl. get_next_step (:308-333) and get_final_step (:335-476).
 * h1_*: hop-1 results [B, N].  Outputs: node6 [B, W, 6], eid3 [B, W, 3], ts3 [B, W, 3],
 * anony [B, W, 3] with W = N * M. */
void or_walks(const or_graph *g, or_rng rng, int32_t N, int32_t M, int32_t B, const int32_t *root,
              const int32_t *h1_node, const int32_t *h1_eid, const float *h1_ts, const uint32_t *event_ids,
              int32_t *node6, int32_t *eid3, float *ts3, int32_t *anony) {
    int64_t W = (int64_t)N * M;
    int64_t *idx = malloc(sizeof(int64_t) * (M > 0 ? M : 1));
    for (int32_t b = 0; b < B; ++b) {
        uint32_t ev = event_ids[b];
        int32_t u = root[b];
        for (int32_t j = 0; j < N; ++j) {
            int32_t v1 = h1_node[b * N + j], e1 = h1_eid[b * N + j];
            float t1 = h1_ts[b * N + j];
            /* ---- step 2: find_before_walk([u, v1], e1) */
            int64_t cu = 0, cv = 0;
            if (u > 0) { int32_t p = or_lookup(g, u, e1); cu = p < 0 ? 0 : p; }
            if (v1 > 0) { int32_t p = or_lookup(g, v1, e1); cv = p < 0 ? 0 : p; }
            int64_t tot = cu + cv;
            int32_t s2[64], n2[64], ee2[64];
            float tt2[64];
            for (int32_t m = 0; m < M; ++m) { s2[m] = 0; n2[m] = 0; ee2[m] = 0; tt2[m] = 0.f; }
            if (tot > 0) {
                for (int32_t m = 0; m < M; ++m) idx[m] = draw(rng, 16, ev, (uint32_t)j, (uint32_t)m, tot);
                qsort(idx, M, sizeof(int64_t), cmp_i64);
                for (int32_t m = 0; m < M; ++m) {
                    int64_t x = idx[m], ent;
                    if (x < cu) { s2[m] = u; ent = g->off[u] + x; }
                    else { s2[m] = v1; ent = g->off[v1] + (x - cu); }
                    n2[m] = g->ngh[ent]; ee2[m] = g->eid[ent]; tt2[m] = (float)g->ts[ent];
                }
            }
            /* ---- step 3 per walk */
            for (int32_t m = 0; m < M; ++m) {
                int64_t w = (int64_t)j * M + m;
                int32_t src1 = u, tgt1 = v1, src2 = s2[m], tgt2 = n2[m], e2 = ee2[m];
                int32_t code, t = 0, o_src = 0, o_ngh = 0, o_e = 0;
                float o_t = 0.f;
                int32_t a_node, a_f1, a_f2, b_node, b_f;     /* list1: a_node filtered to {a_f1,a_f2}; list2: b_node filtered to b_f */
                int filt;
                if (src1 == src2 && tgt1 != tgt2) { code = 2; a_node = src1; a_f1 = tgt1; a_f2 = tgt2; b_node = tgt2; b_f = tgt1; filt = 1; }
                else if (tgt1 == src2 && src1 != tgt2) { code = 3; a_node = tgt1; a_f1 = src1; a_f2 = tgt2; b_node = tgt2; b_f = src1; filt = 1; }
                else { code = 1; a_node = tgt1; a_f1 = a_f2 = 0; b_node = tgt2; b_f = 0; filt = 0; }
                int64_t ca = final_cut(g, a_node, e2), cb = final_cut(g, b_node, e2);
                int64_t sa = g->off[a_node], sb = g->off[b_node];
                int64_t na = 0, nb = 0;
                if (filt) {
                    for (int64_t x = 0; x < ca; ++x) { int32_t y = g->ngh[sa + x]; na += (y == a_f1 || y == a_f2); }
                    for (int64_t x = 0; x < cb; ++x) nb += (g->ngh[sb + x] == b_f);
                } else { na = ca; nb = cb; }
                if (na + nb > 0) {
                    int64_t r = draw(rng, 17, ev, (uint32_t)w, 0, na + nb), ent = -1;
                    if (r < na) {
                        o_src = a_node;
                        if (filt) {
                            int64_t c = 0;
                            for (int64_t x = 0; x < ca; ++x) {
                                int32_t y = g->ngh[sa + x];
                                if (y == a_f1 || y == a_f2) { if (c == r) { ent = sa + x; break; } ++c; }
                            }
                        } else ent = sa + r;
                    } else {
                        int64_t rr = r - na;
                        o_src = b_node;
                        if (filt) {
                            int64_t c = 0;
                            for (int64_t x = 0; x < cb; ++x) {
                                if (g->ngh[sb + x] == b_f) { if (c == rr) { ent = sb + x; break; } ++c; }
                            }
                        } else ent = sb + rr;
                    }
                    o_ngh = g->ngh[ent]; o_e = g->eid[ent]; o_t = (float)g->ts[ent];
                    if (code == 2) {
                        if (o_src == src1 && o_ngh == tgt1) t = 1;
                        else if (o_src == src1 && o_ngh == tgt2) t = 2;
                        else if (o_src == tgt1 && o_ngh == tgt2) t = 3;
                        else t = 0;
                    } else if (code == 3) {
                        if (o_src == tgt1 && o_ngh == src1) t = 1;
                        else if (o_src == tgt1 && o_ngh == tgt2) t = 3;
                        else if (o_src == tgt2 && o_ngh == src1) t = 2;
                        else t = 0;
                    } else {
                        if (o_src == src1 && o_ngh != tgt1) t = 3;
                        else if (o_src == tgt1 && o_ngh != src1) t = 2;
                        else if (o_src == src1 && o_ngh == tgt1) t = 1;
                        else if (o_src == tgt1 && o_ngh == src1) t = 1;
                        else t = 0;
                    }
                }
                int64_t o = (int64_t)b * W + w;
                int32_t *nd = node6 + o * 6;
                nd[0] = o_src; nd[1] = o_ngh; nd[2] = src2; nd[3] = tgt2; nd[4] = src1; nd[5] = tgt1;
                eid3[o * 3 + 0] = o_e; eid3[o * 3 + 1] = e2; eid3[o * 3 + 2] = e1;
                ts3[o * 3 + 0] = o_t; ts3[o * 3 + 1] = tt2[m]; ts3[o * 3 + 2] = t1;
                anony[o * 3 + 0] = 1; anony[o * 3 + 1] = code; anony[o * 3 + 2] = t;
            }
        }
    }
    free(idx);
}

/* anony [1,x,t] -> category id in marginal's order (data_preprocess.py:171-178) */
int32_t or_cat(int32_t x, int32_t t) {
    static const int32_t c2[4] = {3, 0, 1, 2}, c3[4] = {7, 4, 6, 5}, c1[4] = {11, 10, 9, 8};
    if (t < 0 || t > 3) return -1;
    return x == 2 ? c2[t] : x == 3 ? c3[t] : x == 1 ? c1[t] : -1;
}

/* anony [1,x,t] -> null-model key - 1 (utils/null_model.py:90) */
int32_t or_null_bin(int32_t x, int32_t t) {
    static const int32_t n2[4] = {0, 1, 3, 2}, n3[4] = {4, 5, 7, 6}, n1[4] = {8, 9, 10, 11};
    if (t < 0 || t > 3) return -1;
    return x == 2 ? n2[t] : x == 3 ? n3[t] : x == 1 ? n1[t] : -1;
}

void or_cat_hist(const int32_t *anony, int64_t n, int32_t *cat, uint64_t *hist12, int null_order) {
    for (int64_t i = 0; i < n; ++i) {
        int32_t c = null_order ? or_null_bin(anony[i * 3 + 1], anony[i * 3 + 2])
                               : or_cat(anony[i * 3 + 1], anony[i * 3 + 2]);
        if (cat) cat[i] = c;
        if (hist12 && c >= 0) hist12[c]++;
    }
}

/* new_edge_info (data_preprocess.py:327-343): cnt[b,w,p,q] = #{w': eid[b,w',q] == eid[b,w,p]} */
void or_edge_counts(const int32_t *eid3, int32_t B, int32_t W, int32_t *cnt) {
    for (int32_t b = 0; b < B; ++b) {
        const int32_t *e = eid3 + (int64_t)b * W * 3;
        int32_t *o = cnt + (int64_t)b * W * 9;
        for (int32_t w = 0; w < W; ++w)
            for (int32_t p = 0; p < 3; ++p)
                for (int32_t q = 0; q < 3; ++q) {
                    int32_t c = 0, x = e[w * 3 + p];
                    for (int32_t w2 = 0; w2 < W; ++w2) c += (e[w2 * 3 + q] == x);
                    o[(w * 3 + p) * 3 + q] = c;
                }
    }
}

/* RandEdgeSampler.sample (batch_loader.py:39-42): dst_list[randint(len)] with key j=1 */
void or_neg_sample(uint64_t seed, uint32_t split, const int32_t *dst_list, int64_t n_dst,
                   const uint32_t *event_ids, int32_t B, int32_t *out) {
    or_rng g = {seed, split, 0};
    for (int32_t b = 0; b < B; ++b) out[b] = dst_list[draw(g, 32, event_ids[b], 0, 1, n_dst)];
}

/* ------------------------------------------------------------------ per-event pipeline
 * What data_preprocess.py:106-134 + marginal's cat + new_edge_info do for one target
 * event, for n_events events (OpenMP over events when n_threads > 1).  Used as the
 * "port" CPU baseline in bench.py and by the parity tests.
 * Outputs (per event e, side s in {src,tgt,bgd}):
 *   dst_fake [E]; sub1_* [E,3,N]; sub2_* [E,3,N*N]; walk node6 [E,3,W,6], eid3 [E,3,W,3],
 *   ts3 [E,3,W,3], cat [E,3,W]; cnt [E,3,W,3,3]; hist12 (cat order, summed). */
int or_event_pipeline(const or_graph *g, uint64_t seed, uint32_t split, int32_t N, int32_t M,
                      int32_t n_events, const int32_t *src, const int32_t *dst, const double *ts,
                      const int32_t *eidx, const uint32_t *event_ids, const int32_t *dst_list, int64_t n_dst,
                      int32_t *dst_fake, int32_t *sub1_node, int32_t *sub1_eid, float *sub1_ts,
                      int32_t *sub2_node, int32_t *sub2_eid, float *sub2_ts,
                      int32_t *node6, int32_t *eid3, float *ts3, int32_t *cat, int32_t *cnt,
                      uint64_t *hist12, int n_threads) {
    int64_t W = (int64_t)N * M, NN = (int64_t)N * N;
    int err = 0;
    uint64_t hist[12] = {0};
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 4) reduction(| : err)
#endif
    for (int32_t e = 0; e < n_events; ++e) {
        uint32_t ev = event_ids[e];
        int32_t fake;
        or_neg_sample(seed, split, dst_list, n_dst, &ev, 1, &fake);
        dst_fake[e] = fake;
        int32_t roots[3] = {src[e], dst[e], fake};
        int32_t anony[64 * 64 * 3];
        for (int s = 0; s < 3; ++s) {
            or_rng g3 = {seed, split, (uint32_t)(s + 1)};
            int64_t o1 = ((int64_t)e * 3 + s) * N, o2 = ((int64_t)e * 3 + s) * NN, ow = ((int64_t)e * 3 + s) * W;
            int32_t *on[2] = {sub1_node + o1, sub2_node + o2}, *oe[2] = {sub1_eid + o1, sub2_eid + o2};
            float *ot[2] = {sub1_ts + o1, sub2_ts + o2};
            int rc = or_khop(g, g3, 2, N, 1, &roots[s], &ts[e], s < 2 ? &eidx[e] : NULL, &ev, on, oe, ot);
            if (rc) err |= 1;
            or_walks(g, g3, N, M, 1, &roots[s], on[0], oe[0], ot[0], &ev, node6 + ow * 6, eid3 + ow * 3,
                     ts3 + ow * 3, W <= 64 * 64 ? anony : NULL);
            uint64_t h[12] = {0};
            or_cat_hist(anony, W, cat + ow, h, 0);
            for (int c = 0; c < 12; ++c) {
#ifdef _OPENMP
#pragma omp atomic
#endif
                hist[c] += h[c];
            }
            or_edge_counts(eid3 + ow * 3, 1, (int32_t)W, cnt + ow * 9);
        }
    }
    for (int c = 0; c < 12; ++c) hist12[c] += hist[c];
    return err ? -1 : 0;
}
