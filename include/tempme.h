/* tempme.h -- C ABI of libtempme_hip.so, the MI355X (gfx950) TempME explanation hot path.
 *
 * Plain pointers and sizes only; no torch types.  All sampling/encoder entry points
 * take DEVICE pointers and a hipStream_t (passed as void*, NULL = default stream) and
 * are stream-ordered and asynchronous.  Graph build/export and weight creation take
 * HOST pointers.  Every entry point returns TM_OK (0) or a negative TM_E_* code;
 * tm_last_error() gives the message (thread-local).  No C++ exception crosses the ABI.
 *
 * Keyed-RNG contract (replaces the reference's unseeded np.random.randint, see
 * oracle/philox.py):  key = (seed lo, seed hi); counter = (event, split<<16 | side<<8 |
 * stage, row, j>>2); word j&3 of Philox4x32-10; draw(high) = (u32 * high) >> 32.
 *
 * The reference interface each entry point replaces is cited as file:line in
 * dharunm236/TempME.
 */
#ifndef TEMPME_H_
#define TEMPME_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TM_OK 0
#define TM_E_EDGE_NOT_IN_LIST (-1) /* IndexError, utils/graph.py:134-135 */
#define TM_E_SHAPE (-2)            /* assert, utils/graph.py:127, :317, :378; explainer_new.py:180 */
#define TM_E_HIP (-3)              /* HIP runtime failure */
#define TM_E_ARG (-4)              /* bad argument (NULL pointer, negative size, ...) */
#define TM_E_UNSUPPORTED (-5)      /* input outside what the build supports (message says what) */

/* sides and stages of the RNG contract */
#define TM_SIDE_NONE 0
#define TM_SIDE_SRC 1
#define TM_SIDE_TGT 2
#define TM_SIDE_BGD 3
#define TM_STAGE_STEP2 16
#define TM_STAGE_STEP3 17
#define TM_STAGE_NEG 32
#define TM_STAGE_PERM 48
#define TM_SPLIT_TRAIN 0
#define TM_SPLIT_TEST 1
#define TM_SPLIT_NULL 2

typedef struct tm_graph tm_graph;     /* opaque, immutable after build; device-resident */
typedef struct tm_weights tm_weights; /* opaque, packed encoder weights on one device */
typedef struct tm_dropin tm_dropin;   /* opaque, drop-in eval context: side streams, staging ring, workspaces */

typedef struct {
    uint64_t seed;
    uint32_t split;
    uint32_t side;
} tm_rng;

const char *tm_last_error(void);
int tm_version(void);

/* Test / diagnostic options, process-wide, all 0 (off) in the product path -- the library reads no environment
 * variables.  TM_DEBUG_FORCE_UNKEYED: the samplers' two-compare rank kernels on any graph (tests compare them with
 * the keyed one-compare kernels); TM_DEBUG_HOST_BUILD: tm_graph_build_edges on the host builder (tests compare it
 * with the device builder); TM_DEBUG_GRAPH_TIMING: the graph build's phase times on stderr. */
#define TM_DEBUG_FORCE_UNKEYED 1
#define TM_DEBUG_HOST_BUILD 2
#define TM_DEBUG_GRAPH_TIMING 3
#define TM_DEBUG_WALK_BLOCKS 4   /* > 0: cap the persistent walk kernel's grid at this many workgroups (A/B tools) */
#define TM_DEBUG_N_OPTS 5
int tm_debug_set(int32_t opt, int32_t value);
/* Threads of the host-side graph builder (0 = the CPUs this process may run on, at most 64). */
int tm_set_host_threads(int32_t n);

/* ---------------------------------------------------------------- graph (host inputs)
 * Replaces NeighborFinder.__init__ / init_off_set / get_ts2idx (utils/graph.py:13-101).
 * Adjacency lists in insertion order, owner-major: entries [in_off[u], in_off[u+1]) are
 * node u's (ngh, eid, ts) triples in the order the caller appended them
 * (temp_exp_main.py:135-144).  The build stable-sorts every list by ts, simulates
 * get_ts2idx (trailing-tie quirk included) and uploads the CSR to `device`. */
int tm_graph_build(int32_t n_nodes, const int64_t *in_off, const int32_t *ngh, const int32_t *eid,
                   const double *ts, int device, tm_graph **out);
/* The same from raw edge rows (src, dst, e_idx, ts as int64/int64/int64/f64 arrays of n_edges):
 * (dst, e, t) is appended to src's list, then (src, e, t) to dst's, row by row -- the adj_list
 * construction of temp_exp_main.py:135-144 -- by a stable counting sort, then tm_graph_build. */
int tm_graph_build_edges(int32_t n_nodes, int64_t n_edges, const int64_t *src, const int64_t *dst,
                         const int64_t *eidx, const double *ts, int device, tm_graph **out);
int tm_graph_free(tm_graph *g);
int tm_graph_info(const tm_graph *g, int32_t *n_nodes, int64_t *n_entries, int32_t *max_eid);
/* host copy of node_idx_l / edge_idx_l / node_ts_l / off_set_l (utils/graph.py:23-27) and
 * per-entry nodeedge2idx[owner][eid] raw value (may be negative, see get_ts2idx). */
int tm_graph_export(const tm_graph *g, int64_t *off, int32_t *ngh, int32_t *eid, double *ts, int32_t *dict_val);
/* strict_temporal view (SURVEY §7/§8(b) opt-in; the reference has no such mode -- its NeighborFinder is
 * parity mode, which every other entry point reproduces).  The view shares g's device buffers and
 * differs in two lookups: an e_idx slice of node u is bisect_left(ts_u, t(e)) -- every record strictly
 * earlier than the edge -- instead of get_ts2idx's trailing-tie value (utils/graph.py:77-101), and
 * get_final_step's lookup of an edge u does not hold cuts at t(e) instead of taking u's whole list
 * (graph.py:357/:366, a future leak).  Pass the view wherever a tm_graph is taken (tm_sample_khop,
 * tm_sample_walks, tm_sample_events).  TM_E_UNSUPPORTED when an edge id carries more than one timestamp.
 * Free the view (tm_graph_free) before g; export/info of a view report g's CSR. */
int tm_graph_strict_view(const tm_graph *g, tm_graph **out);

/* ---------------------------------------------------------------- sampling (device)
 * find_k_hop (utils/graph.py:233-262) + get_temporal_neighbor (:197-231) for B rows.
 * Hop h (1..k) writes B*N^h entries at offset sum_{i<h} B*N^i of out_*; hop-h row r belongs
 * to event event_ids[r / N^(h-1)], row-in-event r % N^(h-1), RNG stage h.
 * eidx == NULL: hop 1 uses the time path (bisect_left on ts, :129); otherwise the
 * e_idx path (:133); hops >= 2 always use the e_idx path (:247-250).
 * *err_flag (device int32, may be NULL) is set to TM_E_EDGE_NOT_IN_LIST on a missing e_idx. */
int tm_sample_khop(const tm_graph *g, tm_rng rng, int32_t k, int32_t N, int32_t B, const int32_t *root,
                   const double *cut, const int32_t *eidx, const uint32_t *event_ids, int32_t *out_node,
                   int32_t *out_eid, float *out_ts, int32_t *err_flag, void *stream);

/* find_k_walks (utils/graph.py:265-306) = get_next_step (:308-333) + get_final_step (:335-476).
 * h1_*: hop-1 results [B, N]; W = N*M walks per row.  Outputs node6 [B,W,6] = [s3,t3,s2,t2,s1,t1],
 * eid3 [B,W,3] = [e3,e2,e1], ts3 [B,W,3], anony3 [B,W,3] (nullable), cat [B,W] (nullable,
 * marginal's category id, processed/data_preprocess.py:171-178). */
int tm_sample_walks(const tm_graph *g, tm_rng rng, int32_t N, int32_t M, int32_t B, const int32_t *root,
                    const int32_t *h1_node, const int32_t *h1_eid, const float *h1_ts, const uint32_t *event_ids,
                    int32_t *out_node6, int32_t *out_eid3, float *out_ts3, int32_t *out_anony3, int32_t *out_cat,
                    void *stream);

/* RandEdgeSampler.sample (utils/batch_loader.py:39-42): out[i] = list[draw(stage NEG, event_ids[i], row 0,
 * draw j)]; j = 0 is the src draw (:40), j = 1 the dst draw (:41).  rng.side is ignored (NONE). */
int tm_neg_sample(tm_rng rng, const int32_t *list, int64_t n_list, const uint32_t *event_ids, int32_t n, int32_t j,
                  int32_t *out, void *stream);

/* Sort keys of the keyed permutation that replaces np.random.permutation(n) in
 * load_data_shuffle (utils/null_model.py:23): out_keys[i] = Philox word 0 of counter
 * (i, split<<16 | STAGE_PERM, 0, 0); the permutation is the stable argsort of the keys. */
int tm_perm_keys(uint64_t seed, uint32_t split, int64_t n, uint32_t *out_keys, void *stream);

/* Motif histogram over n walks' anony codes [n,3].  null_order=0: marginal's category order
 * (data_preprocess.py:171-193); 1: null-model key order (utils/null_model.py:90, key-1).
 * hist12 (device u64[12]) is accumulated into (zero it first).  out_cat nullable. */
int tm_motif_hist(const int32_t *anony3, int64_t n, int32_t null_order, int32_t *out_cat,
                  unsigned long long *hist12, void *stream);

/* new_edge_info (data_preprocess.py:327-343): cnt[g,w,p,q] = #{w' : eid3[g,w',q] == eid3[g,w,p]}. */
int tm_edge_counts(const int32_t *eid3, int32_t n_groups, int32_t W, float *out_cnt, void *stream);

/* Fused per-target-event sampler: what data_preprocess.py:106-134 + marginal's category id +
 * new_edge_info do, for n_events events and all three sides (src, tgt, bgd) in one launch.
 * Outputs are side-major: sub1_* [3,E,N], sub2_* [3,E,N*N], node6 [3,E,W,6], eid3 [3,E,W,3],
 * ts3 [3,E,W,3], cat [3,E,W], cnt [3,E,W,3,3] (f32), dst_fake [E]; hist12 accumulates the
 * category histogram (device u64[12], marginal order).  Bit-identical to the separate calls. */
int tm_sample_events(const tm_graph *g, uint64_t seed, uint32_t split, int32_t N, int32_t M, int32_t n_events,
                     const int32_t *src, const int32_t *dst, const double *ts, const int32_t *eidx,
                     const uint32_t *event_ids, const int32_t *dst_list, int64_t n_dst, int32_t *dst_fake,
                     int32_t *sub1_node, int32_t *sub1_eid, float *sub1_ts, int32_t *sub2_node, int32_t *sub2_eid,
                     float *sub2_ts, int32_t *node6, int32_t *eid3, float *ts3, int32_t *cat, float *cnt,
                     unsigned long long *hist12, int32_t *err_flag, void *stream);

/* Batch slice of a device-resident pack (utils/batch_loader.py get_item / get_item_edge,
 * :203-242): for each job, dst[side][r] = src[side][rows[r]] (row_bytes per row, a multiple of 4;
 * side strides in bytes; rows[r] checked against src_rows, *err_flag (nullable) set if outside).
 * Up to 24 jobs in one launch. */
typedef struct {
    const void *src;
    void *dst;
    int64_t row_bytes, src_side_stride, dst_side_stride, src_rows;
    int32_t sides, reserved;
} tm_gather_job;
int tm_gather_rows(const tm_gather_job *jobs, int32_t n_jobs, const int64_t *rows, int64_t n_rows, int32_t *err_flag,
                   void *stream);

/* ---------------------------------------------------------------- encoder (device)
 * Weights: the 28 fp32 tensors of TempME (models/explainer_new.py:103-171), row-major as
 * nn.Linear stores them, in this order (DEVICE pointers):
 *   0/1 event_conv.lin_event.{weight,bias}   2/3 event_conv.MLP.0   4/5 event_conv.MLP.2
 *   6/7 attention.W1   8/9 attention.W2   10/11 attention.MLP.0   12/13 attention.MLP.3
 *   14/15 MLP.0   16/17 MLP.3   18/19 MLP.5   20/21 edge_dependency_gcn.0   22/23 .3   24/25 .6
 *   26 time_encoder.basis_freq   27 time_encoder.phase
 * de = edge feature dim, dn = node feature dim (= time dim), h = hid_dim (a multiple of 16 up to 256;
 * the fused register-resident walk kernel covers h = 64 with the category feature, every other shape
 * runs the LDS-tiled kernels).  if_cat = if_cat_feature (explainer_new.py:121-125): 0 -> MLP.0 / MLP.3
 * take h inputs (no one-hot category), tensors 14/15/16 shaped accordingly.
 * Replaces the weights of TempME.__init__ (models/explainer_new.py:103-171; the reference keeps them as
 * nn.Linear modules and calls them per forward). */
#define TM_N_WEIGHTS 28
int tm_weights_create(int32_t de, int32_t dn, int32_t h, int device, tm_weights **out);   /* if_cat = 1 */
int tm_weights_create_ex(int32_t de, int32_t dn, int32_t h, int32_t if_cat, int device, tm_weights **out);
int tm_weights_pack(tm_weights *w, const float *const *tensors, void *stream);
/* TempME constructor variants for the eval kernels (explainer_new.py:103-105, :121, :141-145, :367):
 * temporal_guidance = 0 -> the plain Attention (scores not time-weighted; the batch std is not needed),
 * dependency_gate = 0 -> no dependency gate in retrieve_edge_imp_node (walk importance used as is).
 * Defaults 1, 1.  The training kernels support the defaults only. */
int tm_weights_variant(tm_weights *w, int32_t temporal_guidance, int32_t dependency_gate);
/* The node-feature table the caller passes to the eval encoder calls is all zeros (the TGN-format datasets
 * Enron, UCI, Wikipedia, Reddit and USLegis ship zero node features).  event_gcn's two branches
 * (explainer_new.py:93-96, src + relu(tgt + event) and tgt + relu(src + event)) are then the same expression of
 * the event projection, bit for bit, and tm_encoder_fwd_tab computes one of them and reads no node row.  The
 * caller re-asserts it whenever the table changes; 0 (the default) makes no assumption. */
int tm_weights_set_node_zero(tm_weights *w, int32_t node_zero);
/* A process-wide stamp of the weights' packed state: every create / pack / variant / node-zero change takes
 * the next value of one global counter (never 0), so a cache keyed on it can never confuse two weight states,
 * even of two objects allocated at the same address.  Caches of per-edge-id tables (tm_edge_tables) key on it. */
uint64_t tm_weights_version(const tm_weights *w);
int tm_weights_free(tm_weights *w);

/* Workspace bytes tm_encoder_fwd needs for n_walks walks. */
int64_t tm_encoder_workspace_bytes(const tm_weights *w, int64_t n_walks);

/* TempME.forward (explainer_new.py:174-201), eval, for n_groups groups of B*W walks each
 * (one group = one reference call: one side of one batch; the attention's time std is
 * batch-global per group, :828).  Walk arrays are [G,B,W,...]; cut [G,B] (f64, event time);
 * cnt [G,B,W,3,3] f32.  out_imp [G,B,W] (graphlet importance, sigmoid output).
 * M = walks per hop-1 slot as find_k_walks lays them out (walks w and w' share position 2 iff
 * w/M == w'/M, graph.py:283-289); position 2 is then encoded once per slot.  M = 1 is always safe. */
int tm_encoder_fwd(const tm_weights *w, const float *n_feat, const float *e_feat, int32_t n_groups, int32_t B,
                   int32_t W, int32_t M, const int32_t *node6, const int32_t *eid3, const float *ts3,
                   const int32_t *cat, const double *cut, const float *cnt, void *workspace, float *out_imp,
                   void *stream);

/* tm_encoder_fwd with lin_event's edge-feature product taken from a per-edge-id table (etab from
 * tm_edge_tables, [n_ids][tm_edge_table_cols] f32; every eid3 entry must be < n_ids): the
 * event_conv linear (explainer_new.py:79-96) over [E(e) | cnt | cos] is split as
 * W[:, :de] E(e) (table) + W[:, de:] [cnt | cos] (walk kernel), a re-association of the same sum
 * (outputs within the 1e-5 contract, not bit-identical to tm_encoder_fwd).  etab = NULL is
 * tm_encoder_fwd; TM_E_UNSUPPORTED if the encoder dims have no table mode (tm_edge_table_cols == 0). */
int tm_encoder_fwd_tab(const tm_weights *w, const float *n_feat, const float *e_feat, const float *etab,
                       int32_t n_groups, int32_t B, int32_t W, int32_t M, const int32_t *node6, const int32_t *eid3,
                       const float *ts3, const int32_t *cat, const double *cut, const float *cnt, void *workspace,
                       float *out_imp, void *stream);

/* ---------------------------------------------------------------- encoder training (device)
 * Training forward of TempME.forward (explainer_new.py:174-201) with dropout active: drop (nullable
 * = eval) holds uint8 keep-masks [n_walks][DC], DC = (2 + h + hm) rounded up to 16 (144 for the
 * default h = 64, hm = h + 12 with the category feature, hm = h without): columns 0..1 the attention
 * weights alpha (:839), the next h attention.MLP's hidden layer (:780), the next hm MLP's hidden layer
 * (:122); kept values are scaled by drop_scale = 1/(1-p).  With use_temporal_guidance=False (the plain
 * Attention, :12-43, no dropout) the first 2 + h columns are ignored.  `workspace`
 * (tm_encoder_workspace_bytes) keeps the event_gcn outputs F for tm_encoder_bwd.  Replaces the autograd
 * forward of temp_exp_main.py:605-607.  Every constructor variant (tm_weights_create_ex /
 * tm_weights_variant) whose dims tm_encoder_train_supported accepts. */
int tm_encoder_train_supported(int32_t de, int32_t dn, int32_t hid_dim, int32_t if_cat_feature);
int tm_encoder_train_fwd(const tm_weights *w, const float *n_feat, const float *e_feat, int32_t n_groups, int32_t B,
                         int32_t W, const int32_t *node6, const int32_t *eid3, const float *ts3, const int32_t *cat,
                         const double *cut, const float *cnt, const uint8_t *drop, float drop_scale, void *workspace,
                         float *out_imp, void *stream);

/* Buffers of tm_encoder_bwd (caller-allocated device memory; n = n_walks, R = 3n walk positions,
 * KE = kev rounded up to 16 (kev = de + 3 + dn), DN = dn rounded up to 16).  Shapes below for the
 * default hid_dim h = 64 with the category feature: in general 64 -> h, 128 -> 2h, 76 -> hm and
 * 80 -> KM = hm rounded up to 16.  Each layer's
 * (d pre-activation, input) row pair is written so the weight gradients are dW = dY^T X over all rows
 * and the bias gradients sum(dY) (the caller runs those GEMMs / reductions).  Padding columns are 0. */
typedef struct {
    float *imp;    /* [n] recomputed forward output (nullable) */
    float *dlogit; /* [n]            MLP.5:       dW = dlogit^T M2 */
    float *M2;     /* [n][64] */
    float *dM2;    /* [n][64]        MLP.3:       dW = dM2^T M1d[:, :76] */
    float *M1d;    /* [n][80] */
    float *dM1;    /* [n][80]        MLP.0:       dW = dM1[:, :76]^T X[:, :76] */
    float *X;      /* [n][80] */
    float *dY2;    /* [n][64]        attention.MLP.3: dW = dY2^T H1d */
    float *H1d;    /* [n][64] */
    float *dH1;    /* [n][64]        attention.MLP.0: dW = dH1^T O */
    float *O;      /* [n][128] */
    float *dP;     /* [n][128]       attention.W1: dW = dP^T F[:, 2] */
    float *dQ;     /* [2][n][128]    attention.W2: dW = dQ[0]^T F[:, 0] + dQ[1]^T F[:, 1] */
    float *dF;     /* [n][3][128]    d event_gcn outputs */
    float *ev;     /* [R][KE]        lin_event:   dW = dlev[:, :dn]^T ev[:, :kev] */
    float *AB;     /* [R][2][DN]     event_conv.MLP.0: dW = dZ^T AB (2R rows) */
    float *H;      /* [R][2][64]     event_conv.MLP.2: dW = dF^T H (2R rows of 64) */
    float *dZ;     /* [R][2][64] */
    float *dlev;   /* [R][DN] */
    float *g;      /* [R][DN]        time encoder: d phase = sum_rows g, d basis_freq = dt^T g */
    float *dt;     /* [R] */
} tm_encoder_grad_io;

/* Backward of tm_encoder_train_fwd given d_imp [n] = dL/d out_imp, with the same inputs, masks and
 * workspace: recomputes each tile's forward and writes the buffers above. */
int tm_encoder_bwd(const tm_weights *w, const float *n_feat, const float *e_feat, int32_t n_groups, int32_t B,
                   int32_t W, const int32_t *node6, const int32_t *eid3, const float *ts3, const int32_t *cat,
                   const double *cut, const float *cnt, const uint8_t *drop, float drop_scale, const void *workspace,
                   const float *d_imp, const tm_encoder_grad_io *io, void *stream);

/* Weight gradients of the encoder from tm_encoder_bwd's buffers (io, same n_groups/B/W) and the
 * training forward's workspace: grads = 22 DEVICE pointers, written (not accumulated), in the tm_weights
 * order without the dependency gate: lin_event w/b, event_conv.MLP.0 w/b, .MLP.2 w/b, attention.W1 w/b,
 * .W2 w/b, .MLP.0 w/b, .MLP.3 w/b, MLP.0 w/b, MLP.3 w/b, MLP.5 w/b, time_encoder.basis_freq, .phase.
 * dW = dY^T X over all rows, computed as per-chunk MFMA partials plus one fixed-order reduce
 * (deterministic). */
#define TM_N_ENC_GRADS 22
int tm_encoder_wgrad(const tm_weights *w, int32_t n_groups, int32_t B, int32_t W, const tm_encoder_grad_io *io,
                     const void *workspace, float *const *grads, void *stream);

/* Generic weight-gradient reduction (the launches tm_encoder_wgrad uses): job j contributes
 * dY_j^T X_j over its R rows (dY [R][ldy] with O used columns, X [R][ldx] with I used columns);
 * target t writes w [O][I] = the sum over jobs first_job .. first_job+n_jobs-1 (same O, I) and
 * b [O] = the column sums of their dY.  Deterministic (fixed-order chunk reduction). */
typedef struct {
    const float *dy, *x;
    int32_t ldy, ldx, O, I, R;
} tm_wgrad_job;
typedef struct {
    float *w, *b;
    int32_t first_job, n_jobs;
} tm_wgrad_target;
int tm_wgrad(const tm_wgrad_job *jobs, int32_t n_jobs, const tm_wgrad_target *targets, int32_t n_targets,
             void *stream);

/* retrieve_edge_imp_node in training (explainer_new.py:354-406 with dropout in the dependency gate,
 * :367-386) up to the gathered scatter-max values: p1 [G,B,N] and p2 [G,B,N^2] are the per-edge maxima
 * of imp * (0.5 + 0.5 sigmoid(gate)) gathered at the subgraph edge ids BEFORE beta_sample and the
 * padding mask (the caller applies those, :395-404).  keep1 [R][64] / keep2 [R][32] (R = G*B*3W walk
 * positions; nullable = eval) are the keep-masks of the gate's Dropout(1.5p) and Dropout(p), kept
 * values scaled by scale1 / scale2.  io receives the activations the backward needs. */
typedef struct {
    float *X;      /* [R][KD] gate input [E[e] | cos(t w + phi)], KD = de + dn rounded up to 16 */
    float *G1;     /* [R][64] dropout(relu(edge_dependency_gcn.0 X)) */
    float *G2;     /* [R][32] dropout(relu(edge_dependency_gcn.3 G1)) */
    float *z;      /* [R]     gate logit (edge_dependency_gcn.6 G2) */
    float *gate;   /* [R]     0.5 + 0.5 sigmoid(z) */
    float *d_gate; /* [R]     backward: dL/d gate */
    float *dz;     /* [R]     backward: .6:  dW = dz^T G2 */
    float *dG2;    /* [R][32] backward: .3:  dW = dG2^T G1 */
    float *dG1;    /* [R][64] backward: .0:  dW = dG1^T X[:, :de+dn] */
    float *g;      /* [R][DN] backward: time encoder: d phase = sum g, d basis_freq = t^T g */
    float *t;      /* [R]     walk event times (f32) */
} tm_explain_grad_io;
int tm_explain_train_fwd(const tm_weights *w, const float *e_feat, int32_t n_groups, int32_t B, int32_t W, int32_t N,
                         const int32_t *eid3, const float *ts3, const float *imp, const int32_t *sub1_eid,
                         const int32_t *sub2_eid, const uint8_t *keep1, const uint8_t *keep2, float scale1,
                         float scale2, const tm_explain_grad_io *io, float *p1, float *p2, void *stream);
/* tm_explain_train_fwd plus the padding mask of explainer_new.py:400-404 as factors: pad1 [G,B,N] / pad2
 * [G,B,N^2] = 0 where sub1_node / sub2_node is 0, else 1 (beta_sample's output times the mask = the
 * reference's masked_fill). */
int tm_explain_train_fwd_pad(const tm_weights *w, const float *e_feat, int32_t n_groups, int32_t B, int32_t W,
                             int32_t N, const int32_t *eid3, const float *ts3, const float *imp, const int32_t *sub1_eid,
                             const int32_t *sub2_eid, const uint8_t *keep1, const uint8_t *keep2, float scale1,
                             float scale2, const tm_explain_grad_io *io, float *p1, float *p2, const int32_t *sub1_node,
                             const int32_t *sub2_node, float *pad1, float *pad2, void *stream);
/* Backward given dp1 / dp2: d_imp [G,B,W] (the scatter-max gradient is split evenly among tied walk
 * positions, as torch's scatter_reduce amax backward does) and the gate's weight gradients
 * grads = 8 DEVICE pointers: edge_dependency_gcn.0 w/b, .3 w/b, .6 w/b, time_encoder.basis_freq, .phase
 * (written, not accumulated). */
int tm_explain_train_bwd(const tm_weights *w, int32_t n_groups, int32_t B, int32_t W, int32_t N, const int32_t *eid3,
                         const float *ts3, const float *imp, const int32_t *sub1_eid, const int32_t *sub2_eid,
                         const uint8_t *keep1, const uint8_t *keep2, float scale1, float scale2, const float *dp1,
                         const float *dp2, const tm_explain_grad_io *io, float *d_imp, float *const *grads,
                         void *stream);

/* kl_loss, prior='empirical' (explainer_new.py:432-448) of n_groups groups (one reference call each:
 * prob [G,B,W] graphlet importance, cat [G,B,W] category ids 0..11, null12 the null vector in key order,
 * target the prior): partial [G*B] = each event's share of its group's loss (the step's KL term is
 * their sum) and dprob [G,B,W] = d(sum over groups)/d prob, clamp included.  fp64 inside. */
int tm_kl_loss(const float *prob, const int32_t *cat, const float *null12, float target, int32_t n_groups, int32_t B,
               int32_t W, float *partial, float *dprob, void *stream);

/* beta_sample(p, training=True) (explainer_new.py:420-430) around torch's own Dirichlet sampler and its
 * gradient: tm_beta_params writes conc [n,2] = (clamp(10p, min=1), clamp(10(1-p), min=1)) and total [n,2]
 * = their sum (the inputs of torch._sample_dirichlet / torch._dirichlet_grad); tm_beta_rsample_bwd gives dp
 * [n] from g = d(x[:,0] * pad), the sample x [n,2] and d = torch._dirichlet_grad(x, conc, total) -- the
 * same fp32 operations as torch's autograd graph of Beta(...).rsample() * pad. */
int tm_beta_params(const float *p, int64_t n, float *conc, float *total, void *stream);
int tm_beta_rsample_bwd(const float *g, const float *pad, const float *x, const float *d, const float *p, int64_t n,
                        float *dp, void *stream);

/* Host arrays read in place by the GPU: the drop-in's host-pack path (the reference's eval loop hands
 * TempME.forward / retrieve_explanation float64 / int64 numpy views of its load_subgraph_margin pack and
 * np.load edge array per batch, utils/batch_loader.py:119-242, temp_exp_main.py:441-453).
 * tm_host_register pins and maps [ptr, ptr + bytes) (page-rounded; the caller keeps the memory alive until
 * tm_host_unregister(ptr)) and returns the device address of ptr; tm_stage_cast runs up to 16 jobs in one
 * launch, each gathering an ndim <= 5 strided view (byte strides) of src (a device-accessible address: device
 * memory or a registered host array's device address) into dst contiguous, converting its type (C conversions:
 * truncation toward zero for integers, round to nearest for float32 -- numpy's astype / torch's .to).
 * bound > 0 (int32 destinations: row indices of a table with `bound` rows) clamps each value into [0, bound):
 * a guard for ids the caller validated once per array (values in range are unchanged), so a pack rewritten
 * after that check can never make a later kernel read outside the table. */
#define TM_I32 1
#define TM_F32 2
#define TM_I64 3
#define TM_F64 4
typedef struct tm_stage_job {
    const void *src;
    void *dst;
    int32_t src_type, dst_type, ndim, bound;
    int64_t shape[5];
    int64_t stride[5];   /* bytes */
} tm_stage_job;
int tm_host_register(void *ptr, int64_t bytes, void **dev_ptr);
int tm_host_unregister(void *ptr);
int tm_stage_cast(const tm_stage_job *jobs, int32_t n_jobs, void *stream);

/* The explainer's optimizer step (temp_exp_main.py:631-632: torch.optim.Adam, amsgrad off) in ONE launch over a
 * flat fp32 bucket of n parameters and their gradients (the four buffers at one offset within 16 bytes, so a span of
 * a larger bucket works): exp_avg / exp_avg_sq updated in place,
 * g = grad * grad_scale (+ weight_decay * param), bias corrections from the device step count `step` (the count
 * before this step; a launch with advance != 0 advances it -- the last of a step's launches when a step updates
 * several spans --, so a captured HIP graph replays correctly) and `done`, a device uint32 that must be 0 before the
 * first launch (the kernel leaves it 0).  Replaces torch.optim.Adam.step /
 * torch's fused Adam over the explainer's parameters (tempme_amd/optim.py FusedAdam). */
int tm_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, float lr, float beta1,
                 float beta2, float eps, float weight_decay, float grad_scale, float *step, uint32_t *done,
                 int32_t advance, void *stream);
/* Up to 32 fp32 copies in one launch (dst[0:n) = src[0:n) per job): the parameters' gradients, as autograd
 * produced them, into the flat bucket tm_adam_step and the gradient all-reduce read. */
typedef struct tm_copy_job {
    const float *src;
    float *dst;
    int64_t n;
} tm_copy_job;
int tm_copy_many(const tm_copy_job *jobs, int32_t n_jobs, void *stream);

/* retrieve_edge_imp_node, eval (explainer_new.py:354-406, :420-430) for each of the G*B
 * (group, event) rows: dependency gate, walk->edge scatter-max, gather at the subgraph eids,
 * Beta mean, node==0 mask.  sub1_* [G,B,N], sub2_* [G,B,N*N]; out_h1 [G,B,N], out_h2 [G,B,N*N]
 * (= the [3B,N] / [3B,N^2] of retrieve_explanation when G = the 3 sides of one batch). */
int tm_edge_importance(const tm_weights *w, const float *e_feat, int32_t n_groups, int32_t B, int32_t W, int32_t N,
                       const int32_t *eid3, const float *ts3, const float *imp, const int32_t *sub1_node,
                       const int32_t *sub1_eid, const int32_t *sub2_node, const int32_t *sub2_eid, float *out_h1,
                       float *out_h2, void *stream);

/* Drop-in eval context for the reference's per-side TempME.forward calls (temp_exp_main.py:446-453):
 * three side streams, a device ring for the cut times (host values sent as kernel arguments),
 * per-stream encoder workspaces. */
int tm_dropin_create(int32_t device, tm_dropin **out);
void tm_dropin_free(tm_dropin *d);
/* Use the caller's stream as side stream k (0..2) -- e.g. a torch stream, so that the caller's allocator
 * can hand out a call's outputs from that stream's pool -- instead of the context's own. */
int tm_dropin_set_stream(tm_dropin *d, int32_t k, void *stream);
/* A per-edge-id cache of the dependency-gate factor for edge ids [0, n_edge_rows) (the edge-feature table's
 * rows; 0 = none): tm_dropin_forward's out_gfac then reads the factor of every walk position whose (edge id,
 * fp32 time) was computed before and computes only the others (explainer_new.py:367-386 is a function of
 * (E[e], t) alone: the results are bit-identical).  Emptied whenever the weights (tm_weights_pack /
 * _variant / _set_node_zero: tm_weights_version changes) or the edge-feature table's address change; a
 * caller that rewrites the table IN PLACE calls tm_dropin_gate_cache_clear. */
int tm_dropin_gate_cache(tm_dropin *d, int64_t n_edge_rows);
int tm_dropin_gate_cache_clear(tm_dropin *d);
/* TempME.forward (explainer_new.py:174-201) for one call (B events x W walks) in one library call on side
 * stream k: with sync != 0 every side stream first waits (once) for `stream` (weights / tables prepared
 * there, or a device cut tensor); the cut times come from the host (cut_host, sent as kernel arguments;
 * an array equal to the previous call's is not sent again) or the device (cut_dev); std + encoder run
 * there (tm_encoder_fwd_tab, M = 1, etab as there), and with out_gfac non-NULL the dependency-gate
 * factor 0.5 + 0.5 * gate of every walk position [B, W, 3] (explainer_new.py:367-386) follows; `stream`
 * then waits for the side stream.  out_imp [B*W] and out_gfac must be allocated on side stream k (or be
 * otherwise free of pending work on other streams). */
int tm_dropin_forward(tm_dropin *d, int32_t k, int32_t sync, const tm_weights *w, const float *n_feat,
                      const float *e_feat, const float *etab, int32_t B, int32_t W, const int32_t *node6,
                      const int32_t *eid3, const float *ts3, const int32_t *cat, const double *cut_host,
                      const double *cut_dev, const float *cnt, float *out_imp, float *out_gfac, void *stream);
/* tm_edge_importance from the gate factors of tm_dropin_forward (walk_imp = imp * gfac, the same
 * roundings as tm_edge_importance): bit-identical outputs. */
int tm_edge_importance_gf(const float *gfac, int32_t n_groups, int32_t B, int32_t W, int32_t N, const int32_t *eid3,
                          const float *imp, const int32_t *sub1_node, const int32_t *sub1_eid,
                          const int32_t *sub2_node, const int32_t *sub2_eid, float *out_h1, float *out_h2,
                          void *stream);

/* tm_edge_importance_gf for the three sides of one batch in one launch (retrieve_explanation,
 * explainer_new.py:408-418): side s's gate factors / walk edge ids / graphlet importance / subgraph
 * records at their own addresses (B events each), outputs concatenated: out_h1 [3B, N], out_h2 [3B, N^2]. */
int tm_edge_importance_gf3(int32_t B, int32_t W, int32_t N, const float *gf0, const float *gf1, const float *gf2,
                           const int32_t *e0, const int32_t *e1, const int32_t *e2, const float *i0, const float *i1,
                           const float *i2, const int32_t *n10, const int32_t *n11, const int32_t *n12,
                           const int32_t *x10, const int32_t *x11, const int32_t *x12, const int32_t *n20,
                           const int32_t *n21, const int32_t *n22, const int32_t *x20, const int32_t *x21,
                           const int32_t *x22, float *out_h1, float *out_h2, void *stream);
/* retrieve_explanation(training=True) (explainer_new.py:408-418 with beta_sample's rsample branch :420-430,
 * as eval_one_epoch calls it under --if_bern, temp_exp_main.py:450-453): the same three-side launch, but
 * out_p1 / out_p2 receive the gathered maxima p (before the Beta draw) and keep_h1 / keep_h2 the padding
 * mask (0 where the subgraph node is 0, else 1); the caller draws Beta(max(10p,1), max(10(1-p),1)) and
 * multiplies by keep (= masked_fill(node == 0, 0)). */
int tm_edge_importance_gf3_bern(int32_t B, int32_t W, int32_t N, const float *gf0, const float *gf1, const float *gf2,
                                const int32_t *e0, const int32_t *e1, const int32_t *e2, const float *i0,
                                const float *i1, const float *i2, const int32_t *n10, const int32_t *n11,
                                const int32_t *n12, const int32_t *x10, const int32_t *x11, const int32_t *x12,
                                const int32_t *n20, const int32_t *n21, const int32_t *n22, const int32_t *x20,
                                const int32_t *x21, const int32_t *x22, float *out_p1, float *out_p2, float *keep_h1,
                                float *keep_h2, void *stream);

/* Dependency-gate table (explainer_new.py:367-386 evaluated once per edge id): out_gf[e] =
 * 0.5 + 0.5*sigmoid(depMLP([e_feat[e] | cos(t_e * basis_freq + phase)])) for e in [0, max_eid],
 * t_e the edge's timestamp in g (as f32).  TM_E_UNSUPPORTED if an edge id carries several
 * timestamps in g (then use tm_edge_importance). */
int tm_edge_gate_table(const tm_weights *w, const tm_graph *g, const float *e_feat, float *out_gf, void *stream);

/* Row width of the walk kernel's edge table for these encoder dims (176), or 0 if it has none. */
int tm_edge_table_cols(const tm_weights *w);

/* tm_edge_gate_table plus (out_etab non-NULL) the edge table of tm_encoder_fwd_tab, in one launch
 * over the edge ids [0, max_eid]: out_etab[e][k] = sum_{j < de} lin_event.W[k][j] * e_feat[e][j]
 * (k < dn; columns dn..cols-1 are 0).  out_etab [max_eid + 1][tm_edge_table_cols(w)]. */
int tm_edge_tables(const tm_weights *w, const tm_graph *g, const float *e_feat, float *out_gf, float *out_etab,
                   void *stream);

/* The edge table alone, without a graph (the drop-in TempME.forward's table mode): out_etab [n_ids][cols]
 * for the edge ids [0, n_ids) of the edge-feature table e_feat [n_ids][de]; same values as tm_edge_tables'.
 * Replaces the per-position E(e) product of explainer_new.py:79-96 (event_conv.lin_event). */
int tm_edge_feature_table(const tm_weights *w, const float *e_feat, int32_t n_ids, float *out_etab, void *stream);

/* tm_edge_importance driven by a gate table (n_ids entries): bit-identical outputs, no per-walk
 * gate MLP.  *err_flag (nullable) is set if a walk edge id is outside the table. */
int tm_edge_importance_tab(const float *gf, int32_t n_ids, int32_t n_groups, int32_t B, int32_t W, int32_t N,
                           const int32_t *eid3, const float *imp, const int32_t *sub1_node, const int32_t *sub1_eid,
                           const int32_t *sub2_node, const int32_t *sub2_eid, float *out_h1, float *out_h2,
                           int32_t *err_flag, void *stream);

/* ---------------------------------------------------------------- TGN base model (consumer of the path)
 * One temporal-attention layer of the base TGN's embedding_update_layer
 * (TGN/modules/embedding_module.py:356-393 -> TemporalAttentionLayer :181-216 ->
 * MultiHeadAttention :52-86 -> ScaledDotProductAttention :16-32), the part that touches every
 * neighbour: per source row r and head h
 *     s_j = (qf[r,h] . key[r,j]) / temperature,   s_j = -1e10 where mask_node[m,j] == 0
 *     z[r,h] = sum_j softmax(s)_j * ew[m,j] * key[r,j]
 * with key[r,j] = [node feature (d_node) | edge feature (d_edge) | cos(dt[r,j]*time_w + time_b) (d_time)]
 * built on the fly (never materialised) and m = (r*n_head + h) % rows when head_major_rows
 * (the reference pairs rows with mask/explain-weight rows through .repeat(n_head,1,1),
 * embedding_module.py:74-75 and :211-212), else m = r.
 * The caller supplies qf[r,h] = (W_k,h^T W_q,h) query[r] and applies (fc W_v,h) to z: the
 * per-neighbour key/value projections of the reference fold into one per-row projection on each
 * side (same result up to fp32 reassociation; DESIGN.md "TGN contrast"). */
typedef struct {
    int32_t rows, n_ngh, n_head;
    int32_t d_node, d_edge, d_time;       /* d_key = d_node + d_edge + d_time <= 512 */
    int32_t node_rows, edge_rows;         /* table sizes when gathered (index checks) */
    int32_t head_major_rows;              /* 1 = the reference's row pairing (see above) */
    int32_t seg_rows;                     /* > 0: rows are independent batches of seg_rows rows and the
                                             pairing runs inside each (m = base + ((r-base)*n_head+h) % seg) */
    float temperature;                    /* sqrt(d_key), embedding_module.py:51 */
    const float *node_tab;                /* node_idx != NULL: [node_rows, d_node] table; else dense [rows*n_ngh, d_node] */
    const int32_t *node_idx;              /* [rows*n_ngh] or NULL */
    const float *edge_tab;                /* edge_idx != NULL: [edge_rows, d_edge] table; else dense [rows*n_ngh, d_edge] */
    const int32_t *edge_idx;              /* [rows*n_ngh] or NULL */
    const float *dt;                      /* [rows*n_ngh] time deltas (f32, as the reference casts them) */
    const float *time_w, *time_b;         /* [d_time] TimeEncode Linear(1, d) weight and bias */
    const int32_t *mask_node;             /* [rows*n_ngh]; 0 = padding (masked) */
    const float *ew;                      /* [rows*n_ngh] explanation weights or NULL (= 1) */
    const float *qf;                      /* [rows, n_head*d_key] folded queries */
    int32_t *err_flag;                    /* nullable device flag: set to TM_E_ARG on an out-of-range index */
} tm_tgn_attn;

/* forward: z [rows, n_head*d_key], stats [rows, n_head, 2] (softmax max and sum, for the backward) */
int tm_tgn_attn_fwd(const tm_tgn_attn *a, float *z, float *stats, void *stream);
/* backward given gz = dL/dz: d_ew_parts [rows*n_head, n_ngh] holds the contribution of pair
 * q = r*n_head + h to d ew[m(q), j] (the caller sums the n_head contributions of each row);
 * d_node (nullable; dense node_tab only) [rows*n_ngh, d_node] = dL/d node feature. */
int tm_tgn_attn_bwd(const tm_tgn_attn *a, const float *stats, const float *gz, float *d_ew_parts, float *d_node,
                    void *stream);

/* threshold_test masking (temp_exp_main.py:153-181, tgn branch): for group g and row r,
 * sel = torch.topk(imp[r], k_of_group[g], largest=False).indices as the reference computes it on the
 * CPU -- the index set std::nth_element (or std::partial_sort when 64*k <= n) leaves in front of
 * the (value, index) pairs, ATen TopKImpl.h, so ties resolve exactly as there -- and
 * node_out[g, r, :] = node_in[r, :] with node_out[g, r, sel] = 0 (np.put_along_axis(..., 0)).
 * imp [rows, n] f32, node_in [rows, n] int32, node_out [n_groups, rows, n]; n <= 4096. */
int tm_mask_least_important(const float *imp, int32_t rows, int32_t n, const int32_t *k_of_group, int32_t n_groups,
                            const int32_t *node_in, int32_t *node_out, void *stream);

/* ---------------------------------------------------------------- per-kernel timing
 * tm_profile_enable(1) clears and starts recording a HIP event pair around every kernel
 * launch, on that launch's stream; tm_profile_sync() waits and aggregates, returning the
 * number of kernel names; tm_profile_entry(i) gives name, total ms and launch count. */
int tm_profile_enable(int on);
int tm_profile_sync(void);
int tm_profile_entry(int i, const char **name, double *total_ms, int64_t *count);

/* ---------------------------------------------------------------- base GraphMixer (f4)
 * GraphMixer.compute_node_temporal_embeddings (GM/graphmixer.py:142-193) for R rows (roots) up to the
 * output layer: x_mean [R, C] = the masked token mean of the mixed features (:176-178) and node_out
 * [R, D] = the softmax-weighted neighbour-feature mean plus the root's features (:181-189).  The
 * output layer (Linear(C + D, D)) and MergeLayer score are plain GEMMs on [x_mean | node_out].
 * Explanation weights ew [R, N] (hop-1, NULL: none) are applied as the reference does (input and
 * both branch outputs of every mixer, the token mean, the neighbour mean).  Eval semantics (dropout =
 * identity).  Limits: N <= 32, HT <= 16, L <= 4, C <= 256. */
typedef struct {
    int32_t R, N, C, T, D, L, HT, HC; /* rows, tokens (= n_neighbors), channels (edge dim), time dim, node
                                         dim, mixer layers, token-FFN hidden, channel-FFN hidden */
    const int32_t *node;      /* [R] root node ids */
    const int32_t *nid, *eid; /* [R, N] hop-1 neighbour ids / edge ids (eid unused with edge_attr) */
    const double *cut, *ts;   /* [R] cut times, [R, N] neighbour times */
    const float *ew;          /* [R, N] explanation weights or NULL */
    const float *edge_attr;   /* [R, N, C] or NULL (then e_feat[eid], zeroed on padding neighbours) */
    const float *n_feat;      /* [V, D] */
    const float *e_feat;      /* [E, C] */
    const float *time_w, *time_b; /* [T] TimeEncoder Linear(1, T) weight and bias */
    const float *proj_w;      /* projection_layer.weight [C, C+T] packed by tm_gm_pack */
    const float *proj_b;      /* [C] */
    /* DEVICE array of L x 12 pointers, per mixer: token_norm w/b [N], token ffn.0 w [HT,N] / b, ffn.3 w
       [N,HT] / b, channel_norm w/b [C], channel ffn.0 w [HC,C] packed / b [HC], ffn.3 w [C,HC] packed / b */
    const float *const *layer_table;
    float *x_mean, *node_out; /* outputs */
} tm_gm_embed_args;
/* floats of tm_gm_pack's output for a [n_out, k] weight */
int64_t tm_gm_packed_floats(int32_t n_out, int32_t k);
/* W [n_out, k] row-major (nn.Linear.weight) -> MFMA B-operand fragments */
int tm_gm_pack(const float *w, int32_t n_out, int32_t k, float *packed, void *stream);
int tm_gm_embed(const tm_gm_embed_args *a, void *stream);
/* Backward of tm_gm_embed with respect to the explanation weights (the explainer's training signal through a
 * frozen base GraphMixer, temp_exp_main.py:614-632 with base_type 'graphmixer'; GM/graphmixer.py:142-193,
 * :273-315): d_ew [R, N] from d_x_mean [R, C] and d_node_out [R, D]; zero on padding neighbours.  `a` as for
 * tm_gm_embed with a->ew set, every weight pack by tm_gm_pack (B-operand fragments), and layer_table holding
 * L x 14 pointers: tm_gm_embed's 12, then channel ffn.3 transposed ([HC, C]) and ffn.0 transposed
 * ([C, HC]), both packed by tm_gm_pack.  x_mean / node_out unused.  No parameter gradients. */
int tm_gm_embed_bwd_ok(int32_t N, int32_t C, int32_t T, int32_t L, int32_t HT);
int tm_gm_embed_bwd(const tm_gm_embed_args *a, const float *d_x_mean, const float *d_node_out, float *d_ew,
                    void *stream);
/* 1 when tm_gm_embed runs the register-resident kernel for these dims (C % 4 == 0, T % 4 == 0, N <= 32,
 * C <= 256); its weights are then packed by tm_gm_pack_a instead of tm_gm_pack: proj_w with
 * (n_mult, k_mult) = (1, 4), channel ffn.0 with (2, 1), ffn.3 with (1, 2) */
int tm_gm_fused_ok(int32_t N, int32_t C, int32_t T, int32_t HC);
/* floats of tm_gm_pack_a's output: 16-row / 16-column tiles rounded up to multiples of n_mult / k_mult */
int64_t tm_gm_packed_a_floats(int32_t n_out, int32_t k, int32_t n_mult, int32_t k_mult);
/* W [n_out, k] row-major -> MFMA A-operand fragments (weights as the 16-output-row operand) */
int tm_gm_pack_a(const float *w, int32_t n_out, int32_t k, int32_t n_mult, int32_t k_mult, float *packed, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* TEMPME_H_ */
