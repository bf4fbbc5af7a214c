"""Device-resident explanation scoring of many target events per launch.

One call = what temp_exp_main.py's eval loop does per batch for ``E / B`` batches of
``B`` events (sampling as data_preprocess.py:106-134, TempME.forward x3,
retrieve_explanation(training=False)), without host round trips:

    tm_sample_events        fake dst, 2-hop subgraphs x3, walks x3, categories, edge counts
    tm_edge_tables          per edge id: the dependency gate and lin_event's edge-feature product
                            (EdgeTables: built once per weight state -- tm_weights_version -- edge-feature
                            table and graph, not per call; an eval epoch's weights do not change)
    tm_encoder_fwd_tab      graphlet importance for the 3 * E/B groups (one std per group)
    tm_edge_importance_tab  explanation weights hop-1 [3, E, N] and hop-2 [3, E, N^2]

Outputs are side-major: rows [s, b*B:(b+1)*B] of batch b are the reference's
``retrieve_explanation`` rows [s*B:(s+1)*B].
"""
import time

import torch

from . import _lib as L
from .preprocess import EventBuffers, sample_events


class EdgeTables:
    """The per-edge-id tables of one (explainer, graph): the dependency-gate factor of every edge id
    (retrieve_edge_imp_node's depMLP, explainer_new.py:367-386: a function of (E[e], t_e) and the gate
    weights alone) and lin_event's edge-feature product (event_gcn, :79-96: a function of E[e] and
    lin_event's weights alone).  Both are pure functions of (weight state, edge-feature table, the graph's
    edge timestamps), so they are built once per key -- tm_weights_version (a process-wide stamp taken by
    every repack / variant / node-zero change), the edge-feature table's identity and version, the graph
    handle -- and reused by every call until one of them changes.  The reference recomputes the gate per
    walk position per batch; the values are the same (tests compare against the per-call build bitwise).

    Streams: a build is recorded with an event; a call on another stream waits for it once."""

    def __init__(self, explainer, graph, edge_table=True):
        self.ex, self.graph, self.dev = explainer, graph, graph.device
        n = graph.max_eid + 1
        self.gf = torch.empty(n, dtype=torch.float32, device=self.dev)
        cols = L.lib().tm_edge_table_cols(explainer.packed_weights()) if edge_table else 0
        self.etab = torch.empty((n, cols), dtype=torch.float32, device=self.dev) if cols else None
        self.key = None
        self.builds = 0
        self.build_ms = None           # host-timed duration of the last build (synchronised; see build())
        self._ready = None
        self._waited = set()

    def _key(self):
        w = self.ex.packed_weights()
        _, et = self.ex.feature_tables()
        fn = getattr(L.lib(), "tm_weights_version", None)    # absent in an older A/B build (TEMPME_LIB)
        ver = int(fn(w)) if fn is not None else (w.value, self.ex._packed_key)
        return (ver, et.data_ptr(), getattr(self.ex, "_tables_key", None), self.graph.handle.value)

    def build(self, timed=False):
        """Rebuild on the current stream (one tm_edge_tables launch over every edge id); ``timed`` measures
        it alone (synchronising before and after) for the bench's ``aux.edge_tables_ms``."""
        w = self.ex.packed_weights()
        _, et = self.ex.feature_tables()
        st = torch.cuda.current_stream(self.dev)
        if timed:
            torch.cuda.synchronize(self.dev)
            t0 = time.perf_counter()
        L.check(L.lib().tm_edge_tables(w, self.graph.handle, L.ptr(et), L.ptr(self.gf), L.ptr(self.etab),
                                       st.cuda_stream), "tm_edge_tables")
        if timed:
            torch.cuda.synchronize(self.dev)
            self.build_ms = (time.perf_counter() - t0) * 1e3
        self.key = self._key()
        self.builds += 1
        self._ready = torch.cuda.Event()
        self._ready.record(st)
        self._waited = {st.cuda_stream}

    def ensure(self):
        """The tables for the current weights on the current stream: built if stale, else (once per build and
        stream) the stream waits for the build."""
        if self.key != self._key():
            self.build()
            return
        st = torch.cuda.current_stream(self.dev)
        if st.cuda_stream not in self._waited:
            st.wait_event(self._ready)
            self._waited.add(st.cuda_stream)


class ExplainPipeline:
    def __init__(self, explainer, graph, dst_list, N, M=3, B=100, seed=0, split=L.SPLIT_TEST, edge_table=True,
                 tables=None):
        """``edge_table=False`` keeps lin_event's edge-feature product inside the walk kernel
        (tm_encoder_fwd, bit-identical to the drop-in TempME.forward) instead of reading it from the
        per-edge-id table (a re-association of the same sum, within the 1e-5 contract).  ``tables``: an
        EdgeTables shared with other pipelines of the same explainer and graph."""
        self.ex = explainer
        self.edge_table = bool(edge_table)
        self.graph = graph
        self.tabs = tables if tables is not None else EdgeTables(explainer, graph, edge_table)
        self.dev = graph.device
        self.dst_list = dst_list.to(self.dev, torch.int32).contiguous()
        self.N, self.M, self.B, self.W = int(N), int(M), int(B), int(N) * int(M)
        self.seed, self.split = int(seed), int(split)
        self._E = None

    def _alloc(self, E):
        if self._E == E:
            return
        dev, W, N = self.dev, self.W, self.N
        self.buf = EventBuffers(E, N, self.M, dev)
        n_walks = 3 * E * W
        self.imp = torch.empty(max(n_walks, 1), dtype=torch.float32, device=dev)
        nbytes = L.lib().tm_encoder_workspace_bytes(self.ex.packed_weights(), n_walks)
        self.ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self.h1 = torch.empty(max(3 * E * N, 1), dtype=torch.float32, device=dev)
        self.h2 = torch.empty(max(3 * E * N * N, 1), dtype=torch.float32, device=dev)
        self._E = E

    @property
    def gf(self):
        return self.tabs.gf

    @property
    def etab(self):
        return self.tabs.etab

    def sample(self, src, dst, ts, eidx, event_ids):
        self._alloc(int(src.numel()))
        return sample_events(self.graph, self.seed, self.split, self.N, self.M, src, dst, ts, eidx, event_ids,
                             self.dst_list, out=self.buf, check=False)

    def encode(self, ts):
        E, B, W = self._E, self.B, self.W
        assert E % B == 0, "events per call must be a multiple of the batch size"
        G = 3 * (E // B)
        b = self.buf
        cut = ts.repeat(3).contiguous()
        self.ex.encoder_fwd(b.node6, b.eid3, b.ts3, b.cat, cut, b.cnt, G, B, W, out=self.imp, workspace=self.ws,
                            M=self.M, etab=self.etab)
        return self.imp

    def tables(self, rebuild=False):
        """Per edge id of the graph: the dependency gate (retrieve_edge_imp_node's depMLP,
        explainer_new.py:367-386) and, when the encoder has a table mode, lin_event's edge-feature product
        (event_gcn, :79-96) -- one launch, the edge features read once; rebuilt only when the weights, the
        edge-feature table or the graph changed (EdgeTables), or when ``rebuild``."""
        if rebuild:
            self.tabs.build()
        else:
            self.tabs.ensure()

    def explain(self):
        """retrieve_explanation(training=False) for all groups: the table-driven scatter-max / gather /
        Beta-mean / mask kernel (gate table from ``tables``)."""
        E, B, W, N = self._E, self.B, self.W, self.N
        G = 3 * (E // B)
        b = self.buf
        dev = self.dev
        L.check(L.lib().tm_edge_importance_tab(L.ptr(self.gf), self.gf.numel(), G, B, W, N, L.ptr(b.eid3),
                                               L.ptr(self.imp), L.ptr(b.sub1_node), L.ptr(b.sub1_eid),
                                               L.ptr(b.sub2_node), L.ptr(b.sub2_eid), L.ptr(self.h1), L.ptr(self.h2),
                                               L.ptr(b.err), L.stream_ptr(dev)), "tm_edge_importance_tab")
        return self.h1, self.h2

    def run(self, src, dst, ts, eidx, event_ids):
        """Returns (imp [3,E,W], hop-1 weights [3,E,N], hop-2 weights [3,E,N^2]) device tensors."""
        self.sample(src, dst, ts, eidx, event_ids)
        self.tables()
        self.encode(ts)
        self.explain()
        E, N, W = self._E, self.N, self.W
        return self.imp[:3 * E * W].view(3, E, W), self.h1[:3 * E * N].view(3, E, N), \
            self.h2[:3 * E * N * N].view(3, E, N * N)

    def check_errors(self):
        if getattr(self, "buf", None) is not None:   # nothing sampled yet: nothing to report
            L.raise_device_error(int(self.buf.err.item()), "ExplainPipeline")


class PipelinedExplainer:
    """``depth`` ExplainPipelines in flight on ``depth`` streams (call k on stream k % depth, each
    with its own buffers), for a serving loop over many calls: call k+1's sampling overlaps call k's
    encoder kernel, and call k's explanation overlaps call k+1's encoder.  The encoders themselves
    are chained by an event (each waits for the previous call's encoder) so they never share the
    GPU with each other: the MFMA-bound kernel keeps the whole chip, the latency-bound sampling and
    explanation kernels run in its shadow.

    ``submit`` returns the call's (imp, hop-1, hop-2) device tensors and the stream they are produced
    on (a pipeline stream, not the caller's: ``torch.cuda.current_stream().wait_stream(stream)``
    before using them there); they are overwritten by call k + depth, so consume them first."""

    def __init__(self, explainer, graph, dst_list, N, M=3, B=100, seed=0, split=L.SPLIT_TEST, depth=2,
                 edge_table=True, chain_encoders=True):
        dev = graph.device
        self.depth = max(1, int(depth))
        tabs = EdgeTables(explainer, graph, edge_table)
        self.pipes = [ExplainPipeline(explainer, graph, dst_list, N, M, B, seed, split, edge_table, tables=tabs)
                      for _ in range(self.depth)]
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(self.depth)]
        self._k = 0
        self._enc_done = None
        # chain_encoders=False: call k+1's encoder may start while call k's runs -- its persistent workgroups take
        # the CU slots call k's release at the end of its grid (the walk kernel holds every slot until then)
        self.chain = bool(chain_encoders)

    def submit(self, src, dst, ts, eidx, event_ids):
        i = self._k % self.depth
        p, st = self.pipes[i], self.streams[i]
        ready = torch.cuda.Event()                      # the inputs, produced on the caller's stream
        ready.record(torch.cuda.current_stream(st.device))
        with torch.cuda.stream(st):
            st.wait_event(ready)
            p.sample(src, dst, ts, eidx, event_ids)
            p.tables()
            if self.chain and self._enc_done is not None:
                st.wait_event(self._enc_done)
            p.encode(ts)
            self._enc_done = torch.cuda.Event()
            self._enc_done.record(st)
            p.explain()
        self._k += 1
        E, N, W = p._E, p.N, p.W
        return (p.imp[:3 * E * W].view(3, E, W), p.h1[:3 * E * N].view(3, E, N),
                p.h2[:3 * E * N * N].view(3, E, N * N)), st

    def check_errors(self):
        for p in self.pipes:
            p.check_errors()
