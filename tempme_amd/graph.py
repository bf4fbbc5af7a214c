"""Drop-in ``NeighborFinder`` (utils/graph.py:12) backed by the device-resident CSR of
libtempme_hip.so.

Same constructor, same public attributes (``node_idx_l``, ``node_ts_l``,
``edge_idx_l``, ``off_set_l``, ``nodeedge2idx``), same ``find_before``,
``get_temporal_neighbor``, ``find_k_hop`` and ``find_k_walks`` signatures, return
types and dtypes (int32 nodes/edge ids, float32 times) and the same exceptions
(``IndexError`` for an e_idx missing from its node's list, graph.py:134-135).

Randomness: the reference draws from the unseeded global NumPy RandomState; here
every draw is keyed (Philox4x32-10, include/tempme.h) by ``(seed, split, event,
side, stage, row, j)``.  ``find_k_hop`` / ``find_k_walks`` take optional keyword
arguments ``event_ids`` (one id per target row) and ``side``; without them each
call consumes fresh event ids from a per-finder counter.
"""
import ctypes as C
import math

import numpy as np
import torch

from . import _lib as L

PRECISION = 5


def adjacency_from_edges(src, dst, eidx, ts, n_nodes):
    """Owner-major, insertion-ordered adjacency exactly as temp_exp_main.py:135-144 builds
    ``adj_list``: for every edge row (dst, e, t) is appended to src's list, then (src, e, t)
    to dst's.  Returns (in_off [V+1] int64, ngh int32, eid int32, ts float64)."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    owner = np.stack([src, dst], 1).reshape(-1)
    ngh = np.stack([dst, src], 1).reshape(-1)
    e = np.repeat(np.asarray(eidx, dtype=np.int64), 2)
    t = np.repeat(np.asarray(ts, dtype=np.float64), 2)
    order = np.argsort(owner, kind="stable")
    off = np.zeros(n_nodes + 1, dtype=np.int64)
    np.add.at(off, owner + 1, 1)
    return np.cumsum(off), ngh[order].astype(np.int32), e[order].astype(np.int32), t[order]


def _flatten_adj(adj_list):
    lens = np.fromiter((len(x) for x in adj_list), dtype=np.int64, count=len(adj_list))
    off = np.zeros(len(adj_list) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    n = int(off[-1])
    ngh = np.empty(n, np.int32)
    eid = np.empty(n, np.int32)
    ts = np.empty(n, np.float64)
    k = 0
    for lst in adj_list:
        for (a, e, t) in lst:
            ngh[k] = a
            eid[k] = e
            ts[k] = t
            k += 1
    return off, ngh, eid, ts


class DeviceGraph:
    """Owns one ``tm_graph`` handle (CSR + e_idx table + block search trees on one device)."""

    def __init__(self, in_off, ngh, eid, ts, device=None, *, _edges=None):
        self.device = L.require_device(device)
        h = C.c_void_p()
        if _edges is not None:
            # edge rows: the owner-major adjacency is built by the library (counting sort, C++)
            src, dst, e, t, n_nodes = _edges
            src = np.ascontiguousarray(src, np.int64)
            dst = np.ascontiguousarray(dst, np.int64)
            e = np.ascontiguousarray(e, np.int64)
            t = np.ascontiguousarray(t, np.float64)
            self.n_nodes = int(n_nodes)
            L.check(L.lib().tm_graph_build_edges(self.n_nodes, len(src), src.ctypes.data, dst.ctypes.data,
                                                 e.ctypes.data, t.ctypes.data, self.device.index, C.byref(h)),
                    "tm_graph_build_edges")
        else:
            in_off = np.ascontiguousarray(in_off, np.int64)
            ngh = np.ascontiguousarray(ngh, np.int32)
            eid = np.ascontiguousarray(eid, np.int32)
            ts = np.ascontiguousarray(ts, np.float64)
            self.n_nodes = len(in_off) - 1
            L.check(L.lib().tm_graph_build(self.n_nodes, in_off.ctypes.data, ngh.ctypes.data, eid.ctypes.data,
                                           ts.ctypes.data, self.device.index, C.byref(h)), "tm_graph_build")
        self.handle = h
        n_nodes, n_ent, max_eid = C.c_int32(), C.c_int64(), C.c_int32()
        L.check(L.lib().tm_graph_info(h, C.byref(n_nodes), C.byref(n_ent), C.byref(max_eid)), "tm_graph_info")
        self.n_entries = n_ent.value
        self.max_eid = max_eid.value

    def export(self):
        n = max(self.n_entries, 1)
        off = np.zeros(self.n_nodes + 1, np.int64)
        ngh, eid, dv = np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n, np.int32)
        ts = np.zeros(n, np.float64)
        L.check(L.lib().tm_graph_export(self.handle, off.ctypes.data, ngh.ctypes.data, eid.ctypes.data,
                                        ts.ctypes.data, dv.ctypes.data), "tm_graph_export")
        m = self.n_entries
        return off, ngh[:m], eid[:m], ts[:m], dv[:m]

    def strict_view(self):
        """strict_temporal view (tm_graph_strict_view): the same device CSR with slice lengths
        bisect_left(ts_u, t(e)) and no get_final_step future leak (SURVEY §7 opt-in)."""
        return _StrictGraph(self)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and L._lib is not None:
            L._lib.tm_graph_free(h)
            self.handle = None


class _StrictGraph(DeviceGraph):
    """A ``tm_graph`` view sharing ``parent``'s buffers (held here, so the view is freed first)."""

    def __init__(self, parent):
        self.parent = parent
        self.device = parent.device
        self.n_nodes, self.n_entries, self.max_eid = parent.n_nodes, parent.n_entries, parent.max_eid
        h = C.c_void_p()
        L.check(L.lib().tm_graph_strict_view(parent.handle, C.byref(h)), "tm_graph_strict_view")
        self.handle = h


class NeighborFinder:
    def __init__(self, adj_list, bias=0, ts_precision=PRECISION, use_cache=False, sample_method="multinomial",
                 device=None, *, seed=0, split=L.SPLIT_TEST, strict_temporal=False, _flat=None, _edges=None):
        """graph.py:13-27.  strict_temporal=True (not in the reference, off by default) fixes two of its
        temporal quirks: an e_idx slice keeps exactly the records strictly earlier than the edge (no
        trailing-tie get_ts2idx value, graph.py:77-101), and get_final_step's None lookup cuts at the
        edge's time instead of taking the whole list (graph.py:357/:366)."""
        if not math.isclose(bias, 0) or sample_method != "multinomial":
            # graph.py:219-227 (bias != 0, 'binary') are unreachable from every reference caller
            raise NotImplementedError("only bias=0, sample_method='multinomial' (the reference's only live path)")
        self.bias = bias
        self.ts_precision = ts_precision
        self.use_cache = use_cache
        self.sample_method = sample_method
        self.seed = int(seed)
        self.split = int(split)
        self._next_event = 0
        if _edges is not None:
            self.graph = DeviceGraph(None, None, None, None, device, _edges=_edges)
        else:
            off, ngh, eid, ts = _flat if _flat is not None else _flatten_adj(adj_list)
            self.graph = DeviceGraph(off, ngh, eid, ts, device)
        self.strict_temporal = bool(strict_temporal)
        if self.strict_temporal:
            self.graph = self.graph.strict_view()
        self.device = self.graph.device
        self._host = None
        self._ne2i = None

    # host copies of the CSR (graph.py:23-27), exported on first use: the sampling kernels never need them
    def _export(self):
        if self._host is None:
            o, n, e, t, dv = self.graph.export()
            self._host = (o, n.astype(np.int64), e.astype(np.int64), t, dv)
        return self._host

    off_set_l = property(lambda self: self._export()[0])
    node_idx_l = property(lambda self: self._export()[1])
    edge_idx_l = property(lambda self: self._export()[2])
    node_ts_l = property(lambda self: self._export()[3])
    _dict_val = property(lambda self: self._export()[4])

    @classmethod
    def from_edges(cls, src, dst, eidx, ts, n_nodes=None, **kw):
        """Build from edge rows without materialising Python adjacency lists (same result as
        the adj_list construction of temp_exp_main.py:135-144)."""
        if n_nodes is None:
            n_nodes = int(max(np.max(src), np.max(dst))) + 1
        return cls(None, _edges=(src, dst, eidx, ts, n_nodes), **kw)

    # ------------------------------------------------------------ host-side views
    @property
    def nodeedge2idx(self):
        """{node: {e_idx: position}} exactly as get_ts2idx builds it (graph.py:77-101)."""
        if self._ne2i is None:
            d = {}
            o = self.off_set_l
            for u in range(len(o) - 1):
                s, t = int(o[u]), int(o[u + 1])
                d[u] = {int(e): int(v) for e, v in zip(self.edge_idx_l[s:t], self._dict_val[s:t])}
            self._ne2i = d
        return self._ne2i

    def find_before(self, src_idx, cut_time, e_idx=None, return_binary_prob=False):
        """graph.py:103-146 (host view of the same CSR the kernels read)."""
        s, t = int(self.off_set_l[src_idx]), int(self.off_set_l[src_idx + 1])
        n_i, n_t, n_e = self.node_idx_l[s:t], self.node_ts_l[s:t], self.edge_idx_l[s:t]
        if e_idx is None:
            cut = int(np.searchsorted(n_t, cut_time, side="left"))
        else:
            cut = self.nodeedge2idx[src_idx].get(e_idx) if src_idx > 0 else 0
            if cut is None:
                raise IndexError("e_idx {} not found in edge list of {}".format(e_idx, src_idx))
            if self.strict_temporal and src_idx > 0:
                cut = int(np.searchsorted(n_t, n_t[n_e == e_idx][0], side="left"))
        if return_binary_prob:
            raise NotImplementedError("binary_prob is only used by the dead 'binary' sample method")
        return n_i[:cut], n_e[:cut], n_t[:cut], None

    # ------------------------------------------------------------ device sampling
    def _events(self, B, event_ids):
        if event_ids is None:
            ev = np.arange(self._next_event, self._next_event + B, dtype=np.int64)
            self._next_event += B
        else:
            ev = np.asarray(event_ids, dtype=np.int64).reshape(-1)
            assert len(ev) == B
        return torch.from_numpy(ev.astype(np.uint32).view(np.int32)).to(self.device)

    def _dev(self, a, dtype):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=dtype)).to(self.device)

    def find_k_hop(self, k, src_idx_l, cut_time_l, num_neighbors, e_idx_l=None, *, event_ids=None,
                   side=L.SIDE_NONE, as_tensor=False):
        """graph.py:233-262.  Returns ([node hop1 [B,N], hop2 [B,N^2], ...], [eid ...], [ts ...])."""
        if k == 0:
            return ([], [], [])
        B = len(src_idx_l)
        N = int(num_neighbors)
        assert len(cut_time_l) == B
        sizes = [B * N ** h for h in range(1, k + 1)]
        tot = sum(sizes)
        dev = self.device
        on = torch.zeros(max(tot, 1), dtype=torch.int32, device=dev)
        oe = torch.zeros_like(on)
        ot = torch.zeros(max(tot, 1), dtype=torch.float32, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        root = self._dev(src_idx_l, np.int32)
        cut = self._dev(cut_time_l, np.float64)
        eidx = None if e_idx_l is None else self._dev(e_idx_l, np.int32)
        ev = self._events(B, event_ids)
        rng = L.TmRng(self.seed, self.split, side)
        L.check(L.lib().tm_sample_khop(self.graph.handle, rng, k, N, B, L.ptr(root), L.ptr(cut), L.ptr(eidx),
                                       L.ptr(ev), L.ptr(on), L.ptr(oe), L.ptr(ot), L.ptr(err), L.stream_ptr(dev)),
                "find_k_hop")
        L.raise_device_error(int(err.item()), "find_k_hop")
        outs = ([], [], [])
        o = 0
        for h, sz in enumerate(sizes):
            for lst, arr in zip(outs, (on, oe, ot)):
                v = arr[o:o + sz].view(B, N ** (h + 1))
                lst.append(v if as_tensor else v.cpu().numpy())
            o += sz
        return outs

    def get_temporal_neighbor(self, src_idx_l, cut_time_l, num_neighbor, e_idx_l=None, **kw):
        """graph.py:197-231: one hop, [B, num_neighbor] arrays."""
        n, e, t = self.find_k_hop(1, src_idx_l, cut_time_l, num_neighbor, e_idx_l=e_idx_l, **kw)
        return n[0], e[0], t[0]

    def find_k_walks(self, degree, src_idx_l, num_neighbors, subgraph_src, *, event_ids=None, side=L.SIDE_NONE,
                     as_tensor=False):
        """graph.py:265-306.  Returns (node [B,W,6], eid [B,W,3], ts [B,W,3], anony [B,W,3]), W = degree*num_neighbors."""
        node_records, eidx_records, t_records = subgraph_src
        B = len(src_idx_l)
        N, M = int(degree), int(num_neighbors)
        W = N * M
        dev = self.device

        def as_dev(x, dtype, tdtype):
            if isinstance(x, torch.Tensor):
                return x.to(device=dev, dtype=tdtype).contiguous()
            return self._dev(x, dtype)
        h1n = as_dev(node_records[0], np.int32, torch.int32)
        h1e = as_dev(eidx_records[0], np.int32, torch.int32)
        h1t = as_dev(t_records[0], np.float32, torch.float32)
        assert h1n.numel() == B * N, "hop-1 records must be [B, degree]"
        root = self._dev(src_idx_l, np.int32)
        ev = self._events(B, event_ids)
        node6 = torch.empty(max(B * W * 6, 1), dtype=torch.int32, device=dev)
        eid3 = torch.empty(max(B * W * 3, 1), dtype=torch.int32, device=dev)
        ts3 = torch.empty(max(B * W * 3, 1), dtype=torch.float32, device=dev)
        an3 = torch.empty(max(B * W * 3, 1), dtype=torch.int32, device=dev)
        rng = L.TmRng(self.seed, self.split, side)
        L.check(L.lib().tm_sample_walks(self.graph.handle, rng, N, M, B, L.ptr(root), L.ptr(h1n), L.ptr(h1e),
                                        L.ptr(h1t), L.ptr(ev), L.ptr(node6), L.ptr(eid3), L.ptr(ts3), L.ptr(an3),
                                        None, L.stream_ptr(dev)), "find_k_walks")
        out = (node6[:B * W * 6].view(B, W, 6), eid3[:B * W * 3].view(B, W, 3), ts3[:B * W * 3].view(B, W, 3),
               an3[:B * W * 3].view(B, W, 3))
        if as_tensor:
            return out
        return tuple(x.cpu().numpy() for x in out)
