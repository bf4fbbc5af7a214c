"""Per-event sampling driver + motif bookkeeping with the reference's array layouts.

* ``pre_processing``  processed/data_preprocess.py:99-145 (what it writes to ``{data}_{MODE}.h5``)
* ``marginal``        processed/data_preprocess.py:148-214
* ``calculate_edge``  processed/data_preprocess.py:346-356 (new_edge_info :327-343)

All sampling, category and count work runs on the device (tm_sample_events,
tm_motif_hist, tm_edge_counts); the functions only reshape into the reference's
float64 H5 / .npy layouts.
"""
import numpy as np
import torch

from . import _lib as L

SIDES = ("src", "tgt", "bgd")


class EventBuffers:
    """Device outputs of one tm_sample_events launch (side-major [3, E, ...])."""

    def __init__(self, E, N, M, device):
        W = N * M
        z = lambda *s, dt=torch.int32: torch.zeros(*s, dtype=dt, device=device)  # noqa: E731
        self.E, self.N, self.M, self.W = E, N, M, W
        self.dst_fake = z(max(E, 1))
        self.sub1_node, self.sub1_eid, self.sub1_ts = z(3, E, N), z(3, E, N), z(3, E, N, dt=torch.float32)
        self.sub2_node, self.sub2_eid = z(3, E, N * N), z(3, E, N * N)
        self.sub2_ts = z(3, E, N * N, dt=torch.float32)
        self.node6, self.eid3 = z(3, E, W, 6), z(3, E, W, 3)
        self.ts3 = z(3, E, W, 3, dt=torch.float32)
        self.cat = z(3, E, W)
        self.cnt = z(3, E, W, 3, 3, dt=torch.float32)
        self.hist = torch.zeros(12, dtype=torch.int64, device=device)
        self.err = z(1)


def sample_events(graph, seed, split, N, M, src, dst, ts, eidx, event_ids, dst_list, out=None, check=True):
    """One fused launch over E target events (device tensors in, EventBuffers out)."""
    E = int(src.numel())
    dev = src.device
    if out is None:
        out = EventBuffers(E, N, M, dev)
    L.check(L.lib().tm_sample_events(
        graph.handle, seed, split, N, M, E, L.ptr(src), L.ptr(dst), L.ptr(ts), L.ptr(eidx), L.ptr(event_ids),
        L.ptr(dst_list), dst_list.numel(), L.ptr(out.dst_fake), L.ptr(out.sub1_node), L.ptr(out.sub1_eid),
        L.ptr(out.sub1_ts), L.ptr(out.sub2_node), L.ptr(out.sub2_eid), L.ptr(out.sub2_ts), L.ptr(out.node6),
        L.ptr(out.eid3), L.ptr(out.ts3), L.ptr(out.cat), L.ptr(out.cnt), L.ptr(out.hist), L.ptr(out.err),
        L.stream_ptr(dev)), "tm_sample_events")
    if check:
        L.raise_device_error(int(out.err.item()), "sample_events")
    return out


def _dev(a, dtype, device):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=dtype)).to(device)


def pre_processing(ngh_finder, sampler, src, dst, ts, val_e_idx_l, num_neighbors, walks_per_slot=3, *, seed=None,
                   split=None, event_base=0):
    """data_preprocess.py:99-145 for events 0 .. len(src)-2 (its ``range(num_test_instance-1)``).

    Returns the dict the reference writes to ``{data}_{MODE}.h5``: subgraph_{side}_{0,1}
    ([n, 3N] / [n, 3N^2], node|eid|ts), walks_{side} ([n, W, 15]: 6 node, 3 eid, 3 ts,
    3 anony), dst_fake [n]; float64 like the H5 round trip.  Event k uses event id
    event_base + k."""
    dev = ngh_finder.device
    seed = ngh_finder.seed if seed is None else seed
    split = ngh_finder.split if split is None else split
    n = max(len(src) - 1, 0)
    N, M = int(num_neighbors), int(walks_per_slot)
    ev = np.arange(event_base, event_base + n, dtype=np.int64).astype(np.uint32).view(np.int32)
    b = sample_events(ngh_finder.graph, seed, split, N, M, _dev(src[:n], np.int32, dev), _dev(dst[:n], np.int32, dev),
                      _dev(ts[:n], np.float64, dev), _dev(val_e_idx_l[:n], np.int32, dev), _dev(ev, np.int32, dev),
                      _dev(sampler.dst_list, np.int32, dev))
    h = lambda t: t.cpu().numpy()  # noqa: E731
    out = {"dst_fake": h(b.dst_fake[:n]).astype(np.float64)}
    an = anony_from_cat(h(b.cat))
    for s, side in enumerate(SIDES):
        out[f"subgraph_{side}_0"] = np.concatenate([h(b.sub1_node[s]), h(b.sub1_eid[s]), h(b.sub1_ts[s])], -1).astype(np.float64)
        out[f"subgraph_{side}_1"] = np.concatenate([h(b.sub2_node[s]), h(b.sub2_eid[s]), h(b.sub2_ts[s])], -1).astype(np.float64)
        out[f"walks_{side}"] = np.concatenate([h(b.node6[s]), h(b.eid3[s]), h(b.ts3[s]), an[s]], -1).astype(np.float64)
    return out


# marginal's category order (data_preprocess.py:171-172) as (x, t) of the anony code [1, x, t]
CAT_CODES = ((2, 1), (2, 2), (2, 3), (2, 0), (3, 1), (3, 3), (3, 2), (3, 0), (1, 3), (1, 2), (1, 1), (1, 0))
# null-model key order 1..12 (utils/null_model.py:90)
NULL_CODES = ((2, 0), (2, 1), (2, 3), (2, 2), (3, 0), (3, 1), (3, 3), (3, 2), (1, 0), (1, 1), (1, 2), (1, 3))
CAT_TO_NULL = np.array([CAT_CODES.index(c) for c in NULL_CODES])   # null key k-1 -> cat id


def anony_from_cat(cat):
    tab = np.array([[1, x, t] for (x, t) in CAT_CODES], dtype=np.int32)
    return tab[np.asarray(cat)]


def marginal(walks_src, walks_tgt, walks_bgd, device=None):
    """data_preprocess.py:148-214: [n, W, 15] x3 -> [n, W, 14] x3 (6 node, 3 eid, 3 ts, cat, marginal)."""
    dev = L.require_device(device)
    ws = (walks_src, walks_tgt, walks_bgd)
    n, W = walks_src.shape[0], walks_src.shape[1]
    hist = torch.zeros(12, dtype=torch.int64, device=dev)
    cats = []
    for w in ws:
        an = _dev(w[:, :, 12:15].astype(np.int64), np.int32, dev)
        cat = torch.empty(max(n * W, 1), dtype=torch.int32, device=dev)
        L.check(L.lib().tm_motif_hist(L.ptr(an), n * W, 0, L.ptr(cat), L.ptr(hist), L.stream_ptr(dev)), "marginal")
        cats.append(cat[:n * W])
    freq = hist.cpu().numpy().astype(np.float64) / (n * W * 3)
    out = []
    for w, c in zip(ws, cats):
        c = c.cpu().numpy().reshape(n, W)
        if (c < 0).any():
            raise KeyError("anony code outside the 12 motif categories")
        out.append(np.concatenate([w[:, :, :12], c[..., None].astype(np.float64), freq[c][..., None]], -1))
    return tuple(out)


def edge_counts(eid3, device=None):
    """new_edge_info (data_preprocess.py:327-343) for eid3 [n, W, 3] -> [n, W, 3, 3] float64."""
    dev = L.require_device(device)
    eid3 = np.asarray(eid3)
    n, W = eid3.shape[0], eid3.shape[1]
    e = _dev(eid3.astype(np.int64), np.int32, dev)
    out = torch.empty(max(n * W * 9, 1), dtype=torch.float32, device=dev)
    L.check(L.lib().tm_edge_counts(L.ptr(e), n, W, L.ptr(out), L.stream_ptr(dev)), "new_edge_info")
    return out[:n * W * 9].view(n, W, 3, 3).cpu().numpy().astype(np.float64)


def calculate_edge(walks_src, walks_tgt, walks_bgd, device=None):
    """data_preprocess.py:346-356: -> [3, n, W, 3, 3] (the ``{data}_{MODE}_edge.npy`` array)."""
    return np.stack([edge_counts(w[:, :, 6:9].astype(int), device) for w in (walks_src, walks_tgt, walks_bgd)], 0)
