"""GPU: the device CSR build (graph_dev.hip, tm_graph_build_edges) against the host builder (graph.cpp,
tm_debug_set(TM_DEBUG_HOST_BUILD, 1)) on the same edge rows -- every exported column (off / ngh / eid / ts / get_ts2idx
values) identical, and every sampled output of the fused sampler identical (which exercises the e_idx
table, the block search trees, the block ranks and the block hash table).  Tie-heavy graphs with
self-loops and a node 0, an Enron-shaped hub graph, a sparse 100k-node graph, and rows that repeat an
edge id (the device path hands those to the host builder)."""
import os

import numpy as np
import pytest
import torch

import tempme_amd as tm
from tempme_amd.preprocess import sample_events
from tempme_amd.workload import enron_like

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    return torch.device("cuda", 0)


def _ties(n_nodes, n_edges, n_ts, seed, loops=0.05):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n_nodes, n_edges)
    dst = rng.integers(0, n_nodes, n_edges)
    loop = rng.uniform(size=n_edges) < loops
    dst[loop] = src[loop]
    ts = np.sort(rng.integers(0, n_ts, n_edges)).astype(np.float64)
    return src, dst, np.arange(1, n_edges + 1), ts, n_nodes


def _shuffled(n_nodes, n_edges, n_ts, seed):
    """Rows not in time order (a permutation of a tie-heavy graph): the host builder takes its
    stable_sort path (not the already-sorted copy), the device its radix sorts; ties keep row order."""
    src, dst, eidx, ts, V = _ties(n_nodes, n_edges, n_ts, seed)
    p = np.random.default_rng(seed + 100).permutation(n_edges)
    return src[p], dst[p], eidx[p], ts[p], V


def _enron(n_nodes, n_edges, alpha, seed):
    g = enron_like(n_nodes=n_nodes, n_edges=n_edges, alpha=alpha, de=4, dn=4, seed=seed)
    return g["src"], g["dst"], g["eidx"], g["ts"], g["n_nodes"]


def _build(dev, rows, host):
    from tempme_amd import _lib as L
    L.check(L.lib().tm_debug_set(L.TM_DEBUG_HOST_BUILD, int(host)), "tm_debug_set")
    try:
        return tm.NeighborFinder.from_edges(*rows[:4], rows[4], device=dev, seed=3)
    finally:
        L.check(L.lib().tm_debug_set(L.TM_DEBUG_HOST_BUILD, 0), "tm_debug_set")


CASES = {
    "ties_small": lambda: _ties(12, 400, 9, 1),
    "ties_mid": lambda: _ties(300, 20000, 50, 2),
    "enron_hub": lambda: _enron(184, 60000, 1.2, 3),
    "sparse_100k": lambda: _enron(100000, 200000, 1.5, 4),
    "shuffled_ties": lambda: _shuffled(40, 5000, 12, 6),
    "shuffled_hub": lambda: _shuffled(8, 20000, 300, 7),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_device_build_equals_host_build(dev, case):
    rows = CASES[case]()
    fd, fh = _build(dev, rows, False), _build(dev, rows, True)
    assert fd.graph.handle.value != fh.graph.handle.value
    for a, b, name in zip(fd.graph.export(), fh.graph.export(), ("off", "ngh", "eid", "ts", "dict")):
        assert np.array_equal(a, b), name
    src, dst, eidx, ts, V = rows
    rng = np.random.default_rng(7)
    E = 512
    i = rng.integers(0, len(src), E)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    args = (t(src[i], np.int32), t(dst[i], np.int32), t(ts[i], np.float64), t(eidx[i], np.int32),
            t(np.arange(E, dtype=np.uint32).view(np.int32), np.int32))
    pool = t(np.unique(dst), np.int32)
    outs = []
    for f in (fd, fh):
        b = sample_events(f.graph, 3, tm.SPLIT_TEST, 20, 3, *args, pool, check=False)
        torch.cuda.synchronize()
        outs.append(b)
    for k in ("dst_fake", "sub1_node", "sub1_eid", "sub1_ts", "sub2_node", "sub2_eid", "sub2_ts", "node6", "eid3",
              "ts3", "cat", "cnt", "hist", "err"):
        assert torch.equal(getattr(outs[0], k), getattr(outs[1], k)), k


def test_empty_edge_set(dev):
    """n_edges == 0: the device builder hands over to the host builder (no zero-size device scans)."""
    z = np.zeros(0, dtype=np.int64)
    f = tm.NeighborFinder.from_edges(z, z, z, z.astype(np.float64), 5, device=dev, seed=3)
    off, ngh, eid, ts, dct = f.graph.export()
    assert off.tolist() == [0] * 6 and len(ngh) == len(eid) == len(ts) == 0


def test_repeated_edge_ids_use_the_host_builder(dev):
    src, dst, eidx, ts, V = _ties(50, 2000, 30, 5)
    src, dst, eidx = src.copy(), dst.copy(), eidx.copy()
    src[11], dst[11], eidx[11] = src[10], dst[10], eidx[10]     # one edge id on two rows (same endpoints)
    fd = _build(dev, (src, dst, eidx, ts, V), False)
    fh = _build(dev, (src, dst, eidx, ts, V), True)
    for a, b in zip(fd.graph.export(), fh.graph.export()):
        assert np.array_equal(a, b)
