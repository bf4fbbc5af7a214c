"""Design check: exact deduplication of repeated walks is not worth a kernel change at the
metric config.  Walks are drawn with replacement per hop-1 slot (graph.py:328, :457), so a slot's M walks
can repeat; this measures, on the oracle's sampler output for the full-Enron-shaped graph (N=20, M=3),
how many walks -- and how many walk positions -- repeat an earlier one of the same slot.  Measured at
600 events: 0.12 % of walks, 0.19 % of positions 1, 2.4 % of positions 0 (position 2 is already computed
once per slot by walk_kernel's slot pass)."""
import numpy as np

from oracle import oracle as orc
from oracle import philox as px


def test_repeated_walks_are_rare():
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=184, n_edges=125235, alpha=1.2, seed=0)
    (src, dst, ts, eidx), rows, pool = split(g)
    og = orc.OracleGraph(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"])
    E, N, M = 200, 20, 3
    sel = np.arange(len(src) // 2, len(src) // 2 + E)
    o = orc.event_pipeline(og, 0, px.SPLIT_TEST, N, M, src[sel], dst[sel], ts[sel], eidx[sel], np.arange(E), pool, 8)
    W = N * M
    node6 = o["node6"].reshape(E * 3 * N, M, 6)
    eid3 = o["eid3"].reshape(E * 3 * N, M, 3)
    ts3 = o["ts3"].reshape(E * 3 * N, M, 3)
    cat = o["cat"].reshape(E * 3 * N, M, 1)
    cnt = o["cnt"].reshape(E * 3 * N, M, 9)
    walk = np.concatenate([node6, eid3, ts3.view(np.int32), cat, cnt.astype(np.int32)], -1)   # one row per walk

    def repeats(rows):
        n = 0
        for m in range(1, M):
            earlier = (rows[:, :m] == rows[:, m:m + 1]).all(-1).any(-1)
            n += int(earlier.sum())
        return n

    total = E * 3 * W
    full = repeats(walk)
    pos0 = repeats(np.concatenate([node6[..., 0:2], eid3[..., 0:1], ts3[..., 0:1].view(np.int32)], -1))
    assert full / total < 0.01, full / total
    assert pos0 / total < 0.05, pos0 / total
