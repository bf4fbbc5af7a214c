"""strict_temporal mode (SURVEY §7 opt-in, not in the reference) of the C oracle.

Parity mode is pinned to the reference by tests/test_oracle_golden.py; strict mode has no reference
to pin it (the reference has no such mode), so these tests pin it by its definition: an e_idx slice
is bisect_left(ts_u, t(e)), and nothing a walk or a subgraph of an event's src/tgt side samples is
at or after the event's own time.
"""
import json
import os

import numpy as np
import pandas as pd
import pytest

from oracle import oracle as orc
from oracle import philox as px

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _tie_graph(strict):
    k = json.load(open(os.path.join(G, "kats.json")))["kat_tie"]
    return k, orc.OracleGraph(k["src"], k["dst"], k["eidx"], k["ts"], k["n_nodes"], strict_temporal=strict)


def test_strict_slice_is_bisect_left_of_edge_time():
    k, g = _tie_graph(True)
    _, gp = _tie_graph(False)
    ts = np.asarray(k["ts"])
    for e, t in zip(k["eidx"], ts):
        assert g.find_before(1, 0.0, e) == int(np.searchsorted(ts, t, side="left"))
    # parity mode keeps the trailing-tie value (graph.py:77-101): 6 records before e=7 at t=4, strict 4
    assert gp.find_before(1, 0.0, 7) == 6 and g.find_before(1, 0.0, 7) == 4
    # node 0 stays padding, an edge the node does not hold stays an IndexError (-1)
    assert g.find_before(0, 0.0, 1) == 0
    assert g.find_before(2, 0.0, 7) == -1


def test_strict_needs_one_timestamp_per_edge():
    with pytest.raises(ValueError):
        orc.OracleGraph([1, 2], [2, 3], [5, 5], [1.0, 2.0], 4, strict_temporal=True)


def _uslegis():
    df = pd.read_csv(os.path.join(G, "data", "ml_uslegis_sampled.csv"))
    return df.u.values, df.i.values, df.idx.values, df.ts.values


@pytest.mark.parametrize("strict", [False, True])
def test_strict_pipeline_has_no_future(strict):
    src, dst, eidx, ts = _uslegis()
    g = orc.OracleGraph(src, dst, eidx, ts, 224, strict_temporal=strict)
    rows = np.arange(len(src) - 64, len(src))          # late events: long lists, many ties
    o = orc.event_pipeline(g, 0, px.SPLIT_TEST, 20, 3, src[rows], dst[rows], ts[rows], eidx[rows],
                           np.arange(len(rows)), np.unique(dst), 4)
    t = ts[rows].astype(np.float32)[:, None, None]
    future = 0
    for s in (0, 1):                                    # the src / tgt sides (e_idx path)
        e, w = o["eid3"][:, s], o["ts3"][:, s]
        future += int(((e > 0) & (w >= t)).sum())
        e1, w1 = o["sub1_eid"][:, s], o["sub1_ts"][:, s]
        future += int(((e1 > 0) & (w1 >= t[:, :, 0])).sum())
    if strict:
        assert future == 0
    else:
        assert future > 0    # the reference's ties and step-3 leak show up on this data


def test_strict_equals_parity_without_ties():
    """On a graph whose timestamps are all distinct, get_ts2idx's value is the record's position, which is
    bisect_left of its own time: the e_idx slices of the two modes agree, so the k-hop samples (e_idx path
    for hop 1 and hop 2) are identical; parity mode is pinned to the reference's goldens, so this pins
    strict mode's slices to the reference's wherever the reference has no tie."""
    rng = np.random.default_rng(4)
    V, E = 40, 600
    src = rng.integers(1, V, E)
    dst = 1 + (src - 1 + rng.integers(1, V - 1, E)) % (V - 1)  # in 1..V-1, never src: no self-loop ties
    assert not (dst == src).any()
    ts = rng.permutation(E).astype(np.float64) + 1.0          # distinct times
    eidx = np.arange(1, E + 1)
    gp = orc.OracleGraph(src, dst, eidx, ts, V)
    gs = orc.OracleGraph(src, dst, eidx, ts, V, strict_temporal=True)
    rows = np.arange(E - 80, E)
    for e_l in (eidx[rows], None):
        a = orc.khop(gp, 3, px.SPLIT_TEST, px.SIDE_SRC, 2, 10, src[rows], ts[rows], e_l, np.arange(len(rows)))
        b = orc.khop(gs, 3, px.SPLIT_TEST, px.SIDE_SRC, 2, 10, src[rows], ts[rows], e_l, np.arange(len(rows)))
        for x, y in zip(a, b):
            for u, v in zip(x, y):
                assert np.array_equal(u, v)
