"""Pin the CPU oracle against vectors produced by the reference itself
(tests/golden/make_goldens.py ran /root/reference under the keyed-RNG contract).

CPU only: these are the 'oracle checked against golden vectors' tests.
"""
import json
import os

import numpy as np
import pandas as pd
import pytest

from oracle import oracle as orc
from oracle import philox as px

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_philox_known_answers():
    # Random123 kat_vectors for philox4x32_10
    r = px.philox4x32_10(0, 0, 0, 0, 0, 0)
    assert [int(x) for x in r] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    r = px.philox4x32_10(*([0xffffffff] * 6))
    assert [int(x) for x in r] == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    r = px.philox4x32_10(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0)
    assert [int(x) for x in r] == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_c_philox_matches_python():
    rng = np.random.RandomState(0)
    for _ in range(200):
        seed = int(rng.randint(0, 2**62))
        a = [int(x) for x in rng.randint(0, 2**31, 5)]
        split, side, stage = a[0] % 3, a[1] % 4, a[2] % 64
        ev, row, j = a[3], a[4] % 1000, int(rng.randint(0, 64))
        c = orc.lib().or_draw_u32(seed, split, side, stage, ev, row, j)
        p = int(px.draw_u32(seed, split, side, stage, ev, row, j))
        assert c == p


def test_kat_tie():
    k = json.load(open(os.path.join(G, "kats.json")))["kat_tie"]
    g = orc.OracleGraph(k["src"], k["dst"], k["eidx"], k["ts"], k["n_nodes"])
    for e, v in k["nodeedge2idx_1"].items():
        assert g.dict_raw(1, int(e)) == v
    assert g.find_before(1, 4.0, e=7) == k["find_before_e7"] == 6
    assert g.find_before(1, 4.0) == k["find_before_t4"] == 4
    assert g.find_before(1, 2.5) == k["find_before_t2p5"]


def test_kat_leak():
    k = json.load(open(os.path.join(G, "kats.json")))["kat_leak"]
    g = orc.OracleGraph(k["src"], k["dst"], k["eidx"], k["ts"], k["n_nodes"])
    nodes, eids, tss = orc.khop(g, k["seed"], k["split"], k["side"], 2, k["N"], [1], [10.0], None, [0])
    for h, key in enumerate(("hop1", "hop2")):
        assert nodes[h].tolist() == k[key][0]
        assert eids[h].tolist() == k[key][1]
        assert tss[h].tolist() == k[key][2]
    n6, e3, t3, an = orc.walks(g, k["seed"], k["split"], k["side"], k["N"], k["M"], [1],
                               nodes[0], eids[0], tss[0], [0])
    assert n6.tolist() == k["walk_node"]
    assert e3.tolist() == k["walk_eid"]
    assert t3.tolist() == k["walk_ts"]
    assert an.tolist() == k["walk_anony"]
    # the leak: step 2 is empty (e2 = 0) and step 3 took edges after the hop-1 edge
    assert all(e[1] == 0 for e in k["walk_eid"][0])


def _check_pipeline(g, z, pre, seed, split, N, M, src, dst, ts, eidx, dst_list, n_events):
    o = orc.event_pipeline(g, seed, split, N, M, src[:n_events], dst[:n_events], ts[:n_events],
                           eidx[:n_events], np.arange(n_events), dst_list)
    assert np.array_equal(o["dst_fake"], z[pre + "dst_fake"])
    for s, side in enumerate(("src", "tgt", "bgd")):
        for h, sub in ((0, "sub1"), (1, "sub2")):
            for f in ("node", "eid", "ts"):
                ref = z[f"{pre}subgraph_{side}_{h}_{f}"]
                assert np.array_equal(o[f"{sub}_{f}"][:, s], ref), (side, h, f)
        assert np.array_equal(o["node6"][:, s], z[f"{pre}walks_{side}_node"]), side
        assert np.array_equal(o["eid3"][:, s], z[f"{pre}walks_{side}_eid"]), side
        assert np.array_equal(o["ts3"][:, s], z[f"{pre}walks_{side}_ts"]), side
        assert np.array_equal(o["cat"][:, s], z[f"{pre}walks_{side}_cat"]), side
        assert np.array_equal(o["cnt"][:, s], z[f"{pre}edge"][s]), side
        # marginal (data_preprocess.py:180-208): global frequency of the walk's category
        W = N * M
        freq = o["hist"].astype(np.float64) / (n_events * W * 3)
        assert np.array_equal(freq[o["cat"][:, s]], z[f"{pre}walks_{side}_marg"]), side


def test_synth_small_graph_and_pipeline():
    z = np.load(os.path.join(G, "synth_small.npz"))
    src, dst, ts, eidx = z["src"], z["dst"], z["ts"], z["eidx"]
    g = orc.OracleGraph(src, dst, eidx, ts)
    off, ngh, e, t = g.csr()
    assert np.array_equal(off, z["csr_off"])
    assert np.array_equal(ngh, z["csr_node"]) and np.array_equal(e, z["csr_eid"]) and np.array_equal(t, z["csr_ts"])
    for u, ee, p in z["nodeedge2idx"]:
        assert g.dict_raw(u, ee) == p
    dst_list = np.unique(dst)
    for N in (5, 8):
        _check_pipeline(g, z, f"N{N}_", 11, px.SPLIT_TEST, N, 3, src, dst, ts, eidx, dst_list, 24)
    # 3-hop time-path call
    n_nodes = g.n_nodes
    nodes, eids, tss = orc.khop(g, 3, px.SPLIT_TRAIN, px.SIDE_BGD, 3, 4, np.arange(n_nodes),
                                np.linspace(0, 41, n_nodes), None, 100 + np.arange(n_nodes))
    for h in range(3):
        assert np.array_equal(nodes[h], z[f"khop3_node{h}"])
        assert np.array_equal(eids[h], z[f"khop3_eid{h}"])
        assert np.array_equal(tss[h], z[f"khop3_ts{h}"])


@pytest.mark.parametrize("mode", ["train", "test"])
def test_uslegis_pipeline(mode):
    z = np.load(os.path.join(G, "uslegis_pipeline.npz"))
    src, dst, ts, eidx = z[f"{mode}_src"], z[f"{mode}_dst"], z[f"{mode}_ts"], z[f"{mode}_eidx"]
    if mode == "train":
        g = orc.OracleGraph(src, dst, eidx, ts, 224)
        split = px.SPLIT_TRAIN
    else:
        df = pd.read_csv(os.path.join(G, "data", "ml_uslegis_sampled.csv"))
        g = orc.OracleGraph(df.u.values, df.i.values, df.idx.values, df.ts.values, 224)
        split = px.SPLIT_TEST
    for N, n_ev in ((20, 32), (30, 12)):
        _check_pipeline(g, z, f"{mode}_N{N}_", 0, split, N, 3, src, dst, ts, eidx, z[f"{mode}_sampler_dst"], n_ev)


def test_null_model_oracle():
    """utils/null_model.py:13-128 restated over the C oracle: keyed endpoint shuffle, random.seed(2023)
    masks on the unshuffled columns, 500 test events x 3 sides with one walk per slot."""
    import random
    ref = json.load(open(os.path.join(G, "null_uslegis.json")))
    g_df = pd.read_csv(os.path.join(G, "data", "ml_uslegis_sampled.csv"))
    val_time, test_time = list(np.quantile(g_df.ts, [0.70, 0.85]))
    ts_l, e_l = g_df.ts.values, g_df.idx.values
    perm = px.keyed_permutation(len(ts_l), ref["seed"])
    src_l, dst_l = g_df.u.values[perm], g_df.i.values[perm]
    rnd = random.Random(2023)
    total = set(np.unique(np.hstack([g_df.u.values, g_df.i.values])))
    late = ts_l > val_time
    mask = set(rnd.sample(list(set(src_l[late]).union(set(dst_l[late]))), int(0.1 * len(total))))
    ms, md = g_df.u.map(lambda x: x in mask).values, g_df.i.map(lambda x: x in mask).values
    tr = (ts_l <= val_time) * ((1 - ms) * (1 - md) > 0)
    va, te = (ts_l <= test_time) * (ts_l > val_time), ts_l > test_time
    pool = np.unique(np.concatenate([dst_l[tr], dst_l[va], dst_l[te]]))
    g = orc.OracleGraph(src_l, dst_l, e_l, ts_l, int(max(src_l.max(), dst_l.max())) + 1)
    n, N = 500, ref["N"]
    o = orc.event_pipeline(g, ref["seed"], px.SPLIT_NULL, N, 1, src_l[te][:n], dst_l[te][:n], ts_l[te][:n],
                           e_l[te][:n], np.arange(n), pool)
    an = np.zeros((n * 3 * N, 3), np.int32)
    # categories back to anony codes, then the null-model binning (key order of null_model.py:90)
    codes = [(2, 1), (2, 2), (2, 3), (2, 0), (3, 1), (3, 3), (3, 2), (3, 0), (1, 3), (1, 2), (1, 1), (1, 0)]
    c = o["cat"].reshape(-1)
    an[:, 0] = 1
    an[:, 1] = [codes[x][0] for x in c]
    an[:, 2] = [codes[x][1] for x in c]
    _, hist = orc.cat_hist(an, null_order=True)
    dist = {str(k + 1): int(hist[k]) / (500 * 3 * N) for k in range(12)}
    assert dist == ref["dist"]
