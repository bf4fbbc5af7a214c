"""GPU parity: the HIP path through the C ABI vs (a) vectors produced by the reference
itself (tests/golden) and (b) the CPU oracle on the same seeded inputs.

Bit-exact for every sampled index / id / time / category / count; encoder outputs within
rtol 1e-5, atol 1e-6 (BASELINE.json north_star).
"""
import json
import os

import numpy as np
import pandas as pd
import pytest
import torch

from oracle import encoder_ref as er
from oracle import oracle as orc
from oracle import philox as px

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RTOL, ATOL = 1e-5, 1e-6


@pytest.fixture(scope="module")
def tm():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    import tempme_amd
    return tempme_amd


def _finder(tm, src, dst, eidx, ts, n_nodes=None, seed=0, split=px.SPLIT_TEST):
    return tm.NeighborFinder.from_edges(src, dst, eidx, ts, n_nodes, seed=seed, split=split)


def test_graph_build_matches_oracle(tm):
    z = np.load(os.path.join(G, "synth_small.npz"))
    f = _finder(tm, z["src"], z["dst"], z["eidx"], z["ts"])
    assert np.array_equal(f.off_set_l, z["csr_off"])
    assert np.array_equal(f.node_idx_l, z["csr_node"])
    assert np.array_equal(f.edge_idx_l, z["csr_eid"])
    assert np.array_equal(f.node_ts_l, z["csr_ts"])
    for u, e, p in z["nodeedge2idx"]:
        assert f.nodeedge2idx[int(u)][int(e)] == p


def test_kat_tie(tm):
    k = json.load(open(os.path.join(G, "kats.json")))["kat_tie"]
    adj = [[] for _ in range(k["n_nodes"])]
    for s, d, e, t in zip(k["src"], k["dst"], k["eidx"], k["ts"]):
        adj[s].append((d, e, t))
        adj[d].append((s, e, t))
    f = tm.NeighborFinder(adj)
    assert {str(a): b for a, b in f.nodeedge2idx[1].items()} == k["nodeedge2idx_1"]
    assert len(f.find_before(1, 4.0, e_idx=7)[0]) == 6
    assert len(f.find_before(1, 4.0)[0]) == 4
    # the device e_idx path must agree with the host dict: draw 1 neighbour before e=7 and e=4
    n, e, t = f.get_temporal_neighbor(np.array([1, 1]), np.array([4.0, 4.0]), 8, e_idx_l=np.array([7, 4]),
                                      event_ids=[0, 1])
    assert set(e[0].tolist()) <= {1, 2, 3, 4, 5, 6} and set(e[1].tolist()) <= {1, 2, 3}


def test_kat_leak(tm):
    k = json.load(open(os.path.join(G, "kats.json")))["kat_leak"]
    f = _finder(tm, k["src"], k["dst"], k["eidx"], k["ts"], k["n_nodes"], seed=k["seed"], split=k["split"])
    sub = f.find_k_hop(2, np.array([1]), np.array([10.0]), k["N"], event_ids=[0], side=k["side"])
    for h, key in enumerate(("hop1", "hop2")):
        assert sub[0][h].tolist() == k[key][0] and sub[1][h].tolist() == k[key][1] and sub[2][h].tolist() == k[key][2]
    w = f.find_k_walks(k["N"], np.array([1]), 1, sub, event_ids=[0], side=k["side"])
    assert w[0].tolist() == k["walk_node"] and w[1].tolist() == k["walk_eid"]
    assert w[2].tolist() == k["walk_ts"] and w[3].tolist() == k["walk_anony"]


def test_khop_3hop_time_path(tm):
    z = np.load(os.path.join(G, "synth_small.npz"))
    f = _finder(tm, z["src"], z["dst"], z["eidx"], z["ts"], seed=3, split=px.SPLIT_TRAIN)
    n = f.off_set_l.shape[0] - 1
    sub = f.find_k_hop(3, np.arange(n), np.linspace(0, 41, n), 4, event_ids=100 + np.arange(n), side=px.SIDE_BGD)
    for h in range(3):
        assert np.array_equal(sub[0][h], z[f"khop3_node{h}"])
        assert np.array_equal(sub[1][h], z[f"khop3_eid{h}"])
        assert np.array_equal(sub[2][h], z[f"khop3_ts{h}"])


def _check_events(tm, f, z, pre, seed, split, N, M, src, dst, ts, eidx, dst_list, n):
    from tempme_amd.preprocess import sample_events
    dev = f.device
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:n], dtype=dt)).to(dev)  # noqa: E731
    b = sample_events(f.graph, seed, split, N, M, t(src, np.int32), t(dst, np.int32), t(ts, np.float64),
                      t(eidx, np.int32), torch.arange(n, dtype=torch.int32, device=dev),
                      torch.from_numpy(np.asarray(dst_list, np.int32)).to(dev))
    h = lambda x: x.cpu().numpy()  # noqa: E731
    assert np.array_equal(h(b.dst_fake[:n]), z[pre + "dst_fake"])
    for s, side in enumerate(("src", "tgt", "bgd")):
        for hop, sub in ((0, "sub1"), (1, "sub2")):
            for fld in ("node", "eid", "ts"):
                assert np.array_equal(h(getattr(b, f"{sub}_{fld}")[s]), z[f"{pre}subgraph_{side}_{hop}_{fld}"]), \
                    (side, hop, fld)
        assert np.array_equal(h(b.node6[s]), z[f"{pre}walks_{side}_node"]), side
        assert np.array_equal(h(b.eid3[s]), z[f"{pre}walks_{side}_eid"]), side
        assert np.array_equal(h(b.ts3[s]), z[f"{pre}walks_{side}_ts"]), side
        assert np.array_equal(h(b.cat[s]), z[f"{pre}walks_{side}_cat"]), side
        assert np.array_equal(h(b.cnt[s]).astype(np.int32), z[f"{pre}edge"][s]), side
    W = N * M
    freq = h(b.hist).astype(np.float64) / (n * W * 3)
    for s, side in enumerate(("src", "tgt", "bgd")):
        assert np.array_equal(freq[h(b.cat[s])], z[f"{pre}walks_{side}_marg"])
    return b


def test_fused_events_small(tm):
    z = np.load(os.path.join(G, "synth_small.npz"))
    f = _finder(tm, z["src"], z["dst"], z["eidx"], z["ts"])
    for N in (5, 8):
        _check_events(tm, f, z, f"N{N}_", 11, px.SPLIT_TEST, N, 3, z["src"], z["dst"], z["ts"], z["eidx"],
                      np.unique(z["dst"]), 24)


@pytest.mark.parametrize("mode", ["train", "test"])
def test_fused_events_uslegis(tm, mode):
    z = np.load(os.path.join(G, "uslegis_pipeline.npz"))
    src, dst, ts, eidx = z[f"{mode}_src"], z[f"{mode}_dst"], z[f"{mode}_ts"], z[f"{mode}_eidx"]
    if mode == "train":
        f = _finder(tm, src, dst, eidx, ts, 224, split=px.SPLIT_TRAIN)
    else:
        df = pd.read_csv(os.path.join(G, "data", "ml_uslegis_sampled.csv"))
        f = _finder(tm, df.u.values, df.i.values, df.idx.values, df.ts.values, 224)
    split = px.SPLIT_TRAIN if mode == "train" else px.SPLIT_TEST
    for N, n in ((20, 32), (30, 12)):
        _check_events(tm, f, z, f"{mode}_N{N}_", 0, split, N, 3, src, dst, ts, eidx, z[f"{mode}_sampler_dst"], n)


def test_separate_calls_equal_fused(tm):
    """find_k_hop + find_k_walks + RandEdgeSampler + marginal + calculate_edge drop-ins reproduce
    the reference pipeline (data_preprocess.py:106-134) event by event."""
    z = np.load(os.path.join(G, "uslegis_pipeline.npz"))
    df = pd.read_csv(os.path.join(G, "data", "ml_uslegis_sampled.csv"))
    f = _finder(tm, df.u.values, df.i.values, df.idx.values, df.ts.values, 224)
    sampler = tm.RandEdgeSampler((z["test_sampler_src"],), (z["test_sampler_dst"],), seed=0, split=px.SPLIT_TEST)
    pre, N, n = "test_N20_", 20, 32
    src, dst, ts, eidx = z["test_src"], z["test_dst"], z["test_ts"], z["test_eidx"]
    ws = {s: [] for s in ("src", "tgt", "bgd")}
    for k in range(n):
        _, fake = sampler.sample(1, event_ids=[k])
        assert fake[0] == z[pre + "dst_fake"][k]
        for s_i, (side, root, e_l) in enumerate((("src", src[k:k + 1], eidx[k:k + 1]), ("tgt", dst[k:k + 1], eidx[k:k + 1]),
                                                ("bgd", fake, None))):
            sub = f.find_k_hop(2, root, ts[k:k + 1], N, e_idx_l=e_l, event_ids=[k], side=s_i + 1)
            for hop in (0, 1):
                assert np.array_equal(sub[0][hop][0], z[f"{pre}subgraph_{side}_{hop}_node"][k])
                assert np.array_equal(sub[1][hop][0], z[f"{pre}subgraph_{side}_{hop}_eid"][k])
            w = f.find_k_walks(N, root, 3, sub, event_ids=[k], side=s_i + 1)
            assert np.array_equal(w[0][0], z[f"{pre}walks_{side}_node"][k])
            assert np.array_equal(w[1][0], z[f"{pre}walks_{side}_eid"][k])
            ws[side].append(np.concatenate([w[0], w[1], w[2], w[3]], -1).astype(np.float64))
    wsn = tm.marginal(*[np.concatenate(ws[s]) for s in ("src", "tgt", "bgd")])
    for s_i, side in enumerate(("src", "tgt", "bgd")):
        assert np.array_equal(wsn[s_i][:, :, 12].astype(np.int32), z[f"{pre}walks_{side}_cat"])
        assert np.array_equal(wsn[s_i][:, :, 13], z[f"{pre}walks_{side}_marg"])
    edge = tm.calculate_edge(*wsn)
    assert np.array_equal(edge.astype(np.int32), z[pre + "edge"])


def test_pre_processing_dropin(tm):
    z = np.load(os.path.join(G, "synth_small.npz"))
    f = _finder(tm, z["src"], z["dst"], z["eidx"], z["ts"], seed=11)
    sampler = tm.RandEdgeSampler((z["src"],), (z["dst"],))
    out = tm.pre_processing(f, sampler, z["src"][:25], z["dst"][:25], z["ts"][:25], z["eidx"][:25], 8)
    assert np.array_equal(out["walks_src"][:, :, 6:9].astype(np.int32), z["N8_walks_src_eid"])
    assert np.array_equal(out["walks_bgd"][:, :, 12:15].astype(np.int32), z["N8_walks_bgd_anony"])
    assert np.array_equal(out["subgraph_tgt_1"][:, 64:128].astype(np.int32), z["N8_subgraph_tgt_1_eid"])
    assert np.array_equal(out["dst_fake"].astype(np.int32), z["N8_dst_fake"])


def test_index_error_like_reference(tm):
    f = _finder(tm, [1, 2], [2, 3], [1, 2], [1.0, 2.0], 4)
    with pytest.raises(IndexError):
        f.find_k_hop(2, np.array([1]), np.array([5.0]), 4, e_idx_l=np.array([2]))   # edge 2 is not on node 1
    with pytest.raises(IndexError):
        f.find_before(1, 5.0, e_idx=2)


def test_empty_and_node0(tm):
    f = _finder(tm, [0, 1, 2], [1, 2, 3], [1, 2, 3], [1.0, 2.0, 3.0], 4)
    sub = f.find_k_hop(2, np.array([], np.int64), np.array([]), 4)
    assert sub[0][0].shape == (0, 4) and sub[0][1].shape == (0, 16)
    # node 0 is padding on the e_idx path even though it is a real node here (graph.py:133)
    sub = f.find_k_hop(1, np.array([0]), np.array([9.0]), 4, e_idx_l=np.array([1]))
    assert (sub[0][0] == 0).all()
    # ... but the time path samples its list (graph.py:129)
    sub = f.find_k_hop(1, np.array([0]), np.array([9.0]), 4)
    assert (sub[1][0] == 1).all()


def test_null_model(tm):
    ref = json.load(open(os.path.join(G, "null_uslegis.json")))
    d = tm.get_null_distribution("uslegis_sampled", data_dir=os.path.join(G, "data"), seed=ref["seed"])
    assert {str(k): v for k, v in d.items()} == ref["dist"]


# ------------------------------------------------------------------ encoder
class _Base:
    def __init__(self, n_feat, e_feat, dev):
        self.n_feat_th = torch.as_tensor(n_feat)
        self.e_feat_th = torch.as_tensor(e_feat)
        self.node_raw_features = torch.nn.Embedding.from_pretrained(self.n_feat_th.to(dev), padding_idx=0, freeze=True)
        self.edge_raw_features = torch.nn.Embedding.from_pretrained(self.e_feat_th.to(dev), padding_idx=0, freeze=True)


def _explainer(tm, d):
    dev = torch.device("cuda", 0)
    null = {k + 1: float(v) for k, v in enumerate(d["null"])}
    ex = tm.TempME(_Base(d["n_feat"], d["e_feat"], dev), "tgn", "uslegis_sampled", out_dim=40, hid_dim=64,
                   device=dev, null_model=null)
    missing, unexpected = ex.load_state_dict(d["sd"], strict=False)
    assert not unexpected
    assert all(not k.startswith(("event_conv", "attention.W1", "attention.W2", "attention.MLP", "MLP",
                                 "edge_dependency_gcn", "time_encoder")) for k in missing)
    return ex.to(dev).eval()


@pytest.mark.parametrize("case", ["uslegis", "synth"])
def test_encoder_matches_reference_goldens(tm, case):
    from tests.encoder_inputs import SIDES, load
    d = load(case)
    ex = _explainer(tm, d)
    imps, subs, walks = [], [], []
    for s in SIDES:
        x = d[s]
        w = (x["node"], x["eid"], x["ts"], x["cat"], x["marg"])
        with torch.no_grad():        # eval_one_epoch scores under no_grad (temp_exp_main.py:446-452)
            imp = ex(w, d["ts_cut"], x["cnt"])
        np.testing.assert_allclose(imp.cpu().numpy(), x["imp"], rtol=RTOL, atol=ATOL)
        imps.append(imp)
        subs.append((x["sub_node"], x["sub_eid"], x["sub_ts"]))
        walks.append(w)
    expl = ex.retrieve_explanation(subs[0], imps[0], walks[0], subs[1], imps[1], walks[1], subs[2], imps[2],
                                   walks[2], training=False)
    # (outside no_grad the explanation carries gradients to the dependency gate, as the reference's does)
    assert expl[0].requires_grad
    np.testing.assert_allclose(expl[0].detach().cpu().numpy(), d["expl0"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(expl[1].detach().cpu().numpy(), d["expl1"], rtol=RTOL, atol=ATOL)
    for k, s in enumerate(SIDES):
        kl = ex.kl_loss(imps[k], walks[k], target=0.3)
        np.testing.assert_allclose(float(kl), d["kl"][k], rtol=RTOL, atol=ATOL)


def test_nested_reassignment_repacks(tm):
    """The cached weight list follows nested reassignments: a new Linear deep inside a Sequential, a new
    Parameter on a submodule, and load_state_dict(assign=True) all change the HIP forward's output
    exactly as they change the torch formulation's."""
    from tests.encoder_inputs import SIDES, load
    d = load("uslegis")
    ex = _explainer(tm, d)
    x = d[SIDES[0]]
    w = (x["node"], x["eid"], x["ts"], x["cat"], x["marg"])

    def both():
        with torch.no_grad():
            hip = ex(w, d["ts_cut"], x["cnt"]).cpu().numpy()
            ref = ex._forward_torch(w, d["ts_cut"], x["cnt"]).cpu().numpy()
        np.testing.assert_allclose(hip, ref, rtol=RTOL, atol=ATOL)
        return hip

    base = both()
    torch.manual_seed(11)
    ex.MLP[0] = torch.nn.Linear(ex.mlp_dim, ex.mlp_dim).to(ex.device)
    a = both()
    assert not np.allclose(a, base)
    ex.event_conv.lin_event.weight = torch.nn.Parameter(ex.event_conv.lin_event.weight.detach() * 0.5)
    b = both()
    assert not np.allclose(b, a)
    sd = {k: v.clone() * 1.1 if k.startswith("attention.W1") else v.clone() for k, v in ex.state_dict().items()}
    ex.load_state_dict(sd, assign=True)
    c = both()
    assert not np.allclose(c, b)


def test_pipeline_full_size_vs_oracle(tm):
    """Bench workload shape (enron-like, N=20, B=100): sampled outputs bit-exact vs the C oracle on
    every event of one batch per side, encoder + explanation vs the torch-fp32 oracle."""
    from tempme_amd.pipeline import ExplainPipeline
    from tempme_amd.workload import enron_like, split
    g = enron_like(node_feat="uniform")
    (src, dst, ts, eidx), rows, pool = split(g)
    dev = torch.device("cuda", 0)
    f = _finder(tm, g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"], seed=5)
    torch.manual_seed(0)
    ex = tm.TempME(_Base(g["n_feat"], g["e_feat"], dev), "tgn", "enron_sampled", 40, 64, device=dev,
                   null_model={k: 1 / 12 for k in range(1, 13)}).to(dev).eval()
    N, B, E = 20, 100, 400
    pipe = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=5, split=px.SPLIT_TEST)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:E], dtype=dt)).to(dev)  # noqa: E731
    imp, h1, h2 = pipe.run(t(src, np.int32), t(dst, np.int32), t(ts, np.float64), t(eidx, np.int32),
                           torch.arange(E, dtype=torch.int32, device=dev))
    torch.cuda.synchronize()
    pipe.check_errors()
    og = orc.OracleGraph(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"])
    o = orc.event_pipeline(og, 5, px.SPLIT_TEST, N, 3, src[:E], dst[:E], ts[:E], eidx[:E], np.arange(E), pool, 8)
    b = pipe.buf
    h = lambda x: x.cpu().numpy()  # noqa: E731
    assert np.array_equal(h(b.dst_fake[:E]), o["dst_fake"])
    for name in ("node6", "eid3", "ts3", "cat", "sub1_node", "sub1_eid", "sub1_ts", "sub2_node", "sub2_eid", "sub2_ts"):
        assert np.array_equal(h(getattr(b, name)).swapaxes(0, 1), o[name]), name
    assert np.array_equal(h(b.cnt).swapaxes(0, 1).astype(np.int32), o["cnt"])
    # encoder: one reference batch per side (batch 1 of 4) through the torch-fp32 oracle
    sd = {k: v.detach().cpu() for k, v in ex.state_dict().items()}
    nf, ef = torch.from_numpy(g["n_feat"]), torch.from_numpy(g["e_feat"])
    W = N * 3
    bi = 1
    sl = slice(bi * B, (bi + 1) * B)
    for s in range(3):
        ref = er.forward(sd, nf, ef, o["node6"][sl, s], o["eid3"][sl, s], o["ts3"][sl, s], o["cat"][sl, s],
                         ts[sl], o["cnt"][sl, s].astype(np.float64))
        np.testing.assert_allclose(h(imp[s, sl]), ref.numpy()[..., 0], rtol=RTOL, atol=ATOL)
        e0, e1 = er.edge_importance(sd, ef, ref, o["eid3"][sl, s], o["ts3"][sl, s],
                                    [o["sub1_node"][sl, s], o["sub2_node"][sl, s]],
                                    [o["sub1_eid"][sl, s], o["sub2_eid"][sl, s]])
        np.testing.assert_allclose(h(h1[s, sl]), e0.numpy(), rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(h(h2[s, sl]), e1.numpy(), rtol=RTOL, atol=ATOL)
    assert W == imp.shape[-1]


def test_gate_table_path_bitwise_equals_per_walk_path(tm):
    """tm_edge_importance_tab (gate once per edge id, max before the gate multiply) must equal the
    per-walk-position path (tm_edge_importance, the reference's order of operations) bit for bit."""
    from tempme_amd.pipeline import ExplainPipeline
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=120, n_edges=6000, node_feat="uniform", seed=9)
    (src, dst, ts, eidx), rows, pool = split(g)
    dev = torch.device("cuda", 0)
    f = _finder(tm, g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"], seed=2)
    torch.manual_seed(1)
    ex = tm.TempME(_Base(g["n_feat"], g["e_feat"], dev), "tgn", "x", 40, 64, device=dev,
                   null_model={k: 1 / 12 for k in range(1, 13)}).to(dev).eval()
    N, B, E = 20, 50, 200
    pipe = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=2)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:E], dtype=dt)).to(dev)  # noqa: E731
    imp, h1, h2 = pipe.run(t(src, np.int32), t(dst, np.int32), t(ts, np.float64), t(eidx, np.int32),
                           torch.arange(E, dtype=torch.int32, device=dev))
    b = pipe.buf
    o1, o2 = ex.edge_importance(b.eid3, b.ts3, pipe.imp, b.sub1_node, b.sub1_eid, b.sub2_node, b.sub2_eid,
                                3 * E // B, B, N * 3, N)
    torch.cuda.synchronize()
    pipe.check_errors()
    assert torch.equal(o1[:3 * E * N].view(3, E, N), h1)
    assert torch.equal(o2[:3 * E * N * N].view(3, E, N * N), h2)


def _pareto_finder(tm, seed=4, **kw):
    from tempme_amd.workload import enron_like, split
    g = enron_like(seed=seed, **kw)
    (src, dst, ts, eidx), rows, pool = split(g)
    f = _finder(tm, g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"], seed=seed)
    return g, rows, (src, dst, ts, eidx), pool, f


@pytest.mark.parametrize("N", [7, 20, 30, 64])
def test_khop2_fused_equals_per_level_and_oracle(tm, N):
    """find_k_hop(2) runs the fused 2-hop kernel, find_k_hop(3) the per-level kernel: their first two
    hops share the RNG keys and must be identical, on both the e_idx path and the time path; and
    both equal the C oracle."""
    g, rows, (src, dst, ts, eidx), pool, f = _pareto_finder(tm)
    B = 96
    ev = 1000 + np.arange(B)
    for side, ei in ((px.SIDE_SRC, eidx[:B]), (px.SIDE_BGD, None)):
        two = f.find_k_hop(2, src[:B], ts[:B], N, e_idx_l=ei, event_ids=ev, side=side)
        three = f.find_k_hop(3, src[:B], ts[:B], N, e_idx_l=ei, event_ids=ev, side=side)
        for h in range(2):
            for a in range(3):
                assert np.array_equal(two[a][h], three[a][h]), (side, h, a)
    og = orc.OracleGraph(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"])
    o = orc.khop(og, f.seed, f.split, px.SIDE_SRC, 2, N, src[:B], ts[:B], eidx[:B], ev)
    two = f.find_k_hop(2, src[:B], ts[:B], N, e_idx_l=eidx[:B], event_ids=ev, side=px.SIDE_SRC)
    for h in range(2):
        for a in range(3):
            assert np.array_equal(two[a][h].reshape(-1), np.asarray(o[a][h]).reshape(-1)), (h, a)


def test_unkeyed_kernels_equal_keyed(tm):
    """The one-compare keyed rank kernels (graphs < 2^26 entries) and the two-compare kernels must
    give identical samples (tm_debug_set(TM_DEBUG_FORCE_UNKEYED, 1) selects the latter)."""
    from tempme_amd import _lib as L
    from tempme_amd.preprocess import sample_events
    g, rows, (src, dst, ts, eidx), pool, f = _pareto_finder(tm, seed=6)
    dev = f.device
    E, N = 200, 20
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:E], dtype=dt)).to(dev)  # noqa: E731
    args = (f.graph, 3, px.SPLIT_TEST, N, 3, t(src, np.int32), t(dst, np.int32), t(ts, np.float64),
            t(eidx, np.int32), torch.arange(E, dtype=torch.int32, device=dev), torch.from_numpy(pool).to(dev))
    a = sample_events(*args)
    ka = f.find_k_hop(2, src[:E], ts[:E], N, e_idx_l=eidx[:E], event_ids=np.arange(E), side=px.SIDE_TGT)
    L.check(L.lib().tm_debug_set(L.TM_DEBUG_FORCE_UNKEYED, 1), "tm_debug_set")
    try:
        b = sample_events(*args)
        kb = f.find_k_hop(2, src[:E], ts[:E], N, e_idx_l=eidx[:E], event_ids=np.arange(E), side=px.SIDE_TGT)
    finally:
        L.check(L.lib().tm_debug_set(L.TM_DEBUG_FORCE_UNKEYED, 0), "tm_debug_set")
    for name in ("dst_fake", "node6", "eid3", "ts3", "cat", "cnt", "hist", "sub1_node", "sub1_eid", "sub1_ts",
                 "sub2_node", "sub2_eid", "sub2_ts"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    for x, y in zip(ka, kb):
        for h in range(2):
            assert np.array_equal(x[h], y[h])


@pytest.mark.parametrize("N,alpha", [(30, 1.2), (20, 3.0)])
def test_pipeline_other_configs_vs_oracle(tm, N, alpha):
    """Sampling bit-exact vs the C oracle at N=30 and at Pareto alpha=3 (bench's other configs)."""
    from tempme_amd.pipeline import ExplainPipeline
    g, rows, (src, dst, ts, eidx), pool, f = _pareto_finder(tm, seed=7, alpha=alpha, node_feat="uniform")
    dev = f.device
    torch.manual_seed(0)
    ex = tm.TempME(_Base(g["n_feat"], g["e_feat"], dev), "tgn", "enron_sampled", 40, 64, device=dev,
                   null_model={k: 1 / 12 for k in range(1, 13)}).to(dev).eval()
    B, E = 100, 200
    pipe = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=7, split=px.SPLIT_TEST)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:E], dtype=dt)).to(dev)  # noqa: E731
    imp, h1, h2 = pipe.run(t(src, np.int32), t(dst, np.int32), t(ts, np.float64), t(eidx, np.int32),
                           torch.arange(E, dtype=torch.int32, device=dev))
    torch.cuda.synchronize()
    pipe.check_errors()
    og = orc.OracleGraph(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"])
    o = orc.event_pipeline(og, 7, px.SPLIT_TEST, N, 3, src[:E], dst[:E], ts[:E], eidx[:E], np.arange(E), pool, 8)
    b = pipe.buf
    h = lambda x: x.cpu().numpy()  # noqa: E731
    for name in ("node6", "eid3", "ts3", "cat", "sub1_node", "sub1_eid", "sub2_node", "sub2_eid"):
        assert np.array_equal(h(getattr(b, name)).swapaxes(0, 1), o[name]), name
    assert np.array_equal(h(b.cnt).swapaxes(0, 1).astype(np.int32), o["cnt"])
    x = h(imp)
    assert np.isfinite(x).all() and (x >= 0).all() and (x <= 1).all()


def test_pipeline_wide_edge_features_vs_oracle(tm):
    """BASELINE configs[4] shapes (de = dn = 172, N = 30): the walk kernel's streamed-edge-feature
    instance (lin_event over 22 K steps) vs the torch-fp32 oracle on sampled walks."""
    from tempme_amd.pipeline import ExplainPipeline
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=300, n_edges=6000, alpha=1.5, de=172, dn=172, node_feat="uniform", seed=11)
    (src, dst, ts, eidx), rows, pool = split(g)
    dev = torch.device("cuda", 0)
    f = _finder(tm, g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"], seed=3)
    torch.manual_seed(1)
    ex = tm.TempME(_Base(g["n_feat"], g["e_feat"], dev), "tgn", "synth", 40, 64, device=dev,
                   null_model={k: 1 / 12 for k in range(1, 13)}).to(dev).eval()
    N, B, E = 30, 20, 40
    pipe = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=3, split=px.SPLIT_TEST)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:E], dtype=dt)).to(dev)  # noqa: E731
    imp, h1, h2 = pipe.run(t(src, np.int32), t(dst, np.int32), t(ts, np.float64), t(eidx, np.int32),
                           torch.arange(E, dtype=torch.int32, device=dev))
    torch.cuda.synchronize()
    pipe.check_errors()
    b = pipe.buf
    h = lambda x: x.cpu().numpy()  # noqa: E731
    sd = {k: v.detach().cpu() for k, v in ex.state_dict().items()}
    nf, ef = torch.from_numpy(g["n_feat"]), torch.from_numpy(g["e_feat"])
    for bi in range(E // B):
        sl = slice(bi * B, (bi + 1) * B)
        for s in range(3):
            ref = er.forward(sd, nf, ef, h(b.node6[s, sl]), h(b.eid3[s, sl]), h(b.ts3[s, sl]), h(b.cat[s, sl]),
                             ts[sl], h(b.cnt[s, sl]).astype(np.float64))
            np.testing.assert_allclose(h(imp[s, sl]), ref.numpy()[..., 0], rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("depth", [2, 3])
def test_pipelined_explainer_equals_single_stream(tm, depth):
    """PipelinedExplainer (calls in flight on several streams, encoders chained by events) returns,
    call for call, exactly what ExplainPipeline returns for the same inputs on one stream."""
    from tempme_amd.pipeline import ExplainPipeline, PipelinedExplainer
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=120, n_edges=6000, node_feat="uniform", seed=4)
    (src, dst, ts, eidx), rows, pool = split(g)
    dev = torch.device("cuda", 0)
    f = _finder(tm, g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"], seed=3)
    torch.manual_seed(2)
    ex = tm.TempME(_Base(g["n_feat"], g["e_feat"], dev), "tgn", "x", 40, 64, device=dev,
                   null_model={k: 1 / 12 for k in range(1, 13)}).to(dev).eval()
    N, B, E, calls = 20, 50, 150, 5
    t = lambda a, dt, k: torch.from_numpy(np.ascontiguousarray(a[k * E:(k + 1) * E], dtype=dt)).to(dev)  # noqa: E731
    ins = [(t(src, np.int32, k), t(dst, np.int32, k), t(ts, np.float64, k), t(eidx, np.int32, k),
            torch.arange(k * E, (k + 1) * E, dtype=torch.int32, device=dev)) for k in range(calls)]
    one = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=3)
    want = []
    for x in ins:
        want.append([o.clone() for o in one.run(*x)])
    torch.cuda.synchronize()
    one.check_errors()
    fl = PipelinedExplainer(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=3, depth=depth)
    got = []
    for x in ins:
        outs, st = fl.submit(*x)
        with torch.cuda.stream(st):
            got.append([o.clone() for o in outs])      # before call k + depth reuses the buffers
    torch.cuda.synchronize()
    fl.check_errors()
    for k in range(calls):
        for a, b in zip(want[k], got[k]):
            assert torch.equal(a, b), k


@pytest.mark.parametrize("N,M", [(64, 8), (7, 5), (30, 1), (12, 2)])
def test_fused_events_sizes_vs_oracle(tm, N, M):
    """The fused sampler at the largest supported shape (N=64, M=8: W=512 walks per group, edge-count
    fields at their widest) and at walks-per-slot values outside the specialised M=3 / M=1 kernels,
    bit-exact vs the C oracle (every sampled field, categories, edge counts, histogram)."""
    from tempme_amd.preprocess import sample_events
    g, rows, (src, dst, ts, eidx), pool, f = _pareto_finder(tm, seed=13, alpha=1.2, node_feat="uniform")
    dev = f.device
    E = 24
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:E], dtype=dt)).to(dev)  # noqa: E731
    b = sample_events(f.graph, 13, px.SPLIT_TEST, N, M, t(src, np.int32), t(dst, np.int32), t(ts, np.float64),
                      t(eidx, np.int32), torch.arange(E, dtype=torch.int32, device=dev),
                      torch.from_numpy(np.asarray(pool, np.int32)).to(dev))
    og = orc.OracleGraph(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"])
    o = orc.event_pipeline(og, 13, px.SPLIT_TEST, N, M, src[:E], dst[:E], ts[:E], eidx[:E], np.arange(E), pool, 8)
    h = lambda x: x.cpu().numpy()  # noqa: E731
    assert np.array_equal(h(b.dst_fake[:E]), o["dst_fake"])
    for name in ("node6", "eid3", "ts3", "cat", "sub1_node", "sub1_eid", "sub1_ts", "sub2_node", "sub2_eid",
                 "sub2_ts"):
        assert np.array_equal(h(getattr(b, name)).swapaxes(0, 1), o[name]), name
    assert np.array_equal(h(b.cnt).swapaxes(0, 1).astype(np.int32), o["cnt"])
    assert np.array_equal(h(b.hist).astype(np.uint64), o["hist"])


@pytest.mark.parametrize("de", [32, 172])
def test_edge_table_path(tm, de):
    """tm_edge_tables' edge table = lin_event.W[:, :de] E[e] + lin_event.b (fp64 reference, 1e-5), zero past dn;
    the pipeline's table mode (lin_event's edge part read per edge id) agrees with the per-walk
    product (edge_table=False, the drop-in TempME.forward arithmetic) within the 1e-5 contract, and
    its gate table is unchanged."""
    from tempme_amd.pipeline import ExplainPipeline
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=150, n_edges=5000, alpha=1.5, de=de, dn=172, node_feat="uniform", seed=21)
    (src, dst, ts, eidx), rows, pool = split(g)
    dev = torch.device("cuda", 0)
    f = _finder(tm, g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"], seed=6)
    torch.manual_seed(3)
    ex = tm.TempME(_Base(g["n_feat"], g["e_feat"], dev), "tgn", "x", 40, 64, device=dev,
                   null_model={k: 1 / 12 for k in range(1, 13)}).to(dev).eval()
    N, B, E = 20 if de == 32 else 30, 50, 100
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:E], dtype=dt)).to(dev)  # noqa: E731
    args = (t(src, np.int32), t(dst, np.int32), t(ts, np.float64), t(eidx, np.int32),
            torch.arange(E, dtype=torch.int32, device=dev))
    pt = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=6)
    pp = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=6, edge_table=False)
    a = [x.clone() for x in pt.run(*args)]
    b = [x.clone() for x in pp.run(*args)]
    torch.cuda.synchronize()
    pt.check_errors()
    pp.check_errors()
    assert pt.etab is not None and pp.etab is None
    w = ex.event_conv.lin_event.weight.detach().double().cpu()
    ef = torch.from_numpy(g["e_feat"]).double()[:pt.etab.shape[0]]
    want = ef @ w[:, :de].T + ex.event_conv.lin_event.bias.detach().double().cpu()
    got = pt.etab.double().cpu()
    np.testing.assert_allclose(got[:, :172].numpy(), want.numpy(), rtol=1e-5, atol=1e-6)
    assert (got[:, 172:] == 0).all()
    assert torch.equal(pt.gf, pp.gf)
    np.testing.assert_allclose(a[0].cpu().numpy(), b[0].cpu().numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(a[1].cpu().numpy(), b[1].cpu().numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(a[2].cpu().numpy(), b[2].cpu().numpy(), rtol=RTOL, atol=ATOL)


def test_edge_tables_cached_per_weight_state(tm):
    """The pipeline's per-edge-id tables (gate factor + lin_event's edge product) are built once per weight
    state and reused: repeated calls build nothing and give bitwise the same outputs; the cached tables equal
    a forced rebuild bitwise; an in-place change of the gate weights or of lin_event rebuilds them (the new
    tables equal a fresh pipeline's); two steps in flight share one build."""
    from tempme_amd.pipeline import ExplainPipeline, PipelinedExplainer
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=120, n_edges=4000, alpha=1.3, seed=23)
    (src, dst, ts, eidx), rows, pool = split(g)
    dev = torch.device("cuda", 0)
    f = _finder(tm, g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"], seed=4)
    torch.manual_seed(5)
    ex = tm.TempME(_Base(g["n_feat"], g["e_feat"], dev), "tgn", "x", 40, 64, device=dev,
                   null_model={k: 1 / 12 for k in range(1, 13)}).to(dev).eval()
    N, B, E = 20, 50, 100
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:E], dtype=dt)).to(dev)  # noqa: E731
    args = (t(src, np.int32), t(dst, np.int32), t(ts, np.float64), t(eidx, np.int32),
            torch.arange(E, dtype=torch.int32, device=dev))
    p = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=4)
    a = [x.clone() for x in p.run(*args)]
    b = [x.clone() for x in p.run(*args)]
    assert p.tabs.builds == 1
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    gf0, et0 = p.gf.clone(), p.etab.clone()
    p.tables(rebuild=True)
    torch.cuda.synchronize()
    assert torch.equal(gf0, p.gf) and torch.equal(et0, p.etab)
    with torch.no_grad():
        ex.edge_dependency_gcn[0].weight.mul_(1.25)
    p.run(*args)
    assert p.tabs.builds == 3
    fresh = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=4)
    c = [x.clone() for x in fresh.run(*args)]
    torch.cuda.synchronize()
    assert not torch.equal(gf0, p.gf) and torch.equal(fresh.gf, p.gf)
    with torch.no_grad():
        ex.event_conv.lin_event.weight.mul_(0.75)
    d = [x.clone() for x in p.run(*args)]
    fresh2 = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=4)
    e = [x.clone() for x in fresh2.run(*args)]
    torch.cuda.synchronize()
    assert p.tabs.builds == 4 and torch.equal(fresh2.etab, p.etab) and not torch.equal(et0, p.etab)
    for x, y in zip(d, e):
        assert torch.equal(x, y)
    assert not torch.equal(c[0], d[0])
    fl = PipelinedExplainer(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=4, depth=2)
    outs = []
    for _ in range(4):
        (imp, h1, h2), st = fl.submit(*args)
        torch.cuda.current_stream().wait_stream(st)
        outs.append([imp.clone(), h1.clone(), h2.clone()])
    torch.cuda.synchronize()
    fl.check_errors()
    assert fl.pipes[0].tabs is fl.pipes[1].tabs and fl.pipes[0].tabs.builds == 1
    for o in outs:
        for x, y in zip(o, e):
            assert torch.equal(x, y)


@pytest.mark.parametrize("hid,if_cat,tg", [(128, True, True), (64, False, True), (32, False, False), (48, True, True),
                                             (40, True, True), (20, False, True)])
def test_constructor_shapes_on_hip(tm, hid, if_cat, tg):
    """TempME(hid_dim, if_cat_feature, use_temporal_guidance) shapes outside the fused walk kernel run the
    LDS-tiled HIP kernels (tm_weights_create_ex): forward and retrieve_explanation(eval) within 1e-5 of the
    torch-fp32 oracle, and the HIP path (not the torch formulation) ran.  hid_dim 40 / 20 (not multiples of
    16) run on weights zero-padded to 48 / 32 (TempME._pad_hidden)."""
    from tests.encoder_inputs import SIDES, load
    d = load("synth")
    dev = torch.device("cuda", 0)
    torch.manual_seed(hid + 7 * if_cat)
    ex = tm.TempME(_Base(d["n_feat"], d["e_feat"], dev), "tgn", "x", out_dim=40, hid_dim=hid, device=dev,
                   if_cat_feature=if_cat, use_temporal_guidance=tg,
                   null_model={k + 1: float(v) for k, v in enumerate(d["null"])}).to(dev).eval()
    sd = {k: v.detach().cpu() for k, v in ex.state_dict().items()}
    imps, subs, walks = [], [], []
    for s in SIDES:
        x = d[s]
        w = (x["node"], x["eid"], x["ts"], x["cat"], x["marg"])
        with torch.no_grad():
            imp = ex(w, d["ts_cut"], x["cnt"])
        ref = er.forward(sd, d["n_feat"].float(), d["e_feat"].float(), x["node"], x["eid"], x["ts"], x["cat"],
                         d["ts_cut"], x["cnt"], temporal=tg, if_cat=if_cat)
        np.testing.assert_allclose(imp.cpu().numpy(), ref.numpy(), rtol=RTOL, atol=ATOL, err_msg=s)
        imps.append(imp)
        subs.append((x["sub_node"], x["sub_eid"], x["sub_ts"]))
        walks.append(w)
    with torch.no_grad():
        expl = ex.retrieve_explanation(subs[0], imps[0], walks[0], subs[1], imps[1], walks[1], subs[2], imps[2],
                                       walks[2], training=False)
    for k, s in enumerate(SIDES):
        x = d[s]
        r0, r1 = er.edge_importance(sd, d["e_feat"].float(), imps[k].cpu(), x["eid"], x["ts"], x["sub_node"],
                                    x["sub_eid"])
        B = r0.shape[0]
        np.testing.assert_allclose(expl[0][k * B:(k + 1) * B].cpu().numpy(), r0.numpy(), rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(expl[1][k * B:(k + 1) * B].cpu().numpy(), r1.numpy(), rtol=RTOL, atol=ATOL)
    assert ex._packed is not None, "the HIP encoder did not run"


def test_hid_dim_above_256_fails_loudly(tm):
    """hid_dim > 256 has no HIP kernel instance: the forward raises TempMEError (no silent torch path)."""
    from tempme_amd import _lib as L
    from tests.encoder_inputs import load
    d = load("synth")
    dev = torch.device("cuda", 0)
    ex = tm.TempME(_Base(d["n_feat"], d["e_feat"], dev), "tgn", "x", out_dim=40, hid_dim=272, device=dev,
                   null_model={k + 1: float(v) for k, v in enumerate(d["null"])}).to(dev).eval()
    x = d["src"]
    with pytest.raises(L.TempMEError, match="hid_dim 1..256"):
        with torch.no_grad():
            ex((x["node"], x["eid"], x["ts"], x["cat"], x["marg"]), d["ts_cut"], x["cnt"])


def test_strict_temporal_view_vs_oracle(tm):
    """strict_temporal (tm_graph_strict_view, SURVEY §7 opt-in): the fused sampler on the strict view vs the
    C oracle in strict mode, bit-exact, on uslegis's late events (long lists, many ties); the parity-mode
    graph it views is unchanged, and the host find_before of a strict finder agrees."""
    from tempme_amd.preprocess import sample_events
    df = pd.read_csv(os.path.join(G, "data", "ml_uslegis_sampled.csv"))
    src, dst, eidx, ts = df.u.values, df.i.values, df.idx.values, df.ts.values
    f = tm.NeighborFinder.from_edges(src, dst, eidx, ts, 224, strict_temporal=True)
    fp = _finder(tm, src, dst, eidx, ts, 224)
    rows = np.arange(len(src) - 64, len(src))
    pool = np.unique(dst)
    og = orc.OracleGraph(src, dst, eidx, ts, 224, strict_temporal=True)
    dev = f.device
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[rows], dtype=dt)).to(dev)  # noqa: E731
    h = lambda x: x.cpu().numpy()  # noqa: E731
    for N, M in ((20, 3), (8, 1)):
        o = orc.event_pipeline(og, 0, px.SPLIT_TEST, N, M, src[rows], dst[rows], ts[rows], eidx[rows],
                               np.arange(len(rows)), pool, 8)
        outs = []
        for g in (f.graph, fp.graph):
            outs.append(sample_events(g, 0, px.SPLIT_TEST, N, M, t(src, np.int32), t(dst, np.int32),
                                      t(ts, np.float64), t(eidx, np.int32),
                                      torch.arange(len(rows), dtype=torch.int32, device=dev),
                                      torch.from_numpy(pool.astype(np.int32)).to(dev)))
        b, bp = outs
        for name in ("node6", "eid3", "ts3", "cat", "sub1_node", "sub1_eid", "sub1_ts", "sub2_node", "sub2_eid",
                     "sub2_ts"):
            assert np.array_equal(h(getattr(b, name)).swapaxes(0, 1), o[name]), name
        assert np.array_equal(h(b.cnt).swapaxes(0, 1).astype(np.int32), o["cnt"])
        assert not torch.equal(b.eid3, bp.eid3)        # the view changed the walks, not the parent graph
    ref = orc.event_pipeline(orc.OracleGraph(src, dst, eidx, ts, 224), 0, px.SPLIT_TEST, 8, 1, src[rows],
                             dst[rows], ts[rows], eidx[rows], np.arange(len(rows)), pool, 8)
    assert np.array_equal(h(bp.eid3).swapaxes(0, 1), ref["eid3"])
    for u, e in ((int(src[-1]), int(eidx[-1])), (int(dst[-5]), int(eidx[-5]))):
        assert len(f.find_before(u, 0.0, e_idx=e)[0]) == og.find_before(u, 0.0, e)
