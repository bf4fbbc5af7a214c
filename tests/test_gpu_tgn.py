"""GPU parity of the base-TGN consumer: TGN.contrast with explanation weights,
threshold_test and the explanation-weight gradient, through the C ABI (tm_tgn_attn_fwd / _bwd,
tm_mask_least_important), against the reference's outputs (tests/golden/tgn_uslegis.npz) and the
CPU oracle (oracle/tgn_ref.py).

Tolerance: the reference's own fp32 logits sit up to ~2e-6 from an fp64 evaluation of the same graph
(test_tgn_oracle.test_reference_fp32_envelope); the HIP path folds the per-neighbour projections
(fp32 reassociation of the same sums) and is held to atol 2e-5 + rtol 1e-5 on logits.  Masks
(which entries threshold_test zeroes) are bit-exact, ties included.
"""
import math
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import tgn_inputs as TI
from oracle import tgn_ref as O

pytestmark = pytest.mark.gpu

ATOL, RTOL = 2e-5, 1e-5
CASES = ("uslegis", "synth")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    return torch.device("cuda", 0)


def _model(case, dev, on_device=True):
    m = TI.build_model(case)
    if on_device:
        m = m.to(dev)
    return m


def _sd(m):
    return {k: v.detach().cpu() for k, v in m.state_dict().items()}


def _run(m, d, ew=None, ea=None, dev=None):
    if ew is not None:
        ew = [x.to(dev) for x in ew]
    p, n = m.contrast(d["src"], d["dst"], d["fake"], d["ts_cut"], d["e_idx"], d["sg_src"], d["sg_tgt"], d["sg_bgd"],
                      explain_weights=ew, edge_attr=ea)
    return torch.cat([p, n]).detach().cpu().numpy()


@pytest.mark.parametrize("case", CASES)
def test_contrast_matches_reference(dev, case):
    g, d = TI.golden(), TI.load_batch()
    m = _model(case, dev, on_device=(case == "uslegis"))      # host-resident parameters work too
    tags = [("ori", None, None), ("expl", TI.explanation(case), None), ("rand", TI.rand_weights(case), None)]
    if case == "uslegis":
        tags.append(("attr", TI.explanation(case), TI.edge_attr()))
    for tag, ew, ea in tags:
        out = _run(m, d, ew, ea, dev)
        np.testing.assert_allclose(out, g[f"{case}_{tag}"], atol=ATOL, rtol=RTOL, err_msg=tag)
    m.check_errors()


@pytest.mark.parametrize("case", CASES)
def test_updated_memory_matches_reference(dev, case):
    g = TI.golden()
    m = _model(case, dev)
    np.testing.assert_allclose(m.updated_memory().cpu().numpy(), g[f"{case}_updated_memory"], atol=2e-6, rtol=1e-5)


def test_head_major_pairing_matters(dev):
    """The reference's mask / explanation-weight row pairing is not the identity: turning it off
    changes the logits (so the parity above really exercises it)."""
    d = TI.load_batch()
    m = _model("synth", dev)
    a = _run(m, d, TI.rand_weights("synth"), None, dev)
    m.head_major_rows = False
    b = _run(m, d, TI.rand_weights("synth"), None, dev)
    assert np.abs(a - b).max() > 1e-3


@pytest.mark.parametrize("case", CASES)
def test_threshold_test_matches_reference(dev, case):
    from tempme_amd import fidelity
    g, d = TI.golden(), TI.load_batch()
    B, N = d["B"], d["N"]
    ne = N + N * N
    G = len(g["ratios"])
    m = _model(case, dev)
    expl = [x.to(dev) for x in TI.explanation(case)]
    sgs = (d["sg_src"], d["sg_tgt"], d["sg_bgd"])
    masked = fidelity._masked_nodes(expl, sgs, N, list(g["ratios"]), dev).cpu().numpy()
    bits = np.unpackbits(g[f"{case}_thr_zero_bits"])[:G * 3 * B * ne].reshape(G, 3 * B, ne).astype(bool)
    assert np.array_equal(masked == 0, bits)                  # bit-exact, tie order included
    pos, neg = fidelity.masked_contrast(m, expl, d["src"], d["dst"], d["fake"], d["ts_cut"], *sgs, N, list(g["ratios"]))
    got = torch.cat([pos, neg], dim=1).detach().cpu().numpy()
    np.testing.assert_allclose(got, g[f"{case}_thr_logits"].reshape(G, 2 * B), atol=ATOL, rtol=RTOL)
    ori = torch.from_numpy(g[f"{case}_ori"]).to(dev)
    pos_o, neg_o = ori[:B], ori[B:]
    y_ori = torch.where(ori.sigmoid() > 0.5, 1., 0.).view(-1, 1)
    args = SimpleNamespace(ratios=list(g["ratios"]), base_type="tgn", n_degree=N, bs=B)
    metrics = fidelity.threshold_test(args, expl, m, d["src"], d["dst"], d["fake"], d["ts_cut"], d["e_idx"], pos_o,
                                      neg_o, y_ori, *sgs)
    np.testing.assert_allclose(metrics, g[f"{case}_thr_metrics"], atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("n", [20, 420, 930, 2000])
def test_mask_kernel_equals_cpu_topk(dev, n):
    from tempme_amd import fidelity  # noqa: F401  (loads the library)
    from tempme_amd import _lib as L
    rng = np.random.default_rng(n)
    rows = 96
    imp = (rng.integers(0, 7, (rows, n)) / 7).astype(np.float32)
    imp[rng.uniform(size=imp.shape) < 0.02] = np.nan
    nodes = rng.integers(1, 1000, (rows, n)).astype(np.int32)
    ks = [1, 2, max(1, n // 64), n // 3, n - 3, n]
    out = torch.empty((len(ks), rows, n), dtype=torch.int32, device=dev)
    kd = torch.tensor(ks, dtype=torch.int32, device=dev)
    imp_d, nodes_d = torch.from_numpy(imp).to(dev), torch.from_numpy(nodes).to(dev)
    L.check(L.lib().tm_mask_least_important(L.ptr(imp_d), rows, n, L.ptr(kd), len(ks), L.ptr(nodes_d), L.ptr(out),
                                            L.stream_ptr(dev)))
    out = out.cpu().numpy()
    for gi, k in enumerate(ks):
        ref = nodes.copy()
        np.put_along_axis(ref, torch.topk(torch.from_numpy(imp), k=k, dim=-1, largest=False).indices.numpy(), 0, axis=-1)
        assert np.array_equal(out[gi], ref), k


def test_segments_equal_separate_calls(dev):
    """n_segments stacks independent batches (the batched threshold_test relies on it)."""
    d = TI.load_batch()
    m = _model("synth", dev)
    ew_a, ew_b = [x.to(dev) for x in TI.explanation("synth")], [x.to(dev) for x in TI.rand_weights("synth")]
    sgs = (d["sg_src"], d["sg_tgt"], d["sg_bgd"])
    roots = torch.cat([torch.as_tensor(x).long() for x in (d["src"], d["dst"], d["fake"])]).to(dev)

    def cat(i, h, dt):
        return torch.cat([torch.as_tensor(np.asarray(sg[i][h])).to(dt) for sg in sgs]).to(dev)
    nodes = [roots, cat(0, 0, torch.int32), cat(0, 1, torch.int32)]
    eids = [cat(1, 0, torch.int32), cat(1, 1, torch.int32)]
    times = [cat(2, 0, torch.float64), cat(2, 1, torch.float64)]
    one_a = m.node_embeddings(nodes, eids, times, d["ts_cut"], ew_a)
    one_b = m.node_embeddings(nodes, eids, times, d["ts_cut"], ew_b)
    two = m.node_embeddings([x.repeat(2) if x.dim() == 1 else x.repeat(2, 1) for x in nodes],
                            [x.repeat(2, 1) for x in eids], [x.repeat(2, 1) for x in times], d["ts_cut"],
                            [torch.cat([ew_a[0], ew_b[0]]), torch.cat([ew_a[1], ew_b[1]])], n_segments=2)
    torch.testing.assert_close(two, torch.cat([one_a, one_b]), atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("case", CASES)
def test_explanation_weight_gradient_vs_oracle(dev, case):
    """d BCE(contrast(explain_weights=e), y) / d e through tgn_attn_bwd_kernel + autograd vs torch
    autograd through the literal fp64 oracle (temp_exp_main.py:614-631 trains on exactly this)."""
    d = TI.load_batch()
    m = _model(case, dev)
    nf, ef = TI.feats(case)
    base = TI.rand_weights(case)
    y = torch.cat([torch.ones(d["B"], 1), torch.zeros(d["B"], 1)])
    ew = [x.clone().to(dev).requires_grad_(True) for x in base]
    p, n = m.contrast(d["src"], d["dst"], d["fake"], d["ts_cut"], d["e_idx"], d["sg_src"], d["sg_tgt"], d["sg_bgd"],
                      explain_weights=ew)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(torch.cat([p, n]), y.to(dev))
    loss.backward()
    ew64 = [x.clone().double().requires_grad_(True) for x in base]
    p64, n64 = O.contrast(_sd(m), m.memory.messages, nf, ef, d["src"], d["dst"], d["fake"], d["ts_cut"], d["sg_src"],
                          d["sg_tgt"], d["sg_bgd"], TI.N_DEG, 2, ew64, None, dtype=torch.float64)
    loss64 = torch.nn.functional.binary_cross_entropy_with_logits(torch.cat([p64, n64]), y.double())
    loss64.backward()
    assert abs(loss.item() - loss64.item()) < 1e-5
    for a, b in zip(ew, ew64):
        ga, gb = a.grad.double().cpu(), b.grad
        assert torch.linalg.norm(ga - gb) <= 1e-4 * torch.linalg.norm(gb)
        assert (ga - gb).abs().max() <= 1e-6 + 1e-4 * gb.abs().max()
    assert all(p.grad is None for p in m.parameters())           # frozen base model


def _random_case(seed, V=400, E=5000, N=30, B=16, dn=172, de=32):
    rng = np.random.default_rng(seed)
    nf = rng.uniform(-1, 1, (V, dn)).astype(np.float32)
    nf[0] = 0
    ef = rng.uniform(-1, 1, (E + 1, de)).astype(np.float32)
    ef[0] = 0

    def rec(rows, width, cut):
        node = rng.integers(1, V, (rows, width))
        node[rng.uniform(size=node.shape) < 0.15] = 0
        eid = np.where(node > 0, rng.integers(1, E + 1, node.shape), 0)
        ts = np.where(node > 0, np.floor(cut[:, None] - rng.uniform(0, 5e7, node.shape)), 0.0)
        return node.astype(np.float64), eid.astype(np.float64), ts.astype(np.float64)
    cut = np.floor(rng.uniform(5e7, 1e8, B))
    sgs = []
    for _ in range(3):
        n1, e1, t1 = rec(B, N, cut)
        n2, e2, t2 = rec(B, N * N, np.repeat(cut, 1))
        sgs.append(([n1, n2], [e1, e2], [t1, t2]))
    src, dst, fake = (rng.integers(1, V, B) for _ in range(3))
    ew = [torch.from_numpy(rng.uniform(0, 1, (3 * B, N)).astype(np.float32)),
          torch.from_numpy(rng.uniform(0, 1, (3 * B, N * N)).astype(np.float32))]
    return nf, ef, src, dst, fake, cut, sgs, ew


def test_contrast_n30_enron_dims_vs_oracle(dev):
    """N = 30, de = 32 (Enron-shaped key dim 376), random memory: HIP path vs the fp64 oracle."""
    from tempme_amd.tgn import TGN
    nf, ef, src, dst, fake, cut, sgs, ew = _random_case(3)
    torch.manual_seed(3)
    m = TGN(nf, ef, n_neighbors=30, device=torch.device("cpu"), n_layers=2, n_heads=2, dropout=0.1)
    m.forbidden_memory_update = True
    with torch.no_grad():
        m.memory.memory.normal_(0, 0.5)
        m.time_encoder.w.bias.normal_(0, 0.5)
    m.eval()
    p, n = m.contrast(src, dst, fake, cut, None, *sgs, explain_weights=[x.to(dev) for x in ew])
    got = torch.cat([p, n]).detach().cpu().double().numpy()
    sd = {k: v.detach() for k, v in m.state_dict().items()}
    p64, n64 = O.contrast(sd, m.memory.messages, nf, ef, src, dst, fake, cut, *sgs, 30, 2, ew, None,
                          dtype=torch.float64)
    np.testing.assert_allclose(got, torch.cat([p64, n64]).numpy(), atol=ATOL, rtol=RTOL)
