"""GPU: retrieve_edge_imp_node in training (SURVEY.md §8 a13 with dropout in the dependency gate;
tm_explain_train_fwd / _bwd) against autograd through the oracle's restatement
(oracle/encoder_ref.edge_importance_train, explainer_new.py:354-393) with the SAME keep-masks: gathered
maxima within 1e-5, gradients of imp within 2e-4 and of the 8 gate / time-encoder tensors within 2e-5 of
the fp32 reference's norm (5e-3 of an fp64 one).  Walks repeat an edge (same id and time) at two positions, so tied maxima occur and
the tie-splitting of the scatter-max gradient is exercised."""
import numpy as np
import pytest
import torch

from oracle import encoder_ref as er

pytestmark = pytest.mark.gpu

GATE = ("edge_dependency_gcn.0.weight", "edge_dependency_gcn.0.bias", "edge_dependency_gcn.3.weight",
        "edge_dependency_gcn.3.bias", "edge_dependency_gcn.6.weight", "edge_dependency_gcn.6.bias",
        "time_encoder.basis_freq", "time_encoder.phase")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    return torch.device("cuda", 0)


class _Base:
    def __init__(self, n_feat, e_feat):
        self.n_feat_th = torch.from_numpy(n_feat)
        self.e_feat_th = torch.from_numpy(e_feat)
        self.node_raw_features = torch.nn.Embedding.from_pretrained(self.n_feat_th, padding_idx=0, freeze=True)
        self.edge_raw_features = torch.nn.Embedding.from_pretrained(self.e_feat_th, padding_idx=0, freeze=True)


@pytest.mark.parametrize("de,G,B,N,train", [(32, 3, 12, 20, True), (1, 2, 5, 5, True), (32, 1, 7, 10, False)])
def test_explain_backward_matches_autograd(dev, de, G, B, N, train):
    from tempme_amd import TempME
    rng = np.random.RandomState(de + B)
    V, E, W = 50, 400, 3 * N
    n_feat = rng.uniform(0, 1, (V + 1, 172)).astype(np.float32)
    e_feat = rng.uniform(0, 1, (E + 1, de)).astype(np.float32)
    n_feat[0] = 0
    e_feat[0] = 0
    eid3 = rng.randint(0, E + 1, (G, B, W, 3)).astype(np.int32)
    ts3 = rng.uniform(0, 1e6, (G, B, W, 3)).astype(np.float32)
    dup = rng.uniform(size=(G, B, W)) < 0.3                       # the same edge at positions 0 and 2
    eid3[..., 2][dup] = eid3[..., 0][dup]
    ts3[..., 2][dup] = ts3[..., 0][dup]
    s1e = rng.randint(0, E + 1, (G, B, N)).astype(np.int32)
    s1e[..., : N // 2] = eid3[..., : N // 2, 0]                   # most slots hit a walk edge
    s2e = rng.randint(0, E + 1, (G, B, N * N)).astype(np.int32)
    m2 = min(N * N // 2, 3 * W)
    s2e[..., :m2] = eid3.reshape(G, B, -1)[..., :m2]
    s1n = rng.randint(0, 3, (G, B, N)).astype(np.int32)
    s2n = rng.randint(0, 3, (G, B, N * N)).astype(np.int32)
    imp_np = rng.uniform(0.05, 0.95, (G, B, W)).astype(np.float32)
    torch.manual_seed(9)
    ex = TempME(_Base(n_feat, e_feat), "tgn", "synth", 40, 64, device=dev,
                null_model={k: 1 / 12 for k in range(1, 13)}).to(dev)
    ex.train(train)
    R = G * B * 3 * W
    masks = ex.gate_dropout_masks(R)
    assert (masks[0] is None) == (not train)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    imp = t(imp_np).requires_grad_(True)
    args = (t(eid3), t(ts3), t(s1e), t(s2e), masks, G, B, W, N)
    from tempme_amd.explainer import _ExplainFn
    p, _ = _ExplainFn.apply(ex, args, imp.reshape(-1), *ex._gate_params())
    p1, p2 = p[:G * B * N], p[G * B * N:]
    w1 = torch.from_numpy(rng.uniform(-1, 1, G * B * N).astype(np.float32))
    w2 = torch.from_numpy(rng.uniform(-1, 1, G * B * N * N).astype(np.float32))
    ((p1 * w1.to(dev)).sum() + (p2 * w2.to(dev)).sum()).backward()
    named = dict(ex.named_parameters())
    got = {k: named[k].grad.detach().cpu().double() for k in GATE}
    got_imp = imp.grad.detach().cpu().double()

    # fp32 autograd through the oracle is the tight reference; fp64 a looser sanity bound (a ReLU input
    # within fp32 rounding of 0 can switch sides between fp32 and fp64 evaluation and move ~1e-3 of a
    # gate weight's gradient)
    for dty, tol in ((torch.float32, 2e-5), (torch.float64, 5e-3)):
        sd = {k: v.detach().cpu().to(dty).requires_grad_(k in GATE) for k, v in ex.state_dict().items()}
        ef = torch.from_numpy(e_feat)
        imp_ref = torch.from_numpy(imp_np).to(dty).requires_grad_(True)
        k1 = None if masks[0] is None else masks[0].cpu().numpy().reshape(G, B, 3 * W, -1)
        k2 = None if masks[1] is None else masks[1].cpu().numpy().reshape(G, B, 3 * W, -1)
        loss = 0
        for g in range(G):
            r1, r2 = er.edge_importance_train(sd, ef, imp_ref[g].unsqueeze(-1), eid3[g], ts3[g], [s1e[g], s2e[g]],
                                              None if k1 is None else k1[g], None if k2 is None else k2[g],
                                              masks[2], masks[3])
            np.testing.assert_allclose(p1.detach().cpu().numpy().reshape(G, B, N)[g], r1.detach().numpy(),
                                       rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(p2.detach().cpu().numpy().reshape(G, B, N * N)[g], r2.detach().numpy(),
                                       rtol=1e-5, atol=1e-6)
            loss = loss + (r1.reshape(-1) * w1.to(dty).reshape(G, -1)[g]).sum() \
                + (r2.reshape(-1) * w2.to(dty).reshape(G, -1)[g]).sum()
        loss.backward()
        gi = imp_ref.grad.double().reshape(-1)
        assert float((got_imp.reshape(-1) - gi).norm()) <= 2e-4 * float(gi.norm()) + 1e-9, dty
        for k in GATE:
            gr, ga = sd[k].grad.double(), got[k]
            assert ga.shape == gr.shape, k
            assert float((ga - gr).norm()) <= tol * float(gr.norm()) + 1e-9, (dty, k, float((ga - gr).norm()),
                                                                               float(gr.norm()))


@pytest.mark.parametrize("var", ["nodep", "h32", "h128", "h40"])
def test_explain_backward_variants_match_autograd(dev, var):
    """use_dependency_aware_sampling=False (no gate: d imp through the scatter-max alone, no gradient to the
    time encoder from this path) and the gate at hid_dim 32 / 128 / 40 (40: zero-padded to 48)."""
    from tempme_amd import TempME
    from tempme_amd.explainer import _ExplainFn
    kw = {"nodep": dict(hid_dim=64, use_dependency_aware_sampling=False), "h32": dict(hid_dim=32),
          "h128": dict(hid_dim=128), "h40": dict(hid_dim=40)}[var]
    h = kw.pop("hid_dim")
    rng = np.random.RandomState(h)
    de, G, B, N = 32, 2, 6, 10
    V, E, W = 50, 400, 3 * N
    n_feat = rng.uniform(0, 1, (V + 1, 172)).astype(np.float32)
    e_feat = rng.uniform(0, 1, (E + 1, de)).astype(np.float32)
    n_feat[0] = 0
    e_feat[0] = 0
    eid3 = rng.randint(0, E + 1, (G, B, W, 3)).astype(np.int32)
    ts3 = rng.uniform(0, 1e6, (G, B, W, 3)).astype(np.float32)
    dup = rng.uniform(size=(G, B, W)) < 0.3
    eid3[..., 2][dup] = eid3[..., 0][dup]
    ts3[..., 2][dup] = ts3[..., 0][dup]
    s1e = rng.randint(0, E + 1, (G, B, N)).astype(np.int32)
    s1e[..., : N // 2] = eid3[..., : N // 2, 0]
    s2e = rng.randint(0, E + 1, (G, B, N * N)).astype(np.int32)
    m2 = min(N * N // 2, 3 * W)
    s2e[..., :m2] = eid3.reshape(G, B, -1)[..., :m2]
    imp_np = rng.uniform(0.05, 0.95, (G, B, W)).astype(np.float32)
    torch.manual_seed(3)
    ex = TempME(_Base(n_feat, e_feat), "tgn", "synth", 40, h, device=dev,
                null_model={k: 1 / 12 for k in range(1, 13)}, **kw).to(dev)
    ex.train(True)
    assert ex._hip_ok(), var
    dep = ex.use_dependency_aware_sampling
    masks = ex.gate_dropout_masks(G * B * 3 * W)
    assert (masks[0] is None) == (not dep)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    imp = t(imp_np).requires_grad_(True)
    p, _ = _ExplainFn.apply(ex, (t(eid3), t(ts3), t(s1e), t(s2e), masks, G, B, W, N), imp.reshape(-1),
                            *ex._gate_params())
    p1, p2 = p[:G * B * N], p[G * B * N:]
    w1 = torch.from_numpy(rng.uniform(-1, 1, G * B * N).astype(np.float32))
    w2 = torch.from_numpy(rng.uniform(-1, 1, G * B * N * N).astype(np.float32))
    ((p1 * w1.to(dev)).sum() + (p2 * w2.to(dev)).sum()).backward()
    names = GATE if dep else GATE[-2:]
    named = dict(ex.named_parameters())
    got = {k: named[k].grad.detach().cpu().double() for k in names}
    sd = {k: v.detach().cpu().float().requires_grad_(k in names) for k, v in ex.state_dict().items()}
    imp_ref = torch.from_numpy(imp_np).requires_grad_(True)
    k1 = None if masks[0] is None else masks[0].cpu().numpy().reshape(G, B, 3 * W, -1)
    k2 = None if masks[1] is None else masks[1].cpu().numpy().reshape(G, B, 3 * W, -1)
    loss = 0
    for g in range(G):
        r1, r2 = er.edge_importance_train(sd, torch.from_numpy(e_feat), imp_ref[g].unsqueeze(-1), eid3[g], ts3[g],
                                          [s1e[g], s2e[g]], None if k1 is None else k1[g],
                                          None if k2 is None else k2[g], masks[2], masks[3], dependency=dep)
        np.testing.assert_allclose(p1.detach().cpu().numpy().reshape(G, B, N)[g], r1.detach().numpy(), rtol=1e-5,
                                   atol=1e-6)
        np.testing.assert_allclose(p2.detach().cpu().numpy().reshape(G, B, N * N)[g], r2.detach().numpy(),
                                   rtol=1e-5, atol=1e-6)
        loss = loss + (r1.reshape(-1) * w1.reshape(G, -1)[g]).sum() + (r2.reshape(-1) * w2.reshape(G, -1)[g]).sum()
    loss.backward()
    gi = imp_ref.grad.double().reshape(-1)
    assert float((imp.grad.detach().cpu().double().reshape(-1) - gi).norm()) <= 2e-4 * float(gi.norm()) + 1e-9
    for k in names:
        ga = got[k]
        if not dep:      # the time encoder is not on this path without the gate
            assert float(ga.abs().max()) == 0.0, k
            continue
        gr = sd[k].grad.double()
        assert ga.shape == gr.shape, k
        assert float((ga - gr).norm()) <= 2e-5 * float(gr.norm()) + 1e-9, (var, k)


def test_fused_beta_rsample_equals_torch(dev):
    """_BetaRsampleFn (tm_beta_params + torch._sample_dirichlet, torch._dirichlet_grad + tm_beta_rsample_bwd)
    = Beta(clamp(10p, 1), clamp(10(1-p), 1)).rsample() * pad under autograd, bitwise: same RNG draws, same
    sample, same gradient -- p includes values at the clamp boundaries (10p = 1, 10(1-p) = 1) and 0 / 1."""
    from tempme_amd import TempME
    from tempme_amd.explainer import _BetaRsampleFn
    rng = np.random.RandomState(3)
    n = 50000
    p_np = rng.uniform(0, 1, n).astype(np.float32)
    p_np[:6] = [0.1, 0.9, 0.0, 1.0, 0.05, 0.95]
    pad_np = (rng.uniform(size=n) < 0.8).astype(np.float32)
    g_np = rng.uniform(-1, 1, n).astype(np.float32)
    ex = TempME(_Base(np.zeros((3, 172), np.float32), np.zeros((3, 4), np.float32)), "tgn", "synth", 40, 64, device=dev,
                null_model={k: 1 / 12 for k in range(1, 13)}).to(dev)
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    outs = []
    for fused in (True, False):
        p = t(p_np).requires_grad_(True)
        torch.manual_seed(11)
        e = _BetaRsampleFn.apply(p, t(pad_np)) if fused else ex.beta_sample(p, True) * t(pad_np)
        (e * t(g_np)).sum().backward()
        outs.append((e.detach().clone(), p.grad.detach().clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1]), float((outs[0][1] - outs[1][1]).abs().max())
