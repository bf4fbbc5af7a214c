"""GPU parity of the base-GraphMixer consumer: contrast with hop-1 explanation
weights and threshold_test's graphmixer branch against the reference's outputs
(tests/golden/graphmixer_uslegis.npz) and the fp64 CPU oracle (oracle/graphmixer_ref.py).
Masks bit-exact; logits atol 2e-5 + rtol 1e-5 (as for TGN)."""
import math
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import tgn_inputs as TI
from oracle import graphmixer_ref as O
from tests.test_graphmixer_oracle import build, golden

pytestmark = pytest.mark.gpu
ATOL, RTOL = 2e-5, 1e-5
CASES = ("uslegis", "synth")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("case", CASES)
def test_contrast_matches_reference(dev, case):
    g, d = golden(), TI.load_batch()
    m = build(case).to(dev)
    expl = [TI.explanation(case)[0].to(dev)]
    for tag, ew, ea in (("ori", None, None), ("expl", expl, None),
                        ("rand", [torch.from_numpy(g[f"{case}_ew_rand"]).to(dev)], None),
                        ("attr", expl, torch.from_numpy(g[f"{case}_edge_attr"]).to(dev))):
        p, n = m.contrast(d["src"], d["dst"], d["fake"], d["ts_cut"], d["e_idx"], d["sg_src"], d["sg_tgt"],
                          d["sg_bgd"], explain_weights=ew, edge_attr=ea)
        np.testing.assert_allclose(torch.cat([p, n]).detach().cpu().numpy(), g[f"{case}_{tag}"], atol=ATOL, rtol=RTOL,
                                   err_msg=tag)


@pytest.mark.parametrize("case", CASES)
def test_threshold_test_matches_reference(dev, case):
    from tempme_amd import fidelity
    g, d = golden(), TI.load_batch()
    B, N = d["B"], d["N"]
    G = len(g["ratios"])
    m = build(case).to(dev)
    expl = [TI.explanation(case)[0].to(dev)]
    sgs = (d["sg_src"], d["sg_tgt"], d["sg_bgd"])
    masked = fidelity._masked_nodes(expl, sgs, N, list(g["ratios"]), dev, hops=1).cpu().numpy()
    bits = np.unpackbits(g[f"{case}_thr_zero_bits"])[:G * 3 * B * N].reshape(G, 3 * B, N).astype(bool)
    assert np.array_equal(masked == 0, bits)
    with torch.no_grad():
        pos, neg = fidelity.masked_contrast_graphmixer(m, expl, d["src"], d["dst"], d["fake"], d["ts_cut"], *sgs, N,
                                                       list(g["ratios"]))
    np.testing.assert_allclose(torch.cat([pos, neg], 1).cpu().numpy(), g[f"{case}_thr_logits"].reshape(G, 2 * B),
                               atol=ATOL, rtol=RTOL)
    ori = torch.from_numpy(g[f"{case}_ori"]).to(dev)
    y_ori = torch.where(ori.sigmoid() > 0.5, 1., 0.).view(-1, 1)
    args = SimpleNamespace(ratios=list(g["ratios"]), base_type="graphmixer", n_degree=N, bs=B)
    metrics = fidelity.threshold_test(args, expl, m, d["src"], d["dst"], d["fake"], d["ts_cut"], d["e_idx"], ori[:B],
                                      ori[B:], y_ori, *sgs)
    np.testing.assert_allclose(metrics, g[f"{case}_thr_metrics"], atol=2e-5, rtol=1e-5)


def test_config5_dims_and_gradient_vs_oracle(dev):
    """de = dn = 172, N = 30 (BASELINE configs[4] shapes): logits vs the fp64 oracle, and the
    explanation-weight gradient of a BCE loss vs fp64 autograd through the oracle."""
    from tempme_amd.graphmixer import GraphMixer
    rng = np.random.default_rng(5)
    V, E, N, B, d = 500, 4000, 30, 24, 172
    nf = rng.uniform(0, 1, (V, d)).astype(np.float32)
    ef = rng.uniform(0, 1, (E + 1, d)).astype(np.float32)
    nf[0] = ef[0] = 0
    torch.manual_seed(5)
    m = GraphMixer(nf, ef, n_neighbors=N, device=dev, num_tokens=N, num_layers=2, dropout=0.1).to(dev).eval()
    cut = np.floor(rng.uniform(5e7, 1e8, B))
    sgs = []
    for _ in range(3):
        node = rng.integers(1, V, (B, N))
        node[rng.uniform(size=node.shape) < 0.2] = 0
        eid = np.where(node > 0, rng.integers(1, E + 1, node.shape), 0)
        ts = np.where(node > 0, np.floor(cut[:, None] - rng.uniform(0, 5e7, node.shape)), 0.0)
        sgs.append(([node.astype(np.float64), None], [eid.astype(np.float64), None], [ts, None]))
    src, dst, fake = (rng.integers(1, V, B) for _ in range(3))
    ew0 = rng.uniform(0, 1, (3 * B, N)).astype(np.float32)
    y = torch.cat([torch.ones(B, 1), torch.zeros(B, 1)])
    ew = torch.from_numpy(ew0).to(dev).requires_grad_(True)
    p, n = m.contrast(src, dst, fake, cut, None, *sgs, explain_weights=[ew])
    torch.nn.functional.binary_cross_entropy_with_logits(torch.cat([p, n]), y.to(dev)).backward()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ew64 = torch.from_numpy(ew0).double().requires_grad_(True)
    p64, n64 = O.contrast(sd, 2, src, dst, fake, cut, *sgs, explain_weights=[ew64], dtype=torch.float64)
    torch.nn.functional.binary_cross_entropy_with_logits(torch.cat([p64, n64]), y.double()).backward()
    np.testing.assert_allclose(torch.cat([p, n]).detach().cpu().double().numpy(), torch.cat([p64, n64]).detach().numpy(),
                               atol=ATOL, rtol=RTOL)
    ga, gb = ew.grad.double().cpu(), ew64.grad
    assert torch.linalg.norm(ga - gb) <= 1e-4 * torch.linalg.norm(gb)
    assert getattr(m, "_gmb_key", None) is not None, "the HIP explanation-weight backward did not run"


@pytest.mark.parametrize("N,C,L", [(30, 172, 2), (12, 172, 2), (20, 32, 1), (16, 100, 3), (20, 1, 3)])
def test_hip_ew_gradient_vs_oracle(dev, N, C, L):
    """tm_gm_embed_bwd (the explainer's training signal through a frozen GraphMixer): d ew of a BCE loss on
    contrast's logits vs fp64 autograd through the oracle, for one / two token tiles, channel counts with and
    without padding, 1-3 mixer layers, padding neighbours and a row without any valid neighbour; the embedding's
    parameters get no gradient (frozen base, as the TGN base; the MergeLayer score stays torch autograd)."""
    from tempme_amd.graphmixer import GraphMixer
    rng = np.random.default_rng(N + C + L)
    V, E, B = 300, 2000, 20
    nf = rng.uniform(0, 1, (V, C)).astype(np.float32)
    ef = rng.uniform(0, 1, (E + 1, C)).astype(np.float32)
    nf[0] = ef[0] = 0
    torch.manual_seed(N + L)
    m = GraphMixer(nf, ef, n_neighbors=N, device=dev, num_tokens=N, num_layers=L, dropout=0.1).to(dev).eval()
    cut = np.floor(rng.uniform(5e7, 1e8, B))
    sgs = []
    for _ in range(3):
        node = rng.integers(1, V, (B, N))
        node[rng.uniform(size=node.shape) < 0.25] = 0
        node[1] = 0
        eid = np.where(node > 0, rng.integers(1, E + 1, node.shape), 0)
        ts = np.where(node > 0, np.floor(cut[:, None] - rng.uniform(0, 5e7, node.shape)), 0.0)
        sgs.append(([node.astype(np.float64), None], [eid.astype(np.float64), None], [ts, None]))
    src, dst, fake = (rng.integers(1, V, B) for _ in range(3))
    ew0 = rng.uniform(0, 1, (3 * B, N)).astype(np.float32)
    y = torch.cat([torch.ones(B, 1), torch.zeros(B, 1)])
    ew = torch.from_numpy(ew0).to(dev).requires_grad_(True)
    p, n = m.contrast(src, dst, fake, cut, None, *sgs, explain_weights=[ew])
    torch.nn.functional.binary_cross_entropy_with_logits(torch.cat([p, n]), y.to(dev)).backward()
    assert getattr(m, "_gmb_key", None) is not None, "the HIP explanation-weight backward did not run"
    assert all(q.grad is None for k, q in m.named_parameters() if not k.startswith("affinity_score"))
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ew64 = torch.from_numpy(ew0).double().requires_grad_(True)
    p64, n64 = O.contrast(sd, L, src, dst, fake, cut, *sgs, explain_weights=[ew64], dtype=torch.float64)
    torch.nn.functional.binary_cross_entropy_with_logits(torch.cat([p64, n64]), y.double()).backward()
    np.testing.assert_allclose(torch.cat([p, n]).detach().cpu().double().numpy(), torch.cat([p64, n64]).detach().numpy(),
                               atol=ATOL, rtol=RTOL)
    ga, gb = ew.grad.double().cpu(), ew64.grad
    assert float(torch.linalg.norm(ga - gb)) <= 1e-4 * float(torch.linalg.norm(gb)), \
        (float(torch.linalg.norm(ga - gb)), float(torch.linalg.norm(gb)))
    assert float(ga.abs()[torch.from_numpy(np.concatenate([sg[0][0] for sg in sgs]) == 0)].max()) == 0.0


@pytest.mark.parametrize("case", CASES)
def test_hip_embedding_matches_reference(dev, case):
    """The fused HIP embedding (tm_gm_embed: eval, no gradients) against the reference's outputs, for
    every explanation-weight / edge_attr variant of the golden batch."""
    g, d = golden(), TI.load_batch()
    m = build(case).to(dev).eval()
    expl = [TI.explanation(case)[0].to(dev)]
    with torch.no_grad():
        for tag, ew, ea in (("ori", None, None), ("expl", expl, None),
                            ("rand", [torch.from_numpy(g[f"{case}_ew_rand"]).to(dev)], None),
                            ("attr", expl, torch.from_numpy(g[f"{case}_edge_attr"]).to(dev))):
            p, n = m.contrast(d["src"], d["dst"], d["fake"], d["ts_cut"], d["e_idx"], d["sg_src"], d["sg_tgt"],
                              d["sg_bgd"], explain_weights=ew, edge_attr=ea)
            np.testing.assert_allclose(torch.cat([p, n]).cpu().numpy(), g[f"{case}_{tag}"], atol=ATOL, rtol=RTOL,
                                       err_msg=tag)
    assert getattr(m, "_gm_key", None) is not None, "the HIP embedding did not run"


@pytest.mark.parametrize("N", [30, 12])
def test_hip_embedding_config5_dims_vs_oracle(dev, N):
    """de = dn = 172 (BASELINE configs[4] shapes), N = 30 (two token tiles) and 12 (one): HIP logits vs the
    fp64 oracle, with and without explanation weights, padding neighbours included."""
    from tempme_amd.graphmixer import GraphMixer
    rng = np.random.default_rng(7 + N)
    V, E, B, d = 400, 3000, 40, 172
    nf = rng.uniform(0, 1, (V, d)).astype(np.float32)
    ef = rng.uniform(0, 1, (E + 1, d)).astype(np.float32)
    nf[0] = ef[0] = 0
    torch.manual_seed(11)
    m = GraphMixer(nf, ef, n_neighbors=N, device=dev, num_tokens=N, num_layers=2, dropout=0.1).to(dev).eval()
    cut = np.floor(rng.uniform(5e7, 1e8, B))
    sgs = []
    for _ in range(3):
        node = rng.integers(1, V, (B, N))
        node[rng.uniform(size=node.shape) < 0.25] = 0
        node[0] = 0                                   # a row without any valid neighbour
        eid = np.where(node > 0, rng.integers(1, E + 1, node.shape), 0)
        ts = np.where(node > 0, np.floor(cut[:, None] - rng.uniform(0, 5e7, node.shape)), 0.0)
        sgs.append(([node.astype(np.float64), None], [eid.astype(np.float64), None], [ts, None]))
    src, dst, fake = (rng.integers(1, V, B) for _ in range(3))
    ew0 = rng.uniform(0, 1, (3 * B, N)).astype(np.float32)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    for ew in (None, ew0):
        with torch.no_grad():
            p, n = m.contrast(src, dst, fake, cut, None, *sgs,
                              explain_weights=None if ew is None else [torch.from_numpy(ew).to(dev)])
        p64, n64 = O.contrast(sd, 2, src, dst, fake, cut, *sgs,
                              explain_weights=None if ew is None else [torch.from_numpy(ew).double()],
                              dtype=torch.float64)
        np.testing.assert_allclose(torch.cat([p, n]).cpu().double().numpy(), torch.cat([p64, n64]).numpy(),
                                   atol=ATOL, rtol=RTOL)
    assert getattr(m, "_gm_key", None) is not None, "the HIP embedding did not run"


def test_frozen_base_false_takes_torch_gradients(dev):
    """frozen_base = False: gradients wanted for the base model's own parameters as well -> the torch
    formulation (autograd), so they get a .grad; the default (frozen) HIP backward leaves them None."""
    from tempme_amd.graphmixer import GraphMixer
    rng = np.random.default_rng(5)
    V, E, B, N, C = 100, 500, 8, 12, 32
    nf = rng.uniform(0, 1, (V, C)).astype(np.float32)
    ef = rng.uniform(0, 1, (E + 1, C)).astype(np.float32)
    cut = np.floor(rng.uniform(5e7, 1e8, B))
    sgs = []
    for _ in range(3):
        node = rng.integers(1, V, (B, N))
        eid = rng.integers(1, E + 1, node.shape)
        ts = np.floor(cut[:, None] - rng.uniform(0, 5e7, node.shape))
        sgs.append(([node.astype(np.float64), None], [eid.astype(np.float64), None], [ts, None]))
    src, dst, fake = (rng.integers(1, V, B) for _ in range(3))
    grads = {}
    for frozen in (True, False):
        torch.manual_seed(1)
        m = GraphMixer(nf, ef, n_neighbors=N, device=dev, num_tokens=N, num_layers=1, dropout=0.1).to(dev).eval()
        m.frozen_base = frozen
        ew = torch.full((3 * B, N), 0.5, device=dev, requires_grad=True)
        p, n = m.contrast(src, dst, fake, cut, None, *sgs, explain_weights=[ew])
        torch.cat([p, n]).sum().backward()
        assert (getattr(m, "_gmb_key", None) is not None) == frozen
        assert (m.projection_layer.weight.grad is None) == frozen
        grads[frozen] = ew.grad.detach().clone()
    d = float((grads[True] - grads[False]).norm())
    assert d <= 1e-4 * float(grads[False].norm()) + 1e-9
