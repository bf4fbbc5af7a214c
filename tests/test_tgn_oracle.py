"""Base-TGN consumer on the CPU: the seeded model equals the reference's, and the
oracle (oracle/tgn_ref.py) reproduces the reference's outputs in tests/golden/tgn_uslegis.npz
(make_goldens.py case_tgn ran the reference TGN: contrast without / with explanation weights, with
explicit edge features, and threshold_test over its 16 ratios)."""
import math

import numpy as np
import pytest
import torch

import tgn_inputs as TI
from oracle import tgn_ref as O

CASES = ("uslegis", "synth")
# the reference's own fp32 result differs from its fp64 evaluation by up to ~2e-6 on these logits
# (test_reference_fp32_envelope); the oracle (fp32, same op order) and the HIP path are held to a
# tolerance a few times that envelope
ORACLE_ATOL, ORACLE_RTOL = 5e-6, 1e-5


def _sd(m):
    return {k: v.detach() for k, v in m.state_dict().items()}


def _tags(case):
    tags = [("ori", None, None), ("expl", TI.explanation(case), None), ("rand", TI.rand_weights(case), None)]
    if case == "uslegis":
        tags.append(("attr", TI.explanation(case), TI.edge_attr()))
    return tags


@pytest.mark.parametrize("case", CASES)
def test_seeded_init_matches_reference(case):
    g = TI.golden()
    m = TI.build_model(case)
    torch.manual_seed(TI.SEEDS[case])
    from tempme_amd.tgn import TGN
    nf, ef = TI.feats(case)
    fresh = TGN(nf, ef, n_neighbors=TI.N_DEG, device=torch.device("cpu"), n_layers=3, n_heads=2, dropout=0.5)
    sd = fresh.state_dict()
    keys = {k[len(case) + 4:] for k in g.files if k.startswith(f"{case}_sd_")}
    assert keys == set(sd), "state_dict keys differ from the reference TGN's"
    for k in keys:
        v = sd[k].double()
        c = np.array([v.sum().item(), v.abs().sum().item(), (v * v).sum().item()])
        assert np.allclose(c, g[f"{case}_sd_{k}"], rtol=1e-12, atol=0), k
    assert m.memory.messages and len(m.memory.messages) == 5


@pytest.mark.parametrize("case", CASES)
def test_oracle_updated_memory(case):
    g = TI.golden()
    m = TI.build_model(case)
    nf, _ = TI.feats(case)
    um = O.updated_memory(_sd(m), m.memory.messages, nf.shape[0])
    np.testing.assert_allclose(um.numpy(), g[f"{case}_updated_memory"], atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("case", CASES)
def test_oracle_contrast_matches_reference(case):
    g, d = TI.golden(), TI.load_batch()
    m = TI.build_model(case)
    nf, ef = TI.feats(case)
    for tag, ew, ea in _tags(case):
        p, n = O.contrast(_sd(m), m.memory.messages, nf, ef, d["src"], d["dst"], d["fake"], d["ts_cut"], d["sg_src"],
                          d["sg_tgt"], d["sg_bgd"], TI.N_DEG, 2, ew, ea)
        np.testing.assert_allclose(torch.cat([p, n]).numpy(), g[f"{case}_{tag}"], atol=ORACLE_ATOL,
                                   rtol=ORACLE_RTOL, err_msg=tag)


def test_reference_fp32_envelope():
    """fp64 evaluation of the same graph vs the reference's fp32 outputs: the rounding envelope the
    GPU tolerance is set from."""
    g, d = TI.golden(), TI.load_batch()
    case = "synth"
    m = TI.build_model(case)
    nf, ef = TI.feats(case)
    p, n = O.contrast(_sd(m), m.memory.messages, nf, ef, d["src"], d["dst"], d["fake"], d["ts_cut"], d["sg_src"],
                      d["sg_tgt"], d["sg_bgd"], TI.N_DEG, 2, TI.explanation(case), None, dtype=torch.float64)
    err = np.abs(torch.cat([p, n]).numpy() - g[f"{case}_expl"]).max()
    assert 0 < err < 1e-5


def _golden_masks(case):
    g, d = TI.golden(), TI.load_batch()
    B, N = d["B"], d["N"]
    ne = N + N * N
    G = len(g["ratios"])
    bits = np.unpackbits(g[f"{case}_thr_zero_bits"])[:G * 3 * B * ne].reshape(G, 3 * B, ne).astype(bool)
    return g, d, bits


@pytest.mark.parametrize("case", CASES)
def test_oracle_threshold_contrast(case):
    """Masked-subgraph contrasts of threshold_test: masks from CPU topk (the reference op) equal the
    golden ones, and the oracle's logits on them equal the golden logits."""
    g, d, bits = _golden_masks(case)
    B, N = d["B"], d["N"]
    ne = N + N * N
    m = TI.build_model(case)
    nf, ef = TI.feats(case)
    expl = TI.explanation(case)
    for ri in (0, 7, 15):
        r = g["ratios"][ri]
        topk = min(max(math.ceil(r * ne), 1), ne)
        subs = []
        for si, s in enumerate(TI.SIDES):
            imp = torch.cat([expl[0][si * B:(si + 1) * B], expl[1][si * B:(si + 1) * B]], 1).numpy()
            sub = O.masked_subgraph(d["sg_" + s], O.select_k_smallest(imp, ne - topk), N)
            assert np.array_equal(np.concatenate(sub[0], 1) == 0, bits[ri, si * B:(si + 1) * B])
            subs.append(sub)
        p, n = O.contrast(_sd(m), m.memory.messages, nf, ef, d["src"], d["dst"], d["fake"], d["ts_cut"], *subs,
                          TI.N_DEG, 2)
        np.testing.assert_allclose(torch.cat([p, n]).numpy(), g[f"{case}_thr_logits"][ri], atol=ORACLE_ATOL,
                                   rtol=ORACLE_RTOL)


@pytest.mark.parametrize("case", CASES)
def test_threshold_metrics_from_golden_logits(case):
    """The metric reduction fidelity.threshold_test applies, on the reference's own logits."""
    from sklearn.metrics import average_precision_score, roc_auc_score
    g = TI.golden()
    pos_o, neg_o = np.split(g[f"{case}_ori"].reshape(-1), 2)
    y = (1 / (1 + np.exp(-np.concatenate([pos_o, neg_o]))) > 0.5).astype(np.float32)
    aps, auc, acc, fp, fl = [], [], [], [], []
    for lg in g[f"{case}_thr_logits"]:
        lg = torch.from_numpy(lg.reshape(-1))
        pos, neg = lg[:len(pos_o)], lg[len(pos_o):]
        po, no = torch.from_numpy(pos_o), torch.from_numpy(neg_o)
        pred = torch.cat([pos, neg]).sigmoid()
        fp.append(torch.cat([pos.sigmoid() - po.sigmoid(), no.sigmoid() - neg.sigmoid()]).mean().item())
        fl.append(torch.cat([pos - po, no - neg]).mean().item())
        aps.append(average_precision_score(y, pred.numpy()))
        auc.append(roc_auc_score(y, pred.numpy()))
        acc.append(((pred > 0.5).float().numpy() == y).mean())
    np.testing.assert_allclose([np.mean(aps), np.mean(auc), np.mean(acc), np.mean(fp), np.mean(fl)],
                               g[f"{case}_thr_metrics"], rtol=1e-6, atol=1e-7)


def test_contrast_without_gpu_fails_loudly():
    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    d = TI.load_batch()
    m = TI.build_model("uslegis")
    with pytest.raises(RuntimeError, match="no HIP device"):
        m.contrast(d["src"], d["dst"], d["fake"], d["ts_cut"], d["e_idx"], d["sg_src"], d["sg_tgt"], d["sg_bgd"])
