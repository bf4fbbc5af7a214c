"""Base-GraphMixer consumer on the CPU: the seeded model equals the reference's,
and the oracle (oracle/graphmixer_ref.py) reproduces tests/golden/graphmixer_uslegis.npz (the
reference's contrast without / with explanation, random weights, edge_attr, threshold_test)."""
import math
import os

import numpy as np
import pytest
import torch

import tgn_inputs as TI
from oracle import graphmixer_ref as O

CASES = ("uslegis", "synth")
SEEDS = {"uslegis": 21, "synth": 22}
ATOL, RTOL = 5e-6, 1e-5


def golden():
    return np.load(os.path.join(TI.G, "graphmixer_uslegis.npz"))


def build(case):
    from tempme_amd.graphmixer import GraphMixer
    nf, ef = TI.feats(case)
    torch.manual_seed(SEEDS[case])
    m = GraphMixer(nf, ef, n_neighbors=TI.N_DEG, device=torch.device("cpu"), num_tokens=TI.N_DEG, num_layers=3,
                   dropout=0.5)
    return m.eval()


def _sd(m):
    return {k: v.detach() for k, v in m.state_dict().items()}


@pytest.mark.parametrize("case", CASES)
def test_seeded_init_matches_reference(case):
    g = golden()
    sd = build(case).state_dict()
    keys = {k[len(case) + 4:] for k in g.files if k.startswith(f"{case}_sd_")}
    assert keys == set(sd)
    for k in keys:
        v = sd[k].double()
        c = np.array([v.sum().item(), v.abs().sum().item(), (v * v).sum().item()])
        assert np.allclose(c, g[f"{case}_sd_{k}"], rtol=1e-12, atol=0), k


@pytest.mark.parametrize("case", CASES)
def test_oracle_contrast_matches_reference(case):
    g, d = golden(), TI.load_batch()
    sd = _sd(build(case))
    expl = [TI.explanation(case)[0]]
    for tag, ew, ea in (("ori", None, None), ("expl", expl, None), ("rand", [torch.from_numpy(g[f"{case}_ew_rand"])], None),
                        ("attr", expl, torch.from_numpy(g[f"{case}_edge_attr"]))):
        p, n = O.contrast(sd, 3, d["src"], d["dst"], d["fake"], d["ts_cut"], d["sg_src"], d["sg_tgt"], d["sg_bgd"], ew,
                          ea)
        np.testing.assert_allclose(torch.cat([p, n]).numpy(), g[f"{case}_{tag}"], atol=ATOL, rtol=RTOL, err_msg=tag)


@pytest.mark.parametrize("case", CASES)
def test_oracle_threshold_masks_and_logits(case):
    g, d = golden(), TI.load_batch()
    B, N = d["B"], d["N"]
    G = len(g["ratios"])
    bits = np.unpackbits(g[f"{case}_thr_zero_bits"])[:G * 3 * B * N].reshape(G, 3 * B, N).astype(bool)
    sd = _sd(build(case))
    imp = TI.explanation(case)[0].numpy()
    for ri in (0, 9, 15):
        topk = min(max(math.ceil(g["ratios"][ri] * N), 1), N)
        subs = []
        for si, s in enumerate(TI.SIDES):
            node0 = d["sg_" + s][0][0].copy()
            sel = torch.topk(torch.from_numpy(imp[si * B:(si + 1) * B]), k=N - topk, dim=-1, largest=False).indices
            np.put_along_axis(node0, sel.numpy(), 0, axis=-1)
            assert np.array_equal(node0 == 0, bits[ri, si * B:(si + 1) * B])
            subs.append(([node0, d["sg_" + s][0][1]], d["sg_" + s][1], d["sg_" + s][2]))
        p, n = O.contrast(sd, 3, d["src"], d["dst"], d["fake"], d["ts_cut"], *subs)
        np.testing.assert_allclose(torch.cat([p, n]).numpy(), g[f"{case}_thr_logits"][ri], atol=ATOL, rtol=RTOL)
