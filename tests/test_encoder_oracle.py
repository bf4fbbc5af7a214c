"""Pin the torch-fp32 encoder oracle against outputs of the reference TempME module
(tests/golden/encoder_uslegis.npz).  Tolerance: 1e-5 rel, 1e-6 abs floor (BASELINE north_star)."""
import numpy as np
import pytest
import torch

from oracle import encoder_ref as er
from tests.encoder_inputs import SIDES, load

RTOL, ATOL = 1e-5, 1e-6


@pytest.mark.parametrize("case", ["uslegis", "synth"])
def test_encoder_oracle_matches_reference(case):
    d = load(case)
    imps = []
    for s in SIDES:
        x = d[s]
        imp = er.forward(d["sd"], d["n_feat"], d["e_feat"], x["node"], x["eid"], x["ts"], x["cat"],
                         d["ts_cut"], x["cnt"])
        np.testing.assert_allclose(imp.numpy(), x["imp"], rtol=RTOL, atol=ATOL)
        imps.append(imp)
    e0, e1 = [], []
    for s, imp in zip(SIDES, imps):
        x = d[s]
        a, b = er.edge_importance(d["sd"], d["e_feat"], imp, x["eid"], x["ts"], x["sub_node"], x["sub_eid"])
        e0.append(a)
        e1.append(b)
    np.testing.assert_allclose(torch.cat(e0).numpy(), d["expl0"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(torch.cat(e1).numpy(), d["expl1"], rtol=RTOL, atol=ATOL)
    for k, (s, imp) in enumerate(zip(SIDES, imps)):
        kl = er.kl_loss(imp, d[s]["cat"], d["null"])
        np.testing.assert_allclose(float(kl), d["kl"][k], rtol=RTOL, atol=ATOL)
