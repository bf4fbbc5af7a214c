"""Pin the CPU oracle in the bench regime (timestamps in [0, 1e8), full-Enron graph shape, Enron
feature dims) against outputs of the reference itself (tests/golden/enron_goldens.npz,
make_goldens.py case_enron): the split, every sampled field, categories, marginals and edge counts
bit-exact; the torch-fp32 encoder restatement within rtol 1e-5 / atol 1e-6 for the default
TempME constructor and its use_temporal_guidance=False / use_dependency_aware_sampling=False /
hid_dim=32 variants."""
import numpy as np
import pytest
import torch

import enron_inputs as EI
from oracle import encoder_ref as er
from oracle import oracle as orc
from oracle import philox as px
from tests.test_oracle_golden import _check_pipeline

RTOL, ATOL = 1e-5, 1e-6


@pytest.fixture(scope="module")
def z():
    return EI.golden()


@pytest.fixture(scope="module")
def g(z):
    return EI.graph(z)


def test_split_matches_reference_load_data(z, g):
    """tempme_amd.workload.split (the bench's split) = the reference's load_data on the same edges."""
    from tempme_amd.workload import split
    (src, dst, ts, eidx), rows, pool = split(g)
    assert rows.all()
    assert np.array_equal(src, z["test_src"]) and np.array_equal(dst, z["test_dst"])
    assert np.array_equal(ts, z["test_ts"]) and np.array_equal(eidx, z["test_eidx"])
    assert np.array_equal(pool, z["test_sampler_dst"])
    assert ts.min() > 8e7 and ts.max() < 1e8


@pytest.mark.parametrize("N", sorted(EI.SETS))
def test_oracle_pipeline_enron(z, g, N):
    og = orc.OracleGraph(g["src"], g["dst"], g["eidx"], g["ts"], g["n_nodes"])
    _check_pipeline(og, z, f"test_N{N}_", 0, px.SPLIT_TEST, N, 3, z["test_src"], z["test_dst"], z["test_ts"],
                    z["test_eidx"], z["test_sampler_dst"], EI.SETS[N])


@pytest.mark.parametrize("tag", ["N20_base", "N20_notg", "N20_nodep", "N20_h32", "N30_base"])
def test_encoder_oracle_enron(z, g, tag):
    N, var = int(tag[1:3]), tag[4:]
    kw = EI.VARIANTS[var]
    d = EI.walks(z, N)
    sd = EI.weights(z, tag)
    nf, ef = torch.from_numpy(g["n_feat"]), torch.from_numpy(g["e_feat"])
    imps, e0, e1 = [], [], []
    for s in EI.SIDES:
        x = d[s]
        imp = er.forward(sd, nf, ef, x["node"], x["eid"], x["ts"], x["cat"], d["ts_cut"], x["cnt"],
                         temporal=kw.get("use_temporal_guidance", True))
        np.testing.assert_allclose(imp.numpy(), z[f"{tag}_imp_{s}"], rtol=RTOL, atol=ATOL)
        imps.append(imp)
        a, b = er.edge_importance(sd, ef, imp, x["eid"], x["ts"], x["sub_node"], x["sub_eid"],
                                  dependency=kw.get("use_dependency_aware_sampling", True))
        e0.append(a)
        e1.append(b)
    np.testing.assert_allclose(torch.cat(e0).numpy(), z[f"{tag}_expl0"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(torch.cat(e1).numpy(), z[f"{tag}_expl1"], rtol=RTOL, atol=ATOL)
    for k, (s, imp) in enumerate(zip(EI.SIDES, imps)):
        kl = er.kl_loss(imp, d[s]["cat"], z["null"])
        np.testing.assert_allclose(float(kl), z[f"{tag}_kl"][k], rtol=RTOL, atol=ATOL)
