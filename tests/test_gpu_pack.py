"""GPU: the fused sampler's EventBuffers -> the reference's three files (data_preprocess.py:364-420)
-> DevicePack, bit-exact in both directions, and equal to the drop-in pre_processing / marginal /
calculate_edge outputs (which are themselves pinned to the reference's goldens)."""
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    return torch.device("cuda", 0)


def test_sampled_pack_files_round_trip(dev, tmp_path):
    import tempme_amd as tm
    from tempme_amd import pack as P
    from tempme_amd import preprocess as pp
    from tempme_amd.workload import enron_like, split

    g = enron_like(n_nodes=80, n_edges=4000, seed=5)
    (src, dst, ts, eidx), rows, pool = split(g)
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=3)
    sampler = types.SimpleNamespace(dst_list=pool)
    n = 64
    raw_ref = pp.pre_processing(f, sampler, src[:n + 1], dst[:n + 1], ts[:n + 1], eidx[:n + 1], 20, seed=3,
                                split=tm.SPLIT_TEST)
    d = lambda a, t: torch.from_numpy(np.ascontiguousarray(a[:n], dtype=t)).to(dev)  # noqa: E731
    buf = pp.sample_events(f.graph, 3, tm.SPLIT_TEST, 20, 3, d(src, np.int32), d(dst, np.int32), d(ts, np.float64),
                           d(eidx, np.int32), torch.arange(n, dtype=torch.int32, device=dev),
                           torch.from_numpy(pool.astype(np.int32)).to(dev))
    p_raw, p_cat, p_edge = P.write_split(buf, str(tmp_path), "enron_like", "test")
    with P.open_pack(p_raw) as fh:
        for k in P.RAW_KEYS:
            assert np.array_equal(fh[k][:], raw_ref[k]), k
    cat_ref = pp.marginal(raw_ref["walks_src"], raw_ref["walks_tgt"], raw_ref["walks_bgd"], device=dev)
    edge_ref = pp.calculate_edge(*cat_ref, device=dev)
    with P.open_pack(p_cat) as fh:
        for s, side in enumerate(P.SIDES):
            assert np.array_equal(fh[f"walks_{side}_new"][:], cat_ref[s]), side
    assert np.array_equal(np.load(p_edge), edge_ref)
    dp = P.DevicePack.from_files(p_cat, p_edge, 20, dev)
    for name in ("dst_fake", "sub1_node", "sub1_eid", "sub1_ts", "sub2_node", "sub2_eid", "sub2_ts", "node6", "eid3",
                 "ts3", "cat", "cnt", "hist"):
        assert torch.equal(getattr(dp, name), getattr(buf, name)), name
