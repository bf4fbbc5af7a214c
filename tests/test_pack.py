"""The reference's on-disk pack: writer, h5py-style readers mirroring
utils/batch_loader.py, and the device-resident pack.  CPU only (DevicePack on device='cpu').

Fixtures: tests/golden/uslegis_pipeline.npz holds what the reference's own pre_processing /
marginal / calculate_edge produced on uslegis_sampled (make_goldens.py); the pack arrays are
assembled from those vectors the way data_preprocess.py:114-143 concatenates them, written,
read back through the loaders and compared with the vectors.
"""
import os
import types

import numpy as np
import pytest
import torch

from tempme_amd import pack as P

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SIDES = ("src", "tgt", "bgd")


def _golden_pack(pre="train_N20_"):
    z = np.load(os.path.join(G, "uslegis_pipeline.npz"))
    raw, cat = {"dst_fake": z[pre + "dst_fake"].astype(np.float64)}, {}
    cat["dst_fake"] = raw["dst_fake"]
    for s in SIDES:
        for h in (0, 1):
            k = f"subgraph_{s}_{h}"
            raw[k] = cat[k] = np.concatenate([z[f"{pre}{k}_{f}"] for f in ("node", "eid", "ts")], -1).astype(np.float64)
        base = np.concatenate([z[f"{pre}walks_{s}_{f}"] for f in ("node", "eid", "ts")], -1).astype(np.float64)
        raw[f"walks_{s}"] = np.concatenate([base, z[f"{pre}walks_{s}_anony"]], -1)
        cat[f"walks_{s}_new"] = np.concatenate([base, z[f"{pre}walks_{s}_cat"][..., None],
                                                z[f"{pre}walks_{s}_marg"][..., None]], -1)
    return z, raw, cat, z[pre + "edge"].astype(np.float64)


def test_pack_round_trip_and_loaders(tmp_path):
    z, raw, cat, edge = _golden_pack()
    pre, N = "train_N20_", 20
    p_raw = P.write_pack(str(tmp_path / "uslegis_sampled_train.h5"), raw, P.RAW_KEYS)
    p_cat = P.write_pack(str(tmp_path / "uslegis_sampled_train_cat.h5"), cat, P.CAT_KEYS)
    args = types.SimpleNamespace(n_degree=N)
    with P.open_pack(p_cat) as f:
        assert sorted(f.keys()) == sorted(P.CAT_KEYS)
        for k in P.CAT_KEYS:
            assert f[k][:].dtype == np.float64 and np.array_equal(f[k][:], cat[k])
        pk = P.load_subgraph_margin(args, f)
    bid = np.arange(5, 17)
    sg_src, sg_tgt, sg_bgd, ws, wt, wb, fake = P.get_item(pk, bid)
    for s, sg in zip(SIDES, (sg_src, sg_tgt, sg_bgd)):
        for h in (0, 1):
            for r, fld in zip(sg, ("node", "eid", "ts")):
                assert np.array_equal(r[h], z[f"{pre}subgraph_{s}_{h}_{fld}"][bid])
    for s, w in zip(SIDES, (ws, wt, wb)):
        assert len(w) == 5
        assert w[0].dtype == np.int64 and np.array_equal(w[0], z[f"{pre}walks_{s}_node"][bid])
        assert w[1].dtype == np.int64 and np.array_equal(w[1], z[f"{pre}walks_{s}_eid"][bid])
        assert w[2].dtype == np.float64 and np.array_equal(w[2], z[f"{pre}walks_{s}_ts"][bid])
        assert w[3].shape == (12, 60, 1) and np.array_equal(w[3][..., 0], z[f"{pre}walks_{s}_cat"][bid])
        assert np.array_equal(w[4][..., 0], z[f"{pre}walks_{s}_marg"][bid])
    assert np.array_equal(fake, z[pre + "dst_fake"][bid])
    e_src, e_tgt, e_bgd = P.get_item_edge(edge, bid)
    assert np.array_equal(e_tgt, z[pre + "edge"][1][bid])
    with P.open_pack(p_raw) as f:
        out = P.load_subgraph(args, f, bid)
    for s, w in zip(SIDES, out[3:]):
        assert np.array_equal(w[3], z[f"{pre}walks_{s}_anony"][bid]) and w[3].dtype == np.int64


def test_device_pack_and_buffers_round_trip(tmp_path):
    z, raw, cat, edge = _golden_pack()
    pre = "train_N20_"
    p_cat = P.write_pack(str(tmp_path / "x_train_cat.h5"), cat, P.CAT_KEYS)
    np.save(tmp_path / "x_train_edge.npy", edge)
    dp = P.DevicePack.from_files(p_cat, str(tmp_path / "x_train_edge.npy"), 20, torch.device("cpu"))
    assert (dp.E, dp.N, dp.M, dp.W) == (32, 20, 3, 60)
    for s, side in enumerate(SIDES):
        assert np.array_equal(dp.sub2_eid[s].numpy(), z[f"{pre}subgraph_{side}_1_eid"])
        assert np.array_equal(dp.ts3[s].numpy(), z[f"{pre}walks_{side}_ts"])
        assert np.array_equal(dp.cat[s].numpy(), z[f"{pre}walks_{side}_cat"])
        assert np.array_equal(dp.cnt[s].numpy(), z[pre + "edge"][s])
    # back to the reference's files: both H5 dicts and the edge array reproduce exactly
    raw2, cat2, edge2 = P.buffers_to_arrays(dp)
    for k in P.RAW_KEYS:
        assert np.array_equal(raw2[k], raw[k]), k
    for k in P.CAT_KEYS:
        assert np.array_equal(cat2[k], cat[k]), k
    assert np.array_equal(edge2, edge)
    paths = P.write_split(dp, str(tmp_path), "y", "test")
    assert [os.path.basename(p) for p in paths] == ["y_test.h5", "y_test_cat.h5", "y_test_edge.npy"]


def test_pack_errors(tmp_path):
    _, raw, cat, edge = _golden_pack()
    with pytest.raises(KeyError):
        P.write_pack(str(tmp_path / "a.h5"), {"dst_fake": raw["dst_fake"]}, P.RAW_KEYS)
    bad = tmp_path / "b.h5"
    bad.write_bytes(b"not a pack at all")
    with pytest.raises(ValueError):
        P.open_pack(str(bad))
    p_cat = P.write_pack(str(tmp_path / "c.h5"), cat, P.CAT_KEYS)
    with P.open_pack(p_cat) as f:
        with pytest.raises(AssertionError):
            P.DevicePack(f, edge[:, :3], 20, torch.device("cpu"))
        with pytest.raises(AssertionError):
            P.DevicePack(f, edge, 7, torch.device("cpu"))


def test_get_item_slice_path_matches_fancy_indexing(tmp_path):
    """get_item / get_item_edge index a contiguous np.arange batch by a slice (views, no copies); the
    values must equal fancy indexing with the same ids, and ids past the pack still raise IndexError
    as the reference's fancy indexing does (utils/batch_loader.py:200-242)."""
    _, _, cat, edge = _golden_pack()
    p_cat = P.write_pack(str(tmp_path / "s_cat.h5"), cat, P.CAT_KEYS)
    with P.open_pack(p_cat) as f:
        pk = P.load_subgraph_margin(types.SimpleNamespace(n_degree=20), f)
    bid = np.arange(7, 19)
    fast, ref = P.get_item(pk, bid), P.get_item(pk, list(bid))
    for a, b in zip(fast[:3], ref[:3]):          # subgraphs: (node, eidx, ts) lists per hop
        for x, y in zip(a, b):
            for u, v in zip(x, y):
                assert np.array_equal(u, v)
    for a, b in zip(fast[3:6], ref[3:6]):        # walks
        for u, v in zip(a, b):
            assert u.dtype == v.dtype and np.array_equal(u, v)
    assert np.array_equal(fast[6], ref[6])
    for u, v in zip(P.get_item_edge(edge, bid), P.get_item_edge(edge, list(bid))):
        assert np.array_equal(u, v)
    n = len(pk[-1])
    with pytest.raises(IndexError):
        P.get_item(pk, np.arange(n - 2, n + 2))
    with pytest.raises(IndexError):
        P.get_item_edge(edge, np.arange(n - 2, n + 2))
