"""TempME._pad_hidden (a hid_dim that is not a multiple of 16 runs the HIP kernels on weights zero-padded to
the next one): the padded weights, read back as a state_dict of the wider network, compute the same
graphlet importance (oracle/encoder_ref.forward, explainer_new.py:174-201) and edge importance
(edge_importance, :354-406) as the original ones, on the uslegis golden walks.  CPU only: the GPU side is
tests/test_gpu_parity.py::test_constructor_shapes_on_hip's hid_dim 40 / 20 cases."""
import numpy as np
import pytest
import torch

from oracle import encoder_ref as er
from tests.encoder_inputs import SIDES, load


class _Base:
    def __init__(self, n_feat, e_feat):
        self.n_feat_th = torch.as_tensor(n_feat)
        self.e_feat_th = torch.as_tensor(e_feat)
        self.node_raw_features = torch.nn.Embedding.from_pretrained(self.n_feat_th, padding_idx=0, freeze=True)
        self.edge_raw_features = torch.nn.Embedding.from_pretrained(self.e_feat_th, padding_idx=0, freeze=True)


def _padded_sd(ex):
    """The padded tm_weights-ordered tensors under the state_dict keys they came from."""
    ws = ex._weight_list()
    keys = []
    for path in ex._weight_paths():
        keys += [".".join(path) + ".weight", ".".join(path) + ".bias"]
    keys += ["time_encoder.basis_freq", "time_encoder.phase"]
    raw = ex._pad_hidden([w.detach().float().contiguous() for w in ws])
    assert len(raw) == len(keys) == 28
    return dict(zip(keys, raw))


@pytest.mark.parametrize("hid,if_cat,tg", [(40, True, True), (20, False, True), (36, True, False)])
def test_padded_weights_compute_the_same_function(hid, if_cat, tg):
    from tempme_amd import TempME
    d = load("synth")
    torch.manual_seed(hid)
    ex = TempME(_Base(d["n_feat"], d["e_feat"]), "tgn", "x", out_dim=40, hid_dim=hid, if_cat_feature=if_cat,
                use_temporal_guidance=tg, null_model={k + 1: float(v) for k, v in enumerate(d["null"])}).eval()
    H = ex._hid_packed()
    assert H % 16 == 0 and H > hid
    sd = {k: v.detach() for k, v in ex.state_dict().items()}
    sp = _padded_sd(ex)
    assert sp["MLP.3.weight"].shape[0] == H and sp["attention.W1.weight"].shape == (2 * H, 2 * H)
    assert sp["edge_dependency_gcn.3.weight"].shape == (H // 2, H)
    for s in SIDES:
        x = d[s]
        args = (d["n_feat"].float(), d["e_feat"].float(), x["node"], x["eid"], x["ts"], x["cat"], d["ts_cut"],
                x["cnt"])
        a = er.forward(sd, *args, temporal=tg, if_cat=if_cat)
        b = er.forward(sp, *args, temporal=tg, if_cat=if_cat)
        np.testing.assert_allclose(b.numpy(), a.numpy(), rtol=1e-5, atol=1e-6, err_msg=s)
        ea = er.edge_importance(sd, d["e_feat"].float(), a, x["eid"], x["ts"], x["sub_node"], x["sub_eid"])
        eb = er.edge_importance(sp, d["e_feat"].float(), a, x["eid"], x["ts"], x["sub_node"], x["sub_eid"])
        for u, v in zip(ea, eb):
            np.testing.assert_allclose(v.numpy(), u.numpy(), rtol=1e-5, atol=1e-6, err_msg=s)


@pytest.mark.parametrize("hid,if_cat", [(40, True), (20, False)])
def test_pad_maps_round_trip(hid, if_cat):
    """The training side of the padding: _unpad_grads reads back exactly what _pad_hidden placed, and the
    dropout / gate keep-masks move each hidden unit's column to its padded position."""
    from tempme_amd import TempME
    from tempme_amd.explainer import _ENC_IDX, _GATE_IDX
    d = load("synth")
    torch.manual_seed(hid)
    ex = TempME(_Base(d["n_feat"], d["e_feat"]), "tgn", "x", out_dim=40, hid_dim=hid, if_cat_feature=if_cat,
                null_model={k + 1: float(v) for k, v in enumerate(d["null"])}).train()
    H = ex._hid_packed()
    raw = [w.detach().float().contiguous() for w in ex._weight_list()]
    pad = ex._pad_hidden(raw)
    ex._raw = pad
    for idx in (_ENC_IDX, _GATE_IDX):
        assert ex._padded_shapes(idx) == [tuple(pad[i].shape) for i in idx]
        back = ex._unpad_grads([pad[i] for i in idx], idx)
        for i, b in zip(idx, back):
            assert torch.equal(b, raw[i]), i
    n = 7
    drop = torch.randint(0, 2, (n, ex.dropout_cols()), dtype=torch.uint8)
    dp = ex._drop_packed(drop)
    hm = 12 if if_cat else 0
    assert dp.shape == (n, -(-(2 + H + H + hm) // 16) * 16)
    assert torch.equal(dp[:, :2 + hid], drop[:, :2 + hid])
    assert torch.equal(dp[:, 2 + H:2 + H + hid], drop[:, 2 + hid:2 + 2 * hid])
    if if_cat:
        assert torch.equal(dp[:, 2 + 2 * H:2 + 2 * H + 12], drop[:, 2 + 2 * hid:2 + 2 * hid + 12])
    k1 = torch.randint(0, 2, (n, hid), dtype=torch.uint8)
    k2 = torch.randint(0, 2, (n, hid // 2), dtype=torch.uint8)
    p1, p2, _, _ = ex._gate_masks_packed((k1, k2, 1.0, 1.0))
    assert p1.shape == (n, H) and p2.shape == (n, H // 2)
    assert torch.equal(p1[:, :hid], k1) and torch.equal(p2[:, :hid // 2], k2)
