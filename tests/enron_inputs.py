"""Shared loader for the bench-regime goldens (tests/golden/enron_goldens.npz, make_goldens.py
case_enron): the full-Enron-shaped synthetic graph (regenerated from its parameters and checked
against the stored checksum), the reference's test split of it, the reference pipeline's outputs at
N=20 (100 events) / N=30 (32 events), and reference TempME outputs at Enron dims for the default
constructor and its variants, laid out as batch_loader.get_item hands them to TempME."""
import json
import os

import numpy as np
import torch

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SIDES = ("src", "tgt", "bgd")
SETS = {20: 100, 30: 32}
VARIANTS = {"base": {}, "notg": dict(use_temporal_guidance=False),
            "nodep": dict(use_dependency_aware_sampling=False), "h32": dict(hid_dim=32)}


def golden():
    return np.load(os.path.join(G, "enron_goldens.npz"))


def graph(z=None):
    from tempme_amd.workload import enron_like
    z = golden() if z is None else z
    params = json.loads(str(z["graph_params"]))
    g = enron_like(**params)
    ck = np.array([int(g["src"].sum()), int((g["src"] * g["dst"]).sum() % (1 << 61)), int(g["ts"].sum()),
                   float(g["e_feat"].astype(np.float64).sum()), float(g["n_feat"].astype(np.float64).sum())])
    np.testing.assert_array_equal(ck, z["graph_checksum"])
    return g


def walks(z, n_deg, bsz=None):
    """Per side: the walk record arrays TempME.forward reads plus subgraphs and edge counts."""
    bsz = SETS[n_deg] if bsz is None else bsz
    pre = f"test_N{n_deg}_"
    d = {"ts_cut": z["test_ts"][:bsz].astype(np.float64), "N": n_deg, "B": bsz}
    for s_i, s in enumerate(SIDES):
        w = pre + f"walks_{s}"
        d[s] = dict(
            node=z[w + "_node"][:bsz].astype(np.int64), eid=z[w + "_eid"][:bsz].astype(np.int64),
            ts=z[w + "_ts"][:bsz].astype(np.float64), cat=z[w + "_cat"][:bsz, :, None].astype(np.int64),
            marg=z[w + "_marg"][:bsz, :, None], cnt=z[pre + "edge"][s_i, :bsz].astype(np.float64),
            sub_node=[z[pre + f"subgraph_{s}_{h}_node"][:bsz] for h in (0, 1)],
            sub_eid=[z[pre + f"subgraph_{s}_{h}_eid"][:bsz] for h in (0, 1)],
            sub_ts=[z[pre + f"subgraph_{s}_{h}_ts"][:bsz] for h in (0, 1)])
    return d


def weights(z, tag):
    pref = f"{tag}_w_"
    return {k[len(pref):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(pref)}


def null(z):
    return {k + 1: float(v) for k, v in enumerate(z["null"])}


def build_tgn(z, g, cls=None, n_deg=20):
    """The reference TGN of case_enron's training iteration (make_goldens.tgn_base "enron": seed 13,
    learn_base.py:175-176 defaults) with the committed memory / time-bias / message perturbation."""
    if cls is None:
        from tempme_amd.tgn import TGN as cls
    torch.manual_seed(13)
    m = cls(g["n_feat"], g["e_feat"], n_neighbors=n_deg, device=torch.device("cpu"), n_layers=3, n_heads=2,
            dropout=0.5)
    m.forbidden_memory_update = True
    m.eval()
    p = {k[len("train_pert_"):]: z[k] for k in z.files if k.startswith("train_pert_")}
    with torch.no_grad():
        m.memory.memory.data.copy_(torch.from_numpy(p["memory"]))
        m.memory.last_update.data.copy_(torch.from_numpy(p["last_update"]))
        m.time_encoder.w.bias.data.copy_(torch.from_numpy(p["time_bias"]))
    for i, nd in enumerate(p["msg_nodes"]):
        m.memory.messages[int(nd)] = [(torch.from_numpy(p["msg_raw"][i, k]), torch.tensor(p["msg_ts"][i, k]))
                                      for k in range(2)]
    return m
