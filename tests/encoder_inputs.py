"""Shared loader for the encoder golden inputs (walks of the uslegis test split, N=20,
first 32 events), laid out exactly as batch_loader.get_item hands them to TempME."""
import os

import numpy as np
import torch

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SIDES = ("src", "tgt", "bgd")


def load(case="uslegis", n_deg=20, bsz=32):
    pipe = np.load(os.path.join(G, "uslegis_pipeline.npz"))
    enc = np.load(os.path.join(G, "encoder_uslegis.npz"))
    pre = f"test_N{n_deg}_"
    d = {"ts_cut": enc["ts_cut"], "N": n_deg, "B": bsz}
    for s_i, s in enumerate(SIDES):
        w = pre + f"walks_{s}"
        d[s] = dict(
            node=pipe[w + "_node"][:bsz].astype(np.int64), eid=pipe[w + "_eid"][:bsz].astype(np.int64),
            ts=pipe[w + "_ts"][:bsz].astype(np.float64), cat=pipe[w + "_cat"][:bsz, :, None].astype(np.int64),
            marg=pipe[w + "_marg"][:bsz, :, None],
            cnt=pipe[pre + "edge"][s_i, :bsz].astype(np.float64),
            sub_node=[pipe[pre + f"subgraph_{s}_{h}_node"][:bsz] for h in (0, 1)],
            sub_eid=[pipe[pre + f"subgraph_{s}_{h}_eid"][:bsz] for h in (0, 1)],
            sub_ts=[pipe[pre + f"subgraph_{s}_{h}_ts"][:bsz] for h in (0, 1)],
            imp=enc[f"{case}_imp_{s}"])
    d["n_feat"] = torch.from_numpy(enc[f"{case}_n_feat"])
    d["e_feat"] = torch.from_numpy(enc[f"{case}_e_feat"])
    pref = f"{case}_w_"
    d["sd"] = {k[len(pref):]: torch.from_numpy(enc[k]) for k in enc.files if k.startswith(pref)}
    d["expl0"], d["expl1"] = enc[f"{case}_expl0"], enc[f"{case}_expl1"]
    d["kl"], d["null"] = enc[f"{case}_kl"], enc[f"{case}_null"]
    return d
