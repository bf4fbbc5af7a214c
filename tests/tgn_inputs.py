"""Shared loader for the base-TGN golden case (make_goldens.py case_tgn): the first 32 test events of
uslegis_sampled at N=20, in the layout batch_loader.get_item hands to TGN.contrast (float64 node /
eid / ts records, as after the reference's H5 round trip), the seeded base model and the memory /
time-bias / message perturbation the golden run applied."""
import os

import numpy as np
import torch

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SIDES = ("src", "tgt", "bgd")
SEEDS = {"uslegis": 11, "synth": 12}
N_DEG, BSZ = 20, 32


def load_batch(n_deg=N_DEG, bsz=BSZ):
    pipe = np.load(os.path.join(G, "uslegis_pipeline.npz"))
    enc = np.load(os.path.join(G, "encoder_uslegis.npz"))
    pre = f"test_N{n_deg}_"
    d = {"N": n_deg, "B": bsz, "ts_cut": enc["ts_cut"][:bsz].astype(np.float64),
         "src": pipe["test_src"][:bsz].astype(np.int64), "dst": pipe["test_dst"][:bsz].astype(np.int64),
         "e_idx": pipe["test_eidx"][:bsz].astype(np.int64),
         "fake": pipe[pre + "dst_fake"][:bsz].astype(np.float64)}
    for s in SIDES:
        d["sg_" + s] = tuple([pipe[pre + f"subgraph_{s}_{h}_{k}"][:bsz].astype(np.float64) for h in (0, 1)]
                             for k in ("node", "eid", "ts"))
    return d


def feats(case):
    enc = np.load(os.path.join(G, "encoder_uslegis.npz"))
    return enc[f"{case}_n_feat"], enc[f"{case}_e_feat"]


def explanation(case):
    enc = np.load(os.path.join(G, "encoder_uslegis.npz"))
    return [torch.from_numpy(enc[f"{case}_expl0"]), torch.from_numpy(enc[f"{case}_expl1"])]


def golden():
    return np.load(os.path.join(G, "tgn_uslegis.npz"))


def build_model(case, cls=None):
    """torch.manual_seed(seed); TGN(...) exactly as the golden run (learn_base.py:175-176 defaults),
    then the committed perturbation.  `cls` defaults to tempme_amd.tgn.TGN."""
    if cls is None:
        from tempme_amd.tgn import TGN as cls
    g = golden()
    nf, ef = feats(case)
    torch.manual_seed(SEEDS[case])
    m = cls(nf, ef, n_neighbors=N_DEG, device=torch.device("cpu"), n_layers=3, n_heads=2, dropout=0.5)
    m.forbidden_memory_update = True
    m.eval()
    p = {k[len(case) + 6:]: g[k] for k in g.files if k.startswith(f"{case}_pert_")}
    with torch.no_grad():
        m.memory.memory.data.copy_(torch.from_numpy(p["memory"]))
        m.memory.last_update.data.copy_(torch.from_numpy(p["last_update"]))
        m.time_encoder.w.bias.data.copy_(torch.from_numpy(p["time_bias"]))
    for i, nd in enumerate(p["msg_nodes"]):
        m.memory.messages[int(nd)] = [(torch.from_numpy(p["msg_raw"][i, k]), torch.tensor(p["msg_ts"][i, k]))
                                      for k in range(2)]
    return m


def rand_weights(case):
    g = golden()
    return [torch.from_numpy(g[f"{case}_ew_rand0"]), torch.from_numpy(g[f"{case}_ew_rand1"])]


def edge_attr(case="uslegis"):
    g = golden()
    return [g[f"{case}_edge_attr0"], g[f"{case}_edge_attr1"]]
