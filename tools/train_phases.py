"""GPU time per phase of one eager training step (bench_train workload): events recorded between the
phases of train.train_step's body on the current stream; prints mean ms per phase over the steps."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import tempme_amd as tm  # noqa: E402
from tempme_amd.preprocess import sample_events  # noqa: E402
from tempme_amd.tgn import TGN  # noqa: E402
from tempme_amd.train import batch_from_pack, encode_sides, epoch_spans  # noqa: E402
from tempme_amd.workload import enron_like, split  # noqa: E402

dev = torch.device("cuda", 0)
N, M, B = 20, 3, 100
g = enron_like(n_nodes=184, n_edges=125235, seed=0)
(src, dst, ts, eidx), rows, pool = split(g, mode="train")
f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                 device=dev, seed=0, split=tm.SPLIT_TRAIN)
to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
s_d, d_d, t_d, e_d = to(src, np.int32), to(dst, np.int32), to(ts, np.float64), to(eidx, np.int32)
buf = sample_events(f.graph, 0, tm.SPLIT_TRAIN, N, M, s_d, d_d, t_d, e_d,
                    torch.arange(len(src), dtype=torch.int32, device=dev), to(pool, np.int32))
torch.manual_seed(0)
base = TGN(g["n_feat"], g["e_feat"], n_neighbors=N, device=dev, n_layers=2, n_heads=2, dropout=0.1)
base.forbidden_memory_update = True
base = base.to(dev).eval()
ex = tm.TempME(base, "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
               null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).train()
opt = torch.optim.Adam(ex.parameters(), lr=1e-3)
crit = torch.nn.BCEWithLogitsLoss()
perm = torch.randperm(len(src) - 1).to(dev)
spans = epoch_spans(len(src) - 1, B)[:25]
names = ["pack slice", "contrast (no grad)", "encoder fwd", "explanation fwd", "contrast w/ expl", "losses",
         "backward", "adam"]
acc = np.zeros(len(names))
for k, (a, b) in enumerate(spans):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
    ev[0].record()
    batch = batch_from_pack(buf, s_d, d_d, t_d, e_d, perm[a:b])
    ev[1].record()
    sg_s, sg_t, sg_b = batch.subgraphs
    w_s, w_t, w_b = batch.walks
    with torch.no_grad():
        po, no = base.contrast(batch.src, batch.dst, batch.fake, batch.ts, batch.e_idx, sg_s, sg_t, sg_b)
        y = torch.where(torch.cat([po, no]).sigmoid() > 0.5, 1., 0.).view(-1, 1)
    ev[2].record()
    opt.zero_grad()
    g_s, g_t, g_b = encode_sides(ex, batch)
    ev[3].record()
    expl = ex.retrieve_explanation(sg_s, g_s, w_s, sg_t, g_t, w_t, sg_b, g_b, w_b, training=True)
    ev[4].record()
    pl, nl = base.contrast(batch.src, batch.dst, batch.fake, batch.ts, batch.e_idx, sg_s, sg_t, sg_b,
                           explain_weights=expl)
    ev[5].record()
    loss = crit(torch.cat([pl, nl]), y) + 0.5 * (ex.kl_loss(g_s, w_s) + ex.kl_loss(g_t, w_t) + ex.kl_loss(g_b, w_b))
    ev[6].record()
    loss.backward()
    ev[7].record()
    opt.step()
    ev[8].record()
    torch.cuda.synchronize()
    if k >= 5:
        acc += [ev[i].elapsed_time(ev[i + 1]) for i in range(len(names))]
acc /= len(spans) - 5
for n, v in zip(names, acc):
    print(f"{v:8.3f} ms  {n}")
print(f"{acc.sum():8.3f} ms  total (eager, events between phases)")
