"""Diagnose run_steps (overlapped) vs the serial train_step loop.

Runs the serial loop twice and the overlapped loop once from the same seed, records each step's
gradients (between backward and the optimizer step) and each prepare_step output, and prints, per
step, the relative gradient difference of serial-vs-serial and serial-vs-overlap split by parameter.
If serial-vs-serial already drifts like serial-vs-overlap, the difference is amplification of
summation-order noise, not the schedule."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tempme_amd as tm  # noqa: E402
import tempme_amd.train as T  # noqa: E402
from tempme_amd.preprocess import sample_events  # noqa: E402
from tempme_amd.tgn import TGN  # noqa: E402
from tempme_amd.workload import enron_like, split  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = enron_like(n_nodes=80, n_edges=3000, seed=4)
    (src, dst, ts, eidx), rows, pool = split(g, mode="train")
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=2, split=tm.SPLIT_TRAIN)
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    s_d, d_d, t_d, e_d = to(src, np.int32), to(dst, np.int32), to(ts, np.float64), to(eidx, np.int32)
    buf = sample_events(f.graph, 2, tm.SPLIT_TRAIN, 10, 3, s_d, d_d, t_d, e_d,
                        torch.arange(len(src), dtype=torch.int32, device=dev), to(pool, np.int32))
    torch.manual_seed(3)
    base = TGN(g["n_feat"], g["e_feat"], n_neighbors=10, device=dev, n_layers=2, n_heads=2, dropout=0.1)
    base.forbidden_memory_update = True
    base = base.to(dev).eval()
    B, K = 40, 4
    orig_prep = T.prepare_step

    def one(mode):
        preps = []

        def rec_prep(bm, b):
            out = orig_prep(bm, b)
            preps.append((out[1].clone(), out[2].clone(), out[3].clone()))
            return out
        T.prepare_step = rec_prep
        torch.manual_seed(5)
        ex = tm.TempME(base, "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
                       null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).eval()
        names = [k for k, _ in ex.named_parameters()]
        opt = torch.optim.Adam(ex.parameters(), lr=1e-3)
        steps, params = [], []

        class Rec:
            def start(self):
                steps.append({k: p.grad.detach().clone() for k, p in ex.named_parameters() if p.grad is not None})
                params.append({k: p.detach().clone() for k, p in ex.named_parameters()})

            def finish(self):
                pass
        batches = [T.batch_from_pack(buf, s_d, d_d, t_d, e_d, torch.arange(k * B, (k + 1) * B, device=dev))
                   for k in range(K)]
        if mode == "overlap":
            T.run_steps(ex, base, opt, batches, overlap=True, if_bern=False, grad_sync=Rec())
        else:
            for b in batches:
                T.train_step(ex, base, opt, b, if_bern=False, grad_sync=Rec())
        torch.cuda.synchronize()
        T.prepare_step = orig_prep
        return names, steps, params, preps

    names, s1, p1, q1 = one("serial")
    _, s2, p2, q2 = one("serial")
    _, s3, p3, q3 = one("overlap")
    for k in range(K):
        same = [all(torch.equal(a, b) for a, b in zip(q1[k], q)) for q in (q2[k], q3[k])]
        print(f"step {k}: prepare outputs bitwise equal: serial2={same[0]} overlap={same[1]}")
        for lab, s, p in (("serial2", s2, p2), ("overlap", s3, p3)):
            ga = torch.cat([s1[k][n].reshape(-1) for n in names if n in s1[k]])
            gb = torch.cat([s[k][n].reshape(-1) for n in names if n in s[k]])
            pd = max(float((p1[k][n] - p[k][n]).abs().max()) for n in names)
            print(f"  {lab}: |dg|/|g| = {float((ga - gb).norm()) / float(ga.norm()):.3e}  max|dparam| = {pd:.3e}")
            worst = sorted(((float((s1[k][n] - s[k][n]).norm()) / (float(s1[k][n].norm()) + 1e-30), n)
                            for n in names if n in s1[k]), reverse=True)[:5]
            print("    worst params:", ", ".join(f"{n}={r:.2e}" for r, n in worst))
            pw = sorted(((float((p1[k][n] - p[k][n]).abs().max()), n) for n in names), reverse=True)[:3]
            print("    most-moved params:", ", ".join(f"{n}={r:.2e}" for r, n in pw))


if __name__ == "__main__":
    main()
