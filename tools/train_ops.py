"""Diagnostic: device time of one eager training step (bench_train workload: full-Enron shape, N=20, bs=100,
TGN base, temp_exp_main.py:593-632) attributed to torch ops and to the Python lines that issue them
(torch.profiler with stacks), so the glue kernels between the HIP kernels can be located."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")


def main():
    import tempme_amd as tm
    from tempme_amd.preprocess import sample_events
    from tempme_amd.tgn import TGN
    from tempme_amd.train import batch_from_pack, epoch_spans, train_step
    from tempme_amd.workload import enron_like, split
    dev = torch.device("cuda", 0)
    N, M, B = 20, 3, 100
    g = enron_like(n_nodes=184, n_edges=125235, seed=0)
    (src, dst, ts, eidx), rows, pool = split(g, mode="train")
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=0, split=tm.SPLIT_TRAIN)
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    ev = (to(src, np.int32), to(dst, np.int32), to(ts, np.float64), to(eidx, np.int32))
    buf = sample_events(f.graph, 0, tm.SPLIT_TRAIN, N, M, *ev, torch.arange(len(src), dtype=torch.int32, device=dev),
                        to(pool, np.int32))
    torch.manual_seed(0)
    base = TGN(g["n_feat"], g["e_feat"], n_neighbors=N, device=dev, n_layers=2, n_heads=2, dropout=0.1)
    base.forbidden_memory_update = True
    base = base.to(dev).eval()
    ex = tm.TempME(base, "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
                   null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).train()
    opt = torch.optim.Adam(ex.parameters(), lr=1e-3, fused=True)
    perm = torch.randperm(len(src) - 1).to(dev)
    spans = epoch_spans(len(src) - 1, B)[:12]
    batches = [batch_from_pack(buf, *ev, perm[a:b]) for a, b in spans]
    for b in batches[:4]:
        train_step(ex, base, opt, b)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    steps = batches[4:12]
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
        for b in steps:
            train_step(ex, base, opt, b)
        torch.cuda.synchronize()
    ka = prof.key_averages()
    print("=== ops by device time (per step, us) ===")
    rows_ = sorted(ka, key=lambda e: -e.device_time_total)[:45]
    for e in rows_:
        print("%9.1f us %6.1f calls  %s" % (e.device_time_total / len(steps), e.count / len(steps), e.key[:90]))
    print("=== small glue ops by input shapes (per step) ===")
    glue = ("aten::add", "aten::add_", "aten::cat", "aten::fill_", "aten::zero_", "aten::copy_", "aten::clamp",
            "aten::clamp_min", "aten::mul", "aten::sub", "aten::threshold_backward", "aten::_to_copy", "aten::sum")
    ksh = prof.key_averages(group_by_input_shape=True)
    for e in sorted(ksh, key=lambda e: -e.device_time_total):
        if e.key in glue and e.device_time_total > 0:
            print("%9.1f us %5.1f calls  %-24s %s" % (e.device_time_total / len(steps), e.count / len(steps), e.key,
                                                     str(e.input_shapes)[:150]))
    print("=== by stack (top 40, per step) ===")
    ks = prof.key_averages(group_by_stack_n=4)
    for e in sorted(ks, key=lambda e: -e.device_time_total)[:40]:
        if e.device_time_total <= 0:
            continue
        st = " <- ".join(s.split("/")[-1] for s in (e.stack or [])[:4])
        print("%9.1f us %5.1f calls  %-40s %s" % (e.device_time_total / len(steps), e.count / len(steps), e.key[:40], st))


if __name__ == "__main__":
    main()
