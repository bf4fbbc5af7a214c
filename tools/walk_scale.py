"""walk_kernel duration vs the number of 16-slot units per launch (the grid tail at small shares).

Samples one step of the metric's workload (full-Enron shape, N=20, M=3, 24 reference batches = the 8-rank
share), then times tm_encoder_fwd_tab over the first G groups (one group = one side of one reference batch:
100 events x 60 walks = 125 units) for several G, HIP events on the launch stream, median of reps.
Prints G, units, ms, ms per unit-round (units / resident waves)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import tempme_amd as tm
    from tempme_amd.pipeline import ExplainPipeline
    from tempme_amd.workload import enron_like, split
    dev = torch.device("cuda", 0)
    g = enron_like(n_nodes=184, n_edges=125235, alpha=1.2, seed=0)
    (src, dst, ts, eidx), rows, pool = split(g)
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=0, split=tm.SPLIT_TEST)

    class Base:
        n_feat_th = torch.from_numpy(g["n_feat"])
        e_feat_th = torch.from_numpy(g["e_feat"])
        node_raw_features = torch.nn.Embedding.from_pretrained(n_feat_th, padding_idx=0, freeze=True)
        edge_raw_features = torch.nn.Embedding.from_pretrained(e_feat_th, padding_idx=0, freeze=True)

    torch.manual_seed(0)
    ex = tm.TempME(Base(), "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
                   null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).eval()
    N, M, B = 20, 3, 100
    nb = int(os.environ.get("WS_BATCHES", "24"))
    E = nb * B
    pipe = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, M, B, seed=0)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:E], dtype=dt)).to(dev)  # noqa: E731
    x = (t(src, np.int32), t(dst, np.int32), t(ts, np.float64), t(eidx, np.int32),
         torch.arange(E, dtype=torch.int32, device=dev))
    pipe.run(*x)
    torch.cuda.synchronize()
    b = pipe.buf
    W = N * M
    cut = x[2].repeat(3).contiguous()
    waves = 2048
    Gs = [int(v) for v in os.environ.get("WS_GROUPS", "1,2,4,8,16,17,24,32,33,48,49,64,66,72").split(",")]
    reps = int(os.environ.get("WS_REPS", "9"))
    st = torch.cuda.current_stream()
    print("G units ms ms_per_round")
    for G in Gs:
        if G > 3 * nb:
            continue
        n = G * B * W
        ms = []
        for r in range(reps + 2):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            ex.encoder_fwd(b.node6, b.eid3, b.ts3, b.cat, cut, b.cnt, G, B, W, out=pipe.imp, workspace=pipe.ws, M=M,
                           etab=pipe.etab)
            e.record(st)
            e.synchronize()
            if r >= 2:
                ms.append(a.elapsed_time(e))
        units = n // M // 16
        med = float(np.median(ms))
        print(f"{G} {units} {med:.4f} {med / max(units / waves, 1e-9):.4f}", flush=True)
    _ = n


if __name__ == "__main__":
    main()
