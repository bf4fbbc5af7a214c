"""Debug: run only the k-hop sampling of the bench workload (for rocprofv3 --pmc passes)."""
import sys

import numpy as np
import torch

sys.argv = [sys.argv[0]]
import bench  # noqa: E402
import tempme_amd as tm  # noqa: E402
from tempme_amd import _lib as L  # noqa: E402
from tempme_amd.workload import enron_like, split  # noqa: E402

dev = torch.device("cuda", 0)
N, E = 20, 6400
g = enron_like(alpha=1.2, seed=0)
(src, dst, ts, eidx), rows, pool = split(g)
finder = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                      device=dev, seed=0, split=tm.SPLIT_TEST)
i = np.arange(E) % len(src)
to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
s_, d_, t_, e_ = to(src[i], np.int32), to(dst[i], np.int32), to(ts[i], np.float64), to(eidx[i], np.int32)
ev = to(np.arange(E, dtype=np.uint32).view(np.int32), np.int32)
tot = E * (N + N * N)
on = torch.empty(tot, dtype=torch.int32, device=dev)
oe = torch.empty_like(on)
ot = torch.empty(tot, dtype=torch.float32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
for it in range(10):
    for side, root, ei in ((L.SIDE_SRC, s_, e_), (L.SIDE_TGT, d_, e_), (L.SIDE_BGD, d_, None)):
        L.check(L.lib().tm_sample_khop(finder.graph.handle, L.TmRng(0, 1, side), 2, N, E, L.ptr(root), L.ptr(t_),
                                       L.ptr(ei), L.ptr(ev), L.ptr(on), L.ptr(oe), L.ptr(ot), L.ptr(err),
                                       L.stream_ptr(dev)), "khop")
torch.cuda.synchronize()
print("ok", int(err.item()))
