"""Times NeighborFinder.from_edges (host CSR build + per-edge tables + upload + export)
for the bench graphs, twice each (the first call also pays the device's first allocations)."""
import sys
import time

import torch

sys.path.insert(0, ".")
import tempme_amd as tm  # noqa: E402
from tempme_amd.workload import enron_like, split  # noqa: E402

dev = torch.device("cuda", 0)
torch.zeros(1, device=dev)
for name, kw in (("configs[1]", {}), ("configs[4]", dict(n_nodes=100000, n_edges=1000000, alpha=1.5, de=4, dn=4))):
    g = enron_like(seed=0, **kw)
    (src, dst, ts, eidx), rows, pool = split(g)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                         device=dev)
        torch.cuda.synchronize()
        print(name, "entries", f.graph.n_entries, "build %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
