import numpy as np, torch, time
import tempme_amd as tm
from tempme_amd import _lib as L
from tempme_amd.workload import enron_like, split
dev = torch.device("cuda", 0)
N = 20
g = enron_like(alpha=1.2, seed=0)
(src, dst, ts, eidx), rows, pool = split(g)
finder = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"], device=dev, seed=0, split=tm.SPLIT_TEST)
to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)
for E in (800, 1600, 3200, 6400, 12800, 25600, 51200):
    i = np.arange(E) % len(src)
    s_, t_, e_ = to(src[i], np.int32), to(ts[i], np.float64), to(eidx[i], np.int32)
    ev = to(np.arange(E, dtype=np.uint32).view(np.int32), np.int32)
    tot = E * (N + N * N)
    on = torch.empty(tot, dtype=torch.int32, device=dev); oe = torch.empty_like(on); ot = torch.empty(tot, dtype=torch.float32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    def call():
        L.check(L.lib().tm_sample_khop(finder.graph.handle, L.TmRng(0, 1, 1), 2, N, E, L.ptr(s_), L.ptr(t_), L.ptr(e_), L.ptr(ev), L.ptr(on), L.ptr(oe), L.ptr(ot), L.ptr(err), L.stream_ptr(dev)), "khop")
    for _ in range(3): call()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    a.record()
    for _ in range(reps): call()
    b.record(); b.synchronize()
    ms = a.elapsed_time(b) / reps
    byts = E * ((N + N * N) * 28 + (1 + N) * 32)
    print(f"E={E:6d}  {ms*1e3:8.1f} us/call  {byts/ms/1e6:8.1f} GB/s  ({byts/ms/1e6/8000*100:.1f}% of 8 TB/s)")
