"""walk_kernel wave timeline under a -DTM_TRACE build (TEMPME_LIB=tempme_amd/lib/dbg/trace.so).

For each group count G of tools/walk_scale.py's setup (24 reference batches sampled once), run the encoder a few
times and summarise the last launch's per-wave trace (s_memrealtime, 100 MHz = 10 ns ticks): entry spread,
constant-table load, first vs later unit durations, per-wave end times, lone vs paired waves per SIMD."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def summarise(tr, n_waves):
    tr = tr[:n_waves]
    used = tr[:, 28] > 0
    t0 = tr[:, 0].min()
    ent = (tr[:, 0] - t0) * 0.01                      # us
    cst = (tr[:, 1] - tr[:, 0]) * 0.01
    n = tr[:, 28].astype(np.int64)
    ends = np.full(n_waves, np.nan)
    first = []
    later = []
    for w in np.nonzero(used)[0]:
        k = min(n[w], 12)
        stamps = np.concatenate([[tr[w, 1]], tr[w, 16:16 + k]]).astype(np.int64)
        d = np.diff(stamps) * 0.01
        first.append(d[0])
        later.extend(d[1:].tolist())
        ends[w] = (stamps[-1] - t0) * 0.01
    pct = lambda a: " ".join(f"p{q}={np.percentile(a, q):.1f}" for q in (0, 10, 50, 90, 100))  # noqa: E731
    print(f"  waves {n_waves} used {used.sum()} units/wave {pct(n[used])}")
    print(f"  entry (us after first) {pct(ent)}")
    print(f"  const table (us) {pct(cst)}")
    print(f"  first unit (us) {pct(first)}")
    if later:
        print(f"  later units (us) {pct(later)}")
    e = ends[used]
    print(f"  wave end (us) {pct(e)}  kernel span {(e.max()):.1f} us")
    # per pass of the first two units (pass 0 = the slot pass, then walk m's positions 0 / 1)
    two = used & (n >= 2)
    if two.any():
        st = np.concatenate([tr[two, 1:2], tr[two, 2:16]], axis=1).astype(np.int64)
        d = np.diff(st, axis=1) * 0.01
        print("  unit 0 passes (us, median):", " ".join(f"{np.median(d[:, i]):.1f}" for i in range(7)))
        print("  unit 1 passes (us, median):", " ".join(f"{np.median(d[:, 7 + i]):.1f}" for i in range(7)))
    hw = tr[:, 29].astype(np.uint64)
    xcc = (hw >> np.uint64(32)) & np.uint64(0xF)
    simd = (hw >> np.uint64(4)) & np.uint64(0x3)
    cu = (hw >> np.uint64(8)) & np.uint64(0xF)
    sh = (hw >> np.uint64(12)) & np.uint64(0x1)
    se = (hw >> np.uint64(13)) & np.uint64(0x7)
    key = (((xcc * np.uint64(8) + se) * np.uint64(2) + sh) * np.uint64(16) + cu) * np.uint64(4) + simd
    ku, cnt = np.unique(key[used], return_counts=True)
    print(f"  distinct SIMDs {len(ku)}, waves per SIMD {np.bincount(cnt).tolist()}, XCCs {np.unique(xcc).tolist()}")


def main():
    import tempme_amd as tm
    from tempme_amd import _lib as L
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
    fn = L.lib().tm_debug_trace
    fn.argtypes = [C.c_void_p]
    buf = np.zeros((8192, 32), dtype=np.uint64)
    for G in [int(v) for v in os.environ.get("WS_GROUPS", "16,32,64,72").split(",")]:
        for r in range(4):
            ex.encoder_fwd(b.node6, b.eid3, b.ts3, b.cat, cut, b.cnt, G, B, W, out=pipe.imp, workspace=pipe.ws, M=M,
                           etab=pipe.etab)
            torch.cuda.synchronize()
        assert fn(buf.ctypes.data) == 0
        units = G * B * W // M // 16
        n_waves = min(2048, (units + 3) // 4 * 4)
        print(f"G={G} units={units}")
        summarise(buf.copy(), n_waves)
    # hot: the pipeline's steps back to back (sampler, encoder, explanation), the last step's walk launch
    for _ in range(12):
        pipe.run(*x)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data) == 0
    units = 3 * nb * B * W // M // 16
    print(f"hot pipeline steps, G={3 * nb} units={units}")
    summarise(buf.copy(), min(2048, (units + 3) // 4 * 4))


if __name__ == "__main__":
    main()
