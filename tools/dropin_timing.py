"""Per-segment host timing of the drop-in eval pattern (temp_exp_main.py:446-453) on the metric config:
get_item / get_item_edge, TempME.forward x3, retrieve_explanation, with (a) the free-running loop's
wall time per batch and (b) per-segment host time (perf_counter, no profiler), and (c) the GPU time of
one batch alone (synchronised before and after).  Diagnostic for bench.py's ``dropin`` leg."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")


def main():
    import tempme_amd as tm
    from tempme_amd import pack as P
    from tempme_amd.pipeline import ExplainPipeline
    from tempme_amd.workload import enron_like, split
    dev = torch.device("cuda", 0)
    N, M, B, seed = 20, 3, 100, 0
    g = enron_like(seed=seed, n_nodes=184, n_edges=125235, alpha=1.2)
    (src, dst, ts, eidx), rows, pool = split(g)
    finder = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                          device=dev, seed=seed, split=tm.SPLIT_TEST)

    class Base:
        n_feat_th = torch.from_numpy(g["n_feat"])
        e_feat_th = torch.from_numpy(g["e_feat"])
        node_raw_features = torch.nn.Embedding.from_pretrained(n_feat_th, padding_idx=0, freeze=True)
        edge_raw_features = torch.nn.Embedding.from_pretrained(e_feat_th, padding_idx=0, freeze=True)

    torch.manual_seed(seed)
    ex = tm.TempME(Base(), "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
                   null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).eval()
    nb = 32
    pipe = ExplainPipeline(ex, finder.graph, torch.from_numpy(pool), N, M, B, seed=seed)
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    sl = slice(0, nb * B)
    ev = np.arange(nb * B, dtype=np.int64)
    pipe.sample(to(src[sl], np.int32), to(dst[sl], np.int32), to(ts[sl], np.float64), to(eidx[sl], np.int32),
                to(ev.view(np.int32), np.int32))
    _, cat_d, edge = P.buffers_to_arrays(pipe.buf, nb * B)

    class A:
        n_degree = N
    cut = ts[sl].astype(np.float64)
    host = "host" in sys.argv[1:]     # the reference's host float64 pack (load_subgraph_margin(args, f)) and edge array
    if host:
        pk, ed = P.load_subgraph_margin(A(), cat_d), edge
    else:
        pk, ed = P.load_subgraph_margin(A(), cat_d, device=dev), P.load_edge(edge, dev)
    seg = {k: 0.0 for k in ("get_item", "get_item_edge", "forward_src", "forward_tgt", "forward_bgd", "retrieve")}

    def one(b, t=None):
        idx = np.arange(b * B, (b + 1) * B)
        t0 = time.perf_counter()
        sg_s, sg_t, sg_b, w_s, w_t, w_b, _ = P.get_item(pk, idx)
        t1 = time.perf_counter()
        e_s, e_t, e_b = P.get_item_edge(ed, idx)
        t2 = time.perf_counter()
        i_s = ex(w_s, cut[idx], e_s)
        t3 = time.perf_counter()
        i_t = ex(w_t, cut[idx], e_t)
        t4 = time.perf_counter()
        i_b = ex(w_b, cut[idx], e_b)
        t5 = time.perf_counter()
        out = ex.retrieve_explanation(sg_s, i_s, w_s, sg_t, i_t, w_t, sg_b, i_b, w_b, training=False)
        t6 = time.perf_counter()
        if t is not None:
            for k, d in zip(seg, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
                t[k] += d
        return out

    for b in range(nb):
        one(b)
    torch.cuda.synchronize()
    # time spent inside the two library calls of the fast path (wrapped ctypes functions)
    from tempme_amd import _lib as L
    lib = L.lib()
    ctime, orig = {}, {}
    for name in ("tm_dropin_forward", "tm_edge_importance_gf3"):
        f = orig[name] = getattr(lib, name)

        def wrap(*a, _f=f, _n=name):
            t0 = time.perf_counter()
            r = _f(*a)
            ctime[_n] = ctime.get(_n, 0.0) + time.perf_counter() - t0
            return r
        setattr(lib, name, wrap)
    # the host-pack path's staging (hoststage) and the context's own library entry (bound at context creation)
    from tempme_amd import hoststage as HS
    horig = {n: getattr(HS, n) for n in ("stage", "window_bounds")}
    for name, f in horig.items():
        def wraph(*a, _f=f, _n=name, **kw):
            t0 = time.perf_counter()
            r = _f(*a, **kw)
            ctime["hoststage." + _n] = ctime.get("hoststage." + _n, 0.0) + time.perf_counter() - t0
            return r
        setattr(HS, name, wraph)
    dctx = ex.__dict__.get("_dropin_c")
    if dctx is not None:
        cf = dctx[1].fwd

        def wrapc(*a, _f=cf):
            t0 = time.perf_counter()
            r = _f(*a)
            ctime["ctx.fwd (tm_dropin_forward)"] = ctime.get("ctx.fwd (tm_dropin_forward)", 0.0) + time.perf_counter() - t0
            return r
        dctx[1].fwd = wrapc
    # Python methods of the fast path, timed the same way
    for name in ("_fast_state", "_dropin_ctx", "_hip_eval_ok"):
        f = getattr(ex, name)

        def wrapm(*a, _f=f, _n=name):
            t0 = time.perf_counter()
            r = _f(*a)
            ctime[_n] = ctime.get(_n, 0.0) + time.perf_counter() - t0
            return r
        ex.__dict__[name] = wrapm
    from tempme_amd.explainer import _dropin_ext
    xm = _dropin_ext()
    if xm is not None and hasattr(xm, "prof_enable"):
        xm.prof_enable(True)
    reps = 8
    t0 = time.perf_counter()
    for r in range(reps):
        for b in range(nb):
            one(b, seg)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / (reps * nb)
    print("free-running: %.1f us per batch = %.0f edges/s" % (wall * 1e6, B / wall))
    for k, v in seg.items():
        print("  %-14s %7.1f us" % (k, v / (reps * nb) * 1e6))
    for k, v in ctime.items():
        print("  inside %-22s %7.1f us per batch" % (k, v / (reps * nb) * 1e6))
    if xm is not None and hasattr(xm, "prof_read"):
        segs, n = xm.prof_read()
        xm.prof_enable(False)
        names = ("resident checks", "shape / cut checks", "state check", "output alloc", "recordStream",
                 "tm_dropin_forward", "cache + wrap")
        print("  C++ Fast.forward split (%d calls): " % n + ", ".join("%s %.2f us" % (a, b) for a, b in zip(names, segs)))
    for name, f in orig.items():     # the original function objects (they carry the argtypes)
        setattr(lib, name, f)
    for name in ("_fast_state", "_dropin_ctx", "_hip_eval_ok"):
        del ex.__dict__[name]
    for name, f in horig.items():
        setattr(HS, name, f)
    if dctx is not None:
        dctx[1].fwd = cf
    if "profile" in sys.argv[1:]:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for b in range(nb):
            one(b)
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    # one side's forward, split: the module call, forward() without nn.Module.__call__, and the C++ host
    # side's entry alone (csrc/dropin_ext.cpp Fast.forward: checks, output allocation, tm_dropin_forward)
    fx = ex.__dict__.get("_fastx")
    if fx is not None:
        ins = []
        for b in range(nb):
            idx = np.arange(b * B, (b + 1) * B)
            _, _, _, w_s, _, _, _ = P.get_item(pk, idx)
            e_s, _, _ = P.get_item_edge(ed, idx)
            ins.append((w_s, cut[idx], e_s))
        calls = (("module call", lambda w, c, e: ex(w, c, e)), ("forward()", lambda w, c, e: ex.forward(w, c, e)),
                 ("C++ Fast.forward", lambda w, c, e, _f=fx[0].forward: _f(w[0], w[1], w[2], w[3], c, e)))
        for name, fn in calls[::-1] + calls:     # both orders: the first loop of a run pays any warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for r in range(reps):
                for w, c, e in ins:
                    fn(w, c, e)
            el = time.perf_counter() - t0
            torch.cuda.synchronize()
            print("  one side, %-18s %6.1f us per call" % (name, el / (reps * nb) * 1e6))
    # one batch alone, GPU included
    lat = []
    for b in range(nb):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        one(b)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    print("one batch alone (host + GPU, synchronised): median %.1f us" % (np.median(lat) * 1e6))
    # GPU time of a batch when the host is far ahead: issue all, time with events on the current stream
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e8))          # hold the stream so the host gets ahead of the GPU
    e0.record(s)
    for r in range(2):
        for b in range(nb):
            one(b)
    e1.record(s)
    torch.cuda.synchronize()
    print("GPU-bound (stream held, host ahead): %.1f us per batch" % (e0.elapsed_time(e1) * 1e3 / (2 * nb)))


if __name__ == "__main__":
    main()
