"""bench.py -- explained target-edges/s of the TempME explanation hot path on MI355X.

Metric (BASELINE.json): explained target-edges/sec (TGN+Enron, n_degree=20).  One unit = one
target event with its fake destination, 2-hop subgraphs x3 sides, temporal walks x3 with
motif categories and edge counts, encoder forward x3 and retrieve_explanation (eval)
(SURVEY.md §8(d)); the base TGN's contrast is excluded.

Workload: BASELINE configs[1] = enron_sampled + TGN explainer scoring on 1 MI355X, n_degree=20.
Enron is not available offline, so the graph is a seeded synthetic replica of its shape
(tempme_amd/workload.py: V=183, E=18,780, Pareto(1.2) endpoints, ts in [0, 1e8), de=32,
dn=172); explainer weights are a seeded random init of the TempME architecture.

A step = one pass of the hot path over one batch of synthetic input: --batches reference
batches of --batch-size (default 64 x 100 = 6,400) target events per GPU, all on-device
(tm_sample_events -> tm_encoder_fwd -> tm_edge_importance).  Multi-GPU: one process per GPU
(torch.distributed.run), whole batches sharded across ranks, no data-path collective
(weak scaling); barrier + max-over-ranks timing.

Run:  python bench.py [--gpus N --steps K --warmup W]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "explained target-edges/sec (TGN+Enron, n_degree=20) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
FP32_MFMA_PEAK_TF = 157.3      # MI355X_MICROARCH.md: FP32 matrix (spec)


def flops_model(de, dn, h, N, M, etab=False):
    """Algorithmic MACs per unit for each encoder kernel.  ``etab``: the
    pipeline's edge table (lin_event's de x dn edge part once per edge id in the gate-table launch,
    not per executed walk position)."""
    kev = de + 3 + dn
    per_pos_gcn = kev * dn + 2 * (dn * h + h * h)                       # lin_event + event_gcn MLP x2
    per_walk_head = 3 * (2 * h) ** 2 + (2 * h) * h + h * h + (h + 12) ** 2 + (h + 12) * h + h + 2 * 2 * h
    per_pos_gate = (de + dn) * h + h * (h // 2) + h // 2
    W = N * M
    # walk_kernel executes position 2 once per hop-1 slot (shared by the M walks of the slot), and
    # there the all-time-feature K steps of lin_event (dt = 0: constant) are folded into a bias
    qt = (de + 3 + 15) // 16
    exec_walk = 2 * ((2 + 1.0 / M) * per_pos_gcn + per_walk_head - (1 - 1.0 / M) * (2 * h) ** 2
                     - max(kev - 16 * qt, 0) * dn / M)
    walk = 2 * (3 * per_pos_gcn + per_walk_head)
    if etab:
        # the per-position edge-feature product (de x dn MACs) is done per edge id by the table
        # launch: the walk kernel is credited with the rest of the SURVEY model only
        exec_walk -= 2 * (2 + 1.0 / M) * de * dn
        walk -= 2 * 3 * de * dn
    return dict(gcn_kernel=2 * per_pos_gcn * 3, head_kernel=2 * per_walk_head, explain_kernel=2 * per_pos_gate * 3,
                walk_kernel=walk, walk_kernel_executed=exec_walk,
                gate_per_edge=2 * per_pos_gate + (2 * de * dn if etab else 0),
                per_walk=2 * (3 * per_pos_gcn + per_walk_head + 3 * per_pos_gate), W=W)


def aux_rows(finder, src, dst, ts, eidx, pool, graph_build_ms):
    """SURVEY §8 rows outside the per-step unit, timed once (not part of ``value``): a1 the CSR build
    (NeighborFinder.__init__: host sort + per-edge tables + upload) and a11 the null model's sampling
    and counting (utils/null_model.py pre_processing + statistic: 500 events, num_neighbors 30, one
    walk per slot), which the reference spends 2.7-3.2 s on per TempME construction."""
    from tempme_amd.batch_loader import RandEdgeSampler
    from tempme_amd.null_model import null_counts
    from tempme_amd import _lib as L
    sampler = RandEdgeSampler((pool,), (pool,), seed=0, split=L.SPLIT_NULL, device=finder.device)
    null_counts(finder, sampler, src, dst, ts, eidx, 30)          # warm-up (allocations)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cnt = null_counts(finder, sampler, src, dst, ts, eidx, 30)
    null_ms = (time.perf_counter() - t0) * 1e3
    return {"graph_build_ms": round(graph_build_ms, 2), "graph_entries": int(finder.graph.n_entries),
            "null_model_ms": round(null_ms, 3), "null_model_walks": int(cnt.sum())}


def khop_bytes_per_event(N):
    """SURVEY.md §8(d) compulsory traffic of the k-hop kernel (a1-a4) alone, per target event (3 sides)."""
    return 3 * ((N + N * N) * 16 + (N + N * N) * 12 + (1 + N) * 32)


def khop_alone(pipe, inputs, steps, N, group=8):
    """The (a) kernel measured alone (the >= 50 % HBM target applies to it): 2-hop
    sampling of the three sides of the events of ``group`` steps per call -- src and dst on the e_idx
    path, the pipeline's fake dst on the time path -- as three independent tm_sample_khop calls on
    three streams, timed from the first launch to the last completion (HIP events).  One step's 6,400
    roots per call leave a ~10 us launch/ramp/drain overhead exposed; ``group`` steps per call measure
    the kernel's throughput."""
    from tempme_amd import _lib as L
    g = pipe.graph
    dev = inputs[0][0].device
    plans = []
    for k0 in range(0, steps * group, group):
        chunk = [inputs[(k0 + i) % len(inputs)] for i in range(group)]
        fakes = []
        for src, dst, ts, eidx, ev in chunk:
            pipe.sample(src, dst, ts, eidx, ev)      # fake dst of these events (not timed)
            fakes.append(pipe.buf.dst_fake.clone())
        cat = [torch.cat([c[j] for c in chunk]) for j in range(5)]
        src, dst, ts, eidx, ev = cat
        plans.append((ts, ev, ((L.SIDE_SRC, src, eidx), (L.SIDE_TGT, dst, eidx), (L.SIDE_BGD, torch.cat(fakes), None))))
    E = int(plans[0][0].numel())
    tot = E * (N + N * N)
    outs = [(torch.empty(tot, dtype=torch.int32, device=dev), torch.empty(tot, dtype=torch.int32, device=dev),
             torch.empty(tot, dtype=torch.float32, device=dev)) for _ in range(3)]
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(3)]
    main = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()
    ms = []
    for ts, ev, sides in plans + plans:                # first pass warms the streams, second is timed
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main)
        for st, (side, root, ei), (on, oe, ot) in zip(streams, sides, outs):
            st.wait_event(a)
            L.check(L.lib().tm_sample_khop(g.handle, L.TmRng(pipe.seed, pipe.split, side), 2, N, E, L.ptr(root),
                                           L.ptr(ts), L.ptr(ei), L.ptr(ev), L.ptr(on), L.ptr(oe), L.ptr(ot),
                                           L.ptr(err), st.cuda_stream), "tm_sample_khop")
            main.wait_stream(st)
        b.record(main)
        b.synchronize()
        ms.append(a.elapsed_time(b))
    ms = ms[len(plans):]
    L.raise_device_error(int(err.item()), "khop_alone")
    per_step_ms = sum(ms) / len(ms)
    ach = khop_bytes_per_event(N) * E / (per_step_ms * 1e-3) / 1e9
    return {"kernel": "khop2_kernel (tm_sample_khop k=2), 3 sides on 3 streams", "roots_per_call": E,
            "avg_ms": round(per_step_ms, 4), "launches": 3 * len(ms), "bound": "hbm", "achieved": round(ach, 1),
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_event": khop_bytes_per_event(N)}


def sampling_bytes_per_event(N, M):
    """SURVEY.md §8(d) compulsory-traffic model for (a)+(b), per target event (3 sides)."""
    W = N * M
    khop = (N + N * N) * 16 + (N + N * N) * 12 + (1 + N) * 32
    walks = N * 128 + W * 188
    return 3 * (khop + walks)


def cpu_baseline(g, rows, events, pool, N, M, B, seed, sd, budget_s=12.0, max_batches=400):
    """The oracle port (C sampler + torch-fp32 encoder) on the host cores, bounded sample."""
    from oracle import encoder_ref as er
    from oracle import oracle as orc
    threads = int(os.environ.get("TEMPME_CPU_THREADS", min(16, os.cpu_count() or 1)))
    torch.set_num_threads(threads)
    src, dst, ts, eidx = events
    og = orc.OracleGraph(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"])
    nf, ef = torch.from_numpy(g["n_feat"]), torch.from_numpy(g["e_feat"])
    done, t0 = 0, time.perf_counter()
    while done < max_batches * B and time.perf_counter() - t0 < budget_s:
        sl = slice(done % len(src), done % len(src) + B)
        if sl.stop > len(src):
            sl = slice(0, B)
        o = orc.event_pipeline(og, seed, 1, N, M, src[sl], dst[sl], ts[sl], eidx[sl], np.arange(done, done + B),
                               pool, threads)
        with torch.no_grad():
            for s in range(3):
                imp = er.forward(sd, nf, ef, o["node6"][:, s], o["eid3"][:, s], o["ts3"][:, s], o["cat"][:, s],
                                 ts[sl], o["cnt"][:, s].astype(np.float64))
                er.edge_importance(sd, ef, imp, o["eid3"][:, s], o["ts3"][:, s],
                                   [o["sub1_node"][:, s], o["sub2_node"][:, s]],
                                   [o["sub1_eid"][:, s], o["sub2_eid"][:, s]])
        done += B
    el = time.perf_counter() - t0
    return {"value": round(done / el, 2), "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"{done} target events ({done // B} reference batches of {B}) of the same workload: "
                      f"oracle/tempme_oracle.c sampling+motif ({threads} OpenMP threads) + oracle/encoder_ref.py "
                      f"torch-fp32 encoder+explanation ({threads} threads), {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batches", type=int, default=64, help="reference batches per step per GPU")
    ap.add_argument("--batch-size", type=int, default=100, help="temp_exp_main --test_bs")
    ap.add_argument("--n-degree", type=int, default=20)
    ap.add_argument("--alpha", type=float, default=1.2)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --batches is the whole step, split over the ranks (default: per rank)")
    ap.add_argument("--no-edge-table", action="store_true",
                    help="lin_event's edge-feature product per walk position instead of per edge id")
    ap.add_argument("--streams", type=int, default=1,
                    help="steps in flight (PipelinedExplainer): step k runs on stream k %% S with its own "
                         "buffers, so its sampling and explanation kernels overlap the neighbouring steps' "
                         "encoder kernel (encoders chained: +5 %% at 8 batches per step, none at 64)")
    ap.add_argument("--config", type=int, default=1, choices=(1, 2, 4),
                    help="BASELINE.json configs[i] workload: 1 = enron_sampled + TGN, N=20 (the headline); "
                         "2 = full Enron shape (E=125,235), N=20; 4 = synthetic 1M-edge graph, de=dn=172, "
                         "Pareto 1.5, N=30 (the HBM stress case)")
    args = ap.parse_args()
    if args.config == 4 and args.n_degree == 20:
        args.n_degree = 30

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU; TEMPME_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks
    # sharing the GPUs there are (ranks map to local_rank % device_count)
    backend = os.environ.get("TEMPME_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(dev)

    import tempme_amd as tm
    from tempme_amd import _lib as L
    from tempme_amd.pipeline import ExplainPipeline, PipelinedExplainer
    from tempme_amd.sharding import max_over_ranks, shard_events
    from tempme_amd.workload import enron_like, split

    N, M, B = args.n_degree, 3, args.batch_size
    if args.strong:
        # strong scaling: the step's args.batches reference batches are dealt over the ranks
        if args.batches % world:
            raise SystemExit(f"--strong needs --batches divisible by the {world} ranks")
        E = args.batches // world * B
    else:
        E = args.batches * B
    if args.config == 1:
        g = enron_like(alpha=args.alpha, seed=args.seed)
        workload = ("configs[1]: enron_sampled-shaped synthetic graph (V=183, E=18,780, "
                    f"Pareto {args.alpha}) + TGN explainer scoring, n_degree={args.n_degree}")
    elif args.config == 2:
        g = enron_like(n_nodes=184, n_edges=125235, alpha=args.alpha, seed=args.seed)
        workload = (f"configs[2]: full-Enron-shaped synthetic graph (V=184, E=125,235, Pareto {args.alpha}), "
                    f"TempME encoder + explanation, n_degree={args.n_degree}")
    else:
        g = enron_like(n_nodes=100000, n_edges=1000000, alpha=1.5, de=172, dn=172, seed=args.seed,
                       node_feat="uniform")
        workload = ("configs[4]: synthetic 1M-edge temporal graph (V=100,000, Pareto 1.5, de=dn=172 U(0,1) "
                    f"features), TempME explanation scoring, n_degree={args.n_degree}")
    (src, dst, ts, eidx), rows, pool = split(g)
    torch.zeros(1, device=dev)                     # device context and allocator up before timing the build
    torch.cuda.synchronize()
    tb = time.perf_counter()
    finder = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows],
                                          g["n_nodes"], device=dev, seed=args.seed, split=tm.SPLIT_TEST)
    torch.cuda.synchronize()
    graph_build_ms = (time.perf_counter() - tb) * 1e3

    class Base:
        n_feat_th = torch.from_numpy(g["n_feat"])
        e_feat_th = torch.from_numpy(g["e_feat"])
        node_raw_features = torch.nn.Embedding.from_pretrained(n_feat_th, padding_idx=0, freeze=True)
        edge_raw_features = torch.nn.Embedding.from_pretrained(e_feat_th, padding_idx=0, freeze=True)

    torch.manual_seed(args.seed)
    ex = tm.TempME(Base(), "tgn", "enron_sampled", out_dim=40, hid_dim=64, device=dev,
                   null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).eval()
    S = max(1, args.streams)
    if S == 1:
        pipe = ExplainPipeline(ex, finder.graph, torch.from_numpy(pool), N, M, B, seed=args.seed,
                               edge_table=not args.no_edge_table)
        pipes = [pipe]

        def run_step(k):
            pipe.run(*inputs[k])
    else:
        flight = PipelinedExplainer(ex, finder.graph, torch.from_numpy(pool), N, M, B, seed=args.seed, depth=S,
                                    edge_table=not args.no_edge_table)
        pipes = flight.pipes
        pipe = pipes[0]

        def run_step(k):
            flight.submit(*inputs[k])

    # inputs for every step resident in HBM before timing: events cycle through the test split
    n_steps = args.warmup + args.steps
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    inputs = []
    for k in range(n_steps):
        i, ev = shard_events(k, rank, world, E, len(src))
        inputs.append((to(src[i], np.int32), to(dst[i], np.int32), to(ts[i], np.float64), to(eidx[i], np.int32),
                       to(ev.view(np.int32), np.int32)))

    for k in range(max(args.warmup, S)):        # every stream's buffers allocated before timing
        run_step(k % n_steps)
    torch.cuda.synchronize()
    for p in pipes:
        p.check_errors()

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    L.profile_enable(True)
    t0 = time.perf_counter()
    for k in range(args.warmup, n_steps):
        run_step(k)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    prof = L.profile_read()
    L.profile_enable(False)
    for p in pipes:
        p.check_errors()
    el = max_over_ranks(el, dist, dev if backend == "nccl" else "cpu")

    if rank == 0:
        fm = flops_model(g["e_feat"].shape[1], g["n_feat"].shape[1], 64, N, M, etab=pipe.etab is not None)
        W = fm["W"]
        units = {"events_kernel": ("hbm", sampling_bytes_per_event(N, M) * E),
                 "gcn_kernel": ("mfma", fm["gcn_kernel"] * 3 * E * W),
                 "head_kernel": ("mfma", fm["head_kernel"] * 3 * E * W),
                 "explain_kernel": ("mfma", fm["explain_kernel"] * 3 * E * W),
                 "gate_table_kernel": ("mfma", fm["gate_per_edge"] * (g["eidx"].max() + 1)),
                 "walk_kernel": ("mfma", fm["walk_kernel"] * 3 * E * W)}
        executed = {"walk_kernel": fm["walk_kernel_executed"] * 3 * E * W}
        kernels = {}
        for name, (ms, cnt) in prof.items():
            avg_ms = ms / max(cnt, 1)
            ent = {"avg_ms": round(avg_ms, 4), "launches": cnt}
            if name in units:
                bound, work = units[name]
                if bound == "hbm":
                    ach = work / (avg_ms * 1e-3) / 1e9
                    ent.update(bound="hbm", achieved=round(ach, 1), unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4))
                else:
                    ach = work / (avg_ms * 1e-3) / 1e12
                    ent.update(bound="mfma", achieved=round(ach, 2), unit="TFLOP/s",
                               frac=round(ach / FP32_MFMA_PEAK_TF, 4))
                    if name in executed:
                        ex_tf = executed[name] / (avg_ms * 1e-3) / 1e12
                        ent.update(executed_tflops=round(ex_tf, 2), executed_frac=round(ex_tf / FP32_MFMA_PEAK_TF, 4))
            kernels[name] = ent
        dom = max((k for k in kernels if "bound" in kernels[k]), key=lambda k: kernels[k]["avg_ms"])
        d = kernels[dom]
        roof = {"bound": d["bound"], "achieved": d["achieved"],
                "peak": HBM_PEAK_GBS if d["bound"] == "hbm" else FP32_MFMA_PEAK_TF, "unit": d["unit"],
                "frac": d["frac"], "traffic": None, "kernel": dom}
        pmc = os.path.join(HERE, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            with open(pmc) as fh:
                tr = json.load(fh).get(dom)
            if tr is not None:
                roof["traffic"] = tr
        total = world * args.steps * E
        out = {"metric": METRIC, "value": round(total / el, 2), "unit": "edges/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
               "higher_is_better": True, "scaling": "strong" if args.strong else "weak", "vs_baseline": None,
               "dtype": "fp32",
               "data": "synthetic (seeded graph of the config's shape, random-init TempME weights)",
               "config": {"workload": workload,
                          "n_degree": N, "walks_per_slot": M, "batch_size": B, "batches_per_step_per_gpu": E // B,
                          "events_per_step_per_gpu": E, "parallelism": f"dp{world} (whole batches per rank)",
                          "steps_in_flight": S},
               "roofline": roof, "kernels": kernels,
               "sampling_roofline": kernels.get("events_kernel")}
        if S > 1:
            # with steps in flight the sampling kernel runs in the encoder's shadow (its launch duration
            # then measures co-residency, not the kernel): its roofline comes from a pass with one step
            # in flight, right after the timed region
            L.profile_enable(True)
            for k in range(min(args.steps, 5)):
                pipe.run(*inputs[k])
            torch.cuda.synchronize()
            iso = L.profile_read()
            L.profile_enable(False)
            ms, cnt = iso["events_kernel"]
            avg_ms = ms / max(cnt, 1)
            ach = units["events_kernel"][1] / (avg_ms * 1e-3) / 1e9
            kernels["events_kernel"]["note"] = "launch duration while overlapping the previous step's walk_kernel"
            out["sampling_roofline"] = {"avg_ms": round(avg_ms, 4), "launches": cnt, "bound": "hbm",
                                        "achieved": round(ach, 1), "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                                        "measured": "one step in flight (not overlapped), after the timed region"}
        out["khop_roofline"] = khop_alone(pipe, inputs, min(args.steps, 5), N, group=8)
        out["aux"] = aux_rows(finder, src, dst, ts, eidx, pool, graph_build_ms)
        if world == 1 and not args.no_cpu_baseline:
            sd = {k: v.detach().cpu() for k, v in ex.state_dict().items()}
            out["cpu_baseline"] = cpu_baseline(g, rows, (src, dst, ts, eidx), pool, N, M, B, args.seed, sd)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
