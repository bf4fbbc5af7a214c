"""Explainer training-step throughput (BASELINE.json configs[3]: full Enron + TGN,
target-edge batches sharded across GPUs with one RCCL gradient all-reduce per step).

    python bench_train.py [--gpus N --steps K --warmup W --n-degree 20 --batch-size 100]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench_train.py --gpus N

One train step = temp_exp_main.py:593-632 for one batch of `--batch-size` target events per GPU: base
contrast without explanation (no grad), TempME forward x3 (training mode: dropout, Beta rsample),
retrieve_explanation, contrast with explanation weights, BCE + 0.5 KL, backward, gradient all-reduce,
Adam.  The pack (k-hop subgraphs, walks, categories, edge counts of every training event) is sampled
on the device before timing, as the reference samples it offline (processed/data_preprocess.py).
A timed step is `--global-batches` reference batches over all ranks (strong scaling: N ranks take
global-batches / N train steps each, one all-reduced update per round of N batches; `--weak`: that
many per rank).  Prints one JSON line (rank 0); value = trained target edges per second over all ranks.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch


def kernel_flops(ex, B, N, M, zn=False):
    """Algorithmic FLOPs per training step of the encoder kernels (one launch each covers the three sides of a
    batch: n = 3 B W walks, R = 3 n walk positions; the explanation's gate runs on R positions too).
    gcn_bwd_kernel per position: the recomputed lin_event (kev x dn) and event_gcn first layer (br branches of
    dn x h), then d MLP.2 (h x h per branch), d MLP.0 (h x dn per branch) and the time-feature gradient through
    lin_event (dn x dn); gcn_kernel per position: lin_event + the two MLP layers per branch.  zn: zero node
    features, the kernels' one-branch forms (br = 1; the branch sums fold before the GEMMs).
    wgrad_partial_kernel: dW = dY^T [X | 1] over the rows of every weight-gradient job of the step (the
    encoder's 12 jobs and the gate's 4; tm_encoder_wgrad / tm_explain_train_bwd), 2 rows O (I + 1) each."""
    de, dn, h, hm = ex.edge_dim, ex.node_dim, ex.hid_dim, ex.mlp_dim
    kev = de + 3 + dn
    W = N * M
    n = 3 * B * W
    R = 3 * n
    br = 1 if zn else 2
    gcn_bwd = R * 2 * (kev * dn + br * dn * h + br * h * h + br * h * dn + dn * dn)
    gcn = R * 2 * (kev * dn + br * dn * h + br * h * h)
    h2 = 2 * h
    rows = br * R
    enc = (R * dn * (kev + 1) + rows * h * (dn + 1) + rows * h * (h + 1) + n * h2 * (h2 + 1) + 2 * n * h2 * (h2 + 1)
           + n * h * (h2 + 1) + n * h * (h + 1) + n * hm * (hm + 1) + n * h * (hm + 1) + n * (h + 1) + R * dn * 2)
    gate = R * h * (de + dn + 1) + R * (h // 2) * (h + 1) + R * (h // 2 + 1) + R * dn * 2
    # head_kernel per walk (TemporalAwareAttention :789-846 + the category MLP :122-125; the GEMMs of the wgrad job
    # list above): W1 on position 2 and W2 on positions 0, 1 (h2 x h2 each), the two bmm's (2 h2 each), MLP h2 -> h
    # -> h, the category MLP (hm x hm, hm -> h, h -> 1).  head_bwd_kernel recomputes that forward and runs the
    # data-gradient GEMM of every layer (same sizes): twice the forward.
    head = 2 * n * (3 * h2 * h2 + 4 * h2 + h * h2 + h * h + hm * hm + h * hm + h)
    # gate_train_fwd_kernel per position: [E | cos] (de + dn) -> h -> h/2 -> 1; gate_train_bwd_kernel: d G2 -> d G1
    # (h/2 x h) -> d time features (h x dn)
    gate_fwd = 2 * R * ((de + dn) * h + h * (h // 2) + h // 2)
    gate_bwd = 2 * R * ((h // 2) * h + h * dn)
    return {"gcn_bwd_kernel": gcn_bwd, "gcn_kernel": gcn, "wgrad_partial_kernel": 2 * (enc + gate),
            "head_kernel": head, "head_bwd_kernel": 2 * head, "gate_train_fwd_kernel": gate_fwd,
            "gate_train_bwd_kernel": gate_bwd}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch-size", type=int, default=100, help="temp_exp_main --bs")
    ap.add_argument("--n-degree", type=int, default=20)
    ap.add_argument("--alpha", type=float, default=1.2)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-graph", action="store_true", help="launch every kernel from the host each step "
                    "instead of replaying the step captured as a HIP graph (the default with one GPU)")
    ap.add_argument("--graph", action="store_true", help="capture the step as a HIP graph with several ranks "
                    "too (the RCCL all-reduce is then captured inside the graph)")
    ap.add_argument("--optim", choices=("hip", "torch-fused", "torch"), default="hip",
                    help="hip: tempme_amd.optim.FusedAdam (one HIP kernel over the flat parameter / gradient bucket the "
                         "all-reduce also runs on); torch-fused: torch.optim.Adam(fused=True); torch: its foreach form")
    ap.add_argument("--no-node-zero", action="store_true",
                    help="do not use the zero-node-feature kernel forms (A/B; the graph's node features are zeros)")
    ap.add_argument("--overlap-prepare", action="store_true",
                    help="graphed step with the base model's original contrast as a second graph branch "
                         "(GraphedTrainStep(overlap_prepare=True); measured within noise, round 5)")
    ap.add_argument("--global-batches", type=int, default=8,
                    help="reference batches per timed step over ALL ranks (strong scaling: each rank steps through "
                         "global-batches / N of them, one all-reduced Adam update per round of N batches)")
    ap.add_argument("--weak", action="store_true", help="--global-batches per rank instead (weak scaling)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="eager multi-rank path: run the gradient all-reduce serially instead of overlapping it "
                         "with the next batch's explainer-independent work")
    args = ap.parse_args()

    # one process per GPU: start our own ranks unless a launcher already did (before any GPU call)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        import subprocess
        import socket
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s_:
            s_.bind(("127.0.0.1", 0))
            port = s_.getsockname()[1]
        sys.exit(subprocess.call([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                                  f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
                                  os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench_train.py: --gpus {args.gpus} but the launcher started {world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("TEMPME_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import tempme_amd as tm
    from tempme_amd import _lib as L
    from tempme_amd.preprocess import sample_events
    from tempme_amd.sharding import max_over_ranks
    from tempme_amd.tgn import TGN
    from tempme_amd.train import GradAllReduce, GraphedTrainStep, batch_from_pack, epoch_spans, run_steps
    from tempme_amd.workload import enron_like, split

    N, M, B = args.n_degree, 3, args.batch_size
    g = enron_like(n_nodes=184, n_edges=125235, alpha=args.alpha, seed=args.seed)     # full Enron shape
    (src, dst, ts, eidx), rows, pool = split(g, mode="train")
    finder = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows],
                                          g["n_nodes"], device=dev, seed=args.seed, split=tm.SPLIT_TRAIN)
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    s_d, d_d, t_d, e_d = to(src, np.int32), to(dst, np.int32), to(ts, np.float64), to(eidx, np.int32)
    ev = torch.arange(len(src), dtype=torch.int32, device=dev)
    buf = sample_events(finder.graph, args.seed, tm.SPLIT_TRAIN, N, M, s_d, d_d, t_d, e_d, ev,
                        to(pool, np.int32))

    torch.manual_seed(args.seed)          # identical replicas on every rank
    base = TGN(g["n_feat"], g["e_feat"], n_neighbors=N, device=dev, n_layers=2, n_heads=2, dropout=0.1)
    base.forbidden_memory_update = True
    base = base.to(dev).eval()
    ex = tm.TempME(base, "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
                   null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev)
    ex.node_zero_specialization = not args.no_node_zero
    use_graph = not args.no_graph and (world == 1 or (args.graph and backend == "nccl"))
    # temp_exp_main.py's torch.optim.Adam(lr=1e-3) update rule; default: one HIP kernel over the flat bucket
    if args.optim == "hip":
        from tempme_amd.optim import FusedAdam
        opt = FusedAdam(ex.parameters(), lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0)
        sync = GradAllReduce(ex, bucket=opt)
    else:
        opt = torch.optim.Adam(ex.parameters(), lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                               capturable=use_graph, fused=args.optim == "torch-fused")
        sync = GradAllReduce(ex)
    ex.train()

    if not args.weak and args.global_batches % world:
        raise SystemExit(f"bench_train.py: --global-batches {args.global_batches} is not divisible by {world} ranks")
    per_step = args.global_batches if args.weak else args.global_batches // world   # train_steps per rank per step
    n_steps = (args.warmup + args.steps) * per_step
    gen = torch.Generator().manual_seed(args.seed)
    spans = []
    while len(spans) < n_steps + 4:     # a few spare in case the graphed path drops an epoch's tail batch
        perm = torch.randperm(len(src) - 1, generator=gen).to(dev)
        spans += [(perm, a, b) for a, b in epoch_spans(len(src) - 1, B, rank, world)]
    rows = [perm[a:b] for perm, a, b in spans[:n_steps]]
    if use_graph:
        # whole-batch shape is fixed (epoch tails are dropped), so the step is captured once
        rows = [r for r in rows if r.numel() == B]
        n_steps = min(n_steps, len(rows))
        graphed = GraphedTrainStep(ex, base, opt, buf, s_d, d_d, t_d, e_d, rows[:max(args.warmup, 1)],
                                   grad_sync=sync, overlap_prepare=args.overlap_prepare)

        def step(k):   # one timed step = per_step replays
            out = None
            for i in range(k * per_step, (k + 1) * per_step):
                out = graphed(rows[i])
            return out
    else:
        batches = [batch_from_pack(buf, s_d, d_d, t_d, e_d, r) for r in rows]

        def step(k):   # one timed step = per_step train_steps; the all-reduce overlaps the next batch's prep
            outs = run_steps(ex, base, opt, batches[k * per_step:(k + 1) * per_step], grad_sync=sync,
                             overlap=not args.no_overlap)
            return outs[-1]
        for k in range(args.warmup):
            step(k)
    torch.cuda.synchronize()
    base.check_errors()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    L.profile_enable(True)
    t0 = time.perf_counter()
    losses = []
    n_timed = n_steps // per_step
    for k in range(args.warmup, n_timed):
        losses.append(step(k)["loss"].clone())
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    prof = L.profile_read()
    L.profile_enable(False)
    el = max_over_ranks(el, dist, dev if backend == "nccl" else "cpu")
    if world > 1:   # distinct devices (a gloo rehearsal puts the ranks on one GPU)
        devs = [None] * world
        dist.all_gather_object(devs, dev.index)
        n_gpus = len(set(devs))
    else:
        n_gpus = 1
    losses = [float(x) for x in losses]
    # per-kernel table: a graph replay bypasses the library's launch-site HIP-event timing, so with a
    # captured step the table comes from a few extra EAGER steps (not part of `value`); the dominant kernel's
    # roofline uses its algorithmic FLOPs (kernel_flops below)
    kern_src = "timed steps"
    if use_graph and not prof:
        eager = [batch_from_pack(buf, s_d, d_d, t_d, e_d, r) for r in rows[:3]]
        torch.cuda.synchronize()
        L.profile_enable(True)
        run_steps(ex, base, opt, eager, grad_sync=sync, overlap=False)
        torch.cuda.synchronize()
        prof = L.profile_read()
        L.profile_enable(False)
        kern_src = f"{len(eager)} eager steps after the timed replays (same kernels as the captured step)"
    if rank == 0:
        edges = sum(int(rows[k].numel()) for k in range(args.warmup * per_step, n_timed * per_step)) * world
        timed = n_timed - args.warmup
        out = {"metric": "trained target-edges/sec (explainer training step, TGN + full-Enron-shaped graph)",
               "value": round(edges / el, 2), "unit": "edges/s", "n_gpus": n_gpus, "ranks": world, "steps": timed,
               "warmup": args.warmup, "ms_per_step": round(el / max(timed, 1) * 1e3, 3), "higher_is_better": True,
               "scaling": "weak" if args.weak else "strong", "vs_baseline": None, "dtype": "fp32",
               "data": "synthetic (seeded Enron-shaped graph V=184 E=125,235, random-init TGN and TempME)",
               "config": {"workload": "configs[3]: full Enron + TGN explainer training step", "n_degree": N,
                          "batch_size": B, "train_events": int(len(src)), "parallelism": f"dp{world}",
                          "global_batches_per_step": per_step * world, "train_steps_per_rank_per_step": per_step,
                          "allreduce_overlap": (not args.no_overlap) and not use_graph,
                          "hip_graph": use_graph, "overlap_prepare": bool(args.overlap_prepare and use_graph),
                          "optimizer": args.optim,
                          "zero_node_forms": bool(getattr(ex, "_node_zero", False)) and ex.node_zero_specialization,
                          "grad_bucket_floats": sum(p.numel() for p in ex.parameters() if p.grad is not None)},
               "loss_first_last": [round(losses[0], 5), round(losses[-1], 5)],
               "kernels": {k: {"avg_ms": round(ms / max(c, 1), 4), "launches": c} for k, (ms, c) in prof.items()},
               "kernels_source": kern_src}
        zn = bool(getattr(ex, "_node_zero", False)) and ex.node_zero_specialization
        fl = kernel_flops(ex, B, N, M, zn=zn)
        # per kernel: its FLOPs per training step over its time per training step (the kernel table's launches
        # cover the steps the table was taken over; wgrad_partial_kernel has two launches per step)
        n_tab = len(eager) if use_graph and kern_src != "timed steps" else (n_timed - args.warmup) * per_step
        roofs = {}
        for k, f in fl.items():
            v = out["kernels"].get(k)
            if not v:
                continue
            per_step_ms = v["avg_ms"] * v["launches"] / max(n_tab, 1)
            ach = f / (per_step_ms * 1e-3) / 1e12
            roofs[k] = {"bound": "mfma", "achieved": round(ach, 2), "peak": 157.3, "unit": "TFLOP/s",
                        "frac": round(ach / 157.3, 4), "flop_per_step": f, "ms_per_step": round(per_step_ms, 4)}
        if roofs:
            dom = max(roofs, key=lambda k: roofs[k]["ms_per_step"])
            out["roofline"] = dict(roofs[dom], kernel=dom,
                                   note="algorithmic FLOPs per training step (bench_train.kernel_flops) / the "
                                        "kernel's time per training step")
            out["rooflines"] = roofs
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
