"""bench.py -- explained target-edges/s of the TempME explanation hot path on MI355X.

Metric (BASELINE.json): explained target-edges/sec (TGN+Enron, n_degree=20) at 1/2/4/8 MI355X.  One
unit = one target event with its fake destination, 2-hop subgraphs x3 sides, temporal walks x3 with
motif categories and edge counts, encoder forward x3 and retrieve_explanation (eval);
the base TGN's contrast is excluded.

Workload (default --config 2): the metric's own graph, full Enron (V=184 nodes, E=125,235 edges; the
graph of BASELINE configs[2]/[3]) + TGN explainer scoring at n_degree=20.  Enron is not available
offline, so the graph is a seeded synthetic replica of its shape (tempme_amd/workload.py: Pareto(1.2)
endpoints, ts in [0, 1e8), de=32, dn=172); explainer weights are a seeded random init of the TempME
architecture.  --config 1 = configs[1] (enron_sampled shape, E=18,780), --config 4 = configs[4]
(synthetic 1M-edge graph, de=dn=172, N=30, the HBM stress case).

A step = one pass of the hot path over one global batch of synthetic target events already resident
in HBM: --batches reference batches of --batch-size events (default 192 x 100 = 19,200 = one eval epoch
over the full-Enron test split), all on-device
(tm_sample_events -> tm_edge_tables -> tm_encoder_fwd_tab -> tm_edge_importance_tab).

Multi-GPU: `python bench.py --gpus N` starts its own N ranks (torch.distributed.run, one process per
GPU) when it is not already running under a launcher; the driver's `torch.distributed.run ... bench.py
--gpus N` works the same way.  Whole reference batches are sharded across ranks with no data-path
collective (the graph, tables and weights are replicated per GPU).  The primary line is STRONG scaling:
the global batch of one step is fixed and dealt over the ranks (192 / N batches each); the weak-scaling
figure (192 batches per rank) is reported beside it as "weak".  Barrier + synchronize bracket the timed
region and the time is the max over ranks.

Run:  python bench.py [--gpus N --steps K --warmup W --config {1,2,4}]
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "explained target-edges/sec (TGN+Enron, n_degree=20) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
FP32_MFMA_PEAK_TF = 157.3      # MI355X_MICROARCH.md: FP32 matrix (spec)

CONFIGS = {
    1: dict(name="enron_sampled", graph=dict(n_nodes=183, n_edges=18780), N=20,
            workload="configs[1]: enron_sampled-shaped synthetic graph (V=183, E=18,780, Pareto {alpha}) + TGN "
                     "explainer scoring, n_degree={N}"),
    2: dict(name="enron", graph=dict(n_nodes=184, n_edges=125235), N=20,
            workload="metric config: full Enron shape (V=184, E=125,235, Pareto {alpha}; the graph of configs[2]/[3]) "
                     "+ TGN explainer scoring, n_degree={N}"),
    4: dict(name="synth1m", graph=dict(n_nodes=100000, n_edges=1000000, alpha=1.5, de=172, dn=172,
                                       node_feat="uniform"), N=30,
            workload="configs[4]: synthetic 1M-edge temporal graph (V=100,000, Pareto 1.5, de=dn=172 U(0,1) "
                     "features), TempME explanation scoring, n_degree={N}"),
}


# ----------------------------------------------------------------------------------------------- launcher
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n):
    """Start n ranks of this script under torch.distributed.run as a CHILD process (nothing has touched the
    GPU yet in this process) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


# ----------------------------------------------------------------------------------------------- models
def flops_model(de, dn, h, N, M, etab=False, zn=False):
    """MACs x2 per unit for each encoder kernel.  ``walk_kernel``: the SURVEY.md §8(a) a12 model (3 walk
    positions + head), minus the 3 de x dn edge-feature MACs per walk that the edge table (``etab``) does once
    per edge id.  ``walk_kernel_executed``: what the kernel actually issues (folded form) --
    per walk position 0/1: lin_event, event_gcn's first layer on both branches, the folded attention.MLP.0
    product A1G (h x 2h) and the score dot (2h); per hop-1 slot (shared by its M walks): position 2's
    lin_event over the K steps below qt (the all-time-feature steps are a bias at dt = 0), event_gcn's
    first layer, the folded kv = G^T W1D (2h x 2h), A1D (h x 2h) and the u dot; per walk the head:
    MLP.0 folded with attention.MLP.3 (h+12 x h), MLP.3 (h x h+12) and the last row (h).  ``zn`` (zero node
    features, tm_weights_set_node_zero): event_gcn's first layer runs on one branch (the two are bit-identical)
    and the layers reading both branches (A1D, kv, u, A1G, the score dot) on their column-folded forms."""
    kev = de + 3 + dn
    per_pos_gcn = kev * dn + 2 * (dn * h + h * h)                       # lin_event + event_gcn MLP x2
    per_walk_head = 3 * (2 * h) ** 2 + (2 * h) * h + h * h + (h + 12) ** 2 + (h + 12) * h + h + 2 * 2 * h
    per_pos_gate = (de + dn) * h + h * (h // 2) + h // 2
    W = N * M
    qt = (de + 3 + 15) // 16
    edge = de * dn if etab else 0
    br = 1 if zn else 2           # event_gcn branches computed; the layers reading H take br * h inputs
    pos = kev * dn - edge + br * dn * h
    slot = kev * dn - max(kev - 16 * qt, 0) * dn - edge + br * dn * h + h * br * h + (br * h) ** 2 + br * h
    exec_walk = 2 * (2 * (pos + h * br * h + br * h) + slot / M + (h + 12) * h + h * (h + 12) + h)
    walk = 2 * (3 * per_pos_gcn + per_walk_head)
    if etab:
        walk -= 2 * 3 * de * dn
    return dict(walk_kernel=walk, walk_kernel_executed=exec_walk,
                gate_per_edge=2 * per_pos_gate + (2 * de * dn if etab else 0), W=W,
                per_walk=2 * (3 * per_pos_gcn + per_walk_head + 3 * per_pos_gate))


def sampling_bytes_per_event(N, M):
    """SURVEY.md §8(d) compulsory-traffic model for (a)+(b), per target event (3 sides)."""
    W = N * M
    khop = (N + N * N) * 16 + (N + N * N) * 12 + (1 + N) * 32
    walks = N * 128 + W * 188
    return 3 * (khop + walks)


def khop_bytes_per_event(N):
    """SURVEY.md §8(d) compulsory traffic of the k-hop kernel (a1-a4) alone, per target event (3 sides)."""
    return 3 * ((N + N * N) * 16 + (N + N * N) * 12 + (1 + N) * 32)


def load_traffic(cfg_name):
    """profiles/pmc_traffic_<config>.json (tools/pmc_summary.py --traffic): per-launch HBM bytes (FETCH_SIZE x 2
    + WRITE_SIZE, MI355X_MICROARCH.md §HBM) of every kernel instance of a PMC run of this config, and the
    instance the bench's timing name maps to (the one launched most often)."""
    p = os.path.join(HERE, "profiles", f"pmc_traffic_{cfg_name}.json")
    if not os.path.exists(p):
        return {}, None
    with open(p) as fh:
        d = json.load(fh)
    return d.get("by_bench_name", {}), os.path.relpath(p, HERE)


# ----------------------------------------------------------------------------------------------- legs
def aux_rows(finder, src, dst, ts, eidx, pool, graph_build_ms):
    """SURVEY §8 rows outside the per-step unit, timed once (not part of ``value``): a1 the CSR build
    (NeighborFinder.__init__) and a11 the null model's sampling and counting (utils/null_model.py
    pre_processing + statistic: 500 events, num_neighbors 30, one walk per slot)."""
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


def khop_alone(pipe, inputs, steps, N, group=8):
    """The (a) kernel measured alone (the >= 50 % HBM target applies to it): 2-hop
    sampling of ``group`` steps' events per launch, one tm_sample_khop launch per side -- src and dst on the
    e_idx path, the pipeline's fake dst on the time path -- serialised on one stream, each launch timed with
    HIP events on that stream, so every khop2_kernel duration is its own (a rocprofv3 kernel trace of the
    same run gives the same per-launch average: profiles/r03_*_kernel_stats.csv)."""
    from tempme_amd import _lib as L
    g = pipe.graph
    dev = inputs[0][0].device
    plans = []
    for k0 in range(0, steps * group, group):
        chunk = [inputs[(k0 + i) % len(inputs)] for i in range(group)]
        fakes = []
        for src, dst, ts, eidx, ev in chunk:
            pipe.sample(src, dst, ts, eidx, ev)      # fake dst of these events (not timed)
            fakes.append(pipe.buf.dst_fake[:src.numel()].clone())
        src, dst, ts, eidx, ev = [torch.cat([c[j] for c in chunk]) for j in range(5)]
        plans.append((ts, ev, ((L.SIDE_SRC, src, eidx), (L.SIDE_TGT, dst, eidx), (L.SIDE_BGD, torch.cat(fakes), None))))
    E = int(plans[0][0].numel())
    tot = E * (N + N * N)
    on, oe, ot = (torch.empty(tot, dtype=torch.int32, device=dev), torch.empty(tot, dtype=torch.int32, device=dev),
                  torch.empty(tot, dtype=torch.float32, device=dev))
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    main = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()
    ms = []
    for ts, ev, sides in plans + plans:                # first pass warms up, second is timed
        for side, root, ei in sides:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(main)
            L.check(L.lib().tm_sample_khop(g.handle, L.TmRng(pipe.seed, pipe.split, side), 2, N, E, L.ptr(root),
                                           L.ptr(ts), L.ptr(ei), L.ptr(ev), L.ptr(on), L.ptr(oe), L.ptr(ot),
                                           L.ptr(err), main.cuda_stream), "tm_sample_khop")
            b.record(main)
            ms.append((a, b))
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in ms[3 * len(plans):]]
    L.raise_device_error(int(err.item()), "khop_alone")
    per_launch_ms = sum(ms) / len(ms)
    bytes_per_root = khop_bytes_per_event(N) // 3
    ach = bytes_per_root * E / (per_launch_ms * 1e-3) / 1e9
    return {"kernel": "khop2_kernel (tm_sample_khop k=2), one launch per side, serialised", "roots_per_launch": E,
            "avg_ms": round(per_launch_ms, 4), "launches": len(ms), "bound": "hbm", "achieved": round(ach, 1),
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_root": bytes_per_root}


def dropin_leg(ex, pipe, inputs, B, N, budget_s=3.0):
    """The reference's eval_one_epoch call pattern through the drop-in surface (temp_exp_main.py:441-452):
    per batch ``get_item`` / ``get_item_edge``, TempME.forward x3 (outside no_grad, as the reference calls
    it), then retrieve_explanation(training=False); timed from the pack to device outputs.  The pack is the
    pipeline's own sample of one step's events (tempme_amd/pack.py), held two ways: the reference's host
    float64 arrays (``load_subgraph_margin(args, f)``, ``np.load`` edge counts) and the device pack
    (``load_subgraph_margin(args, f, device=...)``, ``load_edge``) -- ``value`` is the device pack's rate."""
    from tempme_amd import pack as P
    src, dst, ts, eidx, ev = inputs[0]
    dev = src.device
    pipe.sample(src, dst, ts, eidx, ev)
    _, cat_d, edge = P.buffers_to_arrays(pipe.buf, int(src.numel()))

    class A:
        n_degree = N
    cut = ts.cpu().numpy()
    n_b = int(src.numel()) // B

    def run(pk, ed, training=False):
        def one(b):
            idx = np.arange(b * B, (b + 1) * B)
            sg_s, sg_t, sg_b, w_s, w_t, w_b, _ = P.get_item(pk, idx)
            e_s, e_t, e_b = P.get_item_edge(ed, idx)
            i_s, i_t, i_b = ex(w_s, cut[idx], e_s), ex(w_t, cut[idx], e_t), ex(w_b, cut[idx], e_b)
            return ex.retrieve_explanation(sg_s, i_s, w_s, sg_t, i_t, w_t, sg_b, i_b, w_b, training=training)

        for b in range(min(n_b, 4)):
            one(b)
        torch.cuda.synchronize()
        done, t0 = 0, time.perf_counter()
        while True:
            one(done % n_b)
            done += 1
            if done % n_b == 0 or done >= 4 * n_b:
                torch.cuda.synchronize()
                if time.perf_counter() - t0 > budget_s or done >= 4 * n_b:
                    break
        el = time.perf_counter() - t0
        return {"value": round(done * B / el, 2), "batches": done, "ms_per_batch": round(el / done * 1e3, 3)}

    host = run(P.load_subgraph_margin(A(), cat_d), edge)
    dpk, ded = P.load_subgraph_margin(A(), cat_d, device=dev), P.load_edge(edge, dev)
    if os.environ.get("TEMPME_DROPIN_PROFILE"):        # host-side profile of the device-pack loop (stderr)
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        run(dpk, ded)
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(30)
    devp = run(dpk, ded)
    bern = run(dpk, ded, training=True)
    return {"value": devp["value"], "unit": "edges/s", "batch_size": B, "batches": devp["batches"],
            "ms_per_batch": devp["ms_per_batch"], "host_pack": host,
            "bern": dict(bern, what="the same calls with retrieve_explanation(training=True): the reference's default "
                                    "eval call (--if_bern defaults to True, temp_exp_main.py:46, :450-453), Beta rsample"),
            "what": "eval_one_epoch pattern: get_item / get_item_edge, TempME.forward x3 (grad enabled, eval mode), "
                    "retrieve_explanation(training=False) per reference batch; value = device pack "
                    "(load_subgraph_margin(..., device=)), host_pack = the reference's host float64 arrays"}


def _cpu_cores():
    """Cores this process may run on (= nproc), limited by a cgroup CPU quota when one is set."""
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    use = cores if quota is None else max(1, min(cores, int(quota)))
    return use, cores, quota


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(g, rows, events, pool, N, M, B, seed, sd, budget_s=4.0, max_batches=150, reps=3, gm_sd=None):
    """The oracle port (C sampler + torch-fp32 encoder) on the host cores, bounded samples: ``reps`` repeats on the
    process's CPU share (OpenMP and torch threads = the cgroup quota, at most the CPUs it may run on) -- ``value`` is
    their median, ``spread`` min / max -- and one single-thread repeat (the least sensitive to other tenants of the
    box's cores).  ``gm_sd`` (configs[4]): the GraphMixer contrast of every batch with its hop-1 explanation too
    (oracle/graphmixer_ref.py, 2 mixer layers), as the GPU line times it."""
    from oracle import encoder_ref as er
    from oracle import graphmixer_ref as gr
    from oracle import oracle as orc
    use, nproc, quota = _cpu_cores()
    threads = int(os.environ.get("TEMPME_CPU_THREADS", use))
    src, dst, ts, eidx = events
    og = orc.OracleGraph(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"])
    nf, ef = torch.from_numpy(g["n_feat"]), torch.from_numpy(g["e_feat"])

    def one(nthr):
        torch.set_num_threads(nthr)
        done, t0 = 0, time.perf_counter()
        while done < max_batches * B and time.perf_counter() - t0 < budget_s:
            sl = slice(done % len(src), done % len(src) + B)
            if sl.stop > len(src):
                sl = slice(0, B)
            o = orc.event_pipeline(og, seed, 1, N, M, src[sl], dst[sl], ts[sl], eidx[sl], np.arange(done, done + B),
                                   pool, nthr)
            with torch.no_grad():
                h1 = []
                for s in range(3):
                    imp = er.forward(sd, nf, ef, o["node6"][:, s], o["eid3"][:, s], o["ts3"][:, s], o["cat"][:, s],
                                     ts[sl], o["cnt"][:, s].astype(np.float64))
                    h1.append(er.edge_importance(sd, ef, imp, o["eid3"][:, s], o["ts3"][:, s],
                                                 [o["sub1_node"][:, s], o["sub2_node"][:, s]],
                                                 [o["sub1_eid"][:, s], o["sub2_eid"][:, s]])[0])
                if gm_sd is not None:
                    sg = [([o["sub1_node"][:, s]], [o["sub1_eid"][:, s]], [o["sub1_ts"][:, s].astype(np.float64)])
                          for s in range(3)]
                    gr.contrast(gm_sd, 2, src[sl], dst[sl], o["dst_fake"], ts[sl], *sg,
                                explain_weights=[torch.cat(h1).float()])
            done += B
        el = time.perf_counter() - t0
        return done / el, done, el

    one(threads)                                     # warm-up (allocations, page-ins), not reported
    runs = [one(threads) for _ in range(reps)]
    vals = sorted(r[0] for r in runs)
    single = one(1)
    torch.set_num_threads(threads)
    med = vals[len(vals) // 2]
    return {"value": round(med, 2), "unit": "edges/s", "cores": threads, "kind": "port", "nproc": nproc,
            "cgroup_cpu_quota": quota, "cpu_model": _cpu_model(), "repeats": reps,
            "spread": [round(vals[0], 2), round(vals[-1], 2)], "single_thread": round(single[0], 2),
            "sample": f"{reps} repeats (median reported) of up to {max_batches} reference batches of {B} target events or "
                      f"{budget_s:.0f} s each ({sum(r[1] for r in runs)} events in {sum(r[2] for r in runs):.1f} s) of "
                      f"the same workload: oracle/tempme_oracle.c sampling+motif ({threads} OpenMP threads) + "
                      f"oracle/encoder_ref.py torch-fp32 encoder+explanation ({threads} threads)"
                      + (" + oracle/graphmixer_ref.py GraphMixer contrast with the hop-1 explanation" if gm_sd is not None
                         else "") + f"; single_thread = one more repeat on 1 thread ({single[1]} events in "
                      f"{single[2]:.1f} s)"}


# ----------------------------------------------------------------------------------------------- timing
def timed(run_step, pipes, inputs, warmup, steps, dist, backend, dev, L):
    """W untimed warm-up steps, then EXACTLY K steps bracketed by barrier + synchronize; max over ranks."""
    from tempme_amd.sharding import max_over_ranks
    for k in range(warmup):
        run_step(inputs[k % len(inputs)])
    torch.cuda.synchronize()
    for p in pipes:
        p.check_errors()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    L.profile_enable(True)
    t0 = time.perf_counter()
    for k in range(warmup, warmup + steps):
        run_step(inputs[k % len(inputs)])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    prof = L.profile_read()
    L.profile_enable(False)
    for p in pipes:
        p.check_errors()
    return max_over_ranks(el, dist, dev if backend == "nccl" else "cpu"), prof


@torch.no_grad()
def gm_contrast(gm, buf, x, h1):
    """GraphMixer.contrast (GM/graphmixer.py:206-218) of every event of the step with its hop-1
    explanation: the three sides' roots at once (rows are independent, so one call equals the reference's
    per-batch calls), then the MergeLayer scores of (src, dst) and (src, fake)."""
    src, dst, ts, eidx, _ = x
    E = src.numel()
    N = buf.N
    roots = torch.cat([src, dst, buf.dst_fake[:E]])
    cut = ts.repeat(3)
    emb = gm.node_embeddings(roots, cut, buf.sub1_node[:, :E].reshape(3 * E, N), buf.sub1_eid[:, :E].reshape(3 * E, N),
                             buf.sub1_ts[:, :E].reshape(3 * E, N).double(), h1.reshape(3 * E, N))
    s, d, n = emb[:E], emb[E:2 * E], emb[2 * E:]
    return gm.affinity(torch.cat([s, s]), torch.cat([d, n]))


def make_inputs(n_steps, rank, world, per_rank, events, dev):
    from tempme_amd.sharding import shard_events
    src, dst, ts, eidx = events
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    out = []
    for k in range(n_steps):
        i, ev = shard_events(k, rank, world, per_rank, len(src))
        out.append((to(src[i], np.int32), to(dst[i], np.int32), to(ts[i], np.float64), to(eidx[i], np.int32),
                    to(ev.view(np.int32), np.int32)))
    return out


def kernel_table(prof, units, executed):
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
                ent.update(bound="mfma", credited_tflops=round(ach, 2), credited_frac=round(ach / FP32_MFMA_PEAK_TF, 4))
                if name in executed:
                    ex_tf = executed[name] / (avg_ms * 1e-3) / 1e12
                    ent.update(achieved=round(ex_tf, 2), unit="TFLOP/s", frac=round(ex_tf / FP32_MFMA_PEAK_TF, 4))
                else:
                    ent.update(achieved=round(ach, 2), unit="TFLOP/s", frac=round(ach / FP32_MFMA_PEAK_TF, 4))
        kernels[name] = ent
    return kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[i] graph: 2 = full Enron (the metric's config, default), "
                         "1 = enron_sampled, 4 = synthetic 1M-edge de=dn=172 N=30")
    ap.add_argument("--batches", type=int, default=192,
                    help="reference batches of --batch-size events per step (global; strong scaling splits them over "
                         "the ranks).  192 x 100 = 19,200 events = one eval epoch over the full-Enron test split "
                         "(15 %% of 125,235 edges), a multiple of 8 ranks")
    ap.add_argument("--batch-size", type=int, default=100, help="temp_exp_main --test_bs")
    ap.add_argument("--n-degree", type=int, default=None)
    ap.add_argument("--alpha", type=float, default=1.2)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the k-hop-alone, drop-in and aux legs")
    ap.add_argument("--weak", action="store_true", help="primary line weak scaling (--batches per rank)")
    ap.add_argument("--no-edge-table", action="store_true",
                    help="lin_event's edge-feature product per walk position instead of per edge id")
    ap.add_argument("--streams", type=int, default=0,
                    help="steps in flight (PipelinedExplainer); 0 = auto: 1 with one rank (the kernel-level roofline of "
                         "record: every launch alone on the chip; the N=1 line reports the 3-in-flight figure beside "
                         "it as 'pipelined'), 3 with overlapping walk kernels with several ranks (a rank's share of the "
                         "step is small there: 0.99 -> 0.93 ms per step at the 8-rank share, "
                         "profiles/r06_flight_ab.txt)")
    ap.add_argument("--overlap-walk", action="store_true",
                    help="with steps in flight, let one step's walk kernel start while the previous one's grid drains "
                         "(PipelinedExplainer(chain_encoders=False)) instead of chaining the encoders (auto with "
                         "--streams 0 and several ranks)")
    ap.add_argument("--no-node-zero", action="store_true",
                    help="do not specialise the walk kernel for an all-zero node-feature table (A/B)")
    ap.add_argument("--contrast", choices=("auto", "graphmixer", "none"), default="auto",
                    help="base-model contrast with the explanation (auto: GraphMixer for --config 4, as configs[4] "
                         "names it; none elsewhere: SURVEY §8(d) excludes the base contrast from the scoring unit)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, form the process group and report it (no GPU work)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    N = args.n_degree or cfg["N"]

    # ---- one process per GPU: start our own ranks unless a launcher already did (before any GPU call)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    # TEMPME_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks sharing the GPUs there are
    backend = os.environ.get("TEMPME_DIST_BACKEND", "nccl")
    dist = None
    if args.launch_check:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            t = torch.ones(1)
            dist.all_reduce(t)
            if rank == 0:
                print(json.dumps({"n_gpus": world, "ranks_in_group": int(t.item()), "backend": "gloo"}), flush=True)
            dist.destroy_process_group()
        else:
            print(json.dumps({"n_gpus": 1, "ranks_in_group": 1}), flush=True)
        return
    n_dev = torch.cuda.device_count()
    if backend == "nccl" and world > n_dev:
        raise SystemExit(f"bench.py: {world} ranks but {n_dev} GPUs visible")
    dev = torch.device("cuda", local % max(n_dev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import tempme_amd as tm
    from tempme_amd import _lib as L
    from tempme_amd.pipeline import ExplainPipeline, PipelinedExplainer
    from tempme_amd.workload import enron_like, split

    M, B = 3, args.batch_size
    gkw = dict(cfg["graph"])
    gkw.setdefault("alpha", args.alpha)
    g = enron_like(seed=args.seed, **gkw)
    workload = cfg["workload"].format(alpha=gkw["alpha"], N=N)
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
    ex = tm.TempME(Base(), "tgn", cfg["name"], out_dim=40, hid_dim=64, device=dev,
                   null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).eval()
    ex.node_zero_specialization = not args.no_node_zero
    rank_batches = args.batches if args.weak else args.batches // max(1, world)
    S = args.streams if args.streams > 0 else (1 if world == 1 else 3)
    overlap = S > 1 and (args.overlap_walk or args.streams == 0)
    contrast = args.contrast if args.contrast != "auto" else ("graphmixer" if args.config == 4 else "none")
    gm = None
    if contrast == "graphmixer":
        # configs[4]'s base model, random-init (no checkpoint travels), scoring the explanation
        from tempme_amd.graphmixer import GraphMixer
        torch.manual_seed(args.seed + 1)
        gm = GraphMixer(g["n_feat"], g["e_feat"], n_neighbors=N, device=dev, num_tokens=N, num_layers=2,
                        dropout=0.1).to(dev).eval()
        workload += " + GraphMixer contrast with the hop-1 explanation (fused HIP embedding)"
    if S == 1:
        pipe = ExplainPipeline(ex, finder.graph, torch.from_numpy(pool), N, M, B, seed=args.seed,
                               edge_table=not args.no_edge_table)
        pipes = [pipe]

        def run_step(x):
            _, h1, _ = pipe.run(*x)
            if gm is not None:
                gm_contrast(gm, pipe.buf, x, h1)
    else:
        flight = PipelinedExplainer(ex, finder.graph, torch.from_numpy(pool), N, M, B, seed=args.seed, depth=S,
                                    edge_table=not args.no_edge_table, chain_encoders=not overlap)
        pipes = flight.pipes
        pipe = pipes[0]

        def run_step(x):
            flight.submit(*x)

    n_steps = args.warmup + args.steps
    strong = not args.weak
    # distinct devices the ranks run on (a gloo rehearsal puts several ranks on one GPU): n_gpus counts
    # devices, "ranks" the processes
    if world > 1:
        devs = [None] * world
        dist.all_gather_object(devs, dev.index)
        n_gpus = len(set(devs))
    else:
        n_gpus = 1
    if strong and args.batches % world:
        raise SystemExit(f"bench.py: --batches {args.batches} is not divisible by the {world} ranks")
    per_rank = (args.batches // world if strong else args.batches) * B
    inputs = make_inputs(n_steps, rank, world, per_rank, (src, dst, ts, eidx), dev)
    for k in range(S):                             # every stream's buffers allocated before timing
        run_step(inputs[k % n_steps])
    builds0 = pipe.tabs.builds
    el, prof = timed(run_step, pipes, inputs, args.warmup, args.steps, dist, backend, dev, L)
    tab_builds = pipe.tabs.builds - builds0
    weak = None
    if world > 1:
        # the secondary figure: the other scaling mode on the same ranks
        per_rank2 = (args.batches if strong else args.batches // world) * B
        inputs2 = make_inputs(n_steps, rank, world, per_rank2, (src, dst, ts, eidx), dev)
        run_step(inputs2[0])
        el2, _ = timed(run_step, pipes, inputs2, args.warmup, args.steps, dist, backend, dev, L)
        weak = {"scaling": "weak" if strong else "strong", "value": round(world * args.steps * per_rank2 / el2, 2),
                "ms_per_step": round(el2 / args.steps * 1e3, 3), "events_per_step_per_gpu": per_rank2}
    pipelined = None
    if world == 1 and S == 1 and not args.no_extras and gm is None:
        # like-for-like with the multi-rank lines: the same step with 3 steps in flight and overlapping walk kernels
        fl3 = PipelinedExplainer(ex, finder.graph, torch.from_numpy(pool), N, M, B, seed=args.seed, depth=3,
                                 edge_table=not args.no_edge_table, chain_encoders=False)
        for k in range(3):
            fl3.submit(*inputs[k % n_steps])
        el3, _ = timed(lambda x: fl3.submit(*x), fl3.pipes, inputs, args.warmup, args.steps, dist, backend, dev, L)
        pipelined = {"value": round(args.steps * per_rank / el3, 2), "ms_per_step": round(el3 / args.steps * 1e3, 3),
                     "steps_in_flight": 3, "walk_overlap": True,
                     "what": "the same timed steps with 3 steps in flight, consecutive walk kernels overlapping (the "
                             "multi-rank lines' mode); per-launch kernel durations then include the sharing, so the "
                             "kernel roofline of record is the serial line's"}
        del fl3

    if rank == 0:
        E = per_rank
        zn = bool(getattr(ex, "_node_zero", False)) and ex.node_zero_specialization and pipe.etab is not None
        fm = flops_model(g["e_feat"].shape[1], g["n_feat"].shape[1], 64, N, M, etab=pipe.etab is not None, zn=zn)
        W = fm["W"]
        units = {"events_kernel": ("hbm", sampling_bytes_per_event(N, M) * E),
                 "gate_table_kernel": ("mfma", fm["gate_per_edge"] * (int(g["eidx"].max()) + 1)),
                 "walk_kernel": ("mfma", fm["walk_kernel"] * 3 * E * W)}
        executed = {"walk_kernel": fm["walk_kernel_executed"] * 3 * E * W}
        if gm is not None:
            # per row: projection N (C+T) C + per mixer channel FFN 2 N C HC + token FFN 2 N HT C MACs
            C_, T_, HT_, HC_ = gm.num_channels, gm.time_feat_dim, int(0.5 * N), int(4 * gm.num_channels)
            per_row = 2 * (N * (C_ + T_) * C_ + gm.num_layers * (2 * N * C_ * HC_ + 2 * N * HT_ * C_))
            units["gm_embed_kernel"] = ("mfma", per_row * 3 * E)   # LDS-tiled form (dims outside tm_gm_fused_ok)
            units["gm_fused_kernel"] = ("mfma", per_row * 3 * E)   # register-resident form
        kernels = kernel_table(prof, units, executed)
        traffic, tsrc = load_traffic(cfg["name"])
        dom = max((k for k in kernels if "bound" in kernels[k]), key=lambda k: kernels[k]["avg_ms"])
        d = kernels[dom]
        roof = {"bound": d["bound"], "achieved": d["achieved"],
                "peak": HBM_PEAK_GBS if d["bound"] == "hbm" else FP32_MFMA_PEAK_TF, "unit": d["unit"],
                "frac": d["frac"], "traffic": traffic.get(dom), "kernel": dom}
        if dom in executed:
            roof["credited_frac"] = d["credited_frac"]
            roof["note"] = ("achieved/frac = FLOPs the kernel executes (position 2 once per hop-1 slot, time-only "
                            "K steps folded, edge-feature product in the edge table); credited_frac = the SURVEY "
                            "§8(d) per-walk model minus the edge-table MACs, for the same launch time")
        if tsrc:
            roof["traffic_source"] = tsrc
        if overlap and dom in executed:
            # consecutive steps' walk kernels overlap: a launch's duration includes the sharing, so credit the kernel
            # with the whole step time instead (a lower bound on its rate)
            ach = executed[dom] / (el / args.steps) / 1e12
            roof.update(achieved=round(ach, 2), frac=round(ach / FP32_MFMA_PEAK_TF, 4),
                        credited_frac=round(units[dom][1] / (el / args.steps) / 1e12 / FP32_MFMA_PEAK_TF, 4),
                        basis="the step time (walk kernels of consecutive steps overlap, so per-launch durations "
                              "include the sharing): a lower bound on the kernel's rate")
        samp = dict(kernels.get("events_kernel", {}))
        if samp and traffic.get("events_kernel") is not None:
            samp["traffic"] = traffic["events_kernel"]
        # the per-edge-id tables (gate factor + lin_event's edge product over all edge ids) are a function of the
        # weight state, the edge-feature table and the graph: built once (EdgeTables), timed here alone
        pipe.tabs.build(timed=True)
        edge_tables = {"ms": round(pipe.tabs.build_ms, 3), "edge_ids": int(pipe.gf.numel()),
                       "builds_in_timed_region": tab_builds,
                       "what": "tm_edge_tables (gate_reg_kernel) over every edge id: built once per weight state "
                               "(tm_weights_version), edge-feature table and graph, outside the per-step unit; the "
                               "reference recomputes the gate per walk position (same values)"}
        total = world * args.steps * per_rank
        out = {"metric": METRIC, "value": round(total / el, 2), "unit": "edges/s", "n_gpus": n_gpus, "ranks": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
               "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
               "dtype": "fp32",
               "data": "synthetic (seeded graph of the config's shape, random-init TempME weights)",
               "config": {"workload": workload, "config": f"configs[{args.config}]" if args.config != 2 else
                          "metric (full Enron + TGN, n_degree=20)", "n_degree": N, "walks_per_slot": M,
                          "batch_size": B, "global_batches_per_step": per_rank * world // B,
                          "events_per_step_per_gpu": per_rank, "parallelism": f"dp{world} (whole batches per rank)",
                          "steps_in_flight": S, "walk_overlap": overlap, "base_contrast": contrast,
                          "edge_tables": "per weight state (see edge_tables), not per step",
                          "walk_kernel_zero_node_features": zn},
               "roofline": roof, "kernels": kernels, "sampling_roofline": samp or None, "edge_tables": edge_tables}
        if weak is not None:
            out["weak" if strong else "strong"] = weak
        if pipelined is not None:
            out["pipelined"] = pipelined
        if not args.no_extras:
            out["khop_roofline"] = khop_alone(pipe, inputs, min(args.steps, 5), N, group=8)
            out["dropin"] = dropin_leg(ex, pipe, inputs, B, N)
            out["aux"] = aux_rows(finder, src, dst, ts, eidx, pool, graph_build_ms)
        if world == 1 and not args.no_cpu_baseline:
            sd = {k: v.detach().cpu() for k, v in ex.state_dict().items()}
            gm_sd = None if gm is None else {k: v.detach().cpu() for k, v in gm.state_dict().items()}
            out["cpu_baseline"] = cpu_baseline(g, rows, (src, dst, ts, eidx), pool, N, M, B, args.seed, sd, gm_sd=gm_sd)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
