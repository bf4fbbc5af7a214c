"""N>1 path on CPU (gloo, world_size 2): event sharding, keyed-RNG shard independence, max-over-ranks.

The GPU path shards exactly like this (bench.py --gpus N); here the per-rank work is the oracle's
event pipeline (test infrastructure), which follows the same RNG contract as the HIP kernels."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tempme_amd.sharding import max_over_ranks, shard_events


def test_shards_disjoint_and_contiguous():
    for world in (1, 2, 4, 8):
        per, n = 7, 23
        for step in range(3):
            ids = np.concatenate([shard_events(step, r, world, per, n)[1] for r in range(world)]).astype(np.int64)
            first = step * world * per
            assert np.array_equal(ids, np.arange(first, first + world * per))
            rows = np.concatenate([shard_events(step, r, world, per, n)[0] for r in range(world)])
            assert np.array_equal(rows, ids % n)


def test_shard_events_rejects_bad_args():
    with pytest.raises(ValueError):
        shard_events(0, 2, 2, 4, 10)
    with pytest.raises(ValueError):
        shard_events(0, 0, 1, 4, 0)


def test_max_over_ranks_without_group():
    assert max_over_ranks(3.5) == 3.5


def _graph():
    rng = np.random.default_rng(7)
    V, E = 40, 600
    src = rng.integers(1, V, E)
    dst = rng.integers(1, V, E)
    ts = np.sort(rng.integers(0, 400, E)).astype(np.float64)
    eidx = np.arange(1, E + 1)
    return V, src, dst, ts, eidx


def _run_events(rows, ev, N=4, M=2):
    from oracle import oracle as O
    V, src, dst, ts, eidx = _graph()
    cut = len(src) * 3 // 4
    g = O.OracleGraph(src, dst, eidx, ts, V)   # events' own edges are in the graph (temp_exp_main.py)
    test = slice(cut, None)
    s, d, t, e = src[test][rows], dst[test][rows], ts[test][rows], eidx[test][rows]
    o = O.event_pipeline(g, 11, 1, N, M, s, d, t, e, ev, np.unique(dst), n_threads=1)
    return {k: v for k, v in o.items() if k != "hist"}


def _worker(rank, world, port, per, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _work(rank, world, per, steps, q)
    except Exception as exc:  # surface the failure instead of a queue timeout
        q.put(repr(exc))
        raise
    finally:
        dist.destroy_process_group()


def _work(rank, world, per, steps, q):
    n_test = len(_graph()[1]) - len(_graph()[1]) * 3 // 4
    outs = []
    for step in range(steps):
        rows, ev = shard_events(step, rank, world, per, n_test)
        outs.append(_run_events(rows, ev))
    dist.barrier()
    el = max_over_ranks(1.0 + rank, dist)          # per-rank "elapsed" -> max over ranks
    gathered = [None] * world
    dist.all_gather_object(gathered, outs)
    if rank == 0:
        q.put((el, gathered))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gloo_two_ranks_match_single_process():
    world, per, steps = 2, 6, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    assert not isinstance(res, str), res
    el, gathered = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert el == 2.0
    n_test = len(_graph()[1]) - len(_graph()[1]) * 3 // 4
    for step in range(steps):
        # one process over the step's whole block of events == the ranks' shards, concatenated
        rows = np.arange(step * world * per, (step + 1) * world * per)
        full = _run_events(rows % n_test, rows.astype(np.uint32))
        for k, v in full.items():
            got = np.concatenate([gathered[r][step][k] for r in range(world)])
            assert np.array_equal(got, v), k


# ------------------------------------------------------------------ explainer gradient all-reduce (a15)
def test_epoch_spans_deal_whole_batches():
    from tempme_amd.train import epoch_spans
    one = epoch_spans(1000, 100)
    assert one[0] == (0, 100) and one[-1] == (900, 999)          # temp_exp_main.py:584-590 bounds
    for world in (2, 4, 8):
        per = [epoch_spans(1000, 100, r, world) for r in range(world)]
        assert len({len(p) for p in per}) == 1                     # same number of all-reduced steps
        got = sorted(sp for p in per for sp in p)
        assert got == one[:len(one) - len(one) % world]


def _grad_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tempme_amd.train import GradAllReduce
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ReLU(), torch.nn.Linear(7, 1),
                                  torch.nn.Linear(3, 3))                  # last layer gets no gradient
        opt = torch.optim.Adam(net.parameters(), lr=1e-2)
        sync = GradAllReduce(net)
        for step in range(3):
            x = torch.randn(4, 5, generator=torch.Generator().manual_seed(100 * step + rank))
            opt.zero_grad()
            net[2](net[1](net[0](x))).pow(2).mean().backward()
            local = [p.grad.clone() if p.grad is not None else None for p in net.parameters()]
            sync()
            synced = [p.grad.clone() if p.grad is not None else None for p in net.parameters()]
            opt.step()
            gl = [None] * world
            dist.all_gather_object(gl, local)
            if rank == 0:
                for i, s in enumerate(synced):
                    if s is None:
                        assert all(g[i] is None for g in gl)
                        continue
                    torch.testing.assert_close(s, sum(g[i] for g in gl) / world)
        params = [None] * world
        dist.all_gather_object(params, [p.detach().clone() for p in net.parameters()])
        if rank == 0:
            for a, b in zip(params[0], params[1]):
                assert torch.equal(a, b)                                  # replicas stay identical
            q.put("ok")
    except Exception as exc:
        q.put(repr(exc))
        raise
    finally:
        dist.destroy_process_group()


def test_grad_all_reduce_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert res == "ok", res
    assert all(p.exitcode == 0 for p in procs)


def _flat_grad_worker(rank, world, port, q):
    """GradAllReduce(flat_grad=...): every gradient a view of one bucket (optim.FusedAdam's layout), the all-reduce
    on the bucket in place; the averages equal the per-parameter path's."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tempme_amd.train import GradAllReduce
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ReLU(), torch.nn.Linear(7, 1))
        n = sum(p.numel() for p in net.parameters())
        flat = torch.zeros(n)
        off = 0
        for p in net.parameters():
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        class Bucket:                                     # optim.FusedAdam's interface: the gradients already bound
            flat_grad = flat

            @staticmethod
            def sync_grads():
                return []
        sync = GradAllReduce(net, bucket=Bucket())
        for step in range(3):
            x = torch.randn(4, 5, generator=torch.Generator().manual_seed(100 * step + rank))
            flat.zero_()
            net[2](net[1](net[0](x))).pow(2).mean().backward()
            local = flat.clone()
            sync.start()
            sync.finish()
            gl = [None] * world
            dist.all_gather_object(gl, local)
            if rank == 0:
                torch.testing.assert_close(flat, sum(gl) / world)
                off = 0
                for p in net.parameters():                 # the .grad views see the averages
                    assert p.grad.data_ptr() == flat[off:].data_ptr()
                    off += p.numel()
        if rank == 0:
            q.put("ok")
        dist.barrier()
    except Exception as exc:
        q.put(repr(exc))
        raise
    finally:
        dist.destroy_process_group()


def test_grad_all_reduce_flat_bucket_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_flat_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert res == "ok", res
    assert all(p.exitcode == 0 for p in procs)


def _bench_env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    return env


def test_bench_self_launches_ranks():
    """`python bench.py --gpus 2` with no launcher starts its own 2 ranks (torch.distributed.run child) and
    forms a world-2 process group (gloo here: --launch-check does no GPU work)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=240, env=_bench_env(), cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["ranks_in_group"] == 2


def test_bench_rejects_world_mismatch():
    """Under a launcher that started a different number of ranks than --gpus, bench.py refuses to run."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = _bench_env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=repo)
    assert r.returncode != 0 and "--gpus 2" in r.stderr


def _overlap_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tempme_amd.train import GradAllReduce
        nets, opts, syncs = [], [], []
        for _ in range(2):
            torch.manual_seed(0)
            net = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ReLU(), torch.nn.Linear(7, 1))
            nets.append(net)
            opts.append(torch.optim.Adam(net.parameters(), lr=1e-2))
            syncs.append(GradAllReduce(net))
        side = []
        for step in range(4):
            x = torch.randn(4, 5, generator=torch.Generator().manual_seed(100 * step + rank))
            for i, (net, opt, sync) in enumerate(zip(nets, opts, syncs)):
                opt.zero_grad()
                net(x).pow(2).mean().backward()
                if i == 0:
                    sync()                                   # serial: all-reduce, then the optimizer
                else:
                    sync.start()                             # overlapped: the next batch's independent work
                    side.append(torch.randn(64, 64).matmul(torch.randn(64, 64)).sum())   # runs in flight
                    sync.finish()
                opt.step()
        for a, b in zip(nets[0].parameters(), nets[1].parameters()):
            assert torch.equal(a, b)
        got = [None] * world
        dist.all_gather_object(got, [p.detach().clone() for p in nets[1].parameters()])
        if rank == 0:
            for a, b in zip(got[0], got[1]):
                assert torch.equal(a, b)                     # replicas identical
            q.put("ok")
    except Exception as exc:
        q.put(repr(exc))
        raise
    finally:
        dist.destroy_process_group()


def test_overlapped_all_reduce_equals_serial():
    """GradAllReduce.start()/finish() with other work in between (train.run_steps overlaps the next
    batch's prepare_step with the collective) gives exactly the serial step's gradients and updates."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert res == "ok", res
    assert all(p.exitcode == 0 for p in procs)


def _run_steps_worker(rank, world, port, q):
    """train.run_steps with a GradAllReduce over gloo (the orchestration: each batch fetched once, batch
    k+1's prepare_step issued while batch k's all-reduce is in flight) against the serial loop.  The
    step body is a CPU stand-in with train_step's structure (the real one needs the HIP library; its
    multi-rank run on the device is tests/test_gpu_multi_rank.py)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import tempme_amd.train as T

        def prepare_step(base, batch):
            return ("prepared", batch["i"])

        def train_step(ex, base, opt, batch, *, grad_sync=None, prepared=None, overlap=None, **kw):
            assert prepared == ("prepared", batch["i"]), (prepared, batch["i"])
            opt.zero_grad()
            ex(batch["x"]).pow(2).mean().backward()
            grad_sync.start()
            if overlap is not None:
                overlap()
            grad_sync.finish()
            opt.step()
            return batch["i"]

        T.prepare_step, T.train_step = prepare_step, train_step

        class Lazy:
            def __init__(self):
                self.fetched = []

            def __len__(self):
                return 5

            def __getitem__(self, k):
                self.fetched.append(k)
                return {"i": k, "x": torch.randn(6, 5, generator=torch.Generator().manual_seed(10 * k + rank))}

        nets = []
        for mode in ("serial", "run_steps"):
            torch.manual_seed(0)
            net = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ReLU(), torch.nn.Linear(7, 1))
            opt = torch.optim.Adam(net.parameters(), lr=1e-2)
            sync = T.GradAllReduce(net)
            lazy = Lazy()
            if mode == "serial":
                for k in range(len(lazy)):
                    b = lazy[k]
                    train_step(net, None, opt, b, grad_sync=sync, prepared=prepare_step(None, b))
            else:
                outs = T.run_steps(net, None, opt, lazy, grad_sync=sync, overlap=True)
                assert outs == list(range(5))
            assert lazy.fetched == list(range(5)), lazy.fetched      # each batch gathered once, in order
            nets.append(net)
        for a, b in zip(nets[0].parameters(), nets[1].parameters()):
            assert torch.equal(a, b)
        got = [None] * world
        dist.all_gather_object(got, [p.detach().clone() for p in nets[1].parameters()])
        if rank == 0:
            for a, b in zip(got[0], got[1]):
                assert torch.equal(a, b)
            q.put("ok")
    except Exception as exc:
        q.put(repr(exc))
        raise
    finally:
        dist.destroy_process_group()


def test_run_steps_grad_all_reduce_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run_steps_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert res == "ok", res
    assert all(p.exitcode == 0 for p in procs)
