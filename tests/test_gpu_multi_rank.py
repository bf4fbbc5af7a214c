"""N>1 on the HIP path: two spawned ranks on cuda:0 (gloo; RCCL does not run two ranks on one device).

* Sharded scoring: each rank runs ExplainPipeline over its shard of whole reference batches
  (sharding.shard_events, bench.py's split); the shards, concatenated, equal one process over the whole
  block bit for bit -- whole-batch sharding keeps the batch-global attention std
  (models/explainer_new.py:826-836) inside one rank, and every draw is keyed by the global event id.
* Gradient all-reduce: each rank takes the training step (temp_exp_main.py:605-632) on its own batch;
  GradAllReduce over the device gradient buffers equals the average of the ranks' local gradients, which
  equals one process's average of the two batches' gradients, and the replicas stay identical through
  run_steps (the all-reduce overlapped with the next batch's preparation).

The processes are spawned (no fork or exec after the parent touched the GPU; the parent never does)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(target):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    assert res == "ok", res
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


# ------------------------------------------------------------------ sharded scoring
def _scoring_setup(dev):
    import tempme_amd as tm
    from tempme_amd.pipeline import ExplainPipeline
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=60, n_edges=4000, node_feat="uniform", seed=3)
    (src, dst, ts, eidx), rows, pool = split(g)
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=1)

    class Base:
        n_feat_th = torch.from_numpy(g["n_feat"])
        e_feat_th = torch.from_numpy(g["e_feat"])
        node_raw_features = torch.nn.Embedding.from_pretrained(n_feat_th, padding_idx=0, freeze=True)
        edge_raw_features = torch.nn.Embedding.from_pretrained(e_feat_th, padding_idx=0, freeze=True)

    torch.manual_seed(0)
    ex = tm.TempME(Base(), "tgn", "enron_sampled", 40, 64, device=dev,
                   null_model={k: 1 / 12 for k in range(1, 13)}).to(dev).eval()
    return (src, dst, ts, eidx), ex, f, pool, ExplainPipeline


def _score(ex, f, pool, Pipe, events, rows, ev, N, B, dev):
    src, dst, ts, eidx = events
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[rows], dtype=dt)).to(dev)  # noqa: E731
    pipe = Pipe(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=1)
    with torch.no_grad():
        imp, h1, h2 = pipe.run(t(src, np.int32), t(dst, np.int32), t(ts, np.float64), t(eidx, np.int32),
                               torch.from_numpy(ev.astype(np.int32)).to(dev))
    torch.cuda.synchronize()
    pipe.check_errors()
    return [x.cpu().numpy() for x in (imp, h1, h2, pipe.buf.eid3, pipe.buf.sub2_node)]


def _scoring_worker(rank, world, port, q):
    try:
        dev = _init(rank, world, port)
        from tempme_amd.sharding import shard_events
        events, ex, f, pool, Pipe = _scoring_setup(dev)
        N, B, per = 10, 16, 3 * 16                     # three whole batches per rank
        n = len(events[0])
        mine = []
        for step in range(2):
            rows, ev = shard_events(step, rank, world, per, n)
            mine.append(_score(ex, f, pool, Pipe, events, rows, ev, N, B, dev))
        got = [None] * world
        dist.all_gather_object(got, mine)
        if rank == 0:
            for step in range(2):
                # one process over the step's whole block (both ranks' events, in rank order)
                rows, ev = shard_events(step, 0, 1, world * per, n)
                full = _score(ex, f, pool, Pipe, events, rows, ev, N, B, dev)
                for k, name in enumerate(("imp", "hop1", "hop2", "eid3", "sub2_node")):
                    cat = np.concatenate([got[r][step][k] for r in range(world)], axis=1)   # side-major [3, E, ...]
                    assert np.array_equal(cat, full[k]), (step, name)
            q.put("ok")
        dist.barrier()
    except Exception as exc:
        q.put(repr(exc))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_sharded_pipeline_equals_single_process():
    _spawn(_scoring_worker)


# ------------------------------------------------------------------ gradient all-reduce on device buffers
def _train_setup(dev):
    import tempme_amd as tm
    from tempme_amd.preprocess import sample_events
    from tempme_amd.tgn import TGN
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=80, n_edges=3000, seed=4)
    (src, dst, ts, eidx), rows, pool = split(g, mode="train")
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=2, split=tm.SPLIT_TRAIN)
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    ev = (to(src, np.int32), to(dst, np.int32), to(ts, np.float64), to(eidx, np.int32))
    buf = sample_events(f.graph, 2, tm.SPLIT_TRAIN, 10, 3, *ev, torch.arange(len(src), dtype=torch.int32, device=dev),
                        to(pool, np.int32))
    torch.manual_seed(3)
    base = TGN(g["n_feat"], g["e_feat"], n_neighbors=10, device=dev, n_layers=2, n_heads=2, dropout=0.1)
    base.forbidden_memory_update = True
    base = base.to(dev).eval()

    def explainer():
        torch.manual_seed(5)
        return tm.TempME(base, "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
                         null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).eval()
    return buf, ev, base, explainer


def _grads(ex):
    return [p.grad.detach().clone() if p.grad is not None else None for p in ex.parameters()]


def _train_worker(rank, world, port, q):
    try:
        dev = _init(rank, world, port)
        from tempme_amd.train import GradAllReduce, batch_from_pack, run_steps, train_step
        buf, ev, base, explainer = _train_setup(dev)
        B = 40
        batch = lambda k: batch_from_pack(buf, *ev, torch.arange(k * B, (k + 1) * B, device=dev))  # noqa: E731

        class Rec(GradAllReduce):                       # local gradients before, averaged after the collective
            def start(self):
                self.local = _grads(self.module)
                super().start()

            def finish(self):
                super().finish()
                self.synced = _grads(self.module)

        # one step per rank on its own batch (rank r: batch r), deterministic configuration
        ex = explainer()
        opt = torch.optim.Adam(ex.parameters(), lr=1e-3)
        sync = Rec(ex)
        train_step(ex, base, opt, batch(rank), if_bern=False, grad_sync=sync)
        assert any(g is not None and g.is_cuda for g in sync.synced)
        local = [None] * world
        dist.all_gather_object(local, [None if g is None else g.cpu() for g in sync.local])
        synced = [None if g is None else g.cpu() for g in sync.synced]
        # three more steps through run_steps (the all-reduce overlapped with the next batch's preparation)
        run_steps(ex, base, opt, [batch(world * (k + 1) + rank) for k in range(3)], grad_sync=GradAllReduce(ex),
                  overlap=True, if_bern=False)
        params = [None] * world
        dist.all_gather_object(params, [p.detach().cpu() for p in ex.parameters()])
        if rank == 0:
            for i, s in enumerate(synced):
                if s is None:
                    assert all(lg[i] is None for lg in local)
                    continue
                torch.testing.assert_close(s, sum(lg[i] for lg in local) / world, rtol=1e-6, atol=1e-9)
            # = one process's average of the two batches' gradients from the same parameters
            ex1 = explainer()

            class NoStep:                               # train_step without the optimizer step
                def zero_grad(self):
                    ex1.zero_grad()

                def step(self):
                    pass
            ref = []
            for k in range(world):
                train_step(ex1, base, NoStep(), batch(k), if_bern=False)
                ref.append(_grads(ex1))
            for i, s in enumerate(synced):
                if s is None:
                    continue
                avg = sum(r[i] for r in ref).cpu() / world
                assert float((s - avg).norm()) <= 1e-5 * float(avg.norm()) + 1e-9, i
            for a, b in zip(params[0], params[1]):
                assert torch.equal(a, b)                # replicas identical after the all-reduced steps
            q.put("ok")
        dist.barrier()
    except Exception as exc:
        q.put(repr(exc))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_grad_all_reduce_on_device_equals_average():
    _spawn(_train_worker)
