"""The data-parallel eval loop on the device (tempme_amd/evaluate.py, temp_exp_main.py:410-544 with
threshold_test :153-272) and the RCCL backend path.

* world 1: every batch's figures from ``eval_batch`` equal the reference loop body written with the
  drop-in calls (TempME.forward x3, retrieve_explanation, contrast, kl_loss, sklearn, threshold_test).
* world 2 (two spawned gloo ranks on cuda:0): the sharded epoch's figures equal one process's, with
  threshold_test and with the Beta rsample (``if_bern``) reseeded per batch.
* RCCL: a world-1 ``nccl`` group on cuda:0 runs GradAllReduce's collective (force=True) inside a
  training step and the eval gather over device tensors."""
import math
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _args(**kw):
    a = dict(test_bs=40, if_bern=False, beta=0.5, prior_p=0.3, test_threshold=True, base_type="tgn", n_degree=10,
             ratios=[0.01, 0.05, 0.1, 0.2, 0.3])
    a.update(kw)
    return SimpleNamespace(**a)


def _setup(dev):
    import tempme_amd as tm
    from tempme_amd.preprocess import sample_events
    from tempme_amd.tgn import TGN
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=80, n_edges=3000, seed=4, node_feat="uniform")
    (src, dst, ts, eidx), rows, pool = split(g)
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=2)
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    ev = (to(src, np.int32), to(dst, np.int32), to(ts, np.float64), to(eidx, np.int32))
    buf = sample_events(f.graph, 2, tm.SPLIT_TEST, 10, 3, *ev, torch.arange(len(src), dtype=torch.int32, device=dev),
                        to(pool, np.int32))
    torch.manual_seed(3)
    base = TGN(g["n_feat"], g["e_feat"], n_neighbors=10, device=dev, n_layers=2, n_heads=2, dropout=0.1)
    base.forbidden_memory_update = True
    base = base.to(dev).eval()
    torch.manual_seed(5)
    ex = tm.TempME(base, "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
                   null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).eval()
    return buf, ev, base, ex


def _reference_batch(args, base, ex, b):
    """temp_exp_main.py:440-494 written with the drop-in calls, on the batch's device views."""
    from sklearn.metrics import average_precision_score, roc_auc_score

    from tempme_amd import fidelity
    sg_s, sg_t, sg_b = b.subgraphs
    w_s, w_t, w_b = b.walks
    e_s, e_t, e_b = b.edges
    criterion = torch.nn.BCEWithLogitsLoss()
    with torch.no_grad():
        pos_out_ori, neg_out_ori = base.contrast(b.src, b.dst, b.fake, b.ts, b.e_idx, sg_s, sg_t, sg_b)
        y_pred = torch.cat([pos_out_ori, neg_out_ori], dim=0).sigmoid()
        y_ori = torch.where(y_pred > 0.5, 1., 0.).view(y_pred.size(0), 1)
    ex.eval()
    g_s, g_t, g_b = ex(w_s, b.ts, e_s), ex(w_t, b.ts, e_t), ex(w_b, b.ts, e_b)
    expl = ex.retrieve_explanation(sg_s, g_s, w_s, sg_t, g_t, w_t, sg_b, g_b, w_b, training=args.if_bern)
    pos_logit, neg_logit = base.contrast(b.src, b.dst, b.fake, b.ts, b.e_idx, sg_s, sg_t, sg_b, explain_weights=expl)
    pred = torch.cat([pos_logit, neg_logit], dim=0)
    pred_loss = criterion(pred, y_ori)
    kl = (ex.kl_loss(g_s, w_s, target=args.prior_p) + ex.kl_loss(g_t, w_t, target=args.prior_p)
          + ex.kl_loss(g_b, w_b, target=args.prior_p))
    loss = pred_loss + args.beta * kl
    with torch.no_grad():
        y_pred = pred.sigmoid()
        pred_label = torch.where(y_pred > 0.5, 1., 0.).view(y_pred.size(0), 1)
        fp = torch.cat([pos_logit.sigmoid() - pos_out_ori.sigmoid(), neg_out_ori.sigmoid() - neg_logit.sigmoid()]).mean(0)
        fl = torch.cat([pos_logit - pos_out_ori, neg_out_ori - neg_logit]).mean(0)
        row = [average_precision_score(y_ori.cpu(), y_pred.cpu()), roc_auc_score(y_ori.cpu(), y_pred.cpu()),
               float((pred_label.cpu() == y_ori.cpu()).float().mean()), fp.item(), fl.item(), loss.item(),
               pred_loss.item(), kl.item()]
        expl0 = ex.retrieve_explanation(sg_s, g_s, w_s, sg_t, g_t, w_t, sg_b, g_b, w_b, training=False)
        row += list(fidelity.threshold_test(args, expl0, base, b.src, b.dst, b.fake, b.ts, b.e_idx, pos_out_ori,
                                            neg_out_ori, y_ori, sg_s, sg_t, sg_b))
    return np.array(row + [1.0])          # + the THRESHOLD_RAN flag (threshold_test ran)


def test_eval_batch_equals_reference_loop_body():
    from tempme_amd.evaluate import eval_batch, eval_spans
    from tempme_amd.train import batch_from_pack
    dev = torch.device("cuda", 0)
    buf, ev, base, ex = _setup(dev)
    args = _args()
    spans = eval_spans(int(ev[0].shape[0]) - 1, args.test_bs)
    assert len(spans) >= 3
    for k, s, e in spans[:3]:
        rows = torch.arange(s, e, dtype=torch.int64, device=dev)
        got = eval_batch(args, base, ex, batch_from_pack(buf, *ev, rows))
        want = _reference_batch(args, base, ex, batch_from_pack(buf, *ev, rows))
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6, err_msg=f"batch {k}")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(target, world, *extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + extra) for r in range(world)]
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


def _eval_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        from tempme_amd.evaluate import eval_one_epoch
        buf, ev, base, ex = _setup(dev)
        for args, seed in ((_args(), None), (_args(if_bern=True, test_threshold=False), 77)):
            sharded = eval_one_epoch(args, base, ex, buf, *ev, rank=rank, world=world, seed=seed)
            if rank == 0:
                single = eval_one_epoch(args, base, ex, buf, *ev, seed=seed)
                n = int(ev[0].shape[0]) - 1
                assert sharded["n_batches"] == single["n_batches"] == math.ceil(n / args.test_bs) - 1
                # bitwise the same figures (a batch whose y_ori holds one class has no AUC: NaN, as in the reference)
                assert sharded.keys() == single.keys()
                for k in single:
                    a, b = sharded[k], single[k]
                    assert a == b or (np.isnan(a) and np.isnan(b)), (k, a, b)
                assert all(np.isfinite(single[k]) for k in ("aps", "acc", "loss", "kl_loss"))
                if args.test_threshold:   # threshold_test ran (a NaN figure of a batch propagates, as in the reference)
                    assert single["ratio_aps"] != 0.0
        if rank == 0:
            q.put("ok")
        dist.barrier()
    except Exception as exc:      # noqa: BLE001
        q.put(repr(exc))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_sharded_eval_equals_single_process():
    _spawn(_eval_worker, WORLD)


def _nccl_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        assert dist.get_backend() == "nccl"
        from tempme_amd.evaluate import gather_rows
        from tempme_amd.train import GradAllReduce, batch_from_pack, train_step
        buf, ev, base, ex = _setup(dev)

        class Rec(GradAllReduce):
            def start(self):
                self.local = [p.grad.detach().clone() for p in self.module.parameters() if p.grad is not None]
                super().start()

            def finish(self):
                super().finish()
                self.synced = [p.grad.detach().clone() for p in self.module.parameters() if p.grad is not None]
        sync = Rec(ex, force=True)
        opt = torch.optim.Adam(ex.parameters(), lr=1e-3)
        train_step(ex, base, opt, batch_from_pack(buf, *ev, torch.arange(0, 40, device=dev)), if_bern=False,
                   grad_sync=sync)
        torch.cuda.synchronize()
        assert sync._flat is not None and sync._flat.is_cuda          # the collective ran on a device bucket
        assert len(sync.local) == len(sync.synced) > 0
        for a, b in zip(sync.local, sync.synced):
            assert torch.equal(a, b)                                  # the average over one rank
        rows = {3: np.arange(14.0), 1: np.ones(14)}
        allr = gather_rows(rows, world, device=dev, collective=True)
        assert allr.shape == (2, 15) and list(allr[:, 0]) == [1.0, 3.0]
        q.put("ok")
    except Exception as exc:      # noqa: BLE001
        q.put(repr(exc))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_rccl_world1_grad_all_reduce_and_gather():
    _spawn(_nccl_worker, 1)
