"""Data-parallel eval loop (tempme_amd/evaluate.py) on CPU: the reference's test-batch bounds
(temp_exp_main.py:422-431), whole-batch sharding, and the gather + epoch means (:495-507) over a gloo
world of 2 equal one process's figures exactly.  The per-batch device work is in
tests/test_gpu_eval.py."""
import math
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from tempme_amd.evaluate import (FIGURES, RATIO_FIGURES, THRESHOLD_RAN, eval_spans, gather_rows, reduce_epoch,
                                 run_sharded, shard_spans)


def _reference_spans(num_test_instance, test_bs):
    """The loop header of eval_one_epoch, temp_exp_main.py:422-432, restated literally."""
    out = []
    num_test_batch = math.ceil(num_test_instance / test_bs) - 1
    idx_list = np.arange(num_test_instance)
    for k in range(num_test_batch):
        s_idx = k * test_bs
        e_idx = min(num_test_instance - 1, s_idx + test_bs)
        if s_idx == e_idx:
            continue
        b = idx_list[s_idx:e_idx]
        out.append((k, int(b[0]), int(b[-1]) + 1))
    return out


@pytest.mark.parametrize("n,bs", [(1000, 100), (1001, 100), (999, 100), (100, 100), (101, 100), (5, 2), (1, 4),
                                  (19200, 100), (230, 7)])
def test_eval_spans_match_reference_loop(n, bs):
    assert eval_spans(n, bs) == _reference_spans(n, bs)


def test_shards_partition_the_batches():
    spans = eval_spans(2345, 100)
    for world in (1, 2, 3, 8):
        got = sorted(sum((shard_spans(spans, r, world) for r in range(world)), []))
        assert got == spans
        for r in range(world):
            assert all(k % world == r for k, _, _ in shard_spans(spans, r, world))
    with pytest.raises(ValueError):
        shard_spans(spans, 2, 2)


def _row(k, s, e):
    """A deterministic stand-in for eval_batch's figures of batch k (threshold_test only on even k) + the flag."""
    rng = np.random.default_rng(1000 + k)
    r = np.append(rng.random(len(FIGURES)) * (e - s), 1.0)
    if k % 2:
        r[len(FIGURES) - len(RATIO_FIGURES):THRESHOLD_RAN] = np.nan
        r[THRESHOLD_RAN] = 0.0
    return r


def _reference_ratio_means(rows, spans):
    """temp_exp_main.py:479-499 restated: ratio lists appended only for batches that ran threshold_test, then
    np.mean over the list (NaN entries included) or 0 for an empty list."""
    out = {}
    for j, name in enumerate(FIGURES):
        if name in RATIO_FIGURES:
            lst = [rows[k][j] for k, _, _ in spans if rows[k][THRESHOLD_RAN] == 1.0]
            out[name] = np.mean(lst) if len(lst) != 0 else 0
    return out


def test_reduce_epoch_is_the_reference_means():
    spans = eval_spans(1234, 100)
    rows = {k: _row(k, s, e) for k, s, e in spans}
    out = reduce_epoch(gather_rows(rows))
    want = _reference_ratio_means(rows, spans)
    for j, name in enumerate(FIGURES):
        col = [rows[k][j] for k, _, _ in spans]
        if name in RATIO_FIGURES:
            assert out[name] == float(want[name]), name
        else:
            assert out[name] == float(np.mean(col)), name
    assert out["n_batches"] == len(spans)
    # no threshold batches: the reference reports 0 for the ratio figures (:495-499)
    for r in rows.values():
        r[len(FIGURES) - len(RATIO_FIGURES):THRESHOLD_RAN] = np.nan
        r[THRESHOLD_RAN] = 0.0
    out = reduce_epoch(gather_rows(rows))
    assert all(out[n] == 0.0 for n in RATIO_FIGURES)


def test_reduce_epoch_keeps_a_nan_ratio_of_a_batch_that_ran():
    """A batch that ran threshold_test but whose ratio_auc is NaN (one-class y_ori: roc_auc_score undefined) makes
    the epoch's ratio_auc NaN, as np.mean does in the reference; the other ratio figures stay the means
    over the same batches."""
    spans = eval_spans(1234, 100)
    rows = {k: _row(k, s, e) for k, s, e in spans}
    j_auc = FIGURES.index("ratio_auc")
    rows[spans[2][0]][j_auc] = np.nan          # an even batch: threshold_test ran
    out = reduce_epoch(gather_rows(rows))
    want = _reference_ratio_means(rows, spans)
    assert np.isnan(out["ratio_auc"]) and np.isnan(want["ratio_auc"])
    for name in RATIO_FIGURES:
        if name != "ratio_auc":
            assert out[name] == float(want[name]), name


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, bs, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        spans = eval_spans(n, bs)
        seen = []

        def fn(k, s, e):
            seen.append(k)
            return _row(k, s, e)
        out = run_sharded(spans, fn, rank, world)
        assert all(k % world == rank for k in seen)
        q.put((rank, out))
        dist.barrier()
    except Exception as exc:      # noqa: BLE001
        q.put((rank, repr(exc)))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1234), (2, 1134), (3, 450)])
def test_sharded_epoch_equals_one_process(world, n):
    bs = 100
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, bs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    single = run_sharded(eval_spans(n, bs), _row)
    for r in range(world):
        assert res[r] == single, (r, res[r])
