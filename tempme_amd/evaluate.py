"""Data-parallel explainer evaluation: ``eval_one_epoch`` (temp_exp_main.py:410-544) with
``threshold_test`` (:153-272), whole reference batches sharded over ranks.

Per reference batch (eval_one_epoch :432-494), on the device:

    with no_grad: pos_out_ori, neg_out_ori = base.contrast(...)  -> y_ori            (:440-444)
    graphlet_imp_{src,tgt,bgd} = Explainer(walks_*, ts, edge_*)   (Explainer.eval())   (:446-449)
    explanation = retrieve_explanation(..., training=if_bern)                          (:450-453)
    pos_logit, neg_logit = base.contrast(..., explain_weights=explanation)             (:454-456)
    loss = BCEWithLogits(pred, y_ori) + beta * sum(kl_loss)                            (:457-462)
    APS / AUC / acc / fidelity (prob, logit) of the batch                              (:463-478)
    test_threshold: retrieve_explanation(training=False) -> threshold_test ratio-AUCs   (:479-494)

and the epoch's figures are means over batches (:495-507).

Sharding: batch k (the reference's k-th test batch, unshuffled) goes to rank k % world.  Every
batch's figures depend only on its own events (the attention std is batch-global, the RNG is keyed
by global event id in the sampled pack), so a rank computes its batches' rows alone; ONE gather at
the end brings every rank's [k, 13 figures] rows to every rank, which sorts them by k and takes the
means in the reference's batch order -- the same floating-point sums as one process.  With
``if_bern`` (Beta rsample inside retrieve_explanation) the draws come from torch's device RNG; pass
``seed`` to reseed it per batch (seed + k) so the draws, too, do not depend on the shard.
"""
import math

import numpy as np
import torch
import torch.distributed as dist

from .train import batch_from_pack, encode_sides, explain_sides, prepare_step

BATCH_FIGURES = ("aps", "auc", "acc", "fid_prob", "fid_logit", "loss", "pred_loss", "kl_loss")
RATIO_FIGURES = ("ratio_aps", "ratio_auc", "ratio_acc", "ratio_prob", "ratio_logit")
FIGURES = BATCH_FIGURES + RATIO_FIGURES
# a row is FIGURES + this flag: 1.0 when the batch ran threshold_test (the reference appends to its ratio lists only
# then, temp_exp_main.py:479-494), so a NaN ratio figure from threshold_test itself (a one-class y_ori has no AUC)
# is told apart from "not run" and propagates into the epoch mean as in the reference's np.mean
THRESHOLD_RAN = len(FIGURES)


def eval_spans(num_instance, test_bs):
    """[(k, start, end)] of the reference's test batches (temp_exp_main.py:422-431): ceil(n / bs) - 1
    batches, the last event never included, empty batches skipped."""
    num_batch = math.ceil(num_instance / test_bs) - 1
    out = []
    for k in range(num_batch):
        s = k * test_bs
        e = min(num_instance - 1, s + test_bs)
        if s != e:
            out.append((k, s, e))
    return out


def shard_spans(spans, rank, world):
    """Rank ``rank``'s whole batches: batch k -> rank k % world (position in the batch list)."""
    if not (0 <= rank < world):
        raise ValueError("shard_spans: bad rank/world")
    return spans[rank::world]


def _metrics_sklearn(y, yp):
    from sklearn.metrics import average_precision_score, roc_auc_score
    return average_precision_score(y, yp), roc_auc_score(y, yp)


def eval_batch(args, base_model, explainer, batch):
    """The figures of one reference batch (temp_exp_main.py:440-494) as a float64 [14] row: FIGURES (ratio
    figures NaN unless ``args.test_threshold``) and the THRESHOLD_RAN flag."""
    from . import fidelity
    criterion = torch.nn.BCEWithLogitsLoss()
    row = np.full(len(FIGURES) + 1, np.nan)
    row[THRESHOLD_RAN] = 0.0
    with torch.no_grad():
        kw, pos_out_ori, neg_out_ori, y_ori = prepare_step(base_model, batch)
        explainer.eval()
        imps = encode_sides(explainer, batch)
        explanation = explain_sides(explainer, batch, imps, bool(args.if_bern))
        sg_s, sg_t, sg_b = batch.subgraphs
        pos_logit, neg_logit = base_model.contrast(batch.src, batch.dst, batch.fake, batch.ts, batch.e_idx, sg_s,
                                                   sg_t, sg_b, explain_weights=explanation, **kw)
        pred = torch.cat([pos_logit, neg_logit], dim=0)
        pred_loss = criterion(pred, y_ori)
        B, W = imps[0].shape[0], imps[0].shape[1]
        if batch.stacked is not None and explainer._hip_ok() and explainer.prior == "empirical":
            prob = torch.stack([x.reshape(B, W) for x in imps])
            kl_loss = explainer.kl_loss_groups(prob, batch.stacked[3].reshape(3, B, W), target=args.prior_p)
        else:
            kl_loss = sum(explainer.kl_loss(g, w, target=args.prior_p) for g, w in zip(imps, batch.walks))
        loss = pred_loss + args.beta * kl_loss
        y_pred = pred.sigmoid()
        pred_label = torch.where(y_pred > 0.5, 1., 0.).view(y_pred.size(0), 1)
        fid_prob = torch.cat([pos_logit.sigmoid() - pos_out_ori.sigmoid(), neg_out_ori.sigmoid() - neg_logit.sigmoid()],
                             dim=0).mean(0)
        fid_logit = torch.cat([pos_logit - pos_out_ori, neg_out_ori - neg_logit], dim=0).mean(0)
        acc = (pred_label == y_ori).float().mean()
        y_h, yp_h = y_ori.cpu().numpy(), y_pred.cpu().numpy()
        aps, auc = _metrics_sklearn(y_h, yp_h)
        row[:8] = (aps, auc, float(acc), float(fid_prob), float(fid_logit), float(loss), float(pred_loss),
                   float(kl_loss))
        if getattr(args, "test_threshold", False):
            expl0 = explain_sides(explainer, batch, imps, False)
            row[8:THRESHOLD_RAN] = fidelity.threshold_test(args, expl0, base_model, batch.src, batch.dst, batch.fake,
                                                           batch.ts, batch.e_idx, pos_out_ori, neg_out_ori, y_ori,
                                                           sg_s, sg_t, sg_b)
            row[THRESHOLD_RAN] = 1.0
    return row


def gather_rows(rows, world=1, group=None, device=None, collective=None):
    """Every rank's {k: row} (rows of equal length) on every rank, as one [n, 1 + F] float64 array sorted by
    batch index k.  One all_gather of a fixed-size padded tensor (RCCL needs device tensors: ``device``);
    ``collective`` forces (True) or skips (False) the gather, default: world > 1."""
    F = len(next(iter(rows.values()))) if rows else len(FIGURES)
    mine = np.full((len(rows), 1 + F), np.nan)
    for i, (k, r) in enumerate(sorted(rows.items())):
        mine[i, 0], mine[i, 1:] = k, r
    if (world > 1) if collective is None else collective:
        dev = device if device is not None else torch.device("cpu")
        n = torch.tensor([len(rows)], dtype=torch.int64, device=dev)
        counts = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(counts, n, group=group)
        cap = max(int(c.item()) for c in counts)
        pad = np.full((cap, 1 + F), -1.0)
        pad[:len(rows)] = mine
        t = torch.from_numpy(pad).to(dev)
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=group)
        allr = np.concatenate([p.cpu().numpy()[:int(c.item())] for p, c in zip(parts, counts)])
    else:
        allr = mine
    order = np.argsort(allr[:, 0], kind="stable")
    allr = allr[order]
    if len(np.unique(allr[:, 0])) != len(allr):
        raise AssertionError("gather_rows: a batch was evaluated on more than one rank")
    return allr


def reduce_epoch(allr):
    """The epoch's figures from the per-batch rows in batch order (temp_exp_main.py:495-507): means over
    batches; the ratio figures are the mean over the batches that ran threshold_test (THRESHOLD_RAN flag; a NaN
    figure of such a batch makes the mean NaN, as np.mean does in the reference), 0 when none did."""
    out = {}
    n_rows = len(allr)
    if n_rows and allr.shape[1] > 1 + THRESHOLD_RAN:
        ran = allr[:, 1 + THRESHOLD_RAN] == 1.0
    else:   # rows without the flag: a batch ran threshold_test when any of its ratio figures is set
        ran = ~np.isnan(allr[:, 1 + len(BATCH_FIGURES):1 + len(FIGURES)]).all(axis=1) if n_rows else np.zeros(0, bool)
    for j, name in enumerate(FIGURES):
        col = allr[:, 1 + j] if n_rows else np.zeros(0)
        if name in RATIO_FIGURES:
            col = col[ran]
            out[name] = float(np.mean(col)) if len(col) else 0.0
        else:
            out[name] = float(np.mean(col)) if len(col) else float("nan")
    out["n_batches"] = int(len(allr))
    return out


def run_sharded(spans, fn, rank=0, world=1, group=None, device=None):
    """``fn(k, start, end) -> row`` over this rank's whole batches, then every rank's rows gathered and
    reduced (the control flow of eval_one_epoch with the batch loop sharded)."""
    rows = {k: np.asarray(fn(k, s, e), dtype=np.float64) for k, s, e in shard_spans(spans, rank, world)}
    return reduce_epoch(gather_rows(rows, world, group, device))


def eval_one_epoch(args, base_model, explainer, buf, src, dst, ts, e_idx, *, rank=0, world=1, group=None,
                   seed=None):
    """temp_exp_main.py:410-544 over a device-resident sampled test pack (preprocess.EventBuffers, the
    reference's test_pack / test_edge) and the test events (device tensors); returns the epoch's figures
    (identical on every rank).  ``args``: test_bs, if_bern, beta, prior_p, test_threshold, base_type,
    n_degree, ratios (the reference's argparse names)."""
    base_model.eval()
    explainer.eval()
    num_instance = int(src.shape[0]) - 1
    spans = eval_spans(num_instance, int(args.test_bs))
    dev = src.device

    def one(k, s, e):
        if seed is not None:
            torch.manual_seed(int(seed) + int(k))
        rows_idx = torch.arange(s, e, dtype=torch.int64, device=dev)
        return eval_batch(args, base_model, explainer, batch_from_pack(buf, src, dst, ts, e_idx, rows_idx))
    gdev = dev if (world > 1 and dist.get_backend(group) == "nccl") else None
    if seed is None:
        return run_sharded(spans, one, rank, world, group, gdev)
    # per-batch reseeding must not leak into the caller's RNG streams (the reference never reseeds in eval):
    # the CPU and device generators are restored afterwards
    cpu_state = torch.get_rng_state()
    dev_state = torch.cuda.get_rng_state(dev) if dev.type == "cuda" else None
    try:
        return run_sharded(spans, one, rank, world, group, gdev)
    finally:
        torch.set_rng_state(cpu_state)
        if dev_state is not None:
            torch.cuda.set_rng_state(dev_state, dev)


__all__ = ["eval_one_epoch", "eval_batch", "eval_spans", "shard_spans", "gather_rows", "reduce_epoch", "run_sharded",
           "FIGURES", "THRESHOLD_RAN"]
