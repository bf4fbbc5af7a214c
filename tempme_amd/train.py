"""Explainer training on the device: the loop body of temp_exp_main.py:584-632
and its data-parallel driver.

    with no_grad: pos_out_ori, neg_out_ori = base.contrast(...)      original predictions -> y_ori
    graphlet_imp_{src,tgt,bgd} = Explainer(walks_*, ts, edge_*)       TempME.forward x3
    explanation = Explainer.retrieve_explanation(..., training=if_bern)
    pos_logit, neg_logit = base.contrast(..., explain_weights=explanation)
    loss = BCEWithLogits(pred, y_ori) + beta * sum(kl_loss)          backward, Adam step

Everything stays on the device: the batch is a slice of a device-resident pack (the sampler's
EventBuffers, i.e. what the reference reads back from its H5 pack), the base model's contrast runs
the HIP attention kernels forward and backward, and the explainer's forward in training runs its
autograd formulation (dropout and Beta ``rsample`` draw from torch's device RNG, so a stochastic
step matches the reference statistically, not bit for bit; with ``Explainer.eval()`` and
``if_bern=False`` the step is deterministic and tests/test_gpu_train.py holds it to the reference).

Data parallel: one process per GPU, each stepping its own whole batches; after
backward the explainer's gradients (one flat fp32 bucket, ~0.46 MB at uslegis dims) are averaged
with ONE all-reduce over RCCL before the optimizer step, so every rank keeps identical weights.
"""
import numpy as np
import torch
import torch.distributed as dist

SIDES = ("src", "tgt", "bgd")


class Batch:
    """One reference batch (get_item + get_item_edge, utils/batch_loader.py:203-242) as device tensors."""

    def __init__(self, src, dst, ts, e_idx, fake, subgraphs, walks, edges):
        self.src, self.dst, self.ts, self.e_idx, self.fake = src, dst, ts, e_idx, fake
        self.subgraphs, self.walks, self.edges = subgraphs, walks, edges

    def __len__(self):
        return int(self.src.shape[0])


def batch_from_pack(buf, src, dst, ts, e_idx, rows):
    """Rows ``rows`` (device int64 index, or a slice) of a sampled pack (preprocess.EventBuffers,
    side-major [3, E, ...]) and of the event arrays."""
    def take(x, s=None):
        x = x if s is None else x[s]
        return x[rows] if isinstance(rows, slice) else x.index_select(0, rows)
    subgraphs, walks, edges = [], [], []
    for s in range(3):
        subgraphs.append(([take(buf.sub1_node, s), take(buf.sub2_node, s)],
                          [take(buf.sub1_eid, s), take(buf.sub2_eid, s)],
                          [take(buf.sub1_ts, s), take(buf.sub2_ts, s)]))
        walks.append((take(buf.node6, s), take(buf.eid3, s), take(buf.ts3, s), take(buf.cat, s).unsqueeze(-1), None))
        edges.append(take(buf.cnt, s))
    return Batch(take(src), take(dst), take(ts), take(e_idx), take(buf.dst_fake), subgraphs, walks, edges)


class GradAllReduce:
    """Average the explainer's gradients over the process group with one collective per step."""

    def __init__(self, module, group=None):
        self.module, self.group = module, group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._flat = None

    def __call__(self):
        if self.world == 1:
            return
        grads = [p.grad for p in self.module.parameters() if p.grad is not None]
        if not grads:
            return
        n = sum(g.numel() for g in grads)
        if self._flat is None or self._flat.numel() != n or self._flat.device != grads[0].device:
            self._flat = torch.empty(n, dtype=torch.float32, device=grads[0].device)
        off = 0
        for g in grads:
            self._flat[off:off + g.numel()].copy_(g.reshape(-1))
            off += g.numel()
        dist.all_reduce(self._flat, op=dist.ReduceOp.SUM, group=self.group)
        self._flat.div_(self.world)
        off = 0
        for g in grads:
            g.copy_(self._flat[off:off + g.numel()].view_as(g))
            off += g.numel()


def train_step(explainer, base_model, optimizer, batch, *, beta=0.5, prior_p=0.3, if_bern=True, criterion=None,
               grad_sync=None):
    """temp_exp_main.py:593-632 for one batch; returns the step's tensors (no host sync)."""
    criterion = criterion or torch.nn.BCEWithLogitsLoss()
    sg_s, sg_t, sg_b = batch.subgraphs
    w_s, w_t, w_b = batch.walks
    e_s, e_t, e_b = batch.edges
    with torch.no_grad():
        pos_out_ori, neg_out_ori = base_model.contrast(batch.src, batch.dst, batch.fake, batch.ts, batch.e_idx,
                                                       sg_s, sg_t, sg_b)
        y_pred = torch.cat([pos_out_ori, neg_out_ori], dim=0).sigmoid()
        y_ori = torch.where(y_pred > 0.5, 1., 0.).view(y_pred.size(0), 1)
    optimizer.zero_grad()
    g_s = explainer(w_s, batch.ts, e_s)
    g_t = explainer(w_t, batch.ts, e_t)
    g_b = explainer(w_b, batch.ts, e_b)
    explanation = explainer.retrieve_explanation(sg_s, g_s, w_s, sg_t, g_t, w_t, sg_b, g_b, w_b, training=if_bern)
    pos_logit, neg_logit = base_model.contrast(batch.src, batch.dst, batch.fake, batch.ts, batch.e_idx, sg_s, sg_t,
                                               sg_b, explain_weights=explanation)
    pred = torch.cat([pos_logit, neg_logit], dim=0)
    pred_loss = criterion(pred, y_ori)
    kl_loss = (explainer.kl_loss(g_s, w_s, target=prior_p) + explainer.kl_loss(g_t, w_t, target=prior_p)
               + explainer.kl_loss(g_b, w_b, target=prior_p))
    loss = pred_loss + beta * kl_loss
    loss.backward()
    if grad_sync is not None:
        grad_sync()
    optimizer.step()
    return dict(loss=loss.detach(), pred_loss=pred_loss.detach(), kl_loss=kl_loss.detach(),
                pos_logit=pos_logit.detach(), neg_logit=neg_logit.detach(), pos_out_ori=pos_out_ori,
                neg_out_ori=neg_out_ori, y_ori=y_ori)


def step_metrics(out):
    """The per-batch training metrics of temp_exp_main.py:633-649 (host side, like the reference)."""
    from sklearn.metrics import average_precision_score, roc_auc_score
    pos, neg = out["pos_logit"], out["neg_logit"]
    po, no = out["pos_out_ori"], out["neg_out_ori"]
    y_pred = torch.cat([pos, neg], dim=0).sigmoid()
    pred_label = torch.where(y_pred > 0.5, 1., 0.).view(y_pred.size(0), 1)
    fid_prob = torch.cat([pos.sigmoid() - po.sigmoid(), no.sigmoid() - neg.sigmoid()], dim=0).mean(0)
    fid_logit = torch.cat([pos - po, no - neg], dim=0).mean(0)
    y, yp = out["y_ori"].cpu().numpy(), y_pred.cpu().numpy()
    return dict(aps=average_precision_score(y, yp), auc=roc_auc_score(y, yp) if len(np.unique(y)) > 1 else float("nan"),
                acc=float((pred_label == out["y_ori"]).float().mean()), fid_prob=float(fid_prob),
                fid_logit=float(fid_logit), loss=float(out["loss"]), pred_loss=float(out["pred_loss"]),
                kl_loss=float(out["kl_loss"]))


def epoch_spans(num_instance, bs, rank=0, world=1):
    """[start, end) positions in the shuffled order of the batches rank `rank` steps through
    (temp_exp_main.py:584-590 batch bounds; tail batches that do not fill a round of `world` dropped)."""
    num_batch = -(-num_instance // bs)
    spans = [(k * bs, min(num_instance - 1, k * bs + bs)) for k in range(num_batch)]
    spans = [sp for sp in spans if sp[0] != sp[1]]    # :588-589
    if world > 1:
        spans = spans[:len(spans) - len(spans) % world]
    return spans[rank::world]


def train_epoch(explainer, base_model, optimizer, buf, src, dst, ts, e_idx, bs, *, generator=None, beta=0.5,
                prior_p=0.3, if_bern=True, grad_sync=None, rank=0, world=1, metrics=False):
    """One epoch over a sampled pack (temp_exp_main.py:570-632): shuffled batch order; with world > 1
    whole batches are dealt round-robin (batch b -> rank b % world) and the tail that does not fill a
    round is dropped, so every rank takes the same number of all-reduced steps.  Returns per-step outputs."""
    num_instance = int(src.shape[0]) - 1              # the reference leaves the last event out (:560-561)
    perm = torch.randperm(num_instance, generator=generator).to(src.device)
    explainer.train()
    outs = []
    for s_idx, e_end in epoch_spans(num_instance, bs, rank, world):
        batch = batch_from_pack(buf, src, dst, ts, e_idx, perm[s_idx:e_end])
        out = train_step(explainer, base_model, optimizer, batch, beta=beta, prior_p=prior_p, if_bern=if_bern,
                         grad_sync=grad_sync)
        outs.append(step_metrics(out) if metrics else out)
    return outs
