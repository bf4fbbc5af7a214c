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
with ONE all-reduce over RCCL before the optimizer step, so every rank keeps identical weights.  The
all-reduce is issued asynchronously and the next batch's explainer-independent work (``prepare_step``)
runs while it is in flight (``run_steps``).
"""
import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L

SIDES = ("src", "tgt", "bgd")


class Batch:
    """One reference batch (get_item + get_item_edge, utils/batch_loader.py:203-242) as device tensors."""

    def __init__(self, src, dst, ts, e_idx, fake, subgraphs, walks, edges, stacked=None):
        self.src, self.dst, self.ts, self.e_idx, self.fake = src, dst, ts, e_idx, fake
        self.subgraphs, self.walks, self.edges = subgraphs, walks, edges
        # (node6 [3,B,W,6], eid3, ts3, cat [3,B,W], cnt [3,B,W,3,3]) device tensors: the three sides of the
        # batch stacked, so the explainer encodes them in one call (per-side walks are views of these)
        self.stacked = stacked
        self.sub_stacked = None   # (hop-1 nodes, hop-1 eids, hop-2 nodes, hop-2 eids) [3, B, ...] when gathered
        self.imp_all = None       # encode_sides' [3 B W] importances and their per-side views

    def __len__(self):
        return int(self.src.shape[0])


def _gather_pack(arrays, rows, err=None):
    """index_select(dim, rows) of every (tensor, dim) in ``arrays`` (dim 1 for the side-major pack
    arrays, 0 for the event arrays) as ONE tm_gather_rows launch; rows a device int64 tensor; a row
    outside an array sets the int32 device flag ``err`` (the pack's, raised by its check)."""
    outs, jobs = [], []
    n = int(rows.numel())
    for x, dim in arrays:
        shape = list(x.shape)
        shape[dim] = n
        o = torch.empty(shape, dtype=x.dtype, device=x.device)
        row_elems = int(np.prod(x.shape[dim + 1:])) if x.dim() > dim + 1 else 1
        sides = int(x.shape[0]) if dim == 1 else 1
        jobs.append(L.GatherJob(x.data_ptr(), o.data_ptr(), row_elems * x.element_size(),
                                x.stride(0) * x.element_size() if dim == 1 else 0,
                                o.stride(0) * o.element_size() if dim == 1 else 0, int(x.shape[dim]), sides, 0))
        outs.append(o)
    arr = (L.GatherJob * len(jobs))(*jobs)
    L.check(L.lib().tm_gather_rows(arr, len(jobs), L.ptr(rows), n, L.ptr(err), L.stream_ptr(rows.device)),
            "batch_from_pack")
    return outs


def batch_from_pack(buf, src, dst, ts, e_idx, rows):
    """Rows ``rows`` (device int64 index, or a slice) of a sampled pack (preprocess.EventBuffers,
    side-major [3, E, ...]) and of the event arrays (one gather launch for all of them)."""
    packed = [(buf.node6, 1), (buf.eid3, 1), (buf.ts3, 1), (buf.cat, 1), (buf.cnt, 1), (buf.sub1_node, 1),
              (buf.sub1_eid, 1), (buf.sub1_ts, 1), (buf.sub2_node, 1), (buf.sub2_eid, 1), (buf.sub2_ts, 1),
              (src, 0), (dst, 0), (ts, 0), (e_idx, 0), (buf.dst_fake, 0)]
    if (not isinstance(rows, slice) and rows.is_cuda and rows.dtype == torch.int64
            and all(x.is_contiguous() and x.is_cuda and x.element_size() % 4 == 0 for x, _ in packed)):
        g = _gather_pack(packed, rows, getattr(buf, "err", None))
        node6, eid3, ts3, cat, cnt = g[:5]
        s1, s2 = g[5:8], g[8:11]
        return _batch(g[11], g[12], g[13], g[14], g[15], node6, eid3, ts3, cat, cnt, s1, s2)

    def take(x, dim=0):
        return x[(slice(None),) * dim + (rows,)] if isinstance(rows, slice) else x.index_select(dim, rows)
    node6, eid3, ts3, cat, cnt = (take(buf.node6, 1), take(buf.eid3, 1), take(buf.ts3, 1), take(buf.cat, 1),
                                  take(buf.cnt, 1))
    s1 = [take(buf.sub1_node, 1), take(buf.sub1_eid, 1), take(buf.sub1_ts, 1)]
    s2 = [take(buf.sub2_node, 1), take(buf.sub2_eid, 1), take(buf.sub2_ts, 1)]
    return _batch(take(src), take(dst), take(ts), take(e_idx), take(buf.dst_fake), node6, eid3, ts3, cat, cnt, s1, s2)


def _batch(src, dst, ts, e_idx, fake, node6, eid3, ts3, cat, cnt, s1, s2):
    subgraphs, walks, edges = [], [], []
    for s in range(3):
        subgraphs.append(([s1[0][s], s2[0][s]], [s1[1][s], s2[1][s]], [s1[2][s], s2[2][s]]))
        walks.append((node6[s], eid3[s], ts3[s], cat[s].unsqueeze(-1), None))
        edges.append(cnt[s])
    b = Batch(src, dst, ts, e_idx, fake, subgraphs, walks, edges, stacked=(node6, eid3, ts3, cat, cnt))
    # the three sides' hop-1 / hop-2 node and edge ids as the gathered [3, B, ...] tensors (explain_sides)
    b.sub_stacked = (s1[0], s1[1], s2[0], s2[1])
    return b


def _as_dev(x, dev, dtype):
    if isinstance(x, torch.Tensor):
        return x.to(dev, dtype)
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev, dtype)


def encode_sides(explainer, batch):
    """TempME.forward for the src / tgt / bgd walks of one batch (temp_exp_main.py:605-607).  On the HIP
    path the three sides go through ONE forward_groups call (one std group per side, exactly as three
    separate calls); returns the three [B, W, 1] importance tensors."""
    if not explainer._hip_ok():
        return [explainer(w, batch.ts, e) for w, e in zip(batch.walks, batch.edges)]
    dev = explainer._dev()
    if batch.stacked is None:
        st = lambda k, dt: torch.stack([_as_dev(w[k], dev, dt) for w in batch.walks])  # noqa: E731
        cnt = torch.stack([_as_dev(e, dev, torch.float32) for e in batch.edges])
        batch.stacked = (st(0, torch.int32), st(1, torch.int32), st(2, torch.float32), st(3, torch.int32), cnt)
    node6, eid3, ts3, cat, cnt = batch.stacked
    G, B, W = node6.shape[0], node6.shape[1], node6.shape[2]
    cut = _as_dev(batch.ts, dev, torch.float64).reshape(1, B).expand(G, B)
    imp = explainer.forward_groups(node6, eid3, ts3, cat.reshape(G, B, W), cut, cnt, G, B, W)
    sides = list(imp.view(G, B, W, 1).unbind(0))
    batch.imp_all = (imp, sides)      # the three sides' importances as one tensor (explain_sides, kl_loss)
    return sides


def _stacked_imp(batch, imps, G, B, W):
    """[G, B, W] importances: encode_sides' single output when ``imps`` are its per-side views (no copy),
    else a stack of them."""
    ia = getattr(batch, "imp_all", None)
    if ia is not None and len(imps) == len(ia[1]) and all(a is b for a, b in zip(imps, ia[1])):
        return ia[0].view(G, B, W)
    return torch.stack([x.reshape(B, W) for x in imps])


class GradAllReduce:
    """Average the explainer's gradients over the process group with one collective per step.

    ``start()`` flattens the gradients into one bucket and launches the all-reduce asynchronously;
    ``finish()`` waits for it and writes the averages back.  Work issued between the two (the next
    batch's gather and the frozen base model's original-prediction contrast, which read neither the
    explainer's gradients nor its weights) overlaps the collective.  ``__call__`` does
    both back to back.  ``force``: run the collective even in a group of one (exercises the backend's
    path, e.g. RCCL on one GPU; at world size 1 the average is the gradient itself)."""

    def __init__(self, module, group=None, force=False, bucket=None):
        """``bucket``: the module's optimizer when it keeps the gradients in one flat buffer (optim.FusedAdam):
        ``start`` gathers them there (``bucket.sync_grads()``, one launch per 32 parameters) and the all-reduce runs
        on ``bucket.flat_grad`` in place -- no per-parameter packing copies before the collective or after it."""
        self.module, self.group = module, group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.force = bool(force) and dist.is_initialized()
        self.bucket = bucket
        self.flat_grad = None if bucket is None else bucket.flat_grad
        self._flat = None
        self._work = None
        self._grads = None

    def start(self):
        if self.world == 1 and not self.force:
            return
        if self.flat_grad is not None:
            self.bucket.sync_grads()
            self._flat, self._grads = self.flat_grad, None
            self._work = dist.all_reduce(self._flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
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
        self._grads = grads
        self._work = dist.all_reduce(self._flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish(self):
        if self._work is None:
            return
        self._work.wait()
        self._work = None
        self._flat.div_(self.world)
        if self._grads is None:          # the flat bucket IS the gradients
            return
        off = 0
        for g in self._grads:
            g.copy_(self._flat[off:off + g.numel()].view_as(g))
            off += g.numel()
        self._grads = None

    def __call__(self):
        self.start()
        self.finish()


def explain_sides(explainer, batch, imps, training):
    """Explainer.retrieve_explanation(sg_src, imp_src, walks_src, ..., training) (temp_exp_main.py:608-609);
    on the HIP path the three sides run as one explain_groups call.  Returns the reference's list
    [hop-1 [3B, N], hop-2 [3B, N^2]] (hop-1 only for non-TGN bases)."""
    if not explainer._hip_ok() or batch.stacked is None:
        (sg_s, sg_t, sg_b), (w_s, w_t, w_b) = batch.subgraphs, batch.walks
        return explainer.retrieve_explanation(sg_s, imps[0], w_s, sg_t, imps[1], w_t, sg_b, imps[2], w_b,
                                              training=training)
    dev = explainer._dev()
    node6, eid3, ts3, cat, cnt = batch.stacked
    G, B, W = eid3.shape[0], eid3.shape[1], eid3.shape[2]
    ss = getattr(batch, "sub_stacked", None)
    if ss is not None and all(x.is_cuda and x.dtype == torch.int32 and x.is_contiguous() for x in ss):
        s1n, s1e, s2n, s2e = ss
    else:
        s1n = torch.stack([_as_dev(sg[0][0], dev, torch.int32) for sg in batch.subgraphs])
        s1e = torch.stack([_as_dev(sg[1][0], dev, torch.int32) for sg in batch.subgraphs])
        s2n = torch.stack([_as_dev(sg[0][1], dev, torch.int32) for sg in batch.subgraphs])
        s2e = torch.stack([_as_dev(sg[1][1], dev, torch.int32) for sg in batch.subgraphs])
    N = s1n.shape[-1]
    imp = _stacked_imp(batch, imps, G, B, W)
    e1, e2 = explainer.explain_groups(imp, eid3, ts3, s1n, s1e, s2n, s2e, G, B, W, N, training)
    if explainer.base_type == "tgn":
        return [e1.reshape(G * B, N), e2.reshape(G * B, N * N)]
    return [e1.reshape(G * B, N)]


def prepare_step(base_model, batch):
    """The explainer-independent part of a step (temp_exp_main.py:593-603): the base model's contrast
    inputs (TGN: built once for both contrasts) and its original predictions -> y_ori, under no_grad.
    Issued for batch k+1 while batch k's gradient all-reduce is in flight (``train_step(overlap=...)``)."""
    kw = {}
    sg_s, sg_t, sg_b = batch.subgraphs
    with torch.no_grad():
        if hasattr(base_model, "prepare_contrast"):
            kw["prepared"] = base_model.prepare_contrast(batch.src, batch.dst, batch.fake, batch.ts, sg_s, sg_t, sg_b)
        pos_out_ori, neg_out_ori = base_model.contrast(batch.src, batch.dst, batch.fake, batch.ts, batch.e_idx,
                                                       sg_s, sg_t, sg_b, **kw)
        y_pred = torch.cat([pos_out_ori, neg_out_ori], dim=0).sigmoid()
        y_ori = torch.where(y_pred > 0.5, 1., 0.).view(y_pred.size(0), 1)
    return kw, pos_out_ori, neg_out_ori, y_ori


def _record_stream(obj, stream):
    """record_stream(stream) on every tensor inside obj (dicts, lists, tuples)."""
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            obj.record_stream(stream)
    elif isinstance(obj, dict):
        for v in obj.values():
            _record_stream(v, stream)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _record_stream(v, stream)


def train_step(explainer, base_model, optimizer, batch, *, beta=0.5, prior_p=0.3, if_bern=True, criterion=None,
               grad_sync=None, prepared=None, overlap=None, side_stream=None):
    """temp_exp_main.py:593-632 for one batch; returns the step's tensors (no host sync).  ``prepared``:
    this batch's ``prepare_step`` output if it was issued earlier; ``overlap``: a callable run while the
    gradient all-reduce is in flight (between ``grad_sync.start()`` and ``.finish()``); ``side_stream``:
    without ``prepared``, the base model's original-prediction contrast (``prepare_step``, independent of
    the explainer) runs on this stream concurrently with the explainer's encoder and explanation, joined
    before the explained contrast."""
    criterion = criterion or torch.nn.BCEWithLogitsLoss()
    sg_s, sg_t, sg_b = batch.subgraphs
    w_s, w_t, w_b = batch.walks
    fork = prepared is None and side_stream is not None
    if fork:
        cur = torch.cuda.current_stream(side_stream.device)
        side_stream.wait_stream(cur)
        with torch.cuda.stream(side_stream):
            prepared = prepare_step(base_model, batch)
    elif prepared is None:
        prepared = prepare_step(base_model, batch)
    kw, pos_out_ori, neg_out_ori, y_ori = prepared
    optimizer.zero_grad()
    g_s, g_t, g_b = encode_sides(explainer, batch)
    explanation = explain_sides(explainer, batch, (g_s, g_t, g_b), if_bern)
    if fork:
        cur.wait_stream(side_stream)
        if not torch.cuda.is_current_stream_capturing():
            # the side stream's allocations are read here: keep them from its pool until this stream is done
            _record_stream(prepared, cur)
    pos_logit, neg_logit = base_model.contrast(batch.src, batch.dst, batch.fake, batch.ts, batch.e_idx, sg_s, sg_t,
                                               sg_b, explain_weights=explanation, **kw)
    pred = torch.cat([pos_logit, neg_logit], dim=0)
    pred_loss = criterion(pred, y_ori)
    if batch.stacked is not None and explainer._hip_ok() and explainer.prior == "empirical":
        # the three per-side kl_loss calls as one tm_kl_loss launch (value and gradient)
        B, W = g_s.shape[0], g_s.shape[1]
        prob = _stacked_imp(batch, (g_s, g_t, g_b), 3, B, W)
        kl_loss = explainer.kl_loss_groups(prob, batch.stacked[3].reshape(3, B, W), target=prior_p)
    else:
        kl_loss = (explainer.kl_loss(g_s, w_s, target=prior_p) + explainer.kl_loss(g_t, w_t, target=prior_p)
                   + explainer.kl_loss(g_b, w_b, target=prior_p))
    loss = pred_loss + beta * kl_loss
    loss.backward()
    if grad_sync is not None and hasattr(grad_sync, "start"):
        grad_sync.start()
    elif grad_sync is not None:
        grad_sync()
    if overlap is not None:
        overlap()
    if grad_sync is not None and hasattr(grad_sync, "finish"):
        grad_sync.finish()
    optimizer.step()
    batch.imp_all = None      # drop the importances' autograd graph with the step (callers may keep the batch)
    return dict(loss=loss.detach(), pred_loss=pred_loss.detach(), kl_loss=kl_loss.detach(),
                pos_logit=pos_logit.detach(), neg_logit=neg_logit.detach(), pos_out_ori=pos_out_ori,
                neg_out_ori=neg_out_ori, y_ori=y_ori)


def run_steps(explainer, base_model, optimizer, batches, *, grad_sync=None, overlap=True, **kw):
    """``train_step`` over a list of batches; with ``overlap`` (and a process group), batch k+1's gather
    result is prepared (``prepare_step``) while batch k's gradient all-reduce is in flight.  Same
    updates as the serial loop (tests/test_multi_rank.py)."""
    outs = []
    n = len(batches)
    # each batch is fetched once (``batches`` may gather lazily, e.g. _LazyBatches): at most the current and
    # the next gathered batch are alive at a time
    b_next = batches[0] if n else None
    nxt = prepare_step(base_model, b_next) if n else None
    for k in range(n):
        b, cur, box = b_next, nxt, {}
        b_next = batches[k + 1] if k + 1 < n else None
        if overlap and b_next is not None:
            def pre(b1=b_next):
                box["p"] = prepare_step(base_model, b1)
        else:
            pre = None
        outs.append(train_step(explainer, base_model, optimizer, b, grad_sync=grad_sync, prepared=cur, overlap=pre,
                               **kw))
        del b, cur
        nxt = box.get("p") if b_next is not None else None
        if nxt is None and b_next is not None:
            nxt = prepare_step(base_model, b_next)
    return outs


class _LazyBatches:
    """The epoch's batches gathered from the pack on access (``batch_from_pack`` per index), so an epoch
    does not hold a permuted device copy of the whole rank-local pack."""

    def __init__(self, buf, src, dst, ts, e_idx, perm, spans):
        self.args, self.perm, self.spans = (buf, src, dst, ts, e_idx), perm, spans

    def __len__(self):
        return len(self.spans)

    def __getitem__(self, k):
        s_idx, e_end = self.spans[k]
        return batch_from_pack(*self.args, self.perm[s_idx:e_end])


class GraphedTrainStep:
    """``train_step`` on one fixed batch shape captured once as a HIP graph and replayed per batch.

    The step launches ~1,000 kernels (the base model's contrast forward/backward, the explainer's
    encoder and explanation, losses, Adam); replaying a captured graph removes their host-side launch
    cost.  Each call copies the batch's rows into a static index buffer and replays: the pack slice,
    every kernel and the optimizer step run on the device with no host synchronisation.  Needs an
    optimizer built with ``capturable=True`` and no host-side collectives (gloo) inside the step; the
    first ``len(warmup_rows)`` batches are run eagerly on the capture stream first (they are real
    training steps).  Returns the static output dict of ``train_step`` (overwritten by every call)."""

    def __init__(self, explainer, base_model, optimizer, buf, src, dst, ts, e_idx, warmup_rows, *,
                 overlap_prepare=False, **kw):
        dev = src.device
        self.args = (explainer, base_model, optimizer, buf, src, dst, ts, e_idx)
        self.kw = kw
        if overlap_prepare and "prepared" not in kw:
            # the captured graph gets two branches: the base model's original contrast beside the explainer
            self.kw = dict(kw, side_stream=torch.cuda.Stream(device=dev))
        self.rows = torch.empty_like(warmup_rows[0])
        self.stream = torch.cuda.Stream(device=dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self.stream):
            for r in warmup_rows:
                self.rows.copy_(r)
                self._body()
        torch.cuda.current_stream(dev).wait_stream(self.stream)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            self.out = self._body()
        # the capture recorded the repack without running it (the device packs are the last warm-up step's,
        # from before its optimizer step): an eager call before the first replay must repack
        explainer._packed_key = None

    def _body(self):
        ex, base, opt, buf, src, dst, ts, e_idx = self.args
        batch = batch_from_pack(buf, src, dst, ts, e_idx, self.rows)
        ex.packed_weights(force=True)     # the replayed step repacks the weights Adam just updated
        return train_step(ex, base, opt, batch, **self.kw)

    def __call__(self, rows):
        self.rows.copy_(rows)
        self.graph.replay()
        # the replay updated the parameters without bumping their version counters: drop the explainer's
        # pack key so an eager call after this one repacks instead of using the pre-update pack
        self.args[0]._packed_key = None
        return self.out


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
    batches = _LazyBatches(buf, src, dst, ts, e_idx, perm, epoch_spans(num_instance, bs, rank, world))
    outs = run_steps(explainer, base_model, optimizer, batches, grad_sync=grad_sync, beta=beta, prior_p=prior_p,
                     if_bern=if_bern)
    return [step_metrics(o) for o in outs] if metrics else outs
