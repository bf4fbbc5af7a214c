"""The explainer's optimizer (temp_exp_main.py:555, :631-632: ``torch.optim.Adam(explainer.parameters(), lr=...,
weight_decay=...)``) as one HIP kernel over a flat fp32 bucket (csrc/optim.hip, ``tm_adam_step``).

``FusedAdam(params, lr, betas, eps, weight_decay)`` takes the module's parameters and moves them into ONE contiguous
device buffer (``flat_param``; every parameter becomes a view of it, same Parameter objects), their gradients into a
second (``flat_grad``) and the Adam moments into two more.  ``zero_grad()`` sets the gradients to None as torch's
default does, so autograd hands each parameter its gradient tensor without an accumulation kernel;
``sync_grads()`` (called by ``step()`` and by the data-parallel all-reduce, train.GradAllReduce(bucket=opt)) copies
them into ``flat_grad`` in one launch per 32 parameters (``tm_copy_many``) and rebinds each ``.grad`` to its view
of the bucket.  ``step()`` is then one launch (no per-parameter or multi-tensor dispatch), and the all-reduce runs
on ``flat_grad`` itself.  The step count lives on the device, so the step is capturable in a HIP graph
(train.GraphedTrainStep).

Semantics = torch.optim.Adam with amsgrad=False, maximize=False (the reference's arguments).  torch skips a parameter
whose ``.grad`` is None (nothing reached it in backward); a post-accumulate-grad hook records which parameters
autograd reached since ``zero_grad`` and the step updates only their spans (one launch when every parameter was
reached, the common case; a launch per contiguous run otherwise).
One step count is shared by the bucket, as torch's per-parameter counts are equal when the same parameters receive
gradients every step (the reference's training loop).
"""
import torch
from torch.autograd.graph import increment_version

from . import _lib as L


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise ValueError("FusedAdam: amsgrad is not supported (the reference does not use it)")
        if not 0.0 <= lr or not 0.0 <= eps or not all(0.0 <= b < 1.0 for b in betas) or not 0.0 <= weight_decay:
            raise ValueError("FusedAdam: bad hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        if len(self.param_groups) != 1:
            raise ValueError("FusedAdam: one parameter group (the explainer's parameters)")
        # parameters that cannot receive a gradient (frozen feature tables) stay outside the bucket and are never
        # touched -- torch.optim.Adam skips them the same way (their .grad stays None)
        ps = [p for p in self.param_groups[0]["params"] if p.requires_grad]
        if not ps:
            raise ValueError("FusedAdam: no trainable parameters")
        dev = ps[0].device
        if dev.type != "cuda" or any(p.device != dev or p.dtype != torch.float32 for p in ps):
            raise ValueError("FusedAdam: fp32 parameters on one GPU")
        if len({p.data_ptr() for p in ps}) != len(ps):
            raise ValueError("FusedAdam: a parameter is listed twice")
        n = sum(p.numel() for p in ps)
        self.flat_param = torch.empty(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.float32, device=dev)
        self._done = torch.zeros(1, dtype=torch.int32, device=dev)
        self._spans = []
        off = 0
        with torch.no_grad():
            for p in ps:
                k = p.numel()
                self.flat_param[off:off + k].copy_(p.reshape(-1))
                self._spans.append((p, off, k))
                off += k
        self._params = [p for p, _, _ in self._spans]
        self._index = {id(p): i for i, p in enumerate(self._params)}
        self._reached = set()
        for i, p in enumerate(self._params):
            p.register_post_accumulate_grad_hook(lambda _p, i=i: self._reached.add(i))
        self._bind()

    def _bind(self):
        """Every parameter, its gradient and its Adam state as views of the flat buffers."""
        for p, off, k in self._spans:
            p.data = self.flat_param[off:off + k].view_as(p)
            p.grad = self.flat_grad[off:off + k].view_as(p)
            self.state[p] = {"step": self.step_t, "exp_avg": self.exp_avg[off:off + k].view_as(p),
                             "exp_avg_sq": self.exp_avg_sq[off:off + k].view_as(p)}

    def _grads_bound(self):
        for p, off, k in self._spans:
            g = p.grad
            if g is None or g.data_ptr() != self.flat_grad[off:].data_ptr():
                return False
        return True

    @torch.no_grad()
    def zero_grad(self, set_to_none=True):
        """``set_to_none`` (torch's default): every ``.grad`` None, so backward hands each parameter autograd's own
        gradient tensor (no accumulation kernel); else one fill of the bucket with the views bound."""
        self._reached.clear()
        if set_to_none:
            for p in self._params:
                p.grad = None
            return
        self.flat_grad.zero_()
        if not self._grads_bound():
            for p, off, k in self._spans:
                p.grad = self.flat_grad[off:off + k].view_as(p)

    @torch.no_grad()
    def sync_grads(self):
        """Every reached parameter's gradient into the bucket (tm_copy_many, up to 32 per launch) and its
        ``.grad`` rebound to the bucket view; idempotent."""
        jobs, rebind = [], []
        for p, off, k in self._spans:
            g = p.grad
            if g is None:
                continue
            dst = self.flat_grad.data_ptr() + 4 * off
            if g.data_ptr() == dst:
                continue
            if g.dtype != torch.float32 or not g.is_contiguous() or g.device != self.flat_grad.device or \
                    g.numel() != k:
                self.flat_grad[off:off + k].copy_(g.reshape(-1))
            else:
                jobs.append(L.CopyJob(g.data_ptr(), dst, k))
            rebind.append((p, off, k, g))
        st = L.stream_ptr(self.flat_grad.device)
        for i in range(0, len(jobs), 32):
            arr = (L.CopyJob * len(jobs[i:i + 32]))(*jobs[i:i + 32])
            L.check(L.lib().tm_copy_many(arr, len(jobs[i:i + 32]), st), "FusedAdam.sync_grads")
        for p, off, k, g in rebind:
            p.grad = self.flat_grad[off:off + k].view_as(p)
        return rebind

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        # the reached parameters' gradients into the bucket (a .grad set by the caller counts as reached)
        for p, g0 in [(p, p.grad) for p, _, _ in self._spans]:
            if g0 is not None and g0.data_ptr() != self.flat_grad.data_ptr() + 4 * self._spans[self._index[id(p)]][1]:
                self._reached.add(self._index[id(p)])
        self.sync_grads()
        for p, off, k in self._spans:
            if p.data_ptr() != self.flat_param[off:].data_ptr():
                raise RuntimeError("FusedAdam: a parameter was rebound away from the flat bucket")
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        # contiguous runs of the parameters autograd reached (torch.optim.Adam skips the others)
        runs, start = [], None
        for i, (p, off, k) in enumerate(self._spans + [(None, self.flat_param.numel(), 0)]):
            hit = i < len(self._spans) and i in self._reached
            if hit and start is None:
                start = off
            elif not hit and start is not None:
                runs.append((start, off))
                start = None
        fn, st = L.lib().tm_adam_step, L.stream_ptr(self.flat_param.device)
        for r, (a, b) in enumerate(runs):
            L.check(fn(self.flat_param.data_ptr() + 4 * a, self.flat_grad.data_ptr() + 4 * a,
                       self.exp_avg.data_ptr() + 4 * a, self.exp_avg_sq.data_ptr() + 4 * a, b - a, float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                       float(g["weight_decay"]), 1.0, L.ptr(self.step_t), L.ptr(self._done), int(r + 1 == len(runs)),
                       st), "FusedAdam.step")
        # the kernel wrote the parameters behind autograd's back: bump their version counters as torch's in-place
        # update would, so caches keyed on them (the explainer's packed weights) see the change
        increment_version(self._params)
        return loss

    def load_state_dict(self, state_dict):
        """torch.optim's state dict (per-parameter exp_avg / exp_avg_sq / step), copied into the flat buffers."""
        super().load_state_dict(state_dict)
        with torch.no_grad():
            steps = []
            for p, off, k in self._spans:
                st = self.state.get(p, {})
                if "exp_avg" in st:
                    self.exp_avg[off:off + k].copy_(st["exp_avg"].reshape(-1))
                    self.exp_avg_sq[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                else:
                    self.exp_avg[off:off + k].zero_()
                    self.exp_avg_sq[off:off + k].zero_()
                if "step" in st:
                    steps.append(float(st["step"]))
            if len(set(steps)) > 1:
                raise ValueError("FusedAdam: parameters at different step counts cannot share one bucket")
            self.step_t.fill_(steps[0] if steps else 0.0)
        self._bind()


__all__ = ["FusedAdam"]
