"""Drop-in ``RandEdgeSampler`` (utils/batch_loader.py:32-42) with keyed device draws.

``sample(size)`` returns (src, dst) numpy arrays like the reference; draw j=0 picks
the src (:40) and j=1 the dst (:41), keyed by (seed, split, event, stage NEG).
"""
import numpy as np
import torch

from . import _lib as L


class RandEdgeSampler:
    def __init__(self, src_list, dst_list, *, seed=0, split=L.SPLIT_TEST, device=None):
        self.src_list = np.unique(np.concatenate(src_list))
        self.dst_list = np.unique(np.concatenate(dst_list))
        self.seed = int(seed)
        self.split = int(split)
        self.device = L.require_device(device)
        self._next_event = 0
        self._src_dev = torch.from_numpy(self.src_list.astype(np.int32)).to(self.device)
        self._dst_dev = torch.from_numpy(self.dst_list.astype(np.int32)).to(self.device)

    def _draw(self, lst, ev, j):
        out = torch.empty(max(ev.numel(), 1), dtype=torch.int32, device=self.device)
        L.check(L.lib().tm_neg_sample(L.TmRng(self.seed, self.split, L.SIDE_NONE), L.ptr(lst), lst.numel(),
                                      L.ptr(ev), ev.numel(), j, L.ptr(out), L.stream_ptr(self.device)),
                "RandEdgeSampler.sample")
        return out[:ev.numel()]

    def sample(self, size, *, event_ids=None, as_tensor=False):
        if event_ids is None:
            ev = np.arange(self._next_event, self._next_event + size, dtype=np.int64)
            self._next_event += size
        else:
            ev = np.asarray(event_ids, dtype=np.int64).reshape(-1)
        evd = torch.from_numpy(ev.astype(np.uint32).view(np.int32)).to(self.device)
        s, d = self._draw(self._src_dev, evd, 0), self._draw(self._dst_dev, evd, 1)
        if as_tensor:
            return s, d
        return s.cpu().numpy().astype(self.src_list.dtype), d.cpu().numpy().astype(self.dst_list.dtype)

    def dst_device(self):
        return self._dst_dev
