"""Host numpy arrays of the reference's eval loop, read by the GPU in place (csrc/stage.hip).

The reference's ``eval_one_epoch`` (temp_exp_main.py:441-453) hands ``TempME.forward`` and
``retrieve_explanation`` float64 / int64 numpy views of the pack it loaded once (``load_subgraph_margin``,
``np.load`` of the edge counts, utils/batch_loader.py:119-242).  ``stage(device, items, stream)`` turns a
call's views into contiguous int32 / float32 device tensors with ONE ``tm_stage_cast`` launch that reads them
straight from host memory: the whole pages inside each view's owning array (its numpy ``base``, at least
``MIN_BYTES``) are pinned and mapped once (``tm_host_register``; only pages the array holds alone, never a page it
shares with a neighbour allocation) and the array is kept referenced -- so it is never freed while registered -- in
an LRU registry capped at ``CAP_BYTES``; no host-side cast and no staging copy per call.  ``None`` when a view does
not qualify (a small or non-owning base, bytes outside the registered pages -- a view touching the array's first or
last partial page --, an unsupported dtype, more than 5 dims): the caller then stages through the pinned host-cast
path (explainer._to_many), same values.

The GPU reads the arrays after the call returns (asynchronously, in stream order), as a device pack would be
read: the views must not be modified before the launched work has run (the reference's loop never writes them).
"""
import atexit
import ctypes as C
import mmap
import threading
from collections import OrderedDict

import numpy as np
import torch

from . import _lib as L

MIN_BYTES = 1 << 20          # smaller bases (one batch's temporaries) go through the pinned host-cast path
CAP_BYTES = 32 << 30         # registered (pinned) host memory held at once, least recently used released first
_TYPES = {np.dtype(np.int64): L.TM_I64, np.dtype(np.float64): L.TM_F64, np.dtype(np.int32): L.TM_I32,
          np.dtype(np.float32): L.TM_F32}
_DST = {torch.int32: (L.TM_I32, 4), torch.float32: (L.TM_F32, 4), torch.float64: (L.TM_F64, 8)}


class _Registry:
    def __init__(self):
        # id(base) -> [base, registered host range start, its length, device address of the start or None (refused),
        #              {layout: (min, max)} (window_bounds)]
        self.regs = OrderedDict()
        self.bytes = 0
        self.lock = threading.Lock()

    def entry(self, base):
        """[base, lo, length, device address of lo or None, bounds cache, base address]: ``base``'s registration
        (made on first use)."""
        key = id(base)
        e = self.regs.get(key)
        if e is not None and e[0] is base:
            try:
                self.regs.move_to_end(key)
                return e
            except KeyError:             # released meanwhile: the locked path below
                pass
        with self.lock:
            e = self.regs.get(key)
            if e is not None and e[0] is base:
                self.regs.move_to_end(key)
                return e
            ptr, n = base.__array_interface__["data"][0], int(base.nbytes)
            lo, hi = -(-ptr // _PAGE) * _PAGE, (ptr + n) // _PAGE * _PAGE     # the whole pages inside the array
            if n < MIN_BYTES or n > CAP_BYTES or hi - lo < _PAGE:
                return None
            while self.bytes + (hi - lo) > CAP_BYTES and self.regs:
                self._release(next(iter(self.regs)))
            dev = C.c_void_p()
            ok = L.lib().tm_host_register(lo, hi - lo, C.byref(dev)) == 0
            # a refusal is remembered too: the slow path serves that base from then on
            e = self.regs[key] = [base, lo, hi - lo, dev.value if ok else None, {}, ptr]
            if ok:
                self.bytes += hi - lo
            return e

    def _release(self, key):
        base, ptr, n, dev, *_ = self.regs.pop(key)
        if dev is not None:
            # launched work may still read it: the whole device drains first (a release is rare: LRU eviction past
            # CAP_BYTES, clear(), interpreter exit)
            torch.cuda.synchronize()
            L.lib().tm_host_unregister(ptr)
            self.bytes -= n

    def clear(self):
        with self.lock:
            while self.regs:
                self._release(next(iter(self.regs)))


_PAGE = mmap.PAGESIZE
_REG = _Registry()


@atexit.register
def _release_all():
    if L._lib is not None:
        try:
            _REG.clear()
        except Exception:      # noqa: BLE001 -- interpreter shutdown
            pass


def _owner(a):
    b = a.base
    if b is None:
        return a
    if isinstance(b, np.ndarray) and b.base is None and (b.flags.c_contiguous or b.flags.f_contiguous):
        return b
    return None


def window_bounds(a):
    """(min, max) over ``a``'s layout repeated along its owning array's whole first axis -- e.g. the edge-id
    columns of every batch of a pack, when ``a`` is one batch's rows -- computed once per (array, layout) and
    kept with the array's registration; None when ``a`` does not qualify for ``stage``.  A caller that checks
    ids against a table once per array this way passes the table's row count as the staging bound, so ids
    rewritten after the check are clamped instead of read outside the table."""
    if a.__class__ is not np.ndarray or a.ndim < 1 or a.dtype not in _TYPES or a.size == 0:
        return None
    base = _owner(a)
    if base is None or not base.flags.c_contiguous:
        return None
    e = _REG.entry(base)
    if e is None or e[3] is None:
        return None
    s0 = a.strides[0]
    if s0 <= 0 or min(a.strides) < 0:
        return None
    from .explainer import _dropin_ext
    ext = _dropin_ext()
    p = ext.buf_addr(a) if ext is not None else a.__array_interface__["data"][0]
    off0 = (p - e[5]) % s0
    key = (off0, a.shape[1:], a.strides, a.dtype.str)
    hit = e[4].get(key)
    if hit is None:
        inner = sum((n - 1) * st for n, st in zip(a.shape[1:], a.strides[1:])) + a.itemsize
        rows = (base.nbytes - off0 - inner) // s0 + 1
        if rows < 1:
            return None
        win = np.ndarray((rows,) + a.shape[1:], dtype=a.dtype, buffer=base, offset=off0, strides=a.strides)
        hit = e[4][key] = (win.min(), win.max())
    return hit


_CODE = {torch.int32: L.TM_I32, torch.float32: L.TM_F32}
_FN = [None]


def stage(device, items, stream=None):
    """[(numpy view, torch dtype[, bound])] -> contiguous device tensors (views of one fresh allocation on
    ``stream``'s pool, default the current stream), read from host memory by one launch on that stream; None if
    any view does not qualify.  bound (int32 outputs): clamp into [0, bound) (tm_stage_job.bound).  On the
    current stream with the drop-in extension built, the per-view work (buffer geometry, registration bounds,
    job rows, the allocation and its views) runs in C++ (dropin_ext.cpp stage_host); same launch, same bytes."""
    if stream is None and len(items) <= 16 and all(it[1] in _CODE for it in items):
        from .explainer import _dropin_ext
        ext = _dropin_ext()
        if ext is not None:
            rows = []
            for it in items:
                a, dt = it[0], it[1]
                if a.__class__ is not np.ndarray or a.dtype not in _TYPES:
                    return None
                base = _owner(a)
                if base is None:
                    return None
                e = _REG.entry(base)
                if e is None or e[3] is None:
                    return None
                rows.append((a, _CODE[dt], int(it[2]) if len(it) > 2 and dt is torch.int32 else 0, e[1], e[2], e[3]))
            if _FN[0] is None:
                _FN[0] = C.cast(L.lib().tm_stage_cast, C.c_void_p).value
            r = ext.stage_host(rows, device.index, _FN[0])
            if r is None:
                return None
            L.check(r[1], "stage host arrays")
            return r[0]
    return _stage_py(device, items, stream)


def _stage_py(device, items, stream=None):
    addrs = []
    for a, dt, *_ in items:
        if a.__class__ is not np.ndarray or a.dtype not in _TYPES or dt not in _DST or a.ndim > 5:
            return None
        base = _owner(a)
        if base is None:
            return None
        e = _REG.entry(base)
        if e is None or e[3] is None:
            return None
        # the bytes the view spans must lie in the registered pages
        p = a.__array_interface__["data"][0]
        lo = hi = p
        for n, st in zip(a.shape, a.strides):
            if n == 0:
                return None
            lo += min(0, (n - 1) * st)
            hi += max(0, (n - 1) * st)
        if lo < e[1] or hi + a.itemsize > e[1] + e[2]:
            return None
        addrs.append(e[3] + (p - e[1]))
    offs, tot = [], 0
    for a, dt, *_ in items:
        offs.append(tot)
        tot += (int(a.size) * _DST[dt][1] + 15) & ~15
    if stream is None:
        buf = torch.empty(max(tot, 16), dtype=torch.uint8, device=device)
        raw = torch._C._cuda_getCurrentRawStream(device.index)
    else:
        with torch.cuda.stream(stream):
            buf = torch.empty(max(tot, 16), dtype=torch.uint8, device=device)
        raw = stream.cuda_stream
    p0 = buf.data_ptr()
    # tm_stage_job rows as int64 words: src, dst, src_type | dst_type << 32, ndim, shape[5], stride[5] (bytes)
    jobs = np.zeros((len(items), 14), dtype=np.int64)
    for i, (it, src, o) in enumerate(zip(items, addrs, offs)):
        a, dt = it[0], it[1]
        r = jobs[i]
        r[0], r[1] = src, p0 + o
        r[2] = _TYPES[a.dtype] | (_DST[dt][0] << 32)
        if a.ndim:
            r[3] = a.ndim | ((int(it[2]) if len(it) > 2 and dt is torch.int32 else 0) << 32)
            r[4:4 + a.ndim] = a.shape
            r[9:9 + a.ndim] = a.strides
        else:
            r[3], r[4] = 1, 1
    L.check(L.lib().tm_stage_cast(jobs.__array_interface__["data"][0], len(items), raw), "stage host arrays")
    return [buf[o:o + int(it[0].size) * _DST[it[1]][1]].view(it[1]).view(it[0].shape) for it, o in zip(items, offs)]


__all__ = ["stage", "window_bounds", "MIN_BYTES", "CAP_BYTES"]
