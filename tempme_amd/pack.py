"""The reference's on-disk handoff between preprocessing and the explainer loop.

Files (processed/data_preprocess.py:139-143, :393-404, :416-419):

* ``{data}_{mode}.h5``      subgraph_{src,tgt,bgd}_0 [n, 3N] (node | eid | ts), subgraph_*_1 [n, 3N^2],
                            walks_{src,tgt,bgd} [n, W, 15] (6 node, 3 eid, 3 ts, 3 anony), dst_fake [n]
* ``{data}_{mode}_cat.h5``  the same subgraphs and dst_fake, walks_*_new [n, W, 14] (6 node, 3 eid, 3 ts,
                            cat id, marginal) instead of walks_*
* ``{data}_{mode}_edge.npy`` [3, n, W, 3, 3] edge-occurrence counts

every array float64, as the reference's h5py round trip leaves them.  Readers mirror
utils/batch_loader.py: ``load_subgraph`` (:45-116), ``load_subgraph_margin`` (:119-197), ``get_item``
(:200-235), ``get_item_edge`` (:238-242) -- same argument order, same tuple nesting, same dtypes
(``.astype(int)`` on node/eid/cat columns, float64 ts / marginal).

Container: HDF5 through h5py when it is importable; this image has no h5py (nor libhdf5), so the
writer then stores the same dataset names / shapes / dtypes in an ``.npz`` container under the
reference's file name.  ``open_pack`` sniffs the magic bytes, so either container reads back, and
``file[name][:]`` (what the reference's loaders do) works on both.

``DevicePack`` is the MI355X side: a pack (from a file or from ``preprocess.pre_processing`` /
``sample_events`` output) uploaded once into the side-major device layout of
``preprocess.EventBuffers``, which ``train.batch_from_pack`` and the scoring pipeline slice without
host round trips.
"""
import os
import zipfile

import numpy as np
import torch

from .preprocess import SIDES, EventBuffers, anony_from_cat

SUBGRAPH_KEYS = tuple(f"subgraph_{s}_{h}" for s in SIDES for h in (0, 1))
RAW_KEYS = SUBGRAPH_KEYS + tuple(f"walks_{s}" for s in SIDES) + ("dst_fake",)       # data_preprocess.py:139
CAT_KEYS = SUBGRAPH_KEYS + tuple(f"walks_{s}_new" for s in SIDES) + ("dst_fake",)   # :393-402
_HDF5_MAGIC = b"\x89HDF\r\n\x1a\n"


def _h5py():
    try:
        import h5py
        return h5py
    except ImportError:
        return None


def write_pack(path, arrays, keys=None):
    """hf.create_dataset(name, data=...) for every key (data_preprocess.py:139-143), float64."""
    keys = tuple(arrays) if keys is None else keys
    missing = [k for k in keys if k not in arrays]
    if missing:
        raise KeyError(f"pack is missing {missing}")
    data = {k: np.asarray(arrays[k], dtype=np.float64) for k in keys}
    h5 = _h5py()
    if h5 is not None:
        with h5.File(path, "w") as hf:
            for k in keys:
                hf.create_dataset(k, data=data[k])
        return path
    with open(path, "wb") as fh:              # keep the reference's file name (np.savez would add .npz)
        np.savez(fh, **data)
    return path


class _NpzPack:
    """h5py.File-like read view of an .npz pack: ``f[name][:]``, ``keys()``, ``close()``, context manager."""

    def __init__(self, path):
        self._z = np.load(path, allow_pickle=False)

    def __getitem__(self, k):
        return self._z[k]

    def __contains__(self, k):
        return k in self._z.files

    def keys(self):
        return list(self._z.files)

    def close(self):
        self._z.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def open_pack(path, mode="r"):
    """``h5py.File(path, 'r')`` of temp_exp_main.py:705-706 for either container."""
    if mode != "r":
        raise ValueError("open_pack is read-only; use write_pack")
    with open(path, "rb") as fh:
        magic = fh.read(8)
    if magic == _HDF5_MAGIC:
        h5 = _h5py()
        if h5 is None:
            raise ImportError(f"{path} is HDF5 and h5py is not importable here")
        return h5.File(path, "r")
    if magic[:2] == b"PK" and zipfile.is_zipfile(path):
        return _NpzPack(path)
    raise ValueError(f"{path}: neither an HDF5 nor an npz pack")


def _split_cols(a, n):
    return a[..., 0:n], a[..., n:2 * n], a[..., 2 * n:3 * n]


def _subgraph(file, side, n_degree, batch_id=None):
    recs = ([], [], [])
    for h, width in ((0, n_degree), (1, n_degree ** 2)):
        a = file[f"subgraph_{side}_{h}"][:]
        if batch_id is not None:
            a = a[batch_id]
        for r, c in zip(recs, _split_cols(a, width)):
            r.append(c)
    return recs


def load_subgraph(args, file, batch_id):
    """utils/batch_loader.py:45-116: one batch of a ``{data}_{mode}.h5`` pack (raw walks, anony codes)."""
    subs = [_subgraph(file, s, args.n_degree, batch_id) for s in SIDES]
    walks = []
    for s in SIDES:
        w = file[f"walks_{s}"][:][batch_id]
        walks.append((w[:, :, :6].astype(int), w[:, :, 6:9].astype(int), w[:, :, 9:12], w[:, :, 12:15].astype(int)))
    return (*subs, *walks)


def load_subgraph_margin(args, file, device=None):
    """utils/batch_loader.py:119-197: the whole ``{data}_{mode}_cat.h5`` pack ->
    (subgraph_src, subgraph_tgt, subgraph_bgd, walks_src, walks_tgt, walks_bgd, dst_fake).

    ``device`` (MI355X extension, default None = the reference's host arrays): upload the pack once into a
    ``DevicePack``; ``get_item`` then hands out device views in the same tuple layout, so the eval / training
    loop's per-batch slicing and TempME's inputs stay on the GPU."""
    if device is not None:
        return DevicePack(file, None, args.n_degree, device)
    subs = [_subgraph(file, s, args.n_degree) for s in SIDES]
    walks = []
    for s in SIDES:
        w = file[f"walks_{s}_new"][:]
        walks.append((w[:, :, :6].astype(int), w[:, :, 6:9].astype(int), w[:, :, 9:12], w[:, :, 12:13].astype(int),
                      w[:, :, 13:14]))
    return (*subs, *walks, file["dst_fake"][:])


def _as_slice(batch_id, n):
    """A contiguous ascending index array (the eval loop's np.arange(s, e)) as the equivalent slice: the
    rows come back as views instead of fancy-indexing copies (same values; the callers only read them).
    Out-of-range ids keep the array, so fancy indexing raises the reference's IndexError."""
    if isinstance(batch_id, np.ndarray) and batch_id.ndim == 1 and batch_id.size > 1 and \
            np.issubdtype(batch_id.dtype, np.integer) and batch_id[0] >= 0 and batch_id[-1] < n and \
            int(batch_id[-1]) - int(batch_id[0]) + 1 == batch_id.size and bool((np.diff(batch_id) == 1).all()):
        return slice(int(batch_id[0]), int(batch_id[-1]) + 1)
    return batch_id


def get_item(input_pack, batch_id):
    """utils/batch_loader.py:200-235 (a ``DevicePack``: its device views, ``DevicePack.get_item``)."""
    if isinstance(input_pack, DevicePack):
        return input_pack.get_item(batch_id)
    *subs, ws, wt, wb, dst_fake = input_pack
    batch_id = _as_slice(batch_id, len(dst_fake))
    out = []
    for node_records, eidx_records, t_records in subs:
        out.append(([i[batch_id] for i in node_records], [i[batch_id] for i in eidx_records],
                    [i[batch_id] for i in t_records]))
    for w in (ws, wt, wb):
        out.append(tuple(item[batch_id] for item in w))
    out.append(dst_fake[batch_id])
    return tuple(out)


def get_item_edge(edge_features, batch_id):
    """utils/batch_loader.py:238-242: [3, n, W, 3, 3] -> (src_edge, tgt_edge, bgd_edge).  A device tensor
    (``load_edge(..., device)``) or a ``DevicePack`` built with its edge counts gives device views."""
    if isinstance(edge_features, DevicePack):
        edge_features = edge_features.cnt
    if isinstance(edge_features, torch.Tensor):
        sl = _dev_index(batch_id, edge_features.shape[1], edge_features.device)
        grid = getattr(edge_features, "_tm_grid", None)
        if isinstance(sl, slice) and grid is not None:
            n = sl.stop - sl.start
            if not grid and n > 0:   # views of every batch on the first batch size's grid, as DevicePack.get_item
                nb = edge_features.shape[1] // n
                per = [[_resident(v) for v in edge_features[s].split(n, dim=0)][:nb] for s in range(3)]
                grid[:] = [n, [tuple(per[s][k] for s in range(3)) for k in range(nb)]]
            if n == grid[0] and sl.start % n == 0:
                return grid[1][sl.start // n]
        e = edge_features[:, sl]
        return tuple(_resident(e[s]) for s in range(3))
    e = edge_features[:, _as_slice(batch_id, np.shape(edge_features)[1]), :, :, :]
    return e[0], e[1], e[2]


def load_edge(edge, device):
    """``np.load({data}_{mode}_edge.npy)`` uploaded once as float32 [3, n, W, 3, 3] for ``get_item_edge``."""
    t = torch.from_numpy(np.ascontiguousarray(np.asarray(edge), dtype=np.float32)).to(device)
    t._tm_grid = []   # get_item_edge's per-batch views, made on first use
    return t


def _resident(t):
    """Mark a device view as resident pack data (written once at upload, never by the caller's pending
    work), so TempME's eval forward may read it from a side stream without waiting for the caller's."""
    t._tm_resident = True
    return t


def _dev_index(batch_id, n, device):
    sl = _as_slice(np.asarray(batch_id) if not isinstance(batch_id, slice) else batch_id, n)
    if isinstance(sl, slice):
        return sl
    idx = np.asarray(sl)
    if idx.size and (idx.min() < -n or idx.max() >= n):
        raise IndexError(f"index {int(idx.max())} is out of bounds for axis 0 with size {n}")
    return torch.from_numpy(idx.astype(np.int64)).to(device)


# ---------------------------------------------------------------------------------- device side
def buffers_to_arrays(buf, n=None):
    """EventBuffers (device, side-major) -> the float64 arrays of both H5 files and the edge .npy:
    (raw dict of ``{data}_{mode}.h5``, cat dict of ``{data}_{mode}_cat.h5``, edge [3, n, W, 3, 3])."""
    n = buf.E if n is None else n
    h = lambda t: t[:, :n].cpu().numpy()  # noqa: E731
    raw = {"dst_fake": buf.dst_fake[:n].cpu().numpy().astype(np.float64)}
    cat_d = {"dst_fake": raw["dst_fake"]}
    cat = h(buf.cat)
    freq = np.bincount(cat.reshape(-1), minlength=12).astype(np.float64) / max(cat.size, 1)  # marginal :180-208
    an = anony_from_cat(cat)
    s1 = [h(buf.sub1_node), h(buf.sub1_eid), h(buf.sub1_ts)]
    s2 = [h(buf.sub2_node), h(buf.sub2_eid), h(buf.sub2_ts)]
    n6, e3, t3 = h(buf.node6), h(buf.eid3), h(buf.ts3)
    for s, side in enumerate(SIDES):
        raw[f"subgraph_{side}_0"] = cat_d[f"subgraph_{side}_0"] = np.concatenate(
            [x[s] for x in s1], -1).astype(np.float64)
        raw[f"subgraph_{side}_1"] = cat_d[f"subgraph_{side}_1"] = np.concatenate(
            [x[s] for x in s2], -1).astype(np.float64)
        base = np.concatenate([n6[s], e3[s], t3[s]], -1).astype(np.float64)
        raw[f"walks_{side}"] = np.concatenate([base, an[s]], -1)
        cat_d[f"walks_{side}_new"] = np.concatenate([base, cat[s][..., None], freq[cat[s]][..., None]], -1)
    return raw, cat_d, h(buf.cnt).astype(np.float64)


def write_split(buf, out_dir, data, mode, n=None):
    """The three files data_preprocess.py:364-420 writes for one (data, MODE), from one sample_events
    launch's EventBuffers.  Returns their paths."""
    raw, cat_d, edge = buffers_to_arrays(buf, n)
    p_raw = write_pack(os.path.join(out_dir, f"{data}_{mode}.h5"), raw, RAW_KEYS)
    p_cat = write_pack(os.path.join(out_dir, f"{data}_{mode}_cat.h5"), cat_d, CAT_KEYS)
    p_edge = os.path.join(out_dir, f"{data}_{mode}_edge.npy")
    np.save(p_edge, edge)
    return p_raw, p_cat, p_edge


class DevicePack(EventBuffers):
    """A ``_cat.h5`` pack + ``_edge.npy`` resident on the device in EventBuffers' layout
    ([3, n, ...] int32 / float32), i.e. what ``load_subgraph_margin`` + ``get_item`` + ``get_item_edge``
    hand the training loop, without per-batch host copies."""

    def __init__(self, file, edge, n_degree, device, walks_per_slot=3):
        """``edge`` (the ``_edge.npy`` array) may be None: ``get_item_edge`` then reads a separate
        ``load_edge`` tensor and ``cnt`` stays zero."""
        dst_fake = np.asarray(file["dst_fake"][:])
        n, N = int(dst_fake.shape[0]), int(n_degree)
        w0 = np.asarray(file["walks_src_new"][:])
        if w0.shape[1] % N:
            raise AssertionError(f"walks per side {w0.shape[1]} is not a multiple of n_degree {N}")
        super().__init__(n, N, w0.shape[1] // N if w0.shape[1] else walks_per_slot, device)
        if edge is not None:
            edge = np.asarray(edge)
            if edge.shape != (3, n, self.W, 3, 3):
                raise AssertionError(f"edge counts {edge.shape} != (3, {n}, {self.W}, 3, 3)")
        self.marg = torch.zeros(3, n, self.W, dtype=torch.float32, device=device)
        i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).astype(np.int32))  # noqa: E731
        f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).astype(np.float32))  # noqa: E731
        self.dst_fake.copy_(i32(dst_fake))
        for s, side in enumerate(SIDES):
            for h, (nd, ed, td) in ((0, (self.sub1_node, self.sub1_eid, self.sub1_ts)),
                                    (1, (self.sub2_node, self.sub2_eid, self.sub2_ts))):
                x, y, z = _split_cols(np.asarray(file[f"subgraph_{side}_{h}"][:]), N ** (h + 1))
                nd[s].copy_(i32(x))
                ed[s].copy_(i32(y))
                td[s].copy_(f32(z))
            w = np.asarray(w0 if s == 0 else file[f"walks_{side}_new"][:])
            self.node6[s].copy_(i32(w[:, :, :6]))
            self.eid3[s].copy_(i32(w[:, :, 6:9]))
            self.ts3[s].copy_(f32(w[:, :, 9:12]))
            self.cat[s].copy_(i32(w[:, :, 12]))
            self.marg[s].copy_(f32(w[:, :, 13]))
            if edge is not None:
                self.cnt[s].copy_(f32(edge[s]))
        self.hist.copy_(torch.bincount(self.cat.reshape(-1).long().cpu(), minlength=12))

    def __len__(self):
        return self.E

    def get_item(self, batch_id):
        """get_item (utils/batch_loader.py:200-235) on the device: the same tuple nesting -- per side
        ([hop-1, hop-2] node, [..] eid, [..] ts), per side (node [B,W,6], eid [B,W,3], ts [B,W,3],
        cat [B,W,1], marginal [B,W,1]), dst_fake [B] -- as int32 / float32 device views.  A batch on the
        grid of the batch size seen first (the eval loop's np.arange(k * bs, (k + 1) * bs)) comes from views
        of every batch made at once (torch.split, one call per array): the same view objects per batch."""
        sl = _dev_index(batch_id, self.E, self.dst_fake.device)
        if isinstance(sl, slice):
            n = sl.stop - sl.start
            grid = self.__dict__.get("_grid")
            if grid is None and n > 0:
                grid = self._grid = (n, self._split_views(n))
            if grid is not None and n == grid[0] and sl.start % n == 0:
                return grid[1][sl.start // n]
        r = _resident
        out = []
        for s in range(3):
            out.append(([r(self.sub1_node[s, sl]), r(self.sub2_node[s, sl])],
                        [r(self.sub1_eid[s, sl]), r(self.sub2_eid[s, sl])],
                        [r(self.sub1_ts[s, sl]), r(self.sub2_ts[s, sl])]))
        for s in range(3):
            out.append((r(self.node6[s, sl]), r(self.eid3[s, sl]), r(self.ts3[s, sl]),
                        r(self.cat[s, sl].unsqueeze(-1)), r(self.marg[s, sl].unsqueeze(-1))))
        out.append(r(self.dst_fake[:self.E][sl]))
        return tuple(out)

    def _split_views(self, B):
        """get_item's tuple for every batch [k B, (k + 1) B) that fits, from one torch.split per array."""
        def sp(t):
            return [_resident(v) for v in t[:self.E].split(B, dim=0)][:self.E // B]
        s1n, s1e, s1t, s2n, s2e, s2t, n6, e3, t3, ct, mg = (
            [sp(a[s]) for s in range(3)] for a in (self.sub1_node, self.sub1_eid, self.sub1_ts, self.sub2_node,
                                                   self.sub2_eid, self.sub2_ts, self.node6, self.eid3, self.ts3,
                                                   self.cat.unsqueeze(-1), self.marg.unsqueeze(-1)))
        df = sp(self.dst_fake)
        out = []
        for k in range(self.E // B):
            subs = tuple(([s1n[s][k], s2n[s][k]], [s1e[s][k], s2e[s][k]], [s1t[s][k], s2t[s][k]]) for s in range(3))
            walks = tuple((n6[s][k], e3[s][k], t3[s][k], ct[s][k], mg[s][k]) for s in range(3))
            out.append((*subs, *walks, df[k]))
        return out

    @classmethod
    def from_files(cls, cat_path, edge_path, n_degree, device):
        with open_pack(cat_path) as f:
            return cls(f, np.load(edge_path, allow_pickle=False), n_degree, device)
