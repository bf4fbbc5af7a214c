"""Null-model motif distribution (utils/null_model.py), sampled on the device.

``get_null_distribution(data_name)`` restates load_data_shuffle (:13-72): endpoints
shuffled by a keyed permutation (replacing the unseeded ``np.random.permutation``,
:23), event ids and times NOT shuffled (:25-27, the quirk that defines the null
graph), split masks from ``random.seed(2023)`` exactly as the reference computes
them.  pre_processing (:86-121) then samples 500 test events (50 batches of 10) with
one walk per hop-1 slot; the 12-bin histogram is keyed 1..12 in the reference's
order (:90) and normalised by 500 * 3 * N (:119-120).
"""
import os
import random

import numpy as np
import pandas as pd
import torch

from . import _lib as L
from .batch_loader import RandEdgeSampler
from .graph import NeighborFinder
from .preprocess import CAT_TO_NULL, sample_events

degree_dict = {"wikipedia": 20, "reddit": 20, "uci": 30, "mooc": 60, "enron": 30, "enron_sampled": 30,
               "canparl": 30, "uslegis": 30, "uslegis_sampled": 30}


def data_path(data, data_dir=None):
    d = data_dir or os.environ.get("TEMPME_DATA_DIR") or "processed"
    return os.path.join(d, f"ml_{data}.csv")


def keyed_permutation(n, seed, device=None):
    """Stable argsort of one Philox word per position (tm_perm_keys)."""
    dev = L.require_device(device)
    keys = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    L.check(L.lib().tm_perm_keys(seed, L.SPLIT_NULL, n, L.ptr(keys), L.stream_ptr(dev)), "keyed_permutation")
    k = keys[:n].to(torch.int64) & 0xFFFFFFFF
    return torch.argsort(k, stable=True).cpu().numpy()


def load_data_shuffle(mode, data, *, data_dir=None, seed=0, device=None):
    g_df = pd.read_csv(data_path(data, data_dir))
    val_time, test_time = list(np.quantile(g_df.ts, [0.70, 0.85]))
    src_l, dst_l = g_df.u.values, g_df.i.values
    e_idx_l, label_l, ts_l = g_df.idx.values, g_df.label.values, g_df.ts.values
    perm = keyed_permutation(len(ts_l), seed, device)
    src_l, dst_l, label_l = np.array(src_l)[perm], np.array(dst_l)[perm], np.array(label_l)[perm]
    max_idx = max(src_l.max(), dst_l.max())
    rnd = random.Random(2023)                         # == random.seed(2023); random.sample(...)
    total_node_set = set(np.unique(np.hstack([g_df.u.values, g_df.i.values])))
    late = ts_l > val_time
    temp_val = list(set(src_l[late]).union(set(dst_l[late])))
    mask_node_set = set(rnd.sample(temp_val, int(0.1 * len(total_node_set))))
    # the masks are taken on the UNshuffled columns (:37-38)
    mask_src = g_df.u.map(lambda x: x in mask_node_set).values
    mask_dst = g_df.i.map(lambda x: x in mask_node_set).values
    none_node = (1 - mask_src) * (1 - mask_dst)
    train = (ts_l <= val_time) * (none_node > 0)
    val = (ts_l <= test_time) * (ts_l > val_time)
    test = ts_l > test_time
    if mode == "test":
        finder = NeighborFinder.from_edges(src_l, dst_l, e_idx_l, ts_l, max_idx + 1, device=device, seed=seed,
                                           split=L.SPLIT_NULL)
        sampler = RandEdgeSampler((src_l[train], src_l[val], src_l[test]), (dst_l[train], dst_l[val], dst_l[test]),
                                  seed=seed, split=L.SPLIT_NULL, device=device)
        return sampler, src_l[test], dst_l[test], ts_l[test], label_l[test], e_idx_l[test], finder
    finder = NeighborFinder.from_edges(src_l[train], dst_l[train], e_idx_l[train], ts_l[train], max_idx + 1,
                                       device=device, seed=seed, split=L.SPLIT_NULL)
    sampler = RandEdgeSampler((src_l[train],), (dst_l[train],), seed=seed, split=L.SPLIT_NULL, device=device)
    return sampler, src_l[train], dst_l[train], ts_l[train], label_l[train], e_idx_l[train], finder


def null_counts(finder, sampler, src, dst, ts, e_idx, num_neighbors, n_events=500):
    """Integer 12-bin counts (null-model key order) over the first n_events events."""
    dev = finder.device
    n = min(n_events, len(src))
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:n], dtype=dt)).to(dev)  # noqa: E731
    ev = torch.arange(n, dtype=torch.int32, device=dev)
    b = sample_events(finder.graph, finder.seed, L.SPLIT_NULL, int(num_neighbors), 1, t(src, np.int32),
                      t(dst, np.int32), t(ts, np.float64), t(e_idx, np.int32), ev, sampler.dst_device())
    hist = b.hist.cpu().numpy()
    return hist[CAT_TO_NULL]


def get_null_distribution(data_name, *, data_dir=None, seed=0, device=None):
    """utils/null_model.py:124-128 -> {1..12: frequency}."""
    num_neighbors = degree_dict[data_name]
    sampler, src, dst, ts, _, e_idx, finder = load_data_shuffle("test", data_name, data_dir=data_dir, seed=seed,
                                                                device=device)
    cnt = null_counts(finder, sampler, src, dst, ts, e_idx, num_neighbors)
    total = 50 * 10
    return {k + 1: int(cnt[k]) / (total * 3 * num_neighbors) for k in range(12)}
