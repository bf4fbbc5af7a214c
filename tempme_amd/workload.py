"""Synthetic inputs of BASELINE.json's configs: no dataset downloads exist,
so graphs are seeded synthetic replicas of the named shapes.

enron_like(): config 2 'enron_sampled' -- V=183 nodes (ids 1..V, 0 is padding), E=18,780 edges,
timestamps sorted uniform ints on [0, 1e8), endpoints drawn from Pareto(alpha) node weights,
no self-loops, idx = row + 1, edge features U(0,1) (de=32), node features zeros (dn=172).
split(): the train/val/test split and masks of temp_exp_main.py:101-150.
"""
import random

import numpy as np


def enron_like(n_nodes=183, n_edges=18780, alpha=1.2, de=32, dn=172, seed=0, node_feat="zeros"):
    rng = np.random.RandomState(seed)
    w = rng.pareto(alpha, n_nodes) + 1.0
    p = w / w.sum()
    src = rng.choice(n_nodes, n_edges, p=p) + 1
    dst = rng.choice(n_nodes, n_edges, p=p) + 1
    loop = src == dst
    while loop.any():
        dst[loop] = rng.choice(n_nodes, int(loop.sum()), p=p) + 1
        loop = src == dst
    ts = np.sort(rng.randint(0, 10 ** 8, n_edges)).astype(np.float64)
    eidx = np.arange(1, n_edges + 1, dtype=np.int64)
    e_feat = rng.uniform(0, 1, (n_edges + 1, de)).astype(np.float32)
    e_feat[0] = 0
    if node_feat == "zeros":
        n_feat = np.zeros((n_nodes + 1, dn), np.float32)
    else:
        n_feat = rng.uniform(0, 1, (n_nodes + 1, dn)).astype(np.float32)
        n_feat[0] = 0
    return dict(src=src.astype(np.int64), dst=dst.astype(np.int64), ts=ts, eidx=eidx, label=np.zeros(n_edges),
                e_feat=e_feat, n_feat=n_feat, n_nodes=n_nodes + 1)


def split(g, mode="test"):
    """temp_exp_main.load_data (:101-150) on in-memory edge arrays.  Returns
    (src, dst, ts, eidx) of the split, the edge rows of its graph, and the sampler's dst pool."""
    src, dst, ts, eidx = g["src"], g["dst"], g["ts"], g["eidx"]
    val_time, test_time = list(np.quantile(ts, [0.70, 0.85]))
    rnd = random.Random(2023)
    total = set(np.unique(np.hstack([src, dst])))
    late = ts > val_time
    temp_val = list(set(src[late]).union(set(dst[late])))
    mask = set(rnd.sample(temp_val, int(0.1 * len(total))))
    ms = np.array([x in mask for x in src])
    md = np.array([x in mask for x in dst])
    none_node = (1 - ms) * (1 - md)
    tr = (ts <= val_time) * (none_node > 0)
    va = (ts <= test_time) * (ts > val_time)
    te = ts > test_time
    if mode == "test":
        sel, graph_rows = te, np.ones(len(ts), bool)
        dst_pool = np.unique(np.concatenate([dst[tr], dst[va], dst[te]]))
    else:
        sel, graph_rows = tr, tr
        dst_pool = np.unique(dst[tr])
    return (src[sel], dst[sel], ts[sel], eidx[sel]), graph_rows, dst_pool
