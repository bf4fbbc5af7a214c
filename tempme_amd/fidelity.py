"""Fidelity evaluation of an explanation on the base model: ``threshold_test``
(temp_exp_main.py:153-272, tgn and graphmixer branches) on the HIP device.

For each sparsity ratio the reference keeps the top ``ceil(ratio * (N + N^2))`` subgraph entries by
explanation score, zeroes the node ids of the rest (torch.topk(largest=False) + np.put_along_axis),
re-runs ``contrast`` without explanation weights and scores the result against the original
predictions (AP, AUC, accuracy, fidelity of probabilities and logits), then averages over ratios.

Here the masks of all ratios come from one launch of ``mask_least_kernel`` (tm_mask_least_important,
which reproduces the CPU top-k's tie order), and all ratios go through ONE batched contrast
(``TGN.node_embeddings(..., n_segments=len(ratios))``) instead of one call per ratio.  AP and AUC
are computed with scikit-learn on the host, as the reference does, from the 2B predictions per ratio.
"""
import math

import numpy as np
import torch
from sklearn.metrics import average_precision_score, roc_auc_score

from . import _lib as L
from .tgn import _as_dev


def _masked_nodes(explanation, subgraphs, N, ratios, dev, hops=2):
    """[G, 3B, ne] int32 node records with the least important entries of each ratio set to 0;
    hops=2: [hop-1 | hop-2] records, ne = N + N^2 (tgn / tgat branches); hops=1: hop-1 records,
    ne = N (graphmixer branch)."""
    ne = N + N * N if hops == 2 else N
    imp = torch.cat(list(explanation[:hops]), dim=1).to(dev, torch.float32).contiguous()
    nodes = torch.cat([torch.cat([_as_dev(sg[0][h], dev, torch.int32) for h in range(hops)], dim=1)
                       for sg in subgraphs], dim=0).contiguous()
    rows = nodes.shape[0]
    if imp.shape != (rows, ne):
        raise AssertionError(f"explanation rows {tuple(imp.shape)} do not match the subgraphs ({rows}, {ne})")
    ks = [ne - min(max(math.ceil(r * ne), 1), ne) for r in ratios]      # temp_exp_main.py:158-168
    k_dev = torch.tensor(ks, dtype=torch.int32, device=dev)
    out = torch.empty((len(ratios), rows, ne), dtype=torch.int32, device=dev)
    L.check(L.lib().tm_mask_least_important(L.ptr(imp), rows, ne, L.ptr(k_dev), len(ratios), L.ptr(nodes),
                                            L.ptr(out), L.stream_ptr(dev)), "threshold_test masks")
    return out


def masked_contrast(base_model, explanation, src_l_cut, dst_l_cut, dst_l_fake, ts_l_cut, subgraph_src, subgraph_tgt,
                    subgraph_bgd, n_degree, ratios):
    """(pos [G, B], neg [G, B]) logits of contrast on the masked subgraph of every ratio."""
    dev = base_model._dev()
    B, N, G = len(src_l_cut), n_degree, len(ratios)
    sgs = (subgraph_src, subgraph_tgt, subgraph_bgd)
    masked = _masked_nodes(explanation, sgs, N, ratios, dev)                          # [G, 3B, ne]
    roots = torch.cat([_as_dev(x, dev, torch.long).reshape(-1) for x in (src_l_cut, dst_l_cut, dst_l_fake)])
    n1 = masked[:, :, :N].reshape(G * 3 * B, N)
    n2 = masked[:, :, N:].reshape(G * 3 * B, N * N)

    def rep(i, h, dtype):
        x = torch.cat([_as_dev(sg[i][h], dev, dtype) for sg in sgs], dim=0)
        return x.repeat(G, 1)
    emb = base_model.node_embeddings([roots.repeat(G), n1, n2], [rep(1, 0, torch.int32), rep(1, 1, torch.int32)],
                                     [rep(2, 0, torch.float64), rep(2, 1, torch.float64)], ts_l_cut, n_segments=G)
    emb = emb.view(G, 3, B, -1)
    s, d, n = emb[:, 0], emb[:, 1], emb[:, 2]
    x1 = torch.cat([s, s], dim=1).reshape(G * 2 * B, -1)
    x2 = torch.cat([d, n], dim=1).reshape(G * 2 * B, -1)
    score = base_model.affinity(x1, x2).view(G, 2 * B)
    return score[:, :B], score[:, B:]


def masked_contrast_graphmixer(base_model, explanation, src_l_cut, dst_l_cut, dst_l_fake, ts_l_cut, subgraph_src,
                               subgraph_tgt, subgraph_bgd, n_degree, ratios):
    """graphmixer branch (temp_exp_main.py:186-206): hop-1 records masked, all ratios in one batch."""
    dev = base_model._dev()
    B, N, G = len(src_l_cut), n_degree, len(ratios)
    sgs = (subgraph_src, subgraph_tgt, subgraph_bgd)
    masked = _masked_nodes(explanation, sgs, N, ratios, dev, hops=1).reshape(G * 3 * B, N)
    roots = torch.cat([_as_dev(x, dev, torch.long).reshape(-1) for x in (src_l_cut, dst_l_cut, dst_l_fake)])
    cut = _as_dev(ts_l_cut, dev, torch.float64).reshape(-1).repeat(3 * G)

    def rep(i, dtype):
        return torch.cat([_as_dev(sg[i][0], dev, dtype) for sg in sgs], dim=0).repeat(G, 1)
    emb = base_model.node_embeddings(roots.repeat(G), cut, masked, rep(1, torch.long), rep(2, torch.float64))
    emb = emb.view(G, 3, B, -1)
    s, d, n = emb[:, 0], emb[:, 1], emb[:, 2]
    x1 = torch.cat([s, s], dim=1).reshape(G * 2 * B, -1)
    x2 = torch.cat([d, n], dim=1).reshape(G * 2 * B, -1)
    score = base_model.affinity(x1, x2).view(G, 2 * B)
    return score[:, :B], score[:, B:]


def threshold_test(args, explanation, base_model, src_l_cut, dst_l_cut, dst_l_fake, ts_l_cut, e_l_cut,
                   pos_out_ori, neg_out_ori, y_ori, subgraph_src, subgraph_tgt, subgraph_bgd):
    """temp_exp_main.py:153-272 -> (aps_AUC, auc_AUC, acc_AUC, fid_prob_AUC, fid_logit_AUC)."""
    fns = {"tgn": masked_contrast, "graphmixer": masked_contrast_graphmixer}
    if args.base_type not in fns:
        raise NotImplementedError(f"threshold_test for base_type {args.base_type!r}: tgn and graphmixer are built")
    with torch.no_grad():
        pos, neg = fns[args.base_type](base_model, explanation, src_l_cut, dst_l_cut, dst_l_fake, ts_l_cut,
                                       subgraph_src, subgraph_tgt, subgraph_bgd, args.n_degree, list(args.ratios))
        po = pos_out_ori.reshape(1, -1).to(pos.device, torch.float32)
        no = neg_out_ori.reshape(1, -1).to(pos.device, torch.float32)
        fid_prob = torch.cat([pos.sigmoid() - po.sigmoid(), no.sigmoid() - neg.sigmoid()], dim=1).mean(1)
        fid_logit = torch.cat([pos - po, no - neg], dim=1).mean(1)
        y_pred = torch.cat([pos, neg], dim=1).sigmoid()
        pred_label = torch.where(y_pred > 0.5, 1., 0.)
        y = y_ori.reshape(1, -1).to(pos.device, torch.float32)
        acc = (pred_label == y).float().mean(1)
        y_pred_h, y_h = y_pred.cpu().numpy(), y_ori.reshape(-1).cpu().numpy()
    aps = [average_precision_score(y_h, p) for p in y_pred_h]
    auc = [roc_auc_score(y_h, p) for p in y_pred_h]
    return (float(np.mean(aps)), float(np.mean(auc)), float(acc.mean().item()), float(fid_prob.mean().item()),
            float(fid_logit.mean().item()))
