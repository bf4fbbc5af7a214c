"""TEST INFRASTRUCTURE ONLY -- torch CPU restatement of the base TGN's contrast with explanation weights.

Functional restatement (no nn.Module, literal operation order: per-neighbour key/value
projections, softmax then explanation weight, no folding) of dharunm236/TempME:
  TGN.get_node_emb / contrast        TGN/tgn.py:99-218   (forbidden_memory_update=True path)
  get_updated_memory                 TGN/tgn.py:237-248, message_aggregator.py:36-52 ("last"),
                                     message_function.py:13-25 ("mlp"), memory_updater.py:30-58 (GRU)
  embedding_update / _attr / _layer  TGN/modules/embedding_module.py:314-393
  retrieve_time_features             :297-311   (f64 deltas cast to f32, TimeEncode :100-112)
  TemporalAttentionLayer             :181-216   (mask .repeat(n_head,1,1): head-major row pairing)
  MultiHeadAttention                 :52-86     (explain weight .repeat(n_head,1,1))
  ScaledDotProductAttention          :16-32
  threshold_test (tgn branch)        temp_exp_main.py:153-272
Eval semantics (dropout = identity).  `dtype=torch.float64` evaluates the same graph in double
precision: the tests use it to measure the reference's own fp32 rounding envelope.
Pinned against tests/golden/tgn_uslegis.npz (outputs of the reference TGN, make_goldens.py case_tgn).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


def _t(x, dtype):
    if isinstance(x, torch.Tensor):
        return x.to(dtype)
    return torch.as_tensor(np.asarray(x)).to(dtype)


def _lin(sd, name, x, bias=True):
    w = sd[name + ".weight"].to(x.dtype)
    b = sd[name + ".bias"].to(x.dtype) if bias else None
    return F.linear(x, w, b)


def time_encode(sd, t):
    """TimeEncode: Linear(1, d) then cos (embedding_module.py:108-112).  torch's CPU addmm with K=1
    rounds t*w+b once to fp32 (an fma); that rounding is kept at every `dtype` because cos of a large
    argument depends on it, and the fp64 mode is meant to remove arithmetic error, not change inputs."""
    w = sd["time_encoder.w.weight"].reshape(-1)
    b = sd["time_encoder.w.bias"]
    arg = (t.double().unsqueeze(-1) * w.double() + b.double()).float()
    return torch.cos(arg.double()).to(t.dtype)


def updated_memory(sd, messages, n_nodes, dtype=torch.float32, aggregator="last"):
    """get_updated_memory over all nodes (tgn.py:237-248): the stored raw messages of each node
    reduced by the aggregator, the message MLP, then one GRUCell step from the stored memory."""
    mem = sd["memory.memory"].to(dtype).clone()
    nodes = [n for n in sorted(messages) if len(messages[n]) > 0 and n < n_nodes]
    if not nodes:
        return mem
    if aggregator == "last":
        raw = torch.stack([_t(messages[n][-1][0], dtype) for n in nodes])
    else:
        raw = torch.stack([torch.stack([_t(m[0], dtype) for m in messages[n]]).mean(0) for n in nodes])
    msg = _lin(sd, "message_function.mlp.2", F.relu(_lin(sd, "message_function.mlp.0", raw)))
    h = mem[nodes]
    wih, whh = sd["memory_updater.memory_updater.weight_ih"].to(dtype), sd["memory_updater.memory_updater.weight_hh"].to(dtype)
    bih, bhh = sd["memory_updater.memory_updater.bias_ih"].to(dtype), sd["memory_updater.memory_updater.bias_hh"].to(dtype)
    gi = F.linear(msg, wih, bih)
    gh = F.linear(h, whh, bhh)
    ir, iz, inn = gi.chunk(3, 1)
    hr, hz, hn = gh.chunk(3, 1)
    r = torch.sigmoid(ir + hr)
    z = torch.sigmoid(iz + hz)
    n = torch.tanh(inn + r * hn)
    mem[nodes] = (h - n) * z + n
    return mem


def attention_layer(sd, pre, n_head, src_feat, src_time, ngh_feat, ngh_time, edge_feat, mask, explain_weight):
    """TemporalAttentionLayer.forward (embedding_module.py:181-216), literal."""
    query = torch.cat([src_feat.unsqueeze(1), src_time], dim=2)               # [B,1,dq]
    key = torch.cat([ngh_feat, edge_feat, ngh_time], dim=2)                   # [B,N,dk]
    attn_mask = mask.unsqueeze(1).repeat(n_head, 1, 1)                        # head-major (:211-212)
    mh = pre + "multi_head_target."
    B, _, dq = query.shape
    N, dk = key.shape[1], key.shape[2]
    q = _lin(sd, mh + "w_qs", query, bias=False).view(B, 1, 1, n_head, dk).transpose(2, 3).reshape(B * n_head, 1, dk)
    k = _lin(sd, mh + "w_ks", key, bias=False).view(B, 1, N, n_head, dk).transpose(2, 3).reshape(B * n_head, N, dk)
    v = _lin(sd, mh + "w_vs", key, bias=False).view(B, 1, N, n_head, dk).transpose(2, 3).reshape(B * n_head, N, dk)
    ew = None if explain_weight is None else explain_weight.reshape(B, 1, N).repeat(n_head, 1, 1)
    attn = torch.bmm(q, k.transpose(-1, -2)) / math.sqrt(dk)
    attn = attn.masked_fill(attn_mask, -1e10)
    attn = torch.softmax(attn, dim=2)
    if ew is not None:
        attn = attn * ew
    out = torch.bmm(attn, v).view(B, 1, n_head * dk)
    out = _lin(sd, mh + "fc", out)
    out = F.layer_norm(out + query, (dq,), sd[mh + "layer_norm.weight"].to(out.dtype),
                       sd[mh + "layer_norm.bias"].to(out.dtype), 1e-5).squeeze(1)
    x = torch.cat([out, src_feat], dim=1)
    return _lin(sd, pre + "merger.fc2", F.relu(_lin(sd, pre + "merger.fc1", x)))


def node_embeddings(sd, memory, n_feat, e_feat, node_list, edge_list, time_list, cut_time, n_neighbors, n_head=2,
                    explain_weights=None, edge_attr=None, dtype=torch.float32):
    """embedding_update(_attr) + embedding_update_layer (embedding_module.py:314-393) -> [3B, d]."""
    N = n_neighbors
    nodes = [_t(x, torch.long) for x in node_list]
    feats = [n_feat.to(dtype)[x] for x in nodes]
    masks = [x == 0 for x in nodes]
    if edge_attr is None:
        efeats = [e_feat.to(dtype)[_t(x, torch.long)] for x in edge_list]
    else:
        efeats = [_t(x, dtype) for x in edge_attr]
    # retrieve_time_features (:297-311): numpy f64 deltas, then .float()
    cut3 = np.concatenate([cut_time, cut_time, cut_time]).astype(np.float64)
    batch = len(cut3)
    std = cut3[:, None, None]
    tfeats = []
    for t_rec in time_list:
        t_rec = np.asarray(t_rec)
        delta = (std - t_rec.reshape(batch, -1, N)).reshape(batch, -1)
        tfeats.append(time_encode(sd, torch.from_numpy(np.asarray(delta, dtype=np.float64)).float().to(dtype)))
        std = np.expand_dims(t_rec, 2)
    mem = memory.to(dtype) if memory is not None else None
    ngh = feats[-1].reshape(-1, feats[-1].shape[-1])
    if mem is not None:
        ngh = mem[nodes[-1].flatten()] + ngh
    L = len(nodes)
    for i in range(L - 1):
        t = L - 1 - i
        src = feats[t - 1].reshape(-1, feats[t - 1].shape[-1])
        R = src.shape[0]
        if mem is not None:
            src = mem[nodes[t - 1].flatten()] + src
        src_time = time_encode(sd, torch.zeros((R, 1), dtype=dtype))
        ew = None if explain_weights is None else _t(explain_weights[t - 1], dtype).reshape(R, -1)
        ngh = attention_layer(sd, f"embedding_module.attention_models.{i}.", n_head, src, src_time,
                              ngh.reshape(R, N, -1), tfeats[t - 1].reshape(R, N, -1),
                              efeats[t - 1].reshape(R, N, -1), masks[t].reshape(R, -1), ew)
    return ngh


def contrast(sd, messages, n_feat, e_feat, src_idx, tgt_idx, bgd_idx, cut_time, subgraph_src, subgraph_tgt,
             subgraph_bgd, n_neighbors, n_head=2, explain_weights=None, edge_attr=None, use_memory=True,
             dtype=torch.float32):
    """TGN.contrast (tgn.py:201-218) -> (pos [B,1], neg [B,1])."""
    n_feat = _t(n_feat, dtype)
    e_feat = _t(e_feat, dtype)
    B = len(src_idx)
    node_list = [np.concatenate([src_idx, tgt_idx, bgd_idx])[:, None]]
    node_list += [np.concatenate([subgraph_src[0][h], subgraph_tgt[0][h], subgraph_bgd[0][h]], axis=0) for h in (0, 1)]
    edge_list = [np.concatenate([subgraph_src[1][h], subgraph_tgt[1][h], subgraph_bgd[1][h]], axis=0) for h in (0, 1)]
    time_list = [np.concatenate([subgraph_src[2][h], subgraph_tgt[2][h], subgraph_bgd[2][h]], axis=0) for h in (0, 1)]
    mem = updated_memory(sd, messages, n_feat.shape[0], dtype) if use_memory else None
    emb = node_embeddings(sd, mem, n_feat, e_feat, node_list, edge_list, time_list, np.asarray(cut_time),
                          n_neighbors, n_head, explain_weights, edge_attr, dtype)
    s, d, n = emb[:B], emb[B:2 * B], emb[2 * B:]
    x = torch.cat([torch.cat([s, s], 0), torch.cat([d, n], 0)], dim=1)
    score = _lin(sd, "affinity_score.fc2", F.relu(_lin(sd, "affinity_score.fc1", x)))
    return score[:B], score[B:]


def select_k_smallest(imp, k):
    """threshold_test's torch.topk(imp, k, largest=False).indices on the CPU (:166-168): the
    reference op itself.  Which of several tied entries it picks is libstdc++'s std::nth_element /
    std::partial_sort order over (value, index) pairs (ATen TopKImpl.h)."""
    return torch.topk(torch.as_tensor(np.asarray(imp)), k=k, dim=-1, largest=False).indices.numpy()


def masked_subgraph(subgraph, sel, n_deg):
    """threshold_test's np.put_along_axis(..., 0) on the hop-1|hop-2 node records (:170-174)."""
    nodes, eids, ts = subgraph
    cat = np.concatenate(nodes, axis=-1).copy()
    np.put_along_axis(cat, sel, 0, axis=-1)
    return list(np.split(cat, [n_deg], axis=1)), eids, ts
