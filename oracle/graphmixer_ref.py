"""TEST INFRASTRUCTURE ONLY -- torch CPU restatement of the base GraphMixer's contrast with hop-1
explanation weights (dharunm236/TempME GraphM/graphmixer.py):
  get_node_emb / contrast                 :106-140, :206-218
  compute_node_temporal_embeddings        :142-193  (padding masks, mean over tokens, softmax node agg)
  TimeEncoder                             :21-50    (Linear(1, d) -> cos; CPU addmm rounds t*w+b once)
  MLPMixer / FeedForwardNet               :244-315  (explain weight on input and both branches)
Literal operation order, eval semantics (dropout = identity).
Pinned against tests/golden/graphmixer_uslegis.npz (outputs of the reference, make_goldens.py).
"""
import numpy as np
import torch
import torch.nn.functional as F


def _t(x, dtype):
    if isinstance(x, torch.Tensor):
        return x.to(dtype)
    return torch.as_tensor(np.asarray(x)).to(dtype)


def _lin(sd, name, x):
    return F.linear(x, sd[name + ".weight"].to(x.dtype), sd[name + ".bias"].to(x.dtype))


def _ffn(sd, pre, x):
    return _lin(sd, pre + "ffn.3", F.gelu(_lin(sd, pre + "ffn.0", x)))


def mixer(sd, pre, x, ew):
    if ew is not None:
        x = x * ew.unsqueeze(-1)
    n_tok, n_ch = x.shape[1], x.shape[2]
    h = F.layer_norm(x.permute(0, 2, 1), (n_tok,), sd[pre + "token_norm.weight"].to(x.dtype),
                     sd[pre + "token_norm.bias"].to(x.dtype), 1e-5)
    h = _ffn(sd, pre + "token_feedforward.", h).permute(0, 2, 1)
    if ew is not None:
        h = h * ew.unsqueeze(-1)
    out = h + x
    h = F.layer_norm(out, (n_ch,), sd[pre + "channel_norm.weight"].to(x.dtype), sd[pre + "channel_norm.bias"].to(x.dtype),
                     1e-5)
    h = _ffn(sd, pre + "channel_feedforward.", h)
    if ew is not None:
        h = h * ew.unsqueeze(-1)
    return h + out


def node_embeddings(sd, n_layers, node_ids, cut, nid, eid, times, ew=None, edge_attr=None, dtype=torch.float32):
    """compute_node_temporal_embeddings for one side: [B, d]."""
    nf = sd["n_feat_th"].to(dtype)
    ef_tab = sd["e_feat_th"].to(dtype)
    nid_np = np.asarray(nid)
    nid_t = _t(nid_np, torch.long)
    mask = (nid_t != 0).long()
    if ew is not None:
        ew = _t(ew, dtype) * mask
    ef = ef_tab[_t(eid, torch.long)] if edge_attr is None else _t(edge_attr, dtype).clone()
    delta = np.asarray(cut, dtype=np.float64)[:, None] - np.asarray(times, dtype=np.float64)
    w = sd["time_encoder.w.weight"].reshape(-1).double()
    b = sd["time_encoder.w.bias"].double()
    arg = (torch.from_numpy(delta).float().double().unsqueeze(-1) * w + b).float()
    tf = torch.cos(arg.double()).to(dtype)
    pad = torch.from_numpy(nid_np == 0)
    tf[pad] = 0.0
    if edge_attr is None:
        ef[pad] = 0.0
    x = _lin(sd, "projection_layer", torch.cat([ef, tf], dim=-1))
    for i in range(n_layers):
        x = mixer(sd, f"mlp_mixers.{i}.", x, ew)
    x[pad] = 0.0
    if ew is not None:
        x = x * ew.unsqueeze(-1)
    x = torch.mean(x, dim=1)
    valid = torch.from_numpy((nid_np > 0).astype(np.float32)).to(dtype)
    valid[valid == 0] = -1e10
    scores = torch.softmax(valid, dim=1)
    if ew is not None:
        scores = scores * ew
    agg = torch.mean(nf[nid_t] * scores.unsqueeze(-1), dim=1)
    out = agg + nf[_t(node_ids, torch.long)]
    return _lin(sd, "output_layer", torch.cat([x, out], dim=1))


def contrast(sd, n_layers, src_idx, tgt_idx, bgd_idx, cut_time, subgraph_src, subgraph_tgt, subgraph_bgd,
             explain_weights=None, edge_attr=None, dtype=torch.float32):
    """GraphMixer.contrast -> (pos [B,1], neg [B,1])."""
    B = len(src_idx)
    embs = []
    for k, (nodes, sg) in enumerate(((src_idx, subgraph_src), (tgt_idx, subgraph_tgt), (bgd_idx, subgraph_bgd))):
        ew = None if explain_weights is None else explain_weights[0][k * B:(k + 1) * B]
        ea = None if edge_attr is None else edge_attr[k * B:(k + 1) * B]
        embs.append(node_embeddings(sd, n_layers, nodes, cut_time, sg[0][0], sg[1][0], sg[2][0], ew, ea, dtype))
    s, d, n = embs
    x = torch.cat([torch.cat([s, s], 0), torch.cat([d, n], 0)], dim=1)
    score = _lin(sd, "affinity_score.fc2", F.relu(_lin(sd, "affinity_score.fc1", x)))
    return score[:B], score[B:]
