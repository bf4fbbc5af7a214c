"""TEST INFRASTRUCTURE ONLY -- torch-fp32 CPU restatement of the TempME motif encoder.

Functional restatement (no nn.Module) of models/explainer_new.py:
  forward                 :174-201   (event features, event_gcn x2, attention, cat one-hot, MLP, sigmoid)
  retrieve_time_features  :318-330   (dt relative to walk position 2, TimeEncode :45-59)
  TemporalAwareAttention  :789-846   (batch-global unbiased std of |cut - t|)
  retrieve_edge_imp_node  :354-406   (dependency gate, scatter-max walk->edge, gather, Beta mean, mask)
  kl_loss                 :432-453   (empirical prior; null vector in null-model key order)
Eval semantics (dropout = identity, Beta mean instead of rsample); forward() also takes explicit dropout
keep-masks so the training forward / backward can be checked with autograd through this restatement.
Pinned against tests/golden/encoder_uslegis.npz and enron_goldens.npz (outputs of the reference module;
the latter at Enron-scale timestamps and for the constructor variants).
"""
import numpy as np
import torch
import torch.nn.functional as F


def _lin(sd, name, x):
    return F.linear(x, sd[name + ".weight"], sd[name + ".bias"])


def time_encode(sd, t):
    """TimeEncode.forward: cos(t * basis_freq + phase) with the argument rounded in fp32 as the reference
    computes it (explainer_new.py:51-59); the cosine in the weights' dtype (fp64 gradient references)."""
    w, ph = sd["time_encoder.basis_freq"], sd["time_encoder.phase"]
    m = t.float().unsqueeze(-1) * w.float()
    m = m + ph.float()
    return torch.cos(m.to(w.dtype))


def forward(sd, n_feat, e_feat, node, eid, ts, cat, cut, edge_count, drop=None, scale=1.0, temporal=True,
            if_cat=True):
    """graphlet importance [B, W, 1] for one side (explainer_new.py:174-201).  temporal=False: the
    plain ``Attention`` of use_temporal_guidance=False (explainer_new.py:12-43, no time scaling, no dropout).
    drop: optional keep-masks [B, W, >= 2 + h + hm] of the training forward's three dropouts (alpha :839 ->
    cols 0..1, attention.MLP hidden :780 -> the next h, MLP hidden :122 -> the next hm = MLP.0's width;
    144 columns = 2..65 and 66..141 for the default h = 64), kept values scaled by `scale`
    (training-mode parity); the plain Attention ignores the first 2 + h.
    Computes in the dtype of sd's tensors (fp32, or fp64 for gradient references)."""
    node = torch.as_tensor(np.asarray(node), dtype=torch.long)
    eid = torch.as_tensor(np.asarray(eid), dtype=torch.long)
    t = torch.as_tensor(np.asarray(ts, dtype=np.float64)).float()
    cut = torch.as_tensor(np.asarray(cut, dtype=np.float64)).float()
    cnt = torch.as_tensor(np.asarray(edge_count, dtype=np.float64)).float()
    dty = sd["event_conv.lin_event.weight"].dtype
    n_feat, e_feat, cnt = n_feat.to(dty), e_feat.to(dty), cnt.to(dty)
    keep = None if drop is None else torch.as_tensor(np.asarray(drop)).to(dty) * scale
    B, W = eid.shape[0], eid.shape[1]
    h, hm = sd["MLP.3.weight"].shape[0], sd["MLP.0.weight"].shape[0]
    ef = e_feat[eid]                                             # [B,W,3,de]
    dt = t[:, :, 2:3] - t                                        # relative to position 2
    tf = time_encode(sd, dt.reshape(B, -1).to(dty)).reshape(B, W, 3, -1)
    ev = torch.cat([ef, cnt, tf], dim=-1)
    xs = n_feat[node[:, :, [0, 2, 4]]]
    xt = n_feat[node[:, :, [1, 3, 5]]]
    lev = _lin(sd, "event_conv.lin_event", ev)

    def mlp(x):
        return _lin(sd, "event_conv.MLP.2", torch.relu(_lin(sd, "event_conv.MLP.0", x)))
    us = mlp(xs + torch.relu(xt + lev))
    ut = mlp(xt + torch.relu(xs + lev))
    f = torch.cat([us, ut], dim=-1)                              # [B,W,3,2h]
    src = f[:, :, 2, :]
    tgt = f[:, :, 0:2, :]
    wp = _lin(sd, "attention.W1", src)                           # [B,W,2h]
    wq = _lin(sd, "attention.W2", tgt)                           # [B,W,2,2h]
    scores = (wp.unsqueeze(2) * wq).sum(-1)                      # [B,W,2]
    if temporal:
        diff = torch.abs(cut.view(B, 1, 1) - t[:, :, :2])
        tw = torch.exp(-diff / (diff.std() + 1e-6)).to(dty)
        scores = scores * (1.0 - 0.3 + 0.3 * tw)
    alpha = torch.softmax(scores, dim=-1)
    if keep is not None and temporal:
        alpha = alpha * keep[..., 0:2]
    out = src + (alpha.unsqueeze(-1) * wq).sum(2)
    hid = torch.relu(_lin(sd, "attention.MLP.0", out))
    if keep is not None and temporal:
        hid = hid * keep[..., 2:2 + h]
    # TemporalAwareAttention.MLP has a Dropout at index 2 (:777-782), Attention.MLP does not (:18)
    out = _lin(sd, "attention.MLP.3" if "attention.MLP.3.weight" in sd else "attention.MLP.2", hid)
    if if_cat:     # compute_catogory_feautres (:308-315); if_cat_feature=False feeds the attention output alone
        oh = F.one_hot(torch.as_tensor(np.asarray(cat), dtype=torch.long).reshape(B, W), 12).to(dty)
        x = torch.cat([out, oh], dim=-1)
    else:
        x = out
    x = torch.relu(_lin(sd, "MLP.0", x))
    if keep is not None:
        x = x * keep[..., 2 + h:2 + h + hm]
    x = torch.relu(_lin(sd, "MLP.3", x))
    return torch.sigmoid(_lin(sd, "MLP.5", x))


def beta_mean(p):
    a = torch.clamp(p * 10, min=1.0)
    b = torch.clamp((1 - p) * 10, min=1.0)
    return a / (a + b)


def edge_importance(sd, e_feat, imp, walk_eid, walk_ts, sub_node, sub_eid, dependency=True):
    """retrieve_edge_imp_node, eval (explainer_new.py:354-406).  sub_*: [hop1 [B,N], hop2 [B,N^2]].
    dependency=False: use_dependency_aware_sampling=False (no gate, :366-386 skipped)."""
    B = imp.shape[0]
    ew = torch.as_tensor(np.asarray(walk_eid), dtype=torch.long).reshape(B, -1)
    tw = torch.as_tensor(np.asarray(walk_ts, dtype=np.float64)).float().reshape(B, -1)
    wimp = imp.repeat(1, 1, 3).view(B, -1)
    if dependency:
        g = torch.cat([e_feat[ew], time_encode(sd, tw)], dim=-1)
        g = torch.relu(_lin(sd, "edge_dependency_gcn.0", g))
        g = torch.relu(_lin(sd, "edge_dependency_gcn.3", g))
        g = _lin(sd, "edge_dependency_gcn.6", g).squeeze(-1)
        wimp = wimp * (0.5 + 0.5 * torch.sigmoid(g))
    i0 = torch.as_tensor(np.asarray(sub_eid[0]), dtype=torch.long)
    i1 = torch.as_tensor(np.asarray(sub_eid[1]), dtype=torch.long)
    n_e = int(max(ew.max(), i0.max(), i1.max()) + 1)
    dense = torch.zeros(B, n_e).scatter_reduce(-1, ew, wimp, "amax", include_self=False)
    outs = []
    for idx, nd in ((i0, sub_node[0]), (i1, sub_node[1])):
        v = beta_mean(torch.gather(dense, -1, idx))
        outs.append(v.masked_fill(torch.as_tensor(np.asarray(nd)) == 0, 0))
    return outs


def kl_loss(imp, cat, null_vec, target=0.3):
    """kl_loss, prior='empirical' (explainer_new.py:432-448)."""
    p = torch.clamp(imp, 1e-6, 1 - 1e-6)
    B = p.shape[0]
    s = p.mean(dim=1)                                            # [B,1]
    c = torch.as_tensor(np.asarray(cat), dtype=torch.long).reshape(B, -1, 1)
    emp = torch.zeros(B, 12, 1).scatter_reduce(1, c, p, "mean", include_self=False).reshape(B, 12)
    emp = s * emp
    null = target * torch.as_tensor(np.asarray(null_vec), dtype=torch.float32).reshape(-1, 12)
    return ((1 - s) * torch.log((1 - s) / (1 - target + 1e-6) + 1e-6)
            + emp * torch.log(emp / (null + 1e-6) + 1e-6)).mean()


def edge_importance_train(sd, e_feat, imp, walk_eid, walk_ts, sub_eid, keep1=None, keep2=None, sc1=1.0, sc2=1.0,
                          dependency=True):
    """retrieve_edge_imp_node up to the gathered scatter-max (explainer_new.py:354-393), with explicit keep-masks
    for edge_dependency_gcn's two dropouts ([B, 3W, h] / [B, 3W, h/2]); autograd-able in imp's dtype.
    dependency=False: use_dependency_aware_sampling=False (no gate).  Returns (p1 [B, N], p2 [B, N^2])
    before beta_sample and the padding mask."""
    B = imp.shape[0]
    ew = torch.as_tensor(np.asarray(walk_eid), dtype=torch.long).reshape(B, -1)
    tw = torch.as_tensor(np.asarray(walk_ts, dtype=np.float64)).float().reshape(B, -1)
    wimp = imp.repeat(1, 1, 3).view(B, -1)
    i0 = torch.as_tensor(np.asarray(sub_eid[0]), dtype=torch.long)
    i1 = torch.as_tensor(np.asarray(sub_eid[1]), dtype=torch.long)
    n_e = int(max(ew.max(), i0.max(), i1.max()) + 1)
    if not dependency:
        dense = torch.zeros(B, n_e, dtype=wimp.dtype).scatter_reduce(-1, ew, wimp, "amax", include_self=False)
        return torch.gather(dense, -1, i0), torch.gather(dense, -1, i1)
    dty = sd["edge_dependency_gcn.0.weight"].dtype
    g = torch.cat([e_feat.to(dty)[ew], time_encode(sd, tw)], dim=-1)
    g = torch.relu(_lin(sd, "edge_dependency_gcn.0", g))
    if keep1 is not None:
        g = g * (torch.as_tensor(np.asarray(keep1)).to(dty) * sc1)
    g = torch.relu(_lin(sd, "edge_dependency_gcn.3", g))
    if keep2 is not None:
        g = g * (torch.as_tensor(np.asarray(keep2)).to(dty) * sc2)
    g = _lin(sd, "edge_dependency_gcn.6", g).squeeze(-1)
    wimp = wimp * (0.5 + 0.5 * torch.sigmoid(g))
    dense = torch.zeros(B, n_e, dtype=wimp.dtype).scatter_reduce(-1, ew, wimp, "amax", include_self=False)
    return torch.gather(dense, -1, i0), torch.gather(dense, -1, i1)
