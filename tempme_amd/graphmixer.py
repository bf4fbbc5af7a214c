"""Drop-in base ``GraphMixer`` (GraphM/graphmixer.py) for the consumer side of the explanation path
(SURVEY.md §8(f) f4): ``contrast(..., explain_weights=[hop-1 weights [3B, N]])``.

Same constructor, submodule names (a reference ``state_dict`` loads as is) and construction order
(``torch.manual_seed(s); GraphMixer(...)`` draws the reference's initial weights).  The forward is
restated over all three sides at once (3B rows) on the device:

    per row: tokens = the N hop-1 neighbours, channels = d_edge
      x = projection([E[eid] | cos(dt*w+b)])        (padding neighbours: both parts zeroed)
      x = MLPMixer^L(x, ew)                          (token mix LN/FFN/GELU, channel mix; * ew each)
      x = mean_j(x_j * valid_j * ew_j)
      agg = mean_j(N[nid_j] * softmax(valid ? 1 : -1e10)_j * ew_j)
      emb = output_layer([x | agg + N[node]])
    affinity_score MergeLayer over [src, src] vs [dst, neg]

The time-encoder argument is formed as the reference's CPU addmm forms it (one rounding of
t*w+b: computed in fp64, rounded to fp32), since cos of a large argument depends on that rounding.
"""
import ctypes

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L
from .tgn import MergeLayer, _as_dev


class TimeEncoder(nn.Module):
    """graphmixer.py:21-50 (fp32 frequencies, not trainable in GraphMixer)."""

    def __init__(self, time_dim, parameter_requires_grad=True):
        super().__init__()
        self.time_dim = time_dim
        self.w = nn.Linear(1, time_dim)
        self.w.weight = nn.Parameter(torch.from_numpy(1 / 10 ** np.linspace(0, 9, time_dim, dtype=np.float32))
                                     .reshape(time_dim, -1))
        self.w.bias = nn.Parameter(torch.zeros(time_dim))
        if not parameter_requires_grad:
            self.w.weight.requires_grad = False
            self.w.bias.requires_grad = False

    def encode(self, dt):
        """cos(fma(dt, w, b)) for fp32 dt [..., ] -> [..., time_dim]."""
        w = self.w.weight.reshape(-1).to(dt.device, torch.float64)
        b = self.w.bias.to(dt.device, torch.float64)
        arg = (dt.double().unsqueeze(-1) * w + b).float()
        return torch.cos(arg)


class FeedForwardNet(nn.Module):
    """graphmixer.py:244-270: Linear, GELU, Dropout, Linear, Dropout."""

    def __init__(self, input_dim, dim_expansion_factor, dropout=0.0):
        super().__init__()
        self.input_dim = input_dim
        self.dim_expansion_factor = dim_expansion_factor
        self.dropout = dropout
        hid = int(dim_expansion_factor * input_dim)
        self.ffn = nn.Sequential(nn.Linear(input_dim, hid), nn.GELU(), nn.Dropout(dropout), nn.Linear(hid, input_dim),
                                 nn.Dropout(dropout))

    def forward(self, x):
        return self.ffn(x)


class MLPMixer(nn.Module):
    """graphmixer.py:273-315, explanation weight applied to the input and both branch outputs."""

    def __init__(self, num_tokens, num_channels, token_dim_expansion_factor=0.5, channel_dim_expansion_factor=4.0,
                 dropout=0.0):
        super().__init__()
        self.token_norm = nn.LayerNorm(num_tokens)
        self.token_feedforward = FeedForwardNet(num_tokens, token_dim_expansion_factor, dropout)
        self.channel_norm = nn.LayerNorm(num_channels)
        self.channel_feedforward = FeedForwardNet(num_channels, channel_dim_expansion_factor, dropout)

    def forward(self, input_tensor, explain_weights=None):
        ew = None if explain_weights is None else explain_weights.unsqueeze(-1)
        if ew is not None:
            input_tensor = input_tensor * ew
        h = self.token_feedforward(self.token_norm(input_tensor.permute(0, 2, 1))).permute(0, 2, 1)
        if ew is not None:
            h = h * ew
        out = h + input_tensor
        h = self.channel_feedforward(self.channel_norm(out))
        if ew is not None:
            h = h * ew
        return h + out


class _GmEmbedFn(torch.autograd.Function):
    """(x_mean, node_out) of tm_gm_embed as a function of the explanation weights: forward passes the
    kernel's outputs through, backward is tm_gm_embed_bwd (d ew [R, N]; zero on padding neighbours)."""

    @staticmethod
    def forward(ctx, ew, x_mean, node_out, args, keep):
        ctx.args, ctx.keep = args, keep
        ctx.shape = ew.shape
        return x_mean.detach(), node_out.detach()

    @staticmethod
    def backward(ctx, d_xm, d_no):
        a = ctx.args
        dev = ctx.keep[1].device
        R, N = a.R, a.N
        d_xm = (torch.zeros(R, a.C, device=dev) if d_xm is None else d_xm).float().contiguous()
        d_no = (torch.zeros(R, a.D, device=dev) if d_no is None else d_no).float().contiguous()
        d_ew = torch.empty(max(R, 1), N, dtype=torch.float32, device=dev)
        L.check(L.lib().tm_gm_embed_bwd(ctypes.byref(a), L.ptr(d_xm), L.ptr(d_no), L.ptr(d_ew), L.stream_ptr(dev)),
                "GraphMixer explanation-weight backward")
        return d_ew[:R].reshape(ctx.shape), None, None, None, None


class GraphMixer(nn.Module):
    """graphmixer.py:53-101 constructor."""

    def __init__(self, n_feat, e_feat, n_neighbors, device, num_tokens, num_layers=2, token_dim_expansion_factor=0.5,
                 channel_dim_expansion_factor=4.0, dropout=0.1):
        super().__init__()
        self.n_feat_th = nn.Parameter(torch.from_numpy(np.asarray(n_feat).astype(np.float32)), requires_grad=False)
        self.e_feat_th = nn.Parameter(torch.from_numpy(np.asarray(e_feat).astype(np.float32)), requires_grad=False)
        self.node_raw_features = nn.Embedding.from_pretrained(self.n_feat_th, padding_idx=0, freeze=True)
        self.edge_raw_features = nn.Embedding.from_pretrained(self.e_feat_th, padding_idx=0, freeze=True)
        self.num_neighbors = n_neighbors
        self.node_feat_dim = self.n_feat_th.shape[1]
        self.edge_feat_dim = self.e_feat_th.shape[1]
        self.time_feat_dim = self.node_feat_dim
        self.num_tokens = num_tokens
        self.num_layers = num_layers
        self.token_dim_expansion_factor = token_dim_expansion_factor
        self.channel_dim_expansion_factor = channel_dim_expansion_factor
        self.dropout = dropout
        self.device = device
        self.num_channels = self.edge_feat_dim
        self.time_encoder = TimeEncoder(time_dim=self.time_feat_dim, parameter_requires_grad=False)
        self.projection_layer = nn.Linear(self.edge_feat_dim + self.time_feat_dim, self.num_channels)
        self.mlp_mixers = nn.ModuleList([
            MLPMixer(num_tokens=self.num_tokens, num_channels=self.num_channels,
                     token_dim_expansion_factor=self.token_dim_expansion_factor,
                     channel_dim_expansion_factor=self.channel_dim_expansion_factor, dropout=self.dropout)
            for _ in range(self.num_layers)])
        self.output_layer = nn.Linear(self.num_channels + self.node_feat_dim, self.node_feat_dim, bias=True)
        self.affinity_score = MergeLayer(self.node_feat_dim, self.node_feat_dim, self.node_feat_dim, 1)

    def _dev(self):
        p = self.projection_layer.weight
        dev = L.require_device(p.device if p.device.type == "cuda" else self.device)
        if p.device != dev:
            raise RuntimeError("GraphMixer: move the model to the HIP device first (model.to(device)), "
                               "as the reference does after loading it")
        return dev

    def _tables(self, dev):
        key = (dev, self.n_feat_th.data_ptr(), self.e_feat_th.data_ptr())
        if getattr(self, "_tab_key", None) != key:
            self._ntab = self.n_feat_th.detach().to(dev, torch.float32)
            self._etab = self.e_feat_th.detach().to(dev, torch.float32)
            self._tab_key = key
        return self._ntab, self._etab

    # ------------------------------------------------------------------ HIP path (tm_gm_embed)
    def _hip_mode(self, explain_weight, N):
        """"eval": the fused HIP embedding, no gradients (threshold_test, scoring).  "grad": explanation
        weights that require a gradient (the explainer's training step through the frozen base model,
        temp_exp_main.py:614-632): the HIP forward plus tm_gm_embed_bwd for d ew; the base model's
        parameters get no .grad (as the TGN base, tgn.py).  None: the torch formulation below (dropout
        active, unsupported dims, or gradients wanted for the base model's own parameters only)."""
        import os
        if os.environ.get("TEMPME_GM_TORCH") == "1" or self.training:
            return None
        ht = int(self.mlp_mixers[0].token_feedforward.dim_expansion_factor * N) if self.num_layers else 0
        if not (N <= 32 and ht <= 16 and self.num_layers <= 4 and self.num_channels <= 256 and N == self.num_tokens):
            return None
        if not torch.is_grad_enabled():
            return "eval"
        if explain_weight is not None and explain_weight.requires_grad:
            ok = L.lib().tm_gm_embed_bwd_ok(N, self.num_channels, self.time_feat_dim, self.num_layers, ht)
            if not ok:
                return None
            if any(p.requires_grad for p in self.parameters()):
                # the reference's training loop leaves the base's parameters requiring grad but never steps
                # them (its optimizer holds the explainer's only, temp_exp_main.py:555); the HIP backward
                # returns d ew alone.  frozen_base = False asks for their gradients: the torch formulation
                if not getattr(self, "frozen_base", True):
                    return None
                if not getattr(self, "_warned_frozen", False):
                    import warnings
                    warnings.warn("GraphMixer: explanation-weight gradients on HIP; the base model's own "
                                  "parameters get no .grad (set model.frozen_base = False for the torch "
                                  "formulation, which computes them)", stacklevel=3)
                    self._warned_frozen = True
            return "grad"
        if any(p.requires_grad for p in self.parameters()):
            return None
        return "eval"

    def _hip_ok(self, explain_weight, N):
        return self._hip_mode(explain_weight, N) is not None

    def _gm_packed(self, dev):
        """Packed MFMA fragments of projection_layer and every channel FFN (tm_gm_pack), rebuilt when a
        parameter changes (version counters)."""
        ps = list(self.parameters())
        key = (dev, tuple((p.data_ptr(), p._version) for p in ps))
        if getattr(self, "_gm_key", None) != key:
            st = L.stream_ptr(dev)
            keep = []

            N, C = self.num_tokens, self.num_channels
            fused = bool(L.lib().tm_gm_fused_ok(N, C, self.time_feat_dim, int(self.channel_dim_expansion_factor * C)))

            def pack(w, mult=(1, 1)):
                # the register-resident kernel takes A-operand fragments (tm_gm_pack_a), the LDS-tiled one
                # B-operand fragments (tm_gm_pack); tm_gm_embed picks the kernel by the same tm_gm_fused_ok
                w = w.detach().to(dev, torch.float32).contiguous()
                n_out, k = w.shape
                if fused:
                    out = torch.empty(int(L.lib().tm_gm_packed_a_floats(n_out, k, *mult)), dtype=torch.float32,
                                      device=dev)
                    L.check(L.lib().tm_gm_pack_a(L.ptr(w), n_out, k, mult[0], mult[1], L.ptr(out), st), "tm_gm_pack_a")
                else:
                    out = torch.empty(int(L.lib().tm_gm_packed_floats(n_out, k)), dtype=torch.float32, device=dev)
                    L.check(L.lib().tm_gm_pack(L.ptr(w), n_out, k, L.ptr(out), st), "tm_gm_pack")
                keep.append(w)
                return out

            def flat(t):
                t = t.detach().to(dev, torch.float32).contiguous()
                keep.append(t)
                return t

            layers = []
            for m in self.mlp_mixers:
                tf, cf = m.token_feedforward.ffn, m.channel_feedforward.ffn
                layers.append([flat(m.token_norm.weight), flat(m.token_norm.bias), flat(tf[0].weight), flat(tf[0].bias),
                               flat(tf[3].weight), flat(tf[3].bias), flat(m.channel_norm.weight),
                               flat(m.channel_norm.bias), pack(cf[0].weight, (2, 1)), flat(cf[0].bias),
                               pack(cf[3].weight, (1, 2)),
                               flat(cf[3].bias)])
            table = torch.tensor([[t.data_ptr() for t in lw] for lw in layers] or [[0] * 12], dtype=torch.int64)
            self._gm_pack = dict(proj_w=pack(self.projection_layer.weight, (1, 4)), proj_b=flat(self.projection_layer.bias),
                                 tw=flat(self.time_encoder.w.weight.reshape(-1)), tb=flat(self.time_encoder.w.bias),
                                 layers=layers, table=table.to(dev), keep=keep)
            self._gm_key = key
        return self._gm_pack

    def _gm_packed_bwd(self, dev):
        """B-operand packs (tm_gm_pack) for tm_gm_embed_bwd: the projection, each channel FFN's two weights
        and their transposes; layer table [L][14]; rebuilt when a parameter changes."""
        ps = list(self.parameters())
        key = (dev, tuple((p.data_ptr(), p._version) for p in ps))
        if getattr(self, "_gmb_key", None) != key:
            st = L.stream_ptr(dev)
            keep = []

            def pack(w):
                w = w.detach().to(dev, torch.float32).contiguous()
                n_out, k = w.shape
                out = torch.empty(int(L.lib().tm_gm_packed_floats(n_out, k)), dtype=torch.float32, device=dev)
                L.check(L.lib().tm_gm_pack(L.ptr(w), n_out, k, L.ptr(out), st), "tm_gm_pack")
                keep.append(w)
                return out

            def flat(t):
                t = t.detach().to(dev, torch.float32).contiguous()
                keep.append(t)
                return t

            layers = []
            for m in self.mlp_mixers:
                tf, cf = m.token_feedforward.ffn, m.channel_feedforward.ffn
                layers.append([flat(m.token_norm.weight), flat(m.token_norm.bias), flat(tf[0].weight), flat(tf[0].bias),
                               flat(tf[3].weight), flat(tf[3].bias), flat(m.channel_norm.weight),
                               flat(m.channel_norm.bias), pack(cf[0].weight), flat(cf[0].bias), pack(cf[3].weight),
                               flat(cf[3].bias), pack(cf[3].weight.t()), pack(cf[0].weight.t())])
            table = torch.tensor([[t.data_ptr() for t in lw] for lw in layers] or [[0] * 14], dtype=torch.int64)
            self._gmb_pack = dict(proj_w=pack(self.projection_layer.weight), layers=layers, table=table.to(dev),
                                  keep=keep)
            self._gmb_key = key
        return self._gmb_pack

    def _embed_args(self, dev, node, nid32, eid32, cut64, t64, ew, ea, proj_w, proj_b, tw, tb, table):
        ntab, etab = self._tables(dev)
        R, N = nid32.shape
        a = L.GmEmbedArgs()
        a.R, a.N, a.C, a.T, a.D, a.L = R, N, self.num_channels, self.time_feat_dim, self.node_feat_dim, self.num_layers
        a.HT = int(self.mlp_mixers[0].token_feedforward.dim_expansion_factor * N) if self.num_layers else 0
        a.HC = int(self.channel_dim_expansion_factor * self.num_channels)
        a.node, a.nid, a.eid, a.cut, a.ts = L.ptr(node), L.ptr(nid32), L.ptr(eid32), L.ptr(cut64), L.ptr(t64)
        a.ew = None if ew is None else L.ptr(ew)
        a.edge_attr = None if ea is None else L.ptr(ea)
        a.n_feat, a.e_feat = L.ptr(ntab), L.ptr(etab)
        a.time_w, a.time_b = L.ptr(tw), L.ptr(tb)
        a.proj_w, a.proj_b = L.ptr(proj_w), L.ptr(proj_b)
        a.layer_table = L.ptr(table)
        return a

    def _embed_hip(self, dev, node_ids, cut, nid, eid, t, explain_weight, edge_attr, mode="eval"):
        R, N = nid.shape
        pk = self._gm_packed(dev)
        i32 = lambda x: x.to(dev, torch.int32).contiguous()  # noqa: E731
        node, nid32 = i32(node_ids), i32(nid)
        eid32 = i32(eid)
        cut64 = cut.to(dev, torch.float64).reshape(-1).contiguous()
        t64 = t.to(dev, torch.float64).contiguous()
        ew = None if explain_weight is None else explain_weight.detach().to(dev, torch.float32).contiguous()
        ea = None if edge_attr is None else edge_attr.detach().to(dev, torch.float32).contiguous()
        C, D = self.num_channels, self.node_feat_dim
        x_mean = torch.empty(max(R, 1), C, dtype=torch.float32, device=dev)
        node_out = torch.empty(max(R, 1), D, dtype=torch.float32, device=dev)
        a = self._embed_args(dev, node, nid32, eid32, cut64, t64, ew, ea, pk["proj_w"], pk["proj_b"], pk["tw"], pk["tb"],
                             pk["table"])
        a.x_mean, a.node_out = L.ptr(x_mean), L.ptr(node_out)
        L.check(L.lib().tm_gm_embed(ctypes.byref(a), L.stream_ptr(dev)), "GraphMixer.compute_node_temporal_embeddings")
        xm, no = x_mean[:R], node_out[:R]
        if mode == "grad":
            # d ew through tm_gm_embed_bwd; the rest of the graph (output layer, MergeLayer) is torch autograd
            # with the base model's weights detached (frozen base: no parameter gradients)
            bk = self._gm_packed_bwd(dev)
            ab = self._embed_args(dev, node, nid32, eid32, cut64, t64, ew, ea, bk["proj_w"], pk["proj_b"], pk["tw"],
                                  pk["tb"], bk["table"])
            keep = (node, nid32, eid32, cut64, t64, ew, ea, bk, pk)
            xm, no = _GmEmbedFn.apply(explain_weight, xm, no, ab, keep)
            return F.linear(torch.cat([xm, no], dim=1), self.output_layer.weight.detach().to(dev),
                            self.output_layer.bias.detach().to(dev))
        return F.linear(torch.cat([xm, no], dim=1), self.output_layer.weight.to(dev), self.output_layer.bias.to(dev))

    def node_embeddings(self, node_ids, cut_time, nid, eid, times, explain_weight=None, edge_attr=None):
        """compute_node_temporal_embeddings (graphmixer.py:142-193) for R rows at once:
        node_ids [R], cut_time [R] (f64), nid/eid/times [R, N] (hop-1 records), explain_weight [R, N]."""
        dev = self._dev()
        N0 = np.shape(nid)[-1]
        mode = self._hip_mode(explain_weight, N0)
        if mode is not None:
            return self._embed_hip(dev, _as_dev(node_ids, dev, torch.long).reshape(-1),
                                   _as_dev(cut_time, dev, torch.float64).reshape(-1), _as_dev(nid, dev, torch.long),
                                   _as_dev(eid, dev, torch.long), _as_dev(times, dev, torch.float64), explain_weight,
                                   None if edge_attr is None else _as_dev(edge_attr, dev, torch.float32), mode)
        ntab, etab = self._tables(dev)
        node_ids = _as_dev(node_ids, dev, torch.long).reshape(-1)
        nid = _as_dev(nid, dev, torch.long)
        valid = nid != 0
        t = _as_dev(times, dev, torch.float64)
        cut = _as_dev(cut_time, dev, torch.float64).reshape(-1, 1)
        ew = None
        if explain_weight is not None:
            ew = explain_weight.to(dev, torch.float32) * valid.to(torch.float32)
        if edge_attr is None:
            ef = etab[_as_dev(eid, dev, torch.long)] * valid.unsqueeze(-1)
        else:
            ef = _as_dev(edge_attr, dev, torch.float32)
        tf = self.time_encoder.encode((cut - t).float()) * valid.unsqueeze(-1)
        x = F.linear(torch.cat([ef, tf], dim=-1), self.projection_layer.weight.to(dev),
                     self.projection_layer.bias.to(dev))
        for mixer in self.mlp_mixers:
            x = mixer(x, ew)
        x = x * valid.unsqueeze(-1)
        if ew is not None:
            x = x * ew.unsqueeze(-1)
        x = x.mean(dim=1)
        m = torch.where(valid, 1.0, -1e10).to(torch.float32)
        scores = torch.softmax(m, dim=1)
        if ew is not None:
            scores = scores * ew
        agg = (ntab[nid] * scores.unsqueeze(-1)).mean(dim=1)
        out_nf = agg + ntab[node_ids]
        return self.output_layer(torch.cat([x, out_nf], dim=1))

    def get_node_emb(self, src_idx, tgt_idx, bgd_idx, cut_time, e_idx, subgraph_src, subgraph_tgt, subgraph_bgd,
                     explain_weights=None, edge_attr=None, time_gap=2000):
        """graphmixer.py:106-140 -> (source, destination, negative) embeddings [B, d]."""
        B = len(src_idx)
        dev = self._dev()
        sgs = (subgraph_src, subgraph_tgt, subgraph_bgd)
        roots = torch.cat([_as_dev(x, dev, torch.long).reshape(-1) for x in (src_idx, tgt_idx, bgd_idx)])
        cut = _as_dev(cut_time, dev, torch.float64).reshape(-1).repeat(3)
        nid = torch.cat([_as_dev(sg[0][0], dev, torch.long) for sg in sgs])
        eid = torch.cat([_as_dev(sg[1][0], dev, torch.long) for sg in sgs])
        t = torch.cat([_as_dev(sg[2][0], dev, torch.float64) for sg in sgs])
        ew = explain_weights[0] if explain_weights is not None else None
        emb = self.node_embeddings(roots, cut, nid, eid, t, ew, edge_attr)
        return emb[:B], emb[B:2 * B], emb[2 * B:]

    def affinity(self, x1, x2):
        return self.affinity_score(x1, x2)

    def contrast(self, src_idx, tgt_idx, bgd_idx, cut_time, e_idx, subgraph_src, subgraph_tgt, subgraph_bgd,
                 explain_weights=None, edge_attr=None, time_gap=2000):
        """graphmixer.py:206-218 -> (pos_score [B,1], neg_score [B,1])."""
        B = len(src_idx)
        s, d, n = self.get_node_emb(src_idx, tgt_idx, bgd_idx, cut_time, e_idx, subgraph_src, subgraph_tgt,
                                    subgraph_bgd, explain_weights, edge_attr, time_gap)
        score = self.affinity(torch.cat([s, s], dim=0), torch.cat([d, n])).squeeze(dim=0)
        return score[:B], score[B:]

    def retrieve_edge_features(self, subgraph_src, subgraph_tgt, subgraph_bgd):
        """graphmixer.py:196-201."""
        dev = self._dev()
        _, etab = self._tables(dev)
        return torch.cat([etab[_as_dev(sg[1][0], dev, torch.long)] for sg in (subgraph_src, subgraph_tgt,
                                                                              subgraph_bgd)], dim=0)

    def set_neighbor_sampler(self, neighbor_sampler):
        self.neighbor_sampler = neighbor_sampler

    def grab_subgraph(self, src_idx_l, cut_time_l):
        """graphmixer.py:232-234."""
        return self.neighbor_sampler.find_k_hop(2, src_idx_l, cut_time_l, num_neighbors=self.num_neighbors,
                                                e_idx_l=None)
