"""Drop-in base ``TGN`` (TGN/tgn.py) for the consumer side of the explanation path.

TempME's training and evaluation loops hand the explanation to the frozen base model:
``base_model.contrast(src, dst, fake, ts, e_idx, sg_src, sg_tgt, sg_bgd, explain_weights=expl)``
(temp_exp_main.py:614-623, :306-321, threshold_test :153-272).  This module keeps the reference's
constructor, submodule names (a reference ``state_dict`` loads as is), construction order (so
``torch.manual_seed(s); TGN(...)`` draws the reference's initial weights) and the
``contrast`` / ``get_node_emb`` / ``grab_subgraph`` signatures.

``contrast`` runs on the HIP device:
  * per layer, the neighbour-facing part (key construction from the feature tables, scores for all
    heads, masked softmax, explanation weight, weighted key sum) is one launch of
    ``tgn_attn_fwd_kernel`` (csrc/tgn_attn.hip, C ABI ``tm_tgn_attn_fwd``);
  * the reference's per-neighbour projections fold into per-row ones: qf = (W_k^T W_q) query before
    the kernel and (fc W_v) z after it, two hipBLASLt GEMMs over source rows, followed by the
    residual LayerNorm and the merger MLP (torch ops on the device);
  * gradients with respect to the explanation weights (the explainer's training signal,
    temp_exp_main.py:624-631) come from ``tgn_attn_bwd_kernel`` (``tm_tgn_attn_bwd``) and torch
    autograd for the dense per-row algebra.  The base model is frozen: its parameters get no .grad.

Scope: the ``forbidden_memory_update=True`` path TempME uses (temp_exp_main.py:703-704), the
"graph_attention" embedding module, 2-hop subgraphs.  Memory messages stored on the model are
applied through get_updated_memory semantics (tgn.py:237-248) once per memory state.
"""
from collections import defaultdict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L


# ------------------------------------------------------------------ modules (parameter layout)
class TimeEncode(nn.Module):
    """embedding_module.py:100-112: Linear(1, d) with frequencies 10^-linspace(0, 9, d), phase 0."""

    def __init__(self, dimension):
        super().__init__()
        self.dimension = dimension
        self.w = nn.Linear(1, dimension)
        freq = 1.0 / 10 ** np.linspace(0, 9, dimension)
        self.w.weight = nn.Parameter(torch.from_numpy(freq).float().reshape(dimension, -1))
        self.w.bias = nn.Parameter(torch.zeros(dimension).float())

    def forward(self, t):
        return torch.cos(self.w(t.unsqueeze(dim=2)))


class MergeLayer(nn.Module):
    """embedding_module.py:115-128: fc2(relu(fc1([x1 | x2])))."""

    def __init__(self, dim1, dim2, dim3, dim4):
        super().__init__()
        self.fc1 = nn.Linear(dim1 + dim2, dim3)
        self.fc2 = nn.Linear(dim3, dim4)
        self.act = nn.ReLU()
        nn.init.xavier_normal_(self.fc1.weight)
        nn.init.xavier_normal_(self.fc2.weight)

    def forward(self, x1, x2):
        return self.fc2(self.act(self.fc1(torch.cat([x1, x2], dim=1))))


class MultiHeadAttention(nn.Module):
    """Parameters of embedding_module.py:35-60 (d_k = d_v = key dim, no projection bias)."""

    def __init__(self, n_head, d_emb, d_k, d_v, dropout=0.1):
        super().__init__()
        self.n_head, self.d_k, self.d_v = n_head, d_k, d_v
        self.w_qs = nn.Linear(d_emb, n_head * d_k, bias=False)
        self.w_ks = nn.Linear(d_k, n_head * d_k, bias=False)
        self.w_vs = nn.Linear(d_v, n_head * d_v, bias=False)
        nn.init.normal_(self.w_qs.weight, mean=0, std=np.sqrt(2.0 / (d_emb + d_k)))
        nn.init.normal_(self.w_ks.weight, mean=0, std=np.sqrt(2.0 / (d_emb + d_k)))
        nn.init.normal_(self.w_vs.weight, mean=0, std=np.sqrt(2.0 / (d_emb + d_v)))
        self.temperature = float(np.power(d_k, 0.5))
        self.fc = nn.Linear(n_head * d_v, d_emb)
        nn.init.xavier_normal_(self.fc.weight)
        self.layer_norm = nn.LayerNorm(d_emb)
        self.dropout = nn.Dropout(dropout)


class TemporalAttentionLayer(nn.Module):
    """embedding_module.py:130-166: query [node | time], key [node | edge | time]."""

    def __init__(self, n_node_features, n_neighbors_features, n_edge_features, time_dim, output_dimension,
                 n_head=2, dropout=0.1):
        super().__init__()
        self.n_head = n_head
        self.feat_dim = n_node_features
        self.time_dim = time_dim
        self.query_dim = n_node_features + time_dim
        self.key_dim = n_neighbors_features + time_dim + n_edge_features
        self.merger = MergeLayer(self.query_dim, n_node_features, n_node_features, output_dimension)
        self.multi_head_target = MultiHeadAttention(n_head=n_head, d_emb=self.query_dim, d_k=self.key_dim,
                                                    d_v=self.key_dim, dropout=dropout)


class Memory(nn.Module):
    """memory.py:8-75: per-node memory and last-update time (parameters, no grad) + raw messages."""

    def __init__(self, n_nodes, memory_dimension, input_dimension, message_dimension=None, device="cpu",
                 combination_method="sum"):
        super().__init__()
        self.n_nodes = n_nodes
        self.memory_dimension = memory_dimension
        self.input_dimension = input_dimension
        self.message_dimension = message_dimension
        self.device = device
        self.combination_method = combination_method
        self.__init_memory__()

    def __init_memory__(self):
        self.memory = nn.Parameter(torch.zeros((self.n_nodes, self.memory_dimension)), requires_grad=False)
        self.last_update = nn.Parameter(torch.zeros(self.n_nodes), requires_grad=False)
        self.messages = defaultdict(list)

    def store_raw_messages(self, nodes, node_id_to_messages):
        for node in nodes:
            self.messages[node].extend(node_id_to_messages[node])

    def get_memory(self, node_idxs):
        return self.memory[node_idxs, :]

    def get_last_update(self, node_idxs):
        return self.last_update[node_idxs]

    def clear_messages(self, nodes):
        for node in nodes:
            self.messages[node] = []


class MLPMessageFunction(nn.Module):
    """message_function.py:13-25 (registered under both ``mlp`` and ``layers``, as the reference)."""

    def __init__(self, raw_message_dimension, message_dimension):
        super().__init__()
        self.mlp = self.layers = nn.Sequential(
            nn.Linear(raw_message_dimension, raw_message_dimension // 2), nn.ReLU(),
            nn.Linear(raw_message_dimension // 2, message_dimension))

    def compute_message(self, raw_messages):
        return self.mlp(raw_messages)


class IdentityMessageFunction(nn.Module):
    def compute_message(self, raw_messages):
        return raw_messages


class SequenceMemoryUpdater(nn.Module):
    """memory_updater.py:10-49 (the memory module is registered here too, as in the reference)."""

    def __init__(self, memory, message_dimension, memory_dimension, device):
        super().__init__()
        self.memory = memory
        self.layer_norm = nn.LayerNorm(memory_dimension)
        self.message_dimension = message_dimension
        self.device = device


class GRUMemoryUpdater(SequenceMemoryUpdater):
    def __init__(self, memory, message_dimension, memory_dimension, device):
        super().__init__(memory, message_dimension, memory_dimension, device)
        self.memory_updater = nn.GRUCell(input_size=message_dimension, hidden_size=memory_dimension)


class RNNMemoryUpdater(SequenceMemoryUpdater):
    def __init__(self, memory, message_dimension, memory_dimension, device):
        super().__init__(memory, message_dimension, memory_dimension, device)
        self.memory_updater = nn.RNNCell(input_size=message_dimension, hidden_size=memory_dimension)


class GraphAttentionEmbedding(nn.Module):
    """embedding_module.py:239-260 (EmbeddingModule :219-236 registers the shared tables)."""

    def __init__(self, node_features, edge_features, neighbor_finder, num_neighbor, time_encoder, n_layers,
                 n_node_features, n_edge_features, n_time_features, embedding_dimension, device, n_heads=2,
                 dropout=0.1, use_memory=True):
        super().__init__()
        self.node_features = node_features
        self.edge_features = edge_features
        self.neighbor_finder = neighbor_finder
        self.time_encoder = time_encoder
        self.n_layers = n_layers
        self.n_node_features = n_node_features
        self.n_edge_features = n_edge_features
        self.n_time_features = n_time_features
        self.dropout = dropout
        self.embedding_dimension = embedding_dimension
        self.device = device
        self.num_neighbor = num_neighbor
        self.use_memory = use_memory
        self.atten_weights_list = []
        self.n_heads = n_heads
        self.attention_models = nn.ModuleList([TemporalAttentionLayer(
            n_node_features=n_node_features, n_neighbors_features=n_node_features, n_edge_features=n_edge_features,
            time_dim=n_time_features, n_head=n_heads, dropout=dropout, output_dimension=n_node_features)
            for _ in range(n_layers)])


# ------------------------------------------------------------------ the HIP attention op
class _TgnAttnFn(torch.autograd.Function):
    """z = tm_tgn_attn_fwd(...); backward through tm_tgn_attn_bwd (explanation weights and the dense
    neighbour-feature rows of the upper layer)."""

    @staticmethod
    def forward(ctx, qf, ngh_dense, ew, spec):
        dev = qf.device
        R, H, dk = spec["rows"], spec["n_head"], spec["d_key"]
        desc = _desc(spec, qf, ngh_dense, ew)
        z = torch.empty((R, H * dk), dtype=torch.float32, device=dev)
        stats = torch.empty((R, H, 2), dtype=torch.float32, device=dev)
        if R:
            L.check(L.lib().tm_tgn_attn_fwd(L.C.byref(desc), L.ptr(z), L.ptr(stats), L.stream_ptr(dev)),
                    "TGN attention")
        ctx.spec = spec
        ctx.save_for_backward(qf, ngh_dense, ew, stats)
        return z

    @staticmethod
    def backward(ctx, gz):
        qf, ngh_dense, ew, stats = ctx.saved_tensors
        spec = ctx.spec
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("TGN attention: gradient with respect to the queries (base model is frozen)")
        R, H, N = spec["rows"], spec["n_head"], spec["n_ngh"]
        dev = gz.device
        gz = gz.contiguous().float()
        want_node = ngh_dense is not None and ctx.needs_input_grad[1]
        parts = torch.empty((R * H, N), dtype=torch.float32, device=dev)
        d_node = torch.empty_like(ngh_dense) if want_node else None
        if R:
            desc = _desc(spec, qf, ngh_dense, ew)
            L.check(L.lib().tm_tgn_attn_bwd(L.C.byref(desc), L.ptr(stats), L.ptr(gz), L.ptr(parts),
                                            L.ptr(d_node), L.stream_ptr(dev)), "TGN attention backward")
        d_ew = None
        if ew is not None and ctx.needs_input_grad[2]:
            # pair q = r*H + h contributes to explanation-weight row q % R (head-major) or r
            d_ew = parts.view(H, R, N).sum(0) if spec["head_major"] else parts.view(R, H, N).sum(1)
            d_ew = d_ew.reshape(ew.shape)
        return None, d_node, d_ew, None


def _desc(spec, qf, ngh_dense, ew):
    a = L.TgnAttn()
    a.rows, a.n_ngh, a.n_head = spec["rows"], spec["n_ngh"], spec["n_head"]
    a.d_node, a.d_edge, a.d_time = spec["d_node"], spec["d_edge"], spec["d_time"]
    a.node_rows, a.edge_rows = spec["node_rows"], spec["edge_rows"]
    a.head_major_rows = 1 if spec["head_major"] else 0
    a.seg_rows = spec.get("seg_rows", 0)
    a.temperature = spec["temperature"]
    a.node_tab = (ngh_dense if ngh_dense is not None else spec["node_tab"]).data_ptr()
    a.node_idx = spec["node_idx"].data_ptr() if spec["node_idx"] is not None else None
    a.edge_tab = spec["edge_tab"].data_ptr() if spec["edge_tab"] is not None else None
    a.edge_idx = spec["edge_idx"].data_ptr() if spec["edge_idx"] is not None else None
    a.dt = spec["dt"].data_ptr()
    a.time_w, a.time_b = spec["time_w"].data_ptr(), spec["time_b"].data_ptr()
    a.mask_node = spec["mask_node"].data_ptr()
    a.ew = ew.data_ptr() if ew is not None else None
    a.qf = qf.data_ptr()
    a.err_flag = spec["err"].data_ptr()
    return a


def _as_dev(x, device, dtype):
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype)
    return torch.from_numpy(np.ascontiguousarray(np.asarray(x))).to(device=device, dtype=dtype)


def _cat_rows(xs):
    """torch.cat(xs) along dim 0 -- as a view when the tensors are consecutive row blocks of one contiguous
    tensor (a gathered pack's three sides, [3, B, ...]), else a copy.  Only for tensors without autograd
    history (the view would route gradients through the first one's base)."""
    a = xs[0]
    if all(isinstance(x, torch.Tensor) for x in xs) and not any(x.requires_grad for x in xs):
        st = a.untyped_storage().data_ptr()
        adjacent = all(x.is_contiguous() and x.dtype == a.dtype and x.device == a.device and x.dim() == a.dim()
                       and x.shape[1:] == a.shape[1:] and x.untyped_storage().data_ptr() == st for x in xs)
        if adjacent:
            off = a.storage_offset()
            for x in xs:
                if x.storage_offset() != off:
                    adjacent = False
                    break
                off += x.numel()
        if adjacent:
            # explicit contiguous strides: is_contiguous() ignores the stride of a size-1 dim, so a.stride()
            # may not describe consecutive rows when a has one row
            shape = (sum(int(x.shape[0]) for x in xs),) + tuple(a.shape[1:])
            strides, acc = [], 1
            for d in reversed(shape):
                strides.append(acc)
                acc *= int(d)
            return a.as_strided(shape, tuple(reversed(strides)), a.storage_offset())
    return torch.cat(list(xs))


# ------------------------------------------------------------------ the model
class TGN(nn.Module):
    """TGN/tgn.py:14-97 constructor (same arguments, submodules and initialisation order)."""

    def __init__(self, n_feat, e_feat, n_neighbors, device=None, n_layers=2, n_heads=2, dropout=0.1,
                 use_memory=True, forbidden_memory_update=False, memory_update_at_start=True, message_dimension=100,
                 memory_dimension=500, embedding_module_type="graph_attention", message_function="mlp",
                 mean_time_shift_src=0, std_time_shift_src=1, mean_time_shift_dst=0, std_time_shift_dst=1,
                 aggregator_type="last", memory_updater_type="gru", use_destination_embedding_in_message=True,
                 use_source_embedding_in_message=True, head_major_rows=True):
        super().__init__()
        if embedding_module_type != "graph_attention":
            raise NotImplementedError(f"embedding module {embedding_module_type!r}: the reference's contrast "
                                      "only runs with 'graph_attention' (embedding_update)")
        self.num_layers = n_layers
        self.ngh_finder = None
        self.device = device
        self.n_feat_th = nn.Parameter(torch.from_numpy(np.asarray(n_feat).astype(np.float32)), requires_grad=False)
        self.e_feat_th = nn.Parameter(torch.from_numpy(np.asarray(e_feat).astype(np.float32)), requires_grad=False)
        self.node_raw_features = nn.Embedding.from_pretrained(self.n_feat_th, padding_idx=0, freeze=True)
        self.edge_raw_features = nn.Embedding.from_pretrained(self.e_feat_th, padding_idx=0, freeze=True)
        self.n_node_features = self.n_feat_th.shape[1]
        self.n_nodes = self.n_feat_th.shape[0]
        self.n_edge_features = self.e_feat_th.shape[1]
        self.embedding_dimension = self.n_node_features
        self.num_neighbors = n_neighbors
        self.embedding_module_type = embedding_module_type
        self.use_destination_embedding_in_message = use_destination_embedding_in_message
        self.use_source_embedding_in_message = use_source_embedding_in_message
        self.use_memory = use_memory
        self.forbidden_memory_update = forbidden_memory_update
        self.time_encoder = TimeEncode(dimension=self.n_node_features)
        self.memory = None
        self.mean_time_shift_src, self.std_time_shift_src = mean_time_shift_src, std_time_shift_src
        self.mean_time_shift_dst, self.std_time_shift_dst = mean_time_shift_dst, std_time_shift_dst
        self.aggregator_type = aggregator_type
        if self.use_memory:
            self.memory_dimension = self.n_node_features
            self.memory_update_at_start = memory_update_at_start
            raw_message_dimension = 2 * self.memory_dimension + self.n_edge_features + self.time_encoder.dimension
            message_dimension = message_dimension if message_function != "identity" else raw_message_dimension
            self.memory = Memory(n_nodes=self.n_nodes, memory_dimension=self.memory_dimension,
                                 input_dimension=message_dimension, message_dimension=message_dimension,
                                 device=self.device)
            if aggregator_type not in ("last", "mean"):
                raise ValueError(f"Message aggregator {aggregator_type} not implemented")
            self.message_aggregator = nn.Module()   # no parameters (message_aggregator.py)
            if message_function == "mlp":
                self.message_function = MLPMessageFunction(raw_message_dimension, message_dimension)
            else:
                self.message_function = IdentityMessageFunction()
            updater = {"gru": GRUMemoryUpdater, "rnn": RNNMemoryUpdater}[memory_updater_type]
            self.memory_updater = updater(self.memory, message_dimension, self.memory_dimension, self.device)
        self.embedding_module = GraphAttentionEmbedding(
            node_features=self.node_raw_features, edge_features=self.edge_raw_features,
            neighbor_finder=self.ngh_finder, num_neighbor=self.num_neighbors, time_encoder=self.time_encoder,
            n_layers=self.num_layers, n_node_features=self.n_node_features, n_edge_features=self.n_edge_features,
            n_time_features=self.n_node_features, embedding_dimension=self.embedding_dimension, device=self.device,
            n_heads=n_heads, dropout=dropout, use_memory=self.use_memory)
        self.affinity_score = MergeLayer(self.n_node_features, self.n_node_features, self.n_node_features, 1)
        # the reference pairs attention rows with mask / explanation rows head-major through
        # .repeat(n_head, 1, 1) (embedding_module.py:74-75, :211-212); False pairs row r with row r
        self.head_major_rows = head_major_rows
        self._pack_cache = None
        self._pack_key = None

    # -------------------------------------------------------------- device pack
    def _dev(self):
        if self.device is not None and torch.device(self.device).type == "cuda":
            return L.require_device(self.device)
        p = self.n_feat_th
        return L.require_device(p.device if p.device.type == "cuda" else None)

    def _param_key(self):
        key = [(t.data_ptr(), t._version) for t in self.parameters()]
        if self.use_memory:
            key.append(tuple((n, len(v), id(v[-1][0]) if v else 0) for n, v in sorted(self.memory.messages.items())))
        return tuple(key)

    def updated_memory(self, dev=None):
        """get_updated_memory(list(range(n_nodes)), memory.messages) (tgn.py:237-248) on the device:
        each node with stored raw messages gets one memory-updater step from its aggregated message."""
        dev = dev or self._dev()
        mem = self.memory.memory.detach().to(dev, torch.float32).clone()
        if not self.memory_update_at_start:
            return mem
        nodes = [n for n in sorted(self.memory.messages) if len(self.memory.messages[n]) > 0]
        if not nodes:
            return mem
        msgs = self.memory.messages
        if self.aggregator_type == "last":
            raw = torch.stack([msgs[n][-1][0].detach().to(dev, torch.float32) for n in nodes])
        else:
            raw = torch.stack([torch.stack([m[0].detach().to(dev, torch.float32) for m in msgs[n]]).mean(0)
                               for n in nodes])
        idx = torch.tensor(nodes, dtype=torch.long, device=dev)
        with torch.no_grad():
            fn = self.message_function
            if isinstance(fn, MLPMessageFunction):
                l0, l2 = fn.mlp[0], fn.mlp[2]
                raw = F.linear(F.relu(F.linear(raw, l0.weight.to(dev), l0.bias.to(dev))), l2.weight.to(dev),
                               l2.bias.to(dev))
            cell = self.memory_updater.memory_updater
            h = mem[idx]
            if isinstance(cell, nn.GRUCell):
                gi = F.linear(raw, cell.weight_ih.to(dev), cell.bias_ih.to(dev))
                gh = F.linear(h, cell.weight_hh.to(dev), cell.bias_hh.to(dev))
                ir, iz, inn = gi.chunk(3, 1)
                hr, hz, hn = gh.chunk(3, 1)
                r = torch.sigmoid(ir + hr)
                z = torch.sigmoid(iz + hz)
                n = torch.tanh(inn + r * hn)
                mem[idx] = (h - n) * z + n
            else:
                mem[idx] = torch.tanh(F.linear(raw, cell.weight_ih.to(dev), cell.bias_ih.to(dev))
                                      + F.linear(h, cell.weight_hh.to(dev), cell.bias_hh.to(dev)))
        return mem

    def _pack(self):
        """Device-resident tables and folded per-layer weights, rebuilt when a parameter changes."""
        dev = self._dev()
        key = (dev, self._param_key())
        if self._pack_cache is not None and self._pack_key == key:
            return self._pack_cache
        f32 = torch.float32
        with torch.no_grad():
            nf = self.n_feat_th.detach().to(dev, f32)
            tab = (self.updated_memory(dev) + nf) if self.use_memory else nf.clone()
            tw = self.time_encoder.w.weight.detach().to(dev, f32).reshape(-1).contiguous()
            tb = self.time_encoder.w.bias.detach().to(dev, f32).contiguous()
            layers = []
            for lay in self.embedding_module.attention_models[:2]:
                mh = lay.multi_head_target
                H, dk = mh.n_head, mh.d_k
                wq = mh.w_qs.weight.detach().to(dev, torch.float64).view(H, dk, -1)     # [H, dk, dq]
                wk = mh.w_ks.weight.detach().to(dev, torch.float64).view(H, dk, dk)     # [H, dk(out), dk(in)]
                wv = mh.w_vs.weight.detach().to(dev, torch.float64).view(H, dk, dk)
                fc = mh.fc.weight.detach().to(dev, torch.float64)                       # [dq, H*dk]
                P = torch.einsum("hoi,hoq->hiq", wk, wq).reshape(H * dk, -1)             # W_k,h^T W_q,h
                G = torch.einsum("qho,hoi->qhi", fc.view(fc.shape[0], H, dk), wv).reshape(fc.shape[0], H * dk)
                layers.append(dict(
                    P=P.to(f32).contiguous(), G=G.to(f32).contiguous(), fcb=mh.fc.bias.detach().to(dev, f32),
                    lnw=mh.layer_norm.weight.detach().to(dev, f32), lnb=mh.layer_norm.bias.detach().to(dev, f32),
                    m1w=lay.merger.fc1.weight.detach().to(dev, f32), m1b=lay.merger.fc1.bias.detach().to(dev, f32),
                    m2w=lay.merger.fc2.weight.detach().to(dev, f32), m2b=lay.merger.fc2.bias.detach().to(dev, f32),
                    H=H, dk=dk, temperature=mh.temperature))
            aff = self.affinity_score
            pack = dict(dev=dev, tab=tab.contiguous(), etab=self.e_feat_th.detach().to(dev, f32).contiguous(),
                        tw=tw, tb=tb, cosb=torch.cos(tb), layers=layers,
                        a1w=aff.fc1.weight.detach().to(dev, f32), a1b=aff.fc1.bias.detach().to(dev, f32),
                        a2w=aff.fc2.weight.detach().to(dev, f32), a2b=aff.fc2.bias.detach().to(dev, f32),
                        err=torch.zeros(1, dtype=torch.int32, device=dev))
        self._pack_cache, self._pack_key = pack, key
        return pack

    # -------------------------------------------------------------- forward pieces
    def _layer(self, pk, li, src_feat, R, N, node_idx, ngh_dense, edge_idx, edge_dense, dt, mask_node, ew, seg=0,
               cache=None):
        """One TemporalAttentionLayer over R source rows (embedding_module.py:181-216).  ``cache`` (the
        prepared inputs' dict): the query and its folded projection depend on the source rows and the frozen
        weights only, so the training step's two contrasts of one batch (temp_exp_main.py:597, :611) compute
        them once."""
        lw = pk["layers"][li]
        H, dk = lw["H"], lw["dk"]
        dn = self.n_node_features
        key = ("qf", li, id(pk))
        hit = cache.get(key) if cache is not None else None
        if hit is not None and hit[0] is pk:
            query, qf = hit[1], hit[2]
        else:
            query = torch.cat([src_feat(), pk["cosb"].expand(R, dn)], dim=1)    # [R, dq]
            qf = (query @ lw["P"].t()).contiguous()                            # [R, H*dk]
            if cache is not None:
                cache[key] = (pk, query, qf)
        src_feat = query[:, :dn]
        de = edge_dense.shape[-1] if edge_dense is not None else self.n_edge_features
        if dn + de + dn != dk:
            raise AssertionError(f"key dim {dn}+{de}+{dn} != {dk}")
        spec = dict(rows=R, n_ngh=N, n_head=H, d_key=dk, d_node=dn, d_edge=de, d_time=dn,
                    node_rows=pk["tab"].shape[0], edge_rows=pk["etab"].shape[0], head_major=self.head_major_rows,
                    temperature=lw["temperature"], node_tab=pk["tab"], node_idx=node_idx,
                    edge_tab=edge_dense if edge_dense is not None else pk["etab"],
                    edge_idx=None if edge_dense is not None else edge_idx, dt=dt, time_w=pk["tw"],
                    time_b=pk["tb"], mask_node=mask_node, err=pk["err"], seg_rows=seg)
        z = _TgnAttnFn.apply(qf, ngh_dense, ew, spec)
        out = torch.addmm(lw["fcb"], z, lw["G"].t())
        h = F.layer_norm(out + query, (query.shape[1],), lw["lnw"], lw["lnb"], 1e-5)
        x = torch.cat([h, src_feat], dim=1)
        return F.linear(F.relu(F.linear(x, lw["m1w"], lw["m1b"])), lw["m2w"], lw["m2b"])

    def node_embeddings(self, nodes, eids, times, cut_time, explain_weights=None, edge_attr=None, n_segments=1,
                        prepared=None):
        """embedding_update(_attr) + embedding_update_layer (embedding_module.py:314-393) for
        nodes = [n0 [R1], n1 [R1,N], n2 [R1,N^2]], eids/times = [hop1, hop2] -> [R1, d].
        n_segments > 1 stacks independent contrast batches (R1 = n_segments * 3B rows): every row
        gives the same result as in its own call (the head-major pairing stays inside its batch).
        ``prepared``: the output of ``_prep_inputs`` for these inputs (built once when the same
        subgraphs go through several contrasts, as the training step's two do)."""
        if self.use_memory and not self.forbidden_memory_update:
            raise NotImplementedError("stateful memory updates inside contrast (tgn.py:167-199) are not part of "
                                      "this build; set forbidden_memory_update=True as temp_exp_main.py:704 does")
        pk = self._pack()
        x = prepared if prepared is not None else self._prep_inputs(nodes, eids, times, cut_time, edge_attr, n_segments)
        R1, N, seg1 = x["R1"], x["N"], x["seg1"]
        dev = pk["dev"]
        ew1 = ew2 = None
        if explain_weights is not None:
            ew1 = explain_weights[0].to(dev, torch.float32).reshape(R1, N).contiguous()
            ew2 = explain_weights[1].to(dev, torch.float32).reshape(R1 * N, N).contiguous()
        tab = pk["tab"]
        # layer 0 (attention_models[0]): hop-1 nodes attend over their hop-2 neighbours
        cache = x if prepared is not None else None
        y0 = self._layer(pk, 0, lambda: tab[x["n1l"]], R1 * N, N, x["n2f"], None, x["e2"], x["ed2"], x["dt2"],
                         x["n2f"], ew2, seg1 * N, cache)
        # layer 1 (attention_models[1]): roots attend over the hop-1 embeddings
        y1 = self._layer(pk, 1, lambda: tab[x["n0"]], R1, N, None, y0.contiguous(), x["e1"], x["ed1"], x["dt1"],
                         x["n1f"], ew1, seg1, cache)
        return y1

    def _prep_inputs(self, nodes, eids, times, cut_time, edge_attr=None, n_segments=1):
        """node_embeddings' index, time-offset and edge-attribute tensors (retrieve_time_features etc.)."""
        dev = self._dev()
        i32 = torch.int32
        n0 = _as_dev(nodes[0], dev, torch.long).reshape(-1)
        R1 = n0.shape[0]
        n1 = _as_dev(nodes[1], dev, i32).reshape(R1, -1)
        N = n1.shape[1]
        n2 = _as_dev(nodes[2], dev, i32).reshape(R1 * N, N)
        cut = _as_dev(cut_time, dev, torch.float64).reshape(-1)
        if cut.shape[0] * 3 * n_segments == R1:
            cut = cut.repeat(3 * n_segments)
        if cut.shape[0] != R1 or R1 % n_segments:
            raise AssertionError("cut_time must give one time per event (or per root row)")
        seg1 = R1 // n_segments if n_segments > 1 else 0
        t1 = _as_dev(times[0], dev, torch.float64).reshape(R1, N)
        t2 = _as_dev(times[1], dev, torch.float64).reshape(R1, N, N)
        dt1 = (cut.view(R1, 1) - t1).float().contiguous()                     # retrieve_time_features
        dt2 = (t1.view(R1, N, 1) - t2).float().contiguous()
        if edge_attr is None:
            e1 = _as_dev(eids[0], dev, i32).reshape(-1).contiguous()
            e2 = _as_dev(eids[1], dev, i32).reshape(-1).contiguous()
            ed1 = ed2 = None
        else:
            if any(isinstance(x, torch.Tensor) and x.requires_grad for x in edge_attr):
                raise NotImplementedError("gradient with respect to edge_attr")
            e1 = e2 = None
            ed1 = _as_dev(edge_attr[0], dev, torch.float32).reshape(R1 * N, -1).contiguous()
            ed2 = _as_dev(edge_attr[1], dev, torch.float32).reshape(R1 * N * N, -1).contiguous()
        return dict(R1=R1, N=N, seg1=seg1, n0=n0, n1l=n1.reshape(-1).long(), n1f=n1.reshape(-1).contiguous(),
                    n2f=n2.reshape(-1).contiguous(), dt1=dt1.reshape(-1), dt2=dt2.reshape(-1), e1=e1, e2=e2,
                    ed1=ed1, ed2=ed2)

    def check_errors(self):
        """Raise if a kernel saw an out-of-range node or edge index (synchronises)."""
        pk = self._pack_cache
        if pk is not None and int(pk["err"].item()) != 0:
            pk["err"].zero_()
            raise IndexError("TGN: node or edge index out of range of the feature tables")

    # -------------------------------------------------------------- reference API
    def get_node_emb(self, src_idx, tgt_idx, bgd_idx, cut_time, e_idx, subgraph_src, subgraph_tgt, subgraph_bgd,
                     explain_weights=None, edge_attr=None, prepared=None):
        """tgn.py:99-199 -> (source, destination, negative) embeddings [B, d] each."""
        B = len(src_idx)
        if prepared is None:
            prepared = self.prepare_contrast(src_idx, tgt_idx, bgd_idx, cut_time, subgraph_src, subgraph_tgt,
                                             subgraph_bgd, edge_attr)
        emb = self.node_embeddings(None, None, None, None, explain_weights, edge_attr, prepared=prepared)
        # split (one backward: a cat of the three gradients) rather than three slices (a zero-filled full-size
        # gradient, a copy and an add each)
        return tuple(emb.split(B)) if B > 0 else (emb[:0], emb[:0], emb[:0])

    def prepare_contrast(self, src_idx, tgt_idx, bgd_idx, cut_time, subgraph_src, subgraph_tgt, subgraph_bgd,
                         edge_attr=None):
        """The inputs contrast derives from its batch (the three sides' roots and subgraphs
        concatenated, time offsets), built once: the training step's two contrasts of the same batch
        (without and with explanation weights, temp_exp_main.py:597, :611) share them."""
        dev = self._dev()
        roots = torch.cat([_as_dev(x, dev, torch.long).reshape(-1) for x in (src_idx, tgt_idx, bgd_idx)])

        def cat(i, h, dtype):
            xs = [sg[i][h] for sg in (subgraph_src, subgraph_tgt, subgraph_bgd)]
            if all(isinstance(x, torch.Tensor) and x.device == dev for x in xs):
                # the three sides of a gathered pack are consecutive rows of one tensor: one view, and one
                # dtype conversion instead of three (elementwise, so the same values as convert-then-cat)
                return _as_dev(_cat_rows(xs), dev, dtype)
            return torch.cat([_as_dev(x, dev, dtype) for x in xs])
        nodes = [roots, cat(0, 0, torch.int32), cat(0, 1, torch.int32)]
        eids = [cat(1, 0, torch.int32), cat(1, 1, torch.int32)] if edge_attr is None else [None, None]
        times = [cat(2, 0, torch.float64), cat(2, 1, torch.float64)]
        return self._prep_inputs(nodes, eids, times, cut_time, edge_attr)

    def affinity(self, x1, x2):
        pk = self._pack()
        h = F.relu(F.linear(torch.cat([x1, x2], dim=1), pk["a1w"], pk["a1b"]))
        return F.linear(h, pk["a2w"], pk["a2b"])

    def contrast(self, src_idx, tgt_idx, bgd_idx, cut_time, e_idx, subgraph_src, subgraph_tgt, subgraph_bgd,
                 explain_weights=None, edge_attr=None, prepared=None):
        """tgn.py:201-218 -> (pos_score [B,1], neg_score [B,1]).  ``prepared``: prepare_contrast's
        output for these same inputs (optional, shared by several contrasts of one batch)."""
        B = len(src_idx)
        if prepared is None:
            prepared = self.prepare_contrast(src_idx, tgt_idx, bgd_idx, cut_time, subgraph_src, subgraph_tgt,
                                             subgraph_bgd, edge_attr)
        emb = self.node_embeddings(None, None, None, None, explain_weights, edge_attr, prepared=prepared)
        if B == 0:
            return emb[:0, :1], emb[:0, :1]
        # get_node_emb's (s, d, n) as two pieces of one split: [d; n] is emb's tail (no copy), and the backward
        # is one cat instead of a zero-filled full-size gradient, a copy and an add per slice
        s, dn = emb.split([B, 2 * B])
        score = self.affinity(torch.cat([s, s], dim=0), dn).squeeze(dim=0)
        return tuple(score.split(B))

    def retrieve_edge_features(self, subgraph_src, subgraph_tgt, subgraph_bgd):
        """tgn.py:220-228: [E_feat[hop-1 eids], E_feat[hop-2 eids]] for the three sides."""
        dev = self._dev()
        et = self._pack()["etab"]
        out = []
        for h in (0, 1):
            idx = torch.cat([_as_dev(sg[1][h], dev, torch.long) for sg in (subgraph_src, subgraph_tgt, subgraph_bgd)])
            out.append(et[idx])
        return out

    def set_neighbor_sampler(self, neighbor_finder):
        self.embedding_module.neighbor_sampler = neighbor_finder

    def grab_subgraph(self, src_idx_l, cut_time_l):
        """tgn.py:283-285."""
        return self.embedding_module.neighbor_sampler.find_k_hop(2, src_idx_l, cut_time_l,
                                                                 num_neighbors=self.num_neighbors, e_idx_l=None)

    def embedding_temperature(self, layer=0):
        return self.embedding_module.attention_models[layer].multi_head_target.temperature


def node_records_cat(subgraph, dev):
    """[hop-1 | hop-2] node records of one side as one int32 device tensor [B, N + N^2]."""
    return torch.cat([_as_dev(subgraph[0][0], dev, torch.int32), _as_dev(subgraph[0][1], dev, torch.int32)], dim=1)


__all__ = ["TGN", "TimeEncode", "MergeLayer", "TemporalAttentionLayer", "MultiHeadAttention", "Memory",
           "node_records_cat"]
