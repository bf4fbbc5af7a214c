"""Drop-in ``TempME`` explainer (models/explainer_new.py:99-453) on the HIP encoder.

Same constructor, submodule names (so a reference ``state_dict`` loads as is), same
construction order (so ``torch.manual_seed(s); TempME(...)`` draws the same initial
weights as the reference), same ``forward`` / ``retrieve_edge_imp_node`` /
``retrieve_explanation`` / ``beta_sample`` / ``kl_loss`` signatures and shapes.

Eval-mode scoring (``forward`` under ``model.eval()`` and
``retrieve_explanation(..., training=False)``) runs entirely in libtempme_hip.so:
tm_encoder_fwd_tab (event features with lin_event's edge-feature product read from a
per-edge-id table built once per weight version by tm_edge_feature_table, event_gcn x2,
temporal-aware attention, MLP) and tm_edge_importance (dependency gate, walk->edge
scatter-max, gather, Beta mean, mask).  Training-mode calls (dropout, Beta ``rsample``,
gradients) run the HIP forward/backward kernels through autograd Functions
(tm_encoder_train_fwd / tm_encoder_bwd / tm_encoder_wgrad, tm_explain_train_fwd / _bwd,
tm_kl_loss); only Beta ``rsample`` and the padding mask are torch ops.
"""
import operator
import os
import threading
import warnings

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L
from .null_model import get_null_distribution

# the training explanation's padding mask comes from the explanation kernel (tm_explain_train_fwd_pad) instead of
# a torch comparison: bitwise the same mask (tests/test_gpu_variants.py flips this to compare the two)
_EXPLAIN_PAD = True


class TimeEncode(nn.Module):
    """explainer_new.py:45-59."""

    def __init__(self, expand_dim):
        super().__init__()
        self.time_dim = expand_dim
        self.basis_freq = nn.Parameter(torch.from_numpy(1 / 10 ** np.linspace(0, 9, self.time_dim)).float())
        self.phase = nn.Parameter(torch.zeros(self.time_dim).float())

    def forward(self, ts):
        b, s = ts.size(0), ts.size(1)
        m = ts.view(b, s, 1) * self.basis_freq.view(1, 1, -1)
        m = m + self.phase.view(1, 1, -1)
        return torch.cos(m)


class Attention(nn.Module):
    """explainer_new.py:12-43 (use_temporal_guidance=False)."""

    def __init__(self, input_dim, hid_dim):
        super().__init__()
        self.hidden_size = hid_dim
        self.W1 = nn.Linear(input_dim, input_dim)
        self.W2 = nn.Linear(input_dim, input_dim)
        self.MLP = nn.Sequential(nn.Linear(input_dim, hid_dim), nn.ReLU(), nn.Linear(hid_dim, hid_dim))
        nn.init.xavier_uniform_(self.W2.weight.data)
        self.W2.bias.data.fill_(0.1)


class TemporalAwareAttention(nn.Module):
    """explainer_new.py:768-846."""

    def __init__(self, input_dim, hid_dim, dropout_p=0.1):
        super().__init__()
        self.hidden_size = hid_dim
        self.W1 = nn.Linear(input_dim, input_dim)
        self.W2 = nn.Linear(input_dim, input_dim)
        self.W_time = nn.Linear(1, input_dim)
        self.dropout = nn.Dropout(dropout_p)
        self.MLP = nn.Sequential(nn.Linear(input_dim, hid_dim), nn.ReLU(), nn.Dropout(dropout_p),
                                 nn.Linear(hid_dim, hid_dim))
        nn.init.xavier_uniform_(self.W2.weight.data)
        self.W2.bias.data.fill_(0.1)
        nn.init.xavier_uniform_(self.W_time.weight.data)


class _MergeLayer(nn.Module):
    def __init__(self, input_dim, hid_dim):
        super().__init__()
        self.fc1 = nn.Linear(2 * input_dim, hid_dim)
        self.fc2 = nn.Linear(hid_dim, 1)
        nn.init.xavier_normal_(self.fc1.weight)
        nn.init.xavier_normal_(self.fc2.weight)
        self.act = nn.ReLU()


class event_gcn(nn.Module):  # noqa: N801  (reference name, kept for state_dict keys)
    def __init__(self, event_dim, node_dim, hid_dim):
        super().__init__()
        self.lin_event = nn.Linear(event_dim, node_dim)
        self.relu = nn.ReLU()
        self.MLP = nn.Sequential(nn.Linear(node_dim, hid_dim), nn.ReLU(), nn.Linear(hid_dim, hid_dim))

    def forward(self, event_feature, src_features, tgt_features):
        event = self.lin_event(event_feature)
        return self.MLP(src_features + self.relu(tgt_features + event))


def _to(x, device, dtype):
    if isinstance(x, torch.Tensor):
        if x.dtype == dtype and x.device == device:
            return x
        return x.to(device=device, dtype=dtype)
    return torch.from_numpy(np.ascontiguousarray(x)).to(device=device, dtype=dtype)


_NP = {torch.int32: np.int32, torch.float32: np.float32, torch.float64: np.float64}


class _Stager:
    """Host arrays of one drop-in call -> device tensors in ONE host->device copy: each array is cast on
    the host (numpy's float->int truncation and float64->float32 rounding are torch's) into a pinned
    buffer, the buffer is copied asynchronously into a fresh caching-allocator block, and the results
    are views of it.  The reference's loop hands every call float64 numpy arrays; one pageable copy and
    one cast kernel per array (six per forward, six per retrieve_edge_imp_node) dominated a batch.
    Pinned buffers rotate over ``slots``; a slot is rewritten only after its previous copy finished."""

    def __init__(self, slots=4):
        self.slots = [None] * slots
        self.i = 0
        self.lock = threading.Lock()   # the slots are shared by every TempME instance of the process

    def __call__(self, device, items):
        with self.lock:
            return self._stage(device, items)

    def _stage(self, device, items):
        shapes = [np.shape(a) for a, _ in items]
        nbytes = [int(np.prod(s, dtype=np.int64)) * np.dtype(_NP[d]).itemsize for s, (_, d) in zip(shapes, items)]
        offs, tot = [], 0
        for n in nbytes:
            offs.append(tot)
            tot += (n + 15) & ~15
        k = self.i
        self.i = (self.i + 1) % len(self.slots)
        slot = self.slots[k]
        if slot is None or slot[0].numel() < tot:
            slot = [torch.empty(max(tot, 1 << 16) * 2, dtype=torch.uint8, pin_memory=True), None]
            self.slots[k] = slot
        elif slot[1] is not None:
            slot[1].synchronize()
        host = slot[0].numpy()
        for (a, d), s, o, n in zip(items, shapes, offs, nbytes):
            np.copyto(host[o:o + n].view(_NP[d]).reshape(s), a, casting="unsafe")
        # the copy and its event on the current stream of `device` (not of the process's current device),
        # so the slot's next reuse waits for this very copy
        with torch.cuda.device(device):
            dev = torch.empty(max(tot, 1), dtype=torch.uint8, device=device)
            dev.copy_(slot[0][:max(tot, 1)], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(device))
        slot[1] = ev
        return [dev[o:o + n].view(d).view(s) for (_, d), s, o, n in zip(items, shapes, offs, nbytes)]


_STAGE = _Stager()

# Generation of the process's module/parameter registrations (torch's global registration hooks fire on
# every submodule or parameter assignment, load_state_dict(assign=True) included): TempME's cached weight
# list is re-validated only when it moved, instead of walking its ~100 links on every call.
_REG_GEN = [0]


def _bump_gen(*_args):
    _REG_GEN[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump_gen)
torch.nn.modules.module.register_module_module_registration_hook(_bump_gen)


_EXT = [None, False]


def _dropin_ext():
    """tempme_amd/lib/_dropin_ext*.so (csrc/dropin_ext.cpp, built by __graft_entry__.build()): the C++ host
    side of the drop-in fast path (checked against the Python host side on the GPU,
    tests/test_gpu_enron.py::test_dropin_cpp_host_side_equals_python_host_side).  Without it the same fast path
    runs its host side in Python (same kernels, same results), with a warning."""
    if not _EXT[1]:
        _EXT[1] = True
        import importlib.machinery
        import importlib.util
        import os
        import sysconfig
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                            "_dropin_ext" + sysconfig.get_config_var("EXT_SUFFIX"))
        if os.path.exists(path):
            loader = importlib.machinery.ExtensionFileLoader("tempme_amd._dropin_ext", path)
            spec = importlib.util.spec_from_file_location("tempme_amd._dropin_ext", path, loader=loader)
            mod = importlib.util.module_from_spec(spec)
            loader.exec_module(mod)
            _EXT[0] = mod
        else:
            warnings.warn("tempme_amd/lib/_dropin_ext*.so not built (python tempme_amd/_build_ext.py): the drop-in "
                          "fast path's host side runs in Python", RuntimeWarning, stacklevel=3)
    return _EXT[0]


def _hoststage():
    from . import hoststage
    return hoststage


def _to_many(device, *items):
    """[_to(a, device, dtype) for (a, dtype) in items], staged through one pinned copy when every
    array is a host numpy array and the device is a GPU."""
    if device.type == "cuda" and all(isinstance(a, np.ndarray) and d in _NP for a, d in items):
        return _STAGE(device, items)
    return [_to(a, device, d).contiguous() for a, d in items]


class TempME(nn.Module):
    def __init__(self, base, base_model_type, data, out_dim, hid_dim, prior="empirical", temp=0.07,
                 if_cat_feature=True, dropout_p=0.1, device=None, use_temporal_guidance=True,
                 use_dependency_aware_sampling=True, *, null_model=None, data_dir=None, seed=0):
        super().__init__()
        self.node_dim = base.n_feat_th.shape[1]
        self.edge_dim = base.e_feat_th.shape[1]
        self.time_dim = self.node_dim
        self.out_dim = out_dim
        self.hid_dim = hid_dim
        self.base_type = base_model_type
        self.dropout_p = dropout_p
        self.temp = temp
        self.prior = prior
        self.if_cat = if_cat_feature
        self.dropout = nn.Dropout(dropout_p)
        self.device = device
        self.event_dim = self.edge_dim + self.time_dim + 3
        self.event_conv = event_gcn(event_dim=self.event_dim, node_dim=self.node_dim, hid_dim=self.hid_dim)
        self.use_temporal_guidance = use_temporal_guidance
        self.attention = (TemporalAwareAttention(2 * self.hid_dim, self.hid_dim) if use_temporal_guidance
                          else Attention(2 * self.hid_dim, self.hid_dim))
        self.mlp_dim = self.hid_dim + 12 if self.if_cat else self.hid_dim
        self.MLP = nn.Sequential(nn.Linear(self.mlp_dim, self.mlp_dim), nn.ReLU(), nn.Dropout(self.dropout_p),
                                 nn.Linear(self.mlp_dim, self.hid_dim), nn.ReLU(), nn.Linear(self.hid_dim, 1))
        self.final_linear = nn.Linear(2 * self.hid_dim, self.hid_dim)
        self.node_emd_dim = self.hid_dim + 12 + self.node_dim if self.if_cat else self.hid_dim + self.node_dim
        self.affinity_score = _MergeLayer(self.node_emd_dim, self.node_emd_dim)
        self.edge_raw_embed = base.edge_raw_features
        self.node_raw_embed = base.node_raw_features
        self.time_encoder = TimeEncode(expand_dim=self.time_dim)
        self.null_model = (null_model if null_model is not None
                           else get_null_distribution(data, data_dir=data_dir, seed=seed, device=device))
        num_nodes = base.n_feat_th.shape[0]
        self.node_degree = torch.ones(num_nodes, device=device if device else torch.device("cpu"))
        self.use_dependency_aware_sampling = use_dependency_aware_sampling
        if use_dependency_aware_sampling:
            self.edge_dependency_gcn = nn.Sequential(
                nn.Linear(self.edge_dim + self.time_dim, self.hid_dim), nn.ReLU(), nn.Dropout(dropout_p * 1.5),
                nn.Linear(self.hid_dim, self.hid_dim // 2), nn.ReLU(), nn.Dropout(dropout_p),
                nn.Linear(self.hid_dim // 2, 1))
            self.edge_importance_attention = nn.MultiheadAttention(embed_dim=self.hid_dim, num_heads=4,
                                                                   dropout=dropout_p, batch_first=True)
            self.edge_to_node_transform = nn.Sequential(nn.Linear(self.edge_dim, self.hid_dim), nn.ReLU(),
                                                        nn.Linear(self.hid_dim, self.hid_dim))
            self.gumbel_temperature = 1.0
            self.min_gumbel_temperature = 0.5
            self.gumbel_anneal_rate = 0.003
        self._packed = None
        self._packed_key = None

    # ------------------------------------------------------------------ HIP plumbing
    def _dev(self):
        d = self.__dict__.get("_dev_cache")
        if d is None or d[0] is not self.device:
            d = self.__dict__["_dev_cache"] = (self.device, L.require_device(self.device))
        return d[1]

    def _needs_autograd(self):
        """Training mode, or a forward whose result must carry gradients to the explainer's
        parameters (temp_exp_main.py:605-631): the autograd formulation runs then.  Only the parameters
        the forward / explanation read matter (the cached weight list; no walk over every submodule)."""
        if self.training:
            return True
        if not torch.is_grad_enabled():
            return False
        return any(p.requires_grad for p in self._weight_list())

    def _hip_eval_ok(self):
        """The eval kernels cover every constructor variant (use_temporal_guidance /
        use_dependency_aware_sampling through tm_weights_variant, if_cat_feature and hid_dim through
        tm_weights_create_ex) for hid_dim up to 256: the fused walk kernel for the default shape (hid_dim 64
        with the category feature), the LDS-tiled kernels for the others; a hid_dim that is not a multiple of
        16 runs them on weights zero-padded to the next one (_pad_hidden)."""
        if not 0 < self.hid_dim <= 256:
            # no silent fallback: the eval kernels' LDS tiles hold at most a 256-wide hidden layer
            raise L.TempMEError("TempME(hid_dim=%d): the HIP encoder kernels cover hid_dim 1..256 (their LDS tiles "
                                "hold at most a 256-wide hidden layer); no other path exists on the device"
                                % self.hid_dim)
        return True

    def _hip_ok(self):
        """The training kernels (f3) cover every constructor variant (use_temporal_guidance,
        use_dependency_aware_sampling, if_cat_feature) for the dims tm_encoder_train_supported accepts:
        hid_dim a multiple of 16 whose tiles fit the LDS (every hid_dim up to 192 at Enron / Wikipedia
        feature dims)."""
        key = (self.edge_dim, self.node_dim, self._hid_packed(), bool(self.if_cat))
        c = self.__dict__.get("_train_ok")
        if c is None or c[0] != key:
            ok = self._hip_eval_ok() and bool(L.lib().tm_encoder_train_supported(*[int(x) for x in key]))
            c = self.__dict__["_train_ok"] = (key, ok)
        ok = c[1]
        if not ok and not getattr(self, "_warned_torch_train", False):
            warnings.warn("TempME(if_cat_feature=%s, hid_dim=%d, edge_dim=%d, node_dim=%d): no HIP training kernel "
                          "instance for these dims; gradients run through the torch-op formulation on the device"
                          % (self.if_cat, self.hid_dim, self.edge_dim, self.node_dim), RuntimeWarning, stacklevel=3)
            self._warned_torch_train = True
        return ok

    def _weight_list(self):
        """The encoder's parameters in pack order.  Cached: walking the submodules through
        nn.Module.__getattr__ cost ~35 us per call, several calls per drop-in forward.  The cache holds,
        beside the list, every (module dict, key, object) link from the explainer down to each listed
        parameter; it is reused only while every link still holds the same object, so reassigning a
        submodule at any depth (``ex.MLP[0] = nn.Linear(...)``), a parameter (``lin.weight =
        nn.Parameter(...)``, ``load_state_dict(..., assign=True)``) or moving the module rebuilds it."""
        c = self.__dict__.get("_wl_cache")
        if c is not None:
            wl, links, gen = c
            if gen == _REG_GEN[0]:
                return wl
            if all(d.get(k) is v for d, k, v in links):
                self.__dict__["_wl_cache"] = (wl, links, _REG_GEN[0])
                return wl
        wl, links = self._build_weight_list()
        self.__dict__["_wl_cache"] = (wl, links, _REG_GEN[0])
        return wl

    def _weight_paths(self):
        # TemporalAwareAttention.MLP = (Linear, ReLU, Dropout, Linear), Attention.MLP = (Linear, ReLU, Linear)
        a_last = "3" if isinstance(self.attention, TemporalAwareAttention) else "2"
        paths = [("event_conv", "lin_event"), ("event_conv", "MLP", "0"), ("event_conv", "MLP", "2"),
                 ("attention", "W1"), ("attention", "W2"), ("attention", "MLP", "0"), ("attention", "MLP", a_last),
                 ("MLP", "0"), ("MLP", "3"), ("MLP", "5")]
        if self.use_dependency_aware_sampling:
            paths += [("edge_dependency_gcn", "0"), ("edge_dependency_gcn", "3"), ("edge_dependency_gcn", "6")]
        return paths

    def _build_weight_list(self):
        links, ts = [], []

        def param(mod, name):
            p = mod._parameters[name]
            links.append((mod._parameters, name, p))
            return p

        for path in self._weight_paths():
            mod = self
            for k in path:
                child = mod._modules[k]
                links.append((mod._modules, k, child))
                mod = child
            ts += [param(mod, "weight"), param(mod, "bias")]
        if not self.use_dependency_aware_sampling:
            # no gate (tm_weights_variant(dep = 0)): shape-correct zeros keep the pack layout
            h = self.hid_dim
            dev = self.node_raw_embed.weight.device
            zg = getattr(self, "_zero_gate", None)
            if zg is None or zg[0].device != dev:
                z = lambda *sh: torch.zeros(*sh, device=dev)  # noqa: E731
                self._zero_gate = [z(h, self.edge_dim + self.time_dim), z(h), z(h // 2, h), z(h // 2), z(1, h // 2), z(1)]
            ts += self._zero_gate
        te = self._modules["time_encoder"]
        links.append((self._modules, "time_encoder", te))
        ts += [param(te, "basis_freq"), param(te, "phase")]
        return ts, links

    def packed_weights(self, force=False):
        """tm_weights handle, re-packed whenever a parameter changed (version counters) or when forced
        (a step captured as a HIP graph must record its repack launch: GraphedTrainStep)."""
        dev = self._dev()
        ws = self._weight_list()
        key = tuple((w.data_ptr(), w._version) for w in ws)
        if self._packed is None or self._packed_key != key or force:
            if self._packed is None:
                h = L.C.c_void_p()
                L.check(L.lib().tm_weights_create_ex(self.edge_dim, self.node_dim, self._hid_packed(),
                                                     int(bool(self.if_cat)), dev.index, L.C.byref(h)),
                        "tm_weights_create")
                self._packed = _Packed(h)
                L.check(L.lib().tm_weights_variant(h, int(bool(self.use_temporal_guidance)),
                                                   int(bool(self.use_dependency_aware_sampling))), "tm_weights_variant")
                self.feature_tables()
                self._set_node_zero(h)
            self._raw = [w.detach().to(device=dev, dtype=torch.float32).contiguous() for w in ws]
            if self._hid_packed() != self.hid_dim:
                self._raw = self._pad_hidden(self._raw)
            arr = (L.C.c_void_p * L.N_WEIGHTS)(*[w.data_ptr() for w in self._raw])
            L.check(L.lib().tm_weights_pack(self._packed.h, arr, L.stream_ptr(dev)), "tm_weights_pack")
            self._packed_key = key
            self._prep_dirty = self._prep_dirty_fast = True   # side streams must wait for this work
        return self._packed.h

    def _hid_packed(self):
        """The hidden width the kernels run at: hid_dim rounded up to a multiple of 16 (their tile)."""
        return -(-self.hid_dim // 16) * 16

    def _pad_maps(self, dev):
        """Index maps of the zero-padding (_pad_hidden), cached per device: hm = the h hidden units, gm = the
        gate's h // 2, m2 = [u_s | u_t] (2h -> 2H), cm = [out | one-hot 12] (mlp_dim -> H + 12), and per
        tm_weights index i the (rows map, padded rows, cols map, padded cols) of its weight (its bias, at
        i + 1, takes the rows map when padded rows > 1)."""
        c = self.__dict__.get("_pad_c")
        if c is not None and c[0] == dev:
            return c[1]
        h, H = self.hid_dim, self._hid_packed()
        ar = lambda n, o=0: torch.arange(n, device=dev) + o  # noqa: E731
        hm, gm, one = ar(h), ar(h // 2), ar(1)
        m2 = torch.cat([hm, ar(h, H)])
        cm = torch.cat([hm, ar(12, H)]) if self.if_cat else hm
        M2 = H + 12 if self.if_cat else H
        dn, kg = self.node_dim, self.edge_dim + self.time_dim
        spec = {2: (hm, H, ar(dn), dn), 4: (hm, H, hm, H), 6: (m2, 2 * H, m2, 2 * H), 8: (m2, 2 * H, m2, 2 * H),
                10: (hm, H, m2, 2 * H), 12: (hm, H, hm, H), 14: (cm, M2, cm, M2), 16: (hm, H, cm, M2),
                18: (one, 1, hm, H), 20: (hm, H, ar(kg), kg), 22: (gm, H // 2, hm, H), 24: (one, 1, gm, H // 2)}
        maps = dict(hm=hm, gm=gm, m2=m2, cm=cm, M2=M2, spec=spec)
        self.__dict__["_pad_c"] = (dev, maps)
        return maps

    def _pad_hidden(self, raw):
        """The tm_weights-ordered tensors of a hid_dim h that is not a multiple of 16, zero-padded to the
        packed width H (_hid_packed): every hidden unit past h gets zero weights and bias, so it carries
        ReLU(0) = 0 and adds exact zeros to every later sum -- the padded network computes the same function.
        The concatenations keep their parts' offsets at H: [u_s | u_t] (the attention's 2h input,
        explainer_new.py:768-846) maps column j >= h to H + j - h, and [out | one-hot 12] (mlp_dim,
        :174-201) the same; the gate's h // 2 layer pads to H // 2."""
        out = list(raw)
        for i, (rows, nr, cols, nc) in self._pad_maps(raw[0].device)["spec"].items():
            w = raw[i].new_zeros(nr, nc)
            w[rows[:, None], cols[None, :]] = raw[i]
            out[i] = w
            if nr > 1:
                b = raw[i + 1].new_zeros(nr)
                b[rows] = raw[i + 1]
                out[i + 1] = b
        return out

    def _unpad_grads(self, grads, idx):
        """Gradients the kernels wrote for the padded tensors of tm_weights indices ``idx`` -> the
        gradients of the module's own (unpadded) parameters: the rows / columns _pad_hidden placed."""
        if self._hid_packed() == self.hid_dim:
            return grads
        spec = self._pad_maps(grads[0].device)["spec"]
        out = list(grads)
        for k, i in enumerate(idx):
            if i in spec:
                rows, _, cols, _ = spec[i]
                out[k] = grads[k][rows[:, None], cols[None, :]]
            elif i - 1 in spec and spec[i - 1][1] > 1:
                out[k] = grads[k][spec[i - 1][0]]
        return out

    def _padded_shapes(self, idx):
        return [tuple(self._raw[i].shape) for i in idx]

    def _drop_packed(self, drop):
        """A dropout keep-mask in the module's column layout (dropout_cols: alpha 2 | attention.MLP hidden h |
        MLP hidden mlp_dim) -> the padded kernels' layout (2 | H | H + 12); a padded unit's column repeats
        column 0 (its activation is zero either way)."""
        if drop is None or self._hid_packed() == self.hid_dim:
            return drop
        m = self._pad_maps(drop.device)
        h, H = self.hid_dim, self._hid_packed()
        ncol = -(-(2 + H + m["M2"]) // 16) * 16
        src = torch.zeros(ncol, dtype=torch.long, device=drop.device)
        src[:2] = torch.arange(2, device=drop.device)
        src[2 + m["hm"]] = 2 + m["hm"]
        src[2 + H + m["cm"]] = 2 + h + torch.arange(self.mlp_dim, device=drop.device)
        return drop.index_select(1, src).contiguous()

    def _gate_masks_packed(self, masks):
        """edge_dependency_gcn's keep-masks [n_pos, h] / [n_pos, h // 2] -> [n_pos, H] / [n_pos, H // 2]."""
        k1, k2, sc1, sc2 = masks
        if k1 is None or self._hid_packed() == self.hid_dim:
            return masks
        m = self._pad_maps(k1.device)
        H = self._hid_packed()

        def widen(k, idx, n):
            src = torch.zeros(n, dtype=torch.long, device=k.device)
            src[idx] = torch.arange(idx.numel(), device=k.device)
            return k.index_select(1, src).contiguous()
        return widen(k1, m["hm"], H), widen(k2, m["gm"], H // 2), sc1, sc2

    def feature_tables(self):
        dev = self._dev()
        nw, ew = self.node_raw_embed.weight, self.edge_raw_embed.weight
        key = (nw.data_ptr(), nw._version, ew.data_ptr(), ew._version)
        if getattr(self, "_tables_key", None) != key:
            self._n_tab = nw.detach().to(device=dev, dtype=torch.float32).contiguous()
            self._e_tab = ew.detach().to(device=dev, dtype=torch.float32).contiguous()
            # every node-feature bit zero (the TGN-format datasets): the eval encoder computes one event_gcn
            # branch, the other being bit-identical (tm_weights_set_node_zero); one device reduction per table
            self._node_zero = bool((self._n_tab.view(torch.int32) == 0).all().item())
            self._tables_key = key
            self._prep_dirty = self._prep_dirty_fast = True   # side streams must wait for this work
            if getattr(self, "_packed", None) is not None:
                self._set_node_zero(self._packed.h)
            c = self.__dict__.get("_dropin_c")
            if c is not None:
                # the edge-feature table may have been rewritten in place (same address): the drop-in's gate-factor
                # cache keys on the address, so empty it explicitly
                fn = getattr(L.lib(), "tm_dropin_gate_cache_clear", None)   # absent in an older A/B build
                if fn is not None:
                    L.check(fn(c[1].h), "tm_dropin_gate_cache_clear")
        return self._n_tab, self._e_tab

    def _set_node_zero(self, h):
        zero = bool(getattr(self, "_node_zero", False)) and getattr(self, "node_zero_specialization", True)
        fn = getattr(L.lib(), "tm_weights_set_node_zero", None)    # absent in an older A/B build (TEMPME_LIB)
        if fn is not None:
            L.check(fn(h, int(zero)), "tm_weights_set_node_zero")

    def dropin_edge_table(self, w=None):
        """The drop-in forward's table mode: lin_event's edge-feature product W[:, :de] E(e) for every row of
        the edge-feature table (tm_edge_feature_table), rebuilt only when the weights or the table change;
        None when the encoder dims have no table mode or TEMPME_DROPIN_TABLE=0."""
        import os
        if os.environ.get("TEMPME_DROPIN_TABLE", "1") == "0":
            return None
        w = self.packed_weights() if w is None else w
        cols = L.lib().tm_edge_table_cols(w)
        if not cols:
            return None
        _, et = self.feature_tables()
        key = (self._packed_key, et.data_ptr(), tuple(et.shape))
        if getattr(self, "_dropin_etab_key", None) != key:
            dev = self._dev()
            self._dropin_etab = torch.empty((et.shape[0], cols), dtype=torch.float32, device=dev)
            L.check(L.lib().tm_edge_feature_table(w, L.ptr(et), int(et.shape[0]), L.ptr(self._dropin_etab),
                                                  L.stream_ptr(dev)), "tm_edge_feature_table")
            self._dropin_etab_key = key
            self._prep_dirty = self._prep_dirty_fast = True   # side streams must wait for this work
        return self._dropin_etab

    def encoder_fwd(self, node6, eid3, ts3, cat, cut, cnt, n_groups, B, W, out=None, workspace=None, M=1,
                    etab=None, w=None):
        """tm_encoder_fwd on device tensors (int32 node6 [G,B,W,6], eid3, f32 ts3, int32 cat [G,B,W],
        f64 cut [G,B], f32 cnt [G,B,W,3,3]) -> f32 [G,B,W].  ``etab``: the per-edge-id table of
        tm_edge_tables (tm_encoder_fwd_tab: lin_event's edge-feature product read, not recomputed)."""
        dev = self._dev()
        nt, et = self.feature_tables()
        w = self.packed_weights() if w is None else w
        n_walks = n_groups * B * W
        if out is None:
            out = torch.empty(max(n_walks, 1), dtype=torch.float32, device=dev)
        if workspace is None:
            nbytes = L.lib().tm_encoder_workspace_bytes(w, n_walks)
            workspace = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        L.check(L.lib().tm_encoder_fwd_tab(w, L.ptr(nt), L.ptr(et),
                                           None if etab is None else L.ptr(etab), n_groups, B, W, M, L.ptr(node6),
                                           L.ptr(eid3), L.ptr(ts3), L.ptr(cat), L.ptr(cut), L.ptr(cnt),
                                           L.ptr(workspace), L.ptr(out), L.stream_ptr(dev)), "TempME.forward")
        return out

    def edge_importance(self, eid3, ts3, imp, s1n, s1e, s2n, s2e, n_groups, B, W, N, out1=None, out2=None, w=None):
        dev = self._dev()
        w = self.packed_weights() if w is None else w
        _, et = self.feature_tables()
        if out1 is None:
            out1 = torch.empty(max(n_groups * B * N, 1), dtype=torch.float32, device=dev)
            out2 = torch.empty(max(n_groups * B * N * N, 1), dtype=torch.float32, device=dev)
        L.check(L.lib().tm_edge_importance(w, L.ptr(et), n_groups, B, W, N, L.ptr(eid3),
                                           L.ptr(ts3), L.ptr(imp), L.ptr(s1n), L.ptr(s1e), L.ptr(s2n), L.ptr(s2e),
                                           L.ptr(out1), L.ptr(out2), L.stream_ptr(dev)), "retrieve_edge_imp_node")
        return out1, out2

    # ------------------------------------------------------------------ HIP training path (f3)
    def _encoder_params(self):
        """The 22 tensors TempME.forward reads (tm_weights order minus the dependency gate): the cached
        weight list's 10 Linear pairs and the time encoder's frequency and phase."""
        ws = self._weight_list()
        return ws[:20] + ws[-2:]

    def dropout_cols(self):
        """Columns of a dropout keep-mask row (include/tempme.h, tm_encoder_train_fwd): alpha 2, attention.MLP
        hidden h, MLP hidden mlp_dim, rounded up to 16 -- 144 for the default constructor."""
        return -(-(2 + self.hid_dim + self.mlp_dim) // 16) * 16

    def dropout_masks(self, n_walks):
        """Keep-masks of the three dropouts TempME.forward applies in training (explainer_new.py:839 alpha,
        :780 attention.MLP hidden, :122 MLP hidden), uint8 [n_walks, dropout_cols()] from torch's device
        RNG, or None when they are inactive (eval mode or p = 0).  The plain Attention
        (use_temporal_guidance=False) has no alpha / hidden dropout: the kernels ignore those columns."""
        p = self.dropout_p
        if not self.training or p <= 0:
            return None, 1.0
        dev = self._dev()
        return (torch.empty(n_walks, self.dropout_cols(), dtype=torch.uint8, device=dev).bernoulli_(1.0 - p),
                1.0 / (1.0 - p))

    def forward_groups(self, node6, eid3, ts3, cat, cut, cnt, n_groups, B, W, drop=None, drop_scale=1.0,
                       use_module_dropout=True):
        """TempME.forward for n_groups independent reference calls at once (e.g. the src/tgt/bgd sides
        of one batch; the attention's time std is per group) with gradients to the encoder's weights:
        tm_encoder_train_fwd forward, tm_encoder_bwd + weight-gradient GEMMs backward.  Inputs are device
        tensors shaped [G,B,W,...]; returns [G*B*W] graphlet importance."""
        dev = self._dev()
        if drop is None and use_module_dropout:
            drop, drop_scale = self.dropout_masks(n_groups * B * W)
        args = (node6.to(dev, torch.int32).contiguous(), eid3.to(dev, torch.int32).contiguous(),
                ts3.to(dev, torch.float32).contiguous(), cat.to(dev, torch.int32).contiguous(),
                cut.to(dev, torch.float64).contiguous(), cnt.to(dev, torch.float32).contiguous(),
                int(n_groups), int(B), int(W))
        return _EncoderFn.apply(self, args, drop, float(drop_scale), *self._encoder_params())

    def _train_fwd(self, args, drop, drop_scale):
        node6, eid3, ts3, cat, cut, cnt, G, B, W = args
        dev = self._dev()
        nt, et = self.feature_tables()
        n = G * B * W
        drop = self._drop_packed(drop)
        out = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        ws = torch.empty(L.lib().tm_encoder_workspace_bytes(self.packed_weights(), n), dtype=torch.uint8, device=dev)
        L.check(L.lib().tm_encoder_train_fwd(self.packed_weights(), L.ptr(nt), L.ptr(et), G, B, W, L.ptr(node6),
                                             L.ptr(eid3), L.ptr(ts3), L.ptr(cat), L.ptr(cut), L.ptr(cnt), L.ptr(drop),
                                             drop_scale, L.ptr(ws), L.ptr(out), L.stream_ptr(dev)),
                "TempME.forward (training)")
        return out[:n], ws

    def _train_bwd(self, args, drop, drop_scale, ws, d_imp):
        node6, eid3, ts3, cat, cut, cnt, G, B, W = args
        dev = self._dev()
        nt, et = self.feature_tables()
        n = G * B * W
        R = 3 * n
        drop = self._drop_packed(drop)
        de, dn, h = self.edge_dim, self.node_dim, self._hid_packed()   # the packed (padded) widths
        kev = de + 3 + dn
        KE, DN, KM = -(-kev // 16) * 16, -(-dn // 16) * 16, -(-(h + 12 if self.if_cat else h) // 16) * 16
        e = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        b = dict(imp=None, dlogit=e(n), M2=e(n, h), dM2=e(n, h), M1d=e(n, KM), dM1=e(n, KM), X=e(n, KM), dY2=e(n, h),
                 H1d=e(n, h), dH1=e(n, h), O=e(n, 2 * h), dP=e(n, 2 * h), dQ=e(2, n, 2 * h), dF=e(n, 3, 2 * h),
                 ev=e(R, KE), AB=e(R, 2, DN), H=e(R, 2, h), dZ=e(R, 2, h), dlev=e(R, DN), g=e(R, DN), dt=e(R))
        io = L.EncoderGradIO(*[None if b[k] is None else b[k].data_ptr() for k in L.GRAD_IO_FIELDS])
        d_imp = d_imp.to(dev, torch.float32).contiguous()
        L.check(L.lib().tm_encoder_bwd(self.packed_weights(), L.ptr(nt), L.ptr(et), G, B, W, L.ptr(node6),
                                       L.ptr(eid3), L.ptr(ts3), L.ptr(cat), L.ptr(cut), L.ptr(cnt), L.ptr(drop),
                                       drop_scale, L.ptr(ws), L.ptr(d_imp), L.C.byref(io), L.stream_ptr(dev)),
                "TempME.forward backward")
        grads = [e(*s) for s in self._padded_shapes(_ENC_IDX)]
        gp = (L.C.c_void_p * len(grads))(*[t.data_ptr() for t in grads])
        L.check(L.lib().tm_encoder_wgrad(self.packed_weights(), G, B, W, L.C.byref(io), L.ptr(ws), gp,
                                         L.stream_ptr(dev)), "TempME.forward weight gradients")
        return tuple(self._unpad_grads(grads, _ENC_IDX))

    def _gate_params(self):
        """edge_dependency_gcn's three Linear pairs and the time encoder (the cached weight list)."""
        ws = self._weight_list()
        return ws[20:26] + ws[-2:]

    def gate_dropout_masks(self, n_pos):
        """Keep-masks of edge_dependency_gcn's Dropout(1.5p) [n_pos, h] and Dropout(p) [n_pos, h/2]
        (explainer_new.py:136-140) from torch's device RNG, or None in eval mode."""
        p = self.dropout_p
        if not self.training or p <= 0 or not self.use_dependency_aware_sampling:
            return None, None, 1.0, 1.0
        dev = self._dev()
        p1 = min(1.5 * p, 1.0)
        k1 = torch.empty(n_pos, self.hid_dim, dtype=torch.uint8, device=dev).bernoulli_(1.0 - p1)
        k2 = torch.empty(n_pos, self.hid_dim // 2, dtype=torch.uint8, device=dev).bernoulli_(1.0 - p)
        return k1, k2, (1.0 / (1.0 - p1) if p1 < 1 else 0.0), 1.0 / (1.0 - p)

    def explain_groups(self, imp, eid3, ts3, s1n, s1e, s2n, s2e, n_groups, B, W, N, training, masks=None):
        """retrieve_edge_imp_node (explainer_new.py:354-406) for n_groups calls at once with gradients to
        imp and the dependency gate: tm_explain_train_fwd / _bwd up to the gathered maxima, then
        beta_sample and the padding mask in torch ops (the rsample gradient is torch's).  imp
        [G,B,W]; returns hop-1 [G,B,N] and hop-2 [G,B,N^2]."""
        dev = self._dev()
        if masks is None:
            masks = self.gate_dropout_masks(n_groups * B * 3 * W)
        i32 = lambda x: x.to(dev, torch.int32).contiguous()  # noqa: E731
        args = (i32(eid3), ts3.to(dev, torch.float32).contiguous(), i32(s1e), i32(s2e), masks,
                int(n_groups), int(B), int(W), int(N))
        if _EXPLAIN_PAD:
            args = args + (i32(s1n), i32(s2n))
        # p = [hop-1 | hop-2] maxima of the G groups in one buffer (one Beta draw below), pad = the padding mask
        p, pad = _ExplainFn.apply(self, args, imp.reshape(-1).to(dev, torch.float32).contiguous(),
                                  *self._gate_params())
        if pad is None:
            pad = torch.cat([s1n.reshape(-1), s2n.reshape(-1)]).to(dev).ne(0).to(torch.float32)
        n1 = n_groups * B * N
        if training and pad is not None and self._fused_beta():
            e = _BetaRsampleFn.apply(p, pad)
        else:
            e = self.beta_sample(p, training) * pad    # beta_sample then masked_fill(node == 0, 0) (:400-404, :420-430)
        # one split, not two slices: its backward is one cat of the two gradients instead of two zero-filled
        # full-size buffers, two copies and their sum
        e1, e2 = torch.split(e, [n1, e.numel() - n1])
        return e1.view(n_groups, B, N), e2.view(n_groups, B, N * N)

    def _expl_io(self, R):
        dev = self._dev()
        h, dn = self._hid_packed(), self.node_dim
        KD, DN = -(-(self.edge_dim + dn) // 16) * 16, -(-dn // 16) * 16
        e = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        b = dict(X=e(R, KD), G1=e(R, h), G2=e(R, h // 2), z=e(R), gate=e(R), d_gate=e(R), dz=e(R), dG2=e(R, h // 2),
                 dG1=e(R, h), g=e(R, DN), t=e(R))
        return b, L.ExplainGradIO(*[b[k].data_ptr() for k in L.EXPL_IO_FIELDS])

    def _explain_fwd(self, args, imp):
        """-> p [G B N | G B N^2] (hop-1 then hop-2 maxima), and with the subgraph node ids in args their
        padding mask in the same layout (else None), and the backward's buffers."""
        eid3, ts3, s1e, s2e, masks, G, B, W, N = args[:9]
        k1, k2, sc1, sc2 = self._gate_masks_packed(masks)
        dev = self._dev()
        _, et = self.feature_tables()
        b, io = self._expl_io(G * B * 3 * W)
        n1, n2 = G * B * N, G * B * N * N
        pad = len(args) > 9
        p = torch.empty(max((n1 + n2) * (2 if pad else 1), 1), dtype=torch.float32, device=dev)
        pp = p.data_ptr()
        if pad:
            s1n, s2n = args[9], args[10]
            q = pp + 4 * (n1 + n2)
            rc = L.lib().tm_explain_train_fwd_pad(self.packed_weights(), L.ptr(et), G, B, W, N, L.ptr(eid3), L.ptr(ts3),
                                                  L.ptr(imp), L.ptr(s1e), L.ptr(s2e), L.ptr(k1), L.ptr(k2), sc1, sc2,
                                                  L.C.byref(io), pp, pp + 4 * n1, L.ptr(s1n), L.ptr(s2n), q,
                                                  q + 4 * n1, L.stream_ptr(dev))
        else:
            rc = L.lib().tm_explain_train_fwd(self.packed_weights(), L.ptr(et), G, B, W, N, L.ptr(eid3), L.ptr(ts3),
                                              L.ptr(imp), L.ptr(s1e), L.ptr(s2e), L.ptr(k1), L.ptr(k2), sc1, sc2,
                                              L.C.byref(io), pp, pp + 4 * n1, L.stream_ptr(dev))
        L.check(rc, "retrieve_edge_imp_node (training)")
        return p[:n1 + n2], (p[n1 + n2:2 * (n1 + n2)] if pad else None), (b, io)

    def _explain_bwd(self, args, imp, bufs, dp1, dp2):
        eid3, ts3, s1e, s2e, masks, G, B, W, N = args[:9]
        k1, k2, sc1, sc2 = self._gate_masks_packed(masks)
        dev = self._dev()
        b, io = bufs
        d_imp = torch.empty(max(G * B * W, 1), dtype=torch.float32, device=dev)
        grads = [torch.empty(s, dtype=torch.float32, device=dev) for s in self._padded_shapes(_GATE_IDX)]
        gp = (L.C.c_void_p * len(grads))(*[t.data_ptr() for t in grads])
        dp1 = dp1.to(dev, torch.float32).contiguous()
        dp2 = dp2.to(dev, torch.float32).contiguous()
        L.check(L.lib().tm_explain_train_bwd(self.packed_weights(), G, B, W, N, L.ptr(eid3), L.ptr(ts3), L.ptr(imp),
                                             L.ptr(s1e), L.ptr(s2e), L.ptr(k1), L.ptr(k2), sc1, sc2, L.ptr(dp1),
                                             L.ptr(dp2), L.C.byref(io), L.ptr(d_imp), gp, L.stream_ptr(dev)),
                "retrieve_edge_imp_node backward")
        return d_imp[:G * B * W], self._unpad_grads(grads, _GATE_IDX)

    # ------------------------------------------------------------------ reference API
    def forward(self, walks, cut_time_l, edge_identify):
        """explainer_new.py:174-201 -> [bsz, n_walks, 1]."""
        node_idx, edge_idx, time_idx, cat_feat, _ = walks
        if not self.training:
            out = self._dropin_forward(node_idx, edge_idx, time_idx, cat_feat, cut_time_l, edge_identify)
            if out is not None:
                return out
        dev = self._dev()
        B, W = np.shape(edge_idx)[0], np.shape(edge_idx)[1]
        assert np.shape(edge_identify)[-1] == 3 and np.shape(edge_idx)[-1] == 3, "event_dim mismatch (:180)"
        if not self._hip_eval_ok() or (self.training and not self._hip_ok()):
            return self._forward_torch(walks, cut_time_l, edge_identify)
        if self.training:
            out = self.forward_groups(_to(node_idx, dev, torch.int32), _to(edge_idx, dev, torch.int32),
                                      _to(time_idx, dev, torch.float32), _to(cat_feat, dev, torch.int32).reshape(B, W),
                                      _to(cut_time_l, dev, torch.float64), _to(edge_identify, dev, torch.float32), 1, B, W)
            return out.view(B, W, 1)
        wts = self.packed_weights()
        etab = self.dropin_edge_table(wts)
        if etab is not None and isinstance(edge_idx, np.ndarray) and edge_idx.size and \
                (edge_idx.max() >= etab.shape[0] or edge_idx.min() < 0):
            raise IndexError("index out of range in self")     # what the reference's embedding lookup raises
        items = ((node_idx, torch.int32), (edge_idx, torch.int32), (time_idx, torch.float32), (cat_feat, torch.int32),
                 (cut_time_l, torch.float64), (edge_identify, torch.float32))
        side = self._side_stream(dev, items)
        if side is None:
            n6, e3, t3, ct, cu, ei = _to_many(dev, *items)
            out = self.encoder_fwd(n6, e3, t3, ct.reshape(B, W), cu, ei, 1, B, W, etab=etab, w=wts)
        else:
            # eval_one_epoch's three per-side calls are independent: each runs on its own side stream (inputs
            # staged there from host arrays, or device-pack views that are already resident), and the caller's
            # stream waits for it, so the three walk kernels overlap instead of running one after another
            cur = torch.cuda.current_stream(dev)
            with torch.cuda.stream(side):
                n6, e3, t3, ct, cu, ei = _to_many(dev, *items)
                out = self.encoder_fwd(n6, e3, t3, ct.reshape(B, W), cu, ei, 1, B, W, etab=etab, w=wts)
                done = torch.cuda.Event()
                done.record(side)
            cur.wait_event(done)
            out.record_stream(cur)
            if self._needs_autograd():
                # the backward reads the staged inputs on the caller's stream (ctx.args): their blocks came
                # from the side stream's pool, so they must not return to it before that stream is done
                for t in (n6, e3, t3, ct, cu, ei):
                    t.record_stream(cur)
        out = out[:B * W]
        if self._needs_autograd():
            # eval mode with gradients enabled (temp_exp_main.py:446-452 calls the explainer outside no_grad):
            # the eval kernel's output, with a backward that recomputes through the training kernels if asked
            args = (n6, e3, t3, ct.reshape(B, W), cu, ei, 1, B, W)
            out = _EvalEncoderFn.apply(self, args, out, *self._encoder_params())
        return out.view(B, W, 1)

    # ------------------------------------------------------------------ drop-in eval fast path
    def _dropin_ctx(self, dev):
        """(device, context, its three side streams -- torch streams, so outputs can come from their pools --,
        next side) -- created on first use; a new context's side streams first wait for the caller's stream."""
        c = self.__dict__.get("_dropin_c")
        if c is None or c[0] != dev:
            h = L.C.c_void_p()
            L.check(L.lib().tm_dropin_create(dev.index, L.C.byref(h)), "tm_dropin_create")
            ctx = _DropinCtx(h)
            ext = [torch.cuda.Stream(device=dev) for _ in range(3)]
            for k in range(3):
                L.check(L.lib().tm_dropin_set_stream(h, k, ext[k].cuda_stream), "tm_dropin_set_stream")
            ctx.streams = ext      # alive as long as the context
            # the dependency-gate factor per (edge id, time), cached across calls (bit-identical; emptied on new
            # weights or tables)
            _, et = self.feature_tables()
            L.check(L.lib().tm_dropin_gate_cache(h, int(et.shape[0])), "tm_dropin_gate_cache")
            ctx.side_ids = [(x.stream_id, x.device_index, x.device_type) for x in ext]
            ctx.cur_obj = None
            ctx.fwd, ctx.expl = L.lib().tm_dropin_forward, L.lib().tm_edge_importance_gf3
            ctx.bern = L.lib().tm_edge_importance_gf3_bern
            c = self.__dict__["_dropin_c"] = (dev, ctx, ext, [0])
            self._prep_dirty_fast = True
        return c

    def _fast_state(self):
        """What the drop-in fast path derives from the weights and feature tables (packed weights, edge
        table, table pointers, parameter bundles), rebuilt when one key over the packed parameters'
        (data_ptr, version, requires_grad) and the two feature tables' (data_ptr, version) changes."""
        fx = self.__dict__.get("_fastx")
        if fx is not None and fx[0].current():
            # the C++ host side watches the same tensors (data_ptr, version, requires_grad) and the module
            # registrations: its state is the current one
            return fx[1]
        ws = self._weight_list()
        ne = self._modules["node_raw_embed"]._parameters["weight"]
        ee = self._modules["edge_raw_embed"]._parameters["weight"]
        key = (*map(_DP, ws), *map(_VER, ws), *map(_RG, ws), ne.data_ptr(), ne._version, ee.data_ptr(), ee._version)
        fs = self.__dict__.get("_fs")
        if fs is not None and fs[0] == key:
            return fs[1]
        wts = self.packed_weights()
        etab = self.dropin_edge_table(wts)
        nt, et = self.feature_tables()
        st = _FastState(wts, None if etab is None else etab.data_ptr(), nt.data_ptr(), et.data_ptr(),
                        any(map(_RG, ws[:20] + ws[-2:])), any(map(_RG, ws[20:26] + ws[-2:])), self._packed_key)
        st.gate_key = self._gate_key(ws)
        st.keep = (etab, nt, et)
        self.__dict__["_fs"] = (key, st)
        return st

    @staticmethod
    def _gate_key(ws):
        """(data_ptr, version, requires_grad) of the tensors the dependency gate reads (the gate MLP and the
        time encoder), which retrieve_explanation checks before using the gate factors of a forward."""
        g = ws[20:26] + ws[-2:]
        return (*map(_DP, g), *map(_VER, g), *map(_RG, g))

    def _dropin_forward(self, node_idx, edge_idx, time_idx, cat_feat, cut_time_l, edge_identify):
        """Eval forward on resident device-pack views (``pack.DevicePack.get_item`` / ``get_item_edge``) in one
        library call (tm_dropin_forward: side stream, staged cut times, encoder, and the dependency-gate
        factors retrieve_edge_imp_node will need, cached by walk identity).  None when the inputs are not
        such views of one batch (the general path handles them)."""
        fx = self.__dict__.get("_fastx")
        if fx is not None:
            r = fx[0].forward(node_idx, edge_idx, time_idx, cat_feat, cut_time_l, edge_identify)
            if r is not None:
                imp, rc, grad = r
                if rc:
                    L.check(rc, "TempME.forward")
                if grad:
                    B, W = edge_idx.shape[0], edge_idx.shape[1]
                    args = (node_idx, edge_idx, time_idx, cat_feat,
                            np.array(cut_time_l, dtype=np.float64) if cut_time_l.__class__ is np.ndarray else cut_time_l,
                            edge_identify, 1, B, W)
                    imp = _apply(_EvalEncoderBundleFn, self, args, imp, fx[1].bundle(self, "enc"))
                return imp
        # host arrays: the reference's own numpy views of its pack (load_subgraph_margin / np.load), staged on the
        # side stream below (read in place from pinned host memory, hoststage) and then the same launches
        host = node_idx.__class__ is np.ndarray
        if host:
            if not (edge_idx.__class__ is np.ndarray and time_idx.__class__ is np.ndarray and
                    cat_feat.__class__ is np.ndarray and edge_identify.__class__ is np.ndarray and edge_idx.ndim == 3):
                return None
        elif not (getattr(edge_idx, "_tm_resident", False) and getattr(node_idx, "_tm_resident", False) and
                  getattr(time_idx, "_tm_resident", False) and getattr(cat_feat, "_tm_resident", False) and
                  getattr(edge_identify, "_tm_resident", False)):
            return None
        # resident views are int32 / float32 slices of one pack: check that they are one batch's
        B, W, three = edge_idx.shape
        if three != 3 or B == 0 or tuple(node_idx.shape) != (B, W, 6) or tuple(time_idx.shape) != (B, W, 3) or \
                tuple(cat_feat.shape[:2]) != (B, W) or tuple(edge_identify.shape) != (B, W, 3, 3):
            return None
        if not host and (edge_idx.dtype is not torch.int32 or time_idx.dtype is not torch.float32):
            return None
        if host and (cat_feat.size != B * W or edge_idx.dtype.kind not in "iuf" or node_idx.dtype.kind not in "iuf"):
            return None
        dev = self._dev()
        cut_h = cut_d = None
        if cut_time_l.__class__ is np.ndarray:
            c = cut_time_l if cut_time_l.dtype == np.float64 and cut_time_l.flags.c_contiguous else \
                np.ascontiguousarray(cut_time_l, dtype=np.float64)
            if c.size != B or B > 512:
                return None
            cut_h = c.__array_interface__["data"][0]
        elif isinstance(cut_time_l, torch.Tensor) and cut_time_l.device == dev and cut_time_l.dtype is torch.float64 \
                and cut_time_l.numel() == B and cut_time_l.is_contiguous():
            cut_d = cut_time_l.data_ptr()
        else:
            return None
        if not self._hip_eval_ok():
            return None
        fs = self._fast_state()
        if host:
            # ids outside the node / edge tables raise what the reference's embedding lookups raise.  The check
            # runs once per pack array and layout (hoststage.window_bounds: these columns over every batch of the
            # array), per call only when that fails or the array is not registered; staging then clamps the ids
            # into the tables (tm_stage_job.bound), so a pack rewritten after the check is never read out of range
            n_node, n_edge = fs.keep[1].shape[0], fs.keep[2].shape[0]
            for a, n in ((edge_idx, n_edge), (node_idx, n_node)):
                wb = _hoststage().window_bounds(a)
                if (wb is None or not (wb[0] >= 0 and wb[1] < n)) and a.size and (a.max() >= n or a.min() < 0):
                    raise IndexError("index out of range in self")
        _, ctx, ext, nk = self._dropin_ctx(dev)
        k = nk[0]
        nk[0] = (k + 1) % 3
        # the outputs come from the caching allocator's pool of side stream k (the kernels writing them run
        # there) and are recorded as used by the caller's stream, which reads them after the wait
        cur = torch._C._cuda_getCurrentStream(dev.index)
        cobj = ctx.cur_obj
        if cobj is None or cobj[0] != cur:
            st = torch.cuda.Stream(stream_id=cur[0], device_index=cur[1], device_type=cur[2])
            cobj = ctx.cur_obj = (cur, st, st.cuda_stream)
        torch._C._cuda_setStream(*ctx.side_ids[k])
        host_keys = staged = None
        try:
            out = torch.empty(B * W * 4, dtype=torch.float32, device=dev)   # imp [B*W] | gate factors [B*W*3]
            if host:
                items = ((node_idx, torch.int32, n_node), (edge_idx, torch.int32, n_edge), (time_idx, torch.float32),
                         (cat_feat, torch.int32), (edge_identify, torch.float32))
                staged = _hoststage().stage(dev, items)         # the current stream is side stream k here
                if staged is None:                           # small / non-owning bases: pinned host-cast copy
                    staged = _to_many(dev, *[it[:2] for it in items])
                host_keys = (edge_idx, time_idx)
                node_idx, edge_idx, time_idx, cat_feat, edge_identify = staged
        finally:
            torch._C._cuda_setStream(*cur)
        out.record_stream(cobj[1])
        if staged is not None:
            # read on the caller's stream later (retrieve, backward): the views share one allocation
            staged[0].record_stream(cobj[1])
        sync = 1 if (cut_d is not None or self.__dict__.get("_prep_dirty_fast", True)) else 0
        if sync:
            self._prep_dirty_fast = False
        o = out.data_ptr()
        rc = ctx.fwd(ctx.h, k, sync, fs.wts, fs.nt, fs.et, fs.etab, B, W, node_idx.data_ptr(), edge_idx.data_ptr(),
                     time_idx.data_ptr(), cat_feat.data_ptr(), cut_h, cut_d, edge_identify.data_ptr(), o, o + 4 * B * W,
                     cobj[2])
        if rc:
            L.check(rc, "TempME.forward")
        imp = out.as_strided((B, W, 1), (W, 1, 1))
        # the gate factors, for retrieve_explanation with these very walk tensors (identity + version) or host arrays
        # (identity; their staged device copies ride along)
        gcache = self.__dict__.setdefault("_gf_cache", [])
        if host:
            gcache.append((host_keys[0], host_keys[1], 0, 0, fs.gate_key, out, B * W, B, W, fs, (edge_idx, time_idx)))
        else:
            gcache.append((edge_idx, time_idx, edge_idx._version, time_idx._version, fs.gate_key, out, B * W, B, W, fs,
                           None))
        if len(gcache) > 6:
            del gcache[0]
        if fs.enc_grad and torch.is_grad_enabled():
            # the cut times as a host copy (moved to the device only if a backward runs); cat [B, W, 1] is
            # reshaped there too
            args = (node_idx, edge_idx, time_idx, cat_feat,
                    np.array(cut_time_l, dtype=np.float64) if cut_d is None else cut_time_l, edge_identify, 1, B, W)
            imp = _apply(_EvalEncoderBundleFn, self, args, imp, fs.bundle(self, "enc"))
        # the C++ host side for later calls (device-pack views; with host arrays its state check keeps _fast_state
        # cheap); its gate-factor cache entry: the walk tensors the kernels read (host arrays: the staged copies)
        self._make_fastx(fs, ctx, dev, (edge_idx, time_idx, out, B, W))
        return imp

    def _make_fastx(self, fs, ctx, dev, entry):
        """The C++ host side of this fast path (csrc/dropin_ext.cpp) for the current weights / tables / context:
        later forwards and retrieves on device-pack views take one C++ call each; any change of the weights,
        tables or module registrations sends the next call back here."""
        ext = _dropin_ext()
        if ext is None:
            return
        fx = self.__dict__.get("_fastx")
        if fx is not None and fx[1] is fs and fx[2] is ctx and fx[0].current():
            fx[0].push(*entry)
            return
        ws = self._weight_list()
        ne = self._modules["node_raw_embed"]._parameters["weight"]
        ee = self._modules["edge_raw_embed"]._parameters["weight"]
        addr = lambda f: L.C.cast(f, L.C.c_void_p).value  # noqa: E731
        lib = L.lib()
        fast = ext.Fast(list(ws) + [ne, ee], [True] * len(ws) + [False, False], _REG_GEN, _REG_GEN[0], ctx.h.value,
                        addr(lib.tm_dropin_forward), addr(lib.tm_edge_importance_gf3),
                        addr(lib.tm_edge_importance_gf3_bern), fs.wts if isinstance(fs.wts, int) else fs.wts.value,
                        fs.nt, fs.et, fs.etab or 0, list(ctx.side_ids), dev.index, bool(fs.enc_grad))
        fast.push(*entry)
        self.__dict__["_fastx"] = (fast, fs, ctx)

    def _param_bundle(self, which):
        return self._fast_state().bundle(self, which)

    def _dropin_retrieve(self, sides, bern=False):
        """retrieve_explanation(training=False) for the three sides of one reference batch whose walks went
        through _dropin_forward: one tm_edge_importance_gf3 launch from the gate factors cached with those
        walk tensors (same objects, unmodified, gate weights unchanged), written straight into the
        concatenated [3B, N] / [3B, N^2] outputs.  None if any side does not qualify.

        bern (training=True on an eval-mode module, eval_one_epoch under --if_bern, temp_exp_main.py:46,
        :450-453): the launch writes the gathered maxima p and the padding mask of the three sides, and
        beta_sample's rsample (explainer_new.py:420-430) runs ONCE over the concatenated [3B, N + N^2]
        (the reference draws per side; the draws are i.i.d. either way -- parity is statistical, SURVEY.md
        §8(c)), then masked_fill(node == 0, 0) as a multiply by the mask."""
        gc = self.__dict__.get("_gf_cache", ())
        gk = None
        got = []
        host = sides[0][2][1].__class__ is np.ndarray
        for subgraph, imp, walks in sides:
            e3, t3 = walks[1], walks[2]
            h = None
            for ent in reversed(gc):
                if ent[0] is e3 and ent[1] is t3:
                    h = ent
                    break
            if h is None or (h[10] is not None) != host or (not host and (e3._version != h[2] or t3._version != h[3])):
                return None
            if gk is None:
                gk = self._gate_key(self._weight_list())
            if h[4] != gk:
                return None
            B, W = h[7], h[8]
            n1, n2 = subgraph[0]
            x1, x2 = subgraph[1]
            if host:
                if not all(t.__class__ is np.ndarray and t.ndim == 2 for t in (n1, x1, n2, x2)):
                    return None
                e3, t3 = h[10]                           # the forward's staged device copies
            elif not all(getattr(t, "_tm_resident", False) for t in (n1, x1, n2, x2)):
                return None
            N = n1.shape[1]
            if imp.__class__ is not torch.Tensor or imp.dtype is not torch.float32 or imp.numel() != B * W or \
                    not imp.is_contiguous() or n1.shape[0] != B or tuple(x1.shape) != tuple(n1.shape) or \
                    tuple(n2.shape) != (B, N * N) or tuple(x2.shape) != tuple(n2.shape) or \
                    (not host and n1.dtype is not torch.int32):
                return None
            got.append((h, e3, t3, imp, n1, x1, n2, x2, B, W, N))
        B, W, N = got[0][8], got[0][9], got[0][10]
        for g in got:
            if g[8] != B or g[9] != W or g[10] != N:
                return None
        dev = self._dev()
        if host:
            # the three sides' hop-1 / hop-2 node and edge ids (float64 views of the reference's pack) in one launch
            items = [(x, torch.int32) for g in got for x in g[4:8]]
            st = _hoststage().stage(dev, items)
            if st is None:
                st = _to_many(dev, *items)
            got = [g[:4] + tuple(st[4 * i:4 * i + 4]) + g[8:] for i, g in enumerate(got)]
        ctx = self.__dict__["_dropin_c"][1]
        n_out = 3 * B * (N + N * N)
        o = torch.empty(n_out * (2 if bern else 1), dtype=torch.float32, device=dev)
        p1 = o.data_ptr()
        p2 = p1 + 4 * 3 * B * N
        (ha, ea, _, ia, na1, xa1, na2, xa2, *_), (hb, eb, _, ib, nb1, xb1, nb2, xb2, *_), \
            (hc, ec, _, ic, nc1, xc1, nc2, xc2, *_) = got
        args = (B, W, N, ha[5].data_ptr() + 4 * ha[6], hb[5].data_ptr() + 4 * hb[6], hc[5].data_ptr() + 4 * hc[6],
                ea.data_ptr(), eb.data_ptr(), ec.data_ptr(), ia.data_ptr(), ib.data_ptr(), ic.data_ptr(),
                na1.data_ptr(), nb1.data_ptr(), nc1.data_ptr(), xa1.data_ptr(), xb1.data_ptr(), xc1.data_ptr(),
                na2.data_ptr(), nb2.data_ptr(), nc2.data_ptr(), xa2.data_ptr(), xb2.data_ptr(), xc2.data_ptr(), p1, p2)
        if bern:
            k1 = p1 + 4 * n_out
            rc = ctx.bern(*args, k1, k1 + 4 * 3 * B * N, torch._C._cuda_getCurrentRawStream(dev.index))
        else:
            rc = ctx.expl(*args, torch._C._cuda_getCurrentRawStream(dev.index))
        if rc:
            L.check(rc, "retrieve_explanation")
        # the gate bundle of the forward's state (its gate parameters are the current ones: gk matched)
        return self._retrieve_tail(o, [(g[1], g[2], g[4], g[5], g[6], g[7], B, W, N) for g in got], (ia, ib, ic),
                                   any(gk[-8:]), ha[9], bern)

    def _retrieve_tail(self, o, sides, imps, gate_grad, fs, bern):
        """The fast retrieve's outputs from its one launch's buffer o ([hop-1 | hop-2], with bern [p | keep]):
        views [3B, N] / [3B, N^2], the Beta draw for bern, and the autograd node when gradients are wanted.
        sides: per side (e3, t3, n1, x1, n2, x2, B, W, N)."""
        B, N = sides[0][6], sides[0][8]
        ia, ib, ic = imps
        grad = torch.is_grad_enabled() and (gate_grad or ia.requires_grad or ib.requires_grad or ic.requires_grad)
        if bern:
            n_out = 3 * B * (N + N * N)
            p, keep = o[:n_out], o[n_out:]
            if grad:
                args = tuple((g[0], g[1], g[3], g[5], g[6], g[7], g[8]) for g in sides)
                p = _apply(_EvalExplain3RawFn, self, args, ia, ib, ic, p, fs.bundle(self, "gate"))
            x = _BetaRsampleFn.apply(p.contiguous(), keep) if self._fused_beta() else self.beta_sample(p, True) * keep
            o1, o2 = x[:3 * B * N].view(3 * B, N), x[3 * B * N:].view(3 * B, N * N)
        else:
            o1, o2 = o.as_strided((3 * B, N), (N, 1)), o.as_strided((3 * B, N * N), (N * N, 1), 3 * B * N)
            if grad:
                o1, o2 = _apply(_EvalExplain3Fn, self, tuple(sides), ia, ib, ic, o1, o2, fs.bundle(self, "gate"))
        if self.base_type == "tgn":
            return [o1, o2]
        return [o1]

    def _side_stream(self, dev, items):
        """The next of three side streams for an eval forward whose inputs are host arrays or resident
        device-pack views (``pack.DevicePack.get_item``), else None (run on the current stream).  Pending
        weight / table preparation on the current stream is waited for through one recorded event."""
        import os
        if dev.type != "cuda" or os.environ.get("TEMPME_DROPIN_STREAMS", "1") == "0":
            return None
        for a, _ in items:
            if isinstance(a, torch.Tensor) and not getattr(a, "_tm_resident", False):
                return None
            if not isinstance(a, (np.ndarray, torch.Tensor)):
                return None
        # the drop-in context's three streams (shared with the fast path: more streams than the device's
        # hardware queues -- 4 by default -- would be multiplexed onto them)
        ss = self._dropin_ctx(dev)[2]
        if self.__dict__.get("_side_streams") is not ss:
            self.__dict__["_side_streams"] = ss
            self.__dict__["_side_i"] = 0
            self._prep_dirty = True
        if getattr(self, "_prep_dirty", True):
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            self.__dict__["_prep_event"] = ev
            self._prep_dirty = False
        i = self.__dict__["_side_i"]
        self.__dict__["_side_i"] = (i + 1) % len(ss)
        ss[i].wait_event(self.__dict__["_prep_event"])
        return ss[i]

    def retrieve_edge_imp_node(self, subgraph, graphlet_imp, walks, training=True):
        """explainer_new.py:354-406 -> (hop-1 [B,N], hop-2 [B,N^2])."""
        node_record, eidx_record, _ = subgraph
        dev = self._dev()
        needs_grad = training or (torch.is_grad_enabled() and (graphlet_imp.requires_grad or any(
            p.requires_grad for p in self._weight_list()[20:26])))
        if not self._hip_eval_ok() or (training and not self._hip_ok()):
            return self._edge_imp_torch(subgraph, graphlet_imp, walks, training)
        B, N = np.shape(node_record[0])[0], np.shape(node_record[0])[1]
        W = np.shape(walks[1])[1]
        if training:
            e0, e1 = self.explain_groups(graphlet_imp.reshape(1, B, W), _to(walks[1], dev, torch.int32),
                                         _to(walks[2], dev, torch.float32), _to(node_record[0], dev, torch.int32),
                                         _to(eidx_record[0], dev, torch.int32), _to(node_record[1], dev, torch.int32),
                                         _to(eidx_record[1], dev, torch.int32), 1, B, W, N, training)
            return e0.view(B, N), e1.view(B, N * N)
        e3, t3, n1, x1, n2, x2 = _to_many(dev, (walks[1], torch.int32), (walks[2], torch.float32),
                                          (node_record[0], torch.int32), (eidx_record[0], torch.int32),
                                          (node_record[1], torch.int32), (eidx_record[1], torch.int32))
        o1, o2 = self.edge_importance(e3, t3, graphlet_imp.detach().to(dev, torch.float32).contiguous(), n1, x1, n2, x2,
                                      1, B, W, N)
        o1, o2 = o1[:B * N].view(B, N), o2[:B * N * N].view(B, N * N)
        if needs_grad:
            # eval (Beta mean) with gradients enabled (eval_one_epoch, temp_exp_main.py:447-449): the eval
            # kernels' values, backward through the HIP training kernels on demand
            o1, o2 = _EvalExplainFn.apply(self, (e3, t3, n1, x1, n2, x2, B, W, N), graphlet_imp, o1, o2,
                                          *self._gate_params())
        return o1, o2

    def retrieve_explanation(self, subgraph_src, graphlet_imp_src, walks_src, subgraph_tgt, graphlet_imp_tgt,
                             walks_tgt, subgraph_bgd, graphlet_imp_bgd, walks_bgd, training=True):
        """explainer_new.py:408-418."""
        # the gate factors cached by eval-mode forwards (dropout off, as in the module's eval mode)
        if not self.training:
            sides = ((subgraph_src, graphlet_imp_src, walks_src), (subgraph_tgt, graphlet_imp_tgt, walks_tgt),
                     (subgraph_bgd, graphlet_imp_bgd, walks_bgd))
            fx = self.__dict__.get("_fastx")
            if fx is not None and fx[0].cached:
                r = fx[0].retrieve(sides, bool(training))
                if r is not None:
                    o, rc, args = r
                    if rc:
                        L.check(rc, "retrieve_explanation")
                    fs = fx[1]
                    return self._retrieve_tail(o, args, (graphlet_imp_src, graphlet_imp_tgt, graphlet_imp_bgd),
                                               fs.gate_grad, fs, bool(training))
            if self.__dict__.get("_gf_cache") and self._hip_eval_ok():
                r = self._dropin_retrieve(sides, bern=bool(training))
                if r is not None:
                    return r
        s0, s1 = self.retrieve_edge_imp_node(subgraph_src, graphlet_imp_src, walks_src, training=training)
        t0, t1 = self.retrieve_edge_imp_node(subgraph_tgt, graphlet_imp_tgt, walks_tgt, training=training)
        b0, b1 = self.retrieve_edge_imp_node(subgraph_bgd, graphlet_imp_bgd, walks_bgd, training=training)
        if self.base_type == "tgn":
            return [torch.cat([s0, t0, b0], dim=0), torch.cat([s1, t1, b1], dim=0)]
        return [torch.cat([s0, t0, b0], dim=0)]

    def _fused_beta(self):
        """beta_sample(p, True) * mask may go through _BetaRsampleFn (bitwise the same as torch's Beta rsample):
        not when the module's beta_sample is overridden (an instance attribute or a subclass)."""
        return "beta_sample" not in self.__dict__ and type(self).beta_sample is TempME.beta_sample

    def beta_sample(self, prob, training):
        """explainer_new.py:420-430."""
        alpha = torch.clamp(prob * 10, min=1.0)
        beta = torch.clamp((1 - prob) * 10, min=1.0)
        if training:
            # validate_args=False: the argument check is a host sync (the values are valid by construction)
            return torch.distributions.Beta(alpha, beta, validate_args=False).rsample()
        return alpha / (alpha + beta)

    def _null_vec(self, device):
        """torch.tensor(list(null_model.values())) on the device, built once (no per-step host copy)."""
        key = (tuple(self.null_model.items()), str(device))
        if getattr(self, "_null_key", None) != key:
            self._null_dev = torch.tensor(list(self.null_model.values())).to(device)
            self._null_key = key
        return self._null_dev

    def kl_loss(self, prob, walks, target=0.3):
        """explainer_new.py:432-453.  With the empirical prior over the 12 motif categories and a device
        tensor prob [B, W(, 1)]: one tm_kl_loss launch (value and d/d prob; fp64 inside, within 1e-5 of the
        torch formulation below, which serves other priors / category counts and host tensors)."""
        _, _, _, cat_feat, _ = walks
        if self.prior == "empirical" and len(self.null_model) == 12 and isinstance(prob, torch.Tensor) and \
                prob.is_cuda and prob.dim() >= 2 and prob.numel() == prob.shape[0] * prob.shape[1] and \
                prob.dtype == torch.float32:
            B, W = prob.shape[0], prob.shape[1]
            cat = _to(cat_feat, prob.device, torch.int32)
            if cat.numel() == B * W:
                return _KLFn.apply(prob.reshape(1, B, W), cat.reshape(1, B, W), self._null_vec(prob.device),
                                   float(target))
        return self._kl_loss_torch(prob, walks, target)

    def _kl_loss_torch(self, prob, walks, target=0.3):
        _, _, _, cat_feat, _ = walks
        prob = torch.clamp(prob, 1e-6, 1 - 1e-6)
        if self.prior == "empirical":
            s = torch.mean(prob, dim=1)
            null = self._null_vec(prob.device)
            num_cat = len(self.null_model.keys())
            cat = _to(cat_feat, prob.device, torch.long).reshape(prob.shape[0], -1, 1)
            emp = torch.zeros(prob.shape[0], num_cat, 1, device=prob.device, dtype=prob.dtype)
            emp = emp.scatter_reduce(1, cat, prob, "mean", include_self=False)
            emp = s * emp.reshape(-1, num_cat)
            null = target * null.reshape(-1, num_cat)
            return ((1 - s) * torch.log((1 - s) / (1 - target + 1e-6) + 1e-6)
                    + emp * torch.log(emp / (null + 1e-6) + 1e-6)).mean()
        return (prob * torch.log(prob / target + 1e-6)
                + (1 - prob) * torch.log((1 - prob) / (1 - target + 1e-6) + 1e-6)).mean()

    def kl_loss_groups(self, prob, cat, target=0.3):
        """sum_g kl_loss(prob[g], walks with categories cat[g]) for G groups at once (the training step's
        three per-side calls, temp_exp_main.py:618-620) on the HIP path: prob [G,B,W] (autograd input),
        cat [G,B,W] int.  prior='empirical' only (the reference default); value and gradient from
        tm_kl_loss (fp64 inside), within 1e-5 of the per-side torch formulation."""
        if self.prior != "empirical" or not self._hip_ok():
            return sum(self._kl_loss_torch(prob[g].unsqueeze(-1), (None, None, None, cat[g], None), target=target)
                       for g in range(prob.shape[0]))
        return _KLFn.apply(prob, cat, self._null_vec(prob.device), float(target))

    # ------------------------------------------------------------------ autograd formulation (training)
    def _forward_torch(self, walks, cut_time_l, edge_identify):
        node_idx, edge_idx, time_idx, cat_feat, _ = walks
        dev = self.node_raw_embed.weight.device if self.device is None else self.device
        eid = _to(edge_idx, dev, torch.long)
        t = _to(time_idx, dev, torch.float32)
        B, W = eid.shape[0], eid.shape[1]
        ef = self.edge_raw_embed(eid)
        cnt = _to(edge_identify, dev, torch.float32)
        dt = t[:, :, 2:3] - t
        tf = self.time_encoder(dt.reshape(B, -1)).reshape(B, W, 3, -1)
        ev = torch.cat([ef, cnt, tf], dim=-1)
        node = _to(node_idx, dev, torch.long)
        xs = self.node_raw_embed(node[:, :, [0, 2, 4]])
        xt = self.node_raw_embed(node[:, :, [1, 3, 5]])
        us = self.event_conv(ev, xs, xt)
        ut = self.event_conv(ev, xt, xs)
        f = torch.cat([us, ut], dim=-1)
        at = self.attention
        src = f[:, :, 2, :]
        wq = at.W2(f[:, :, 0:2, :])
        scores = (at.W1(src).unsqueeze(2) * wq).sum(-1)
        if isinstance(at, TemporalAwareAttention):
            cut = _to(cut_time_l, dev, torch.float32)
            diff = torch.abs(cut.view(B, 1, 1) - t[:, :, :2])
            tw = torch.exp(-diff / (diff.std() + 1e-6))
            scores = scores * (1.0 - 0.3 + 0.3 * tw)
        alpha = torch.softmax(scores, dim=-1)
        if isinstance(at, TemporalAwareAttention):
            alpha = at.dropout(alpha)
        out = at.MLP(src + (alpha.unsqueeze(-1) * wq).sum(2))
        if self.if_cat:
            oh = F.one_hot(_to(cat_feat, dev, torch.long).reshape(B, W), num_classes=12)
            out = torch.cat([out, oh.to(out.dtype)], dim=-1)
        return self.MLP(out).sigmoid()

    def _edge_imp_torch(self, subgraph, graphlet_imp, walks, training):
        node_record, eidx_record, _ = subgraph
        dev = graphlet_imp.device
        i0 = _to(eidx_record[0], dev, torch.long)
        i1 = _to(eidx_record[1], dev, torch.long)
        B = graphlet_imp.shape[0]
        ew = _to(walks[1], dev, torch.long).reshape(B, -1)
        # dense width: the reference sizes it by the batch's largest edge id (a host sync, :362); every id
        # indexes the edge-feature table, so its row count bounds them and gives the same values
        n_e = self.edge_raw_embed.weight.shape[0]
        wimp = graphlet_imp.repeat(1, 1, 3).view(B, -1)
        if self.use_dependency_aware_sampling:
            tw = _to(walks[2], dev, torch.float32).reshape(B, -1)
            g = torch.cat([self.edge_raw_embed(ew), self.time_encoder(tw.unsqueeze(-1)).squeeze(-1)], dim=-1)
            wimp = wimp * (0.5 + 0.5 * torch.sigmoid(self.edge_dependency_gcn(g).squeeze(-1)))
        dense = torch.zeros(B, n_e, device=dev, dtype=wimp.dtype).scatter_reduce(-1, ew, wimp, "amax",
                                                                                  include_self=False)
        e0 = self.beta_sample(torch.gather(dense, -1, i0), training)
        e1 = self.beta_sample(torch.gather(dense, -1, i1), training)
        e0 = e0.masked_fill(_to(node_record[0], dev, torch.long) == 0, 0)
        e1 = e1.masked_fill(_to(node_record[1], dev, torch.long) == 0, 0)
        return e0, e1


class _Packed:
    def __init__(self, h):
        self.h = h

    def __del__(self):
        if self.h is not None and L._lib is not None:
            L._lib.tm_weights_free(self.h)
            self.h = None


class _EncoderFn(torch.autograd.Function):
    """TempME.forward with its backward on the HIP kernels (tm_encoder_train_fwd / tm_encoder_bwd)."""

    @staticmethod
    def forward(ctx, ex, args, drop, drop_scale, *params):
        out, ws = ex._train_fwd(args, drop, drop_scale)
        ctx.ex, ctx.args, ctx.drop, ctx.drop_scale, ctx.ws = ex, args, drop, drop_scale, ws
        return out

    @staticmethod
    def backward(ctx, d_imp):
        grads = ctx.ex._train_bwd(ctx.args, ctx.drop, ctx.drop_scale, ctx.ws, d_imp)
        ctx.ws = None
        return (None, None, None, None, *grads)


class _EvalEncoderFn(torch.autograd.Function):
    """Eval-mode TempME.forward with gradients enabled: forward = the eval kernel's output (no dropout in
    eval, so it is the function the training kernels compute); backward recomputes through
    tm_encoder_train_fwd (without dropout masks) and runs tm_encoder_bwd -- only if a backward is asked for."""

    @staticmethod
    def forward(ctx, ex, args, out, *params):
        ctx.ex, ctx.args = ex, args
        return out.detach()

    @staticmethod
    def backward(ctx, d_imp):
        ex = ctx.ex
        if ex._hip_ok():
            _, ws = ex._train_fwd(ctx.args, None, 1.0)
            grads = ex._train_bwd(ctx.args, None, 1.0, ws, d_imp)
        else:   # constructor variants without HIP training kernels: recompute through the torch formulation
            node6, eid3, ts3, cat, cut, cnt, G, B, W = ctx.args
            params = ex._encoder_params()
            with torch.enable_grad():
                out = ex._forward_torch((node6, eid3, ts3, cat, None), cut, cnt)
                grads = torch.autograd.grad(out.reshape(-1), params, grad_outputs=d_imp.reshape(-1).to(out.dtype),
                                            allow_unused=True)
        return (None, None, None, *grads)


def _apply(fn, *args):
    """fn.apply without the Python wrapper's per-argument pass (unwrap_dead_wrappers): the C++ apply of
    torch.autograd.Function, used when no functorch transform is active (as Function.apply itself does)."""
    if torch._C._are_functorch_transforms_active():
        return fn.apply(*args)
    return _C_APPLY(fn)(*args)


def _C_APPLY(fn):
    a = fn.__dict__.get("_c_apply")
    if a is None:
        a = super(torch.autograd.Function, fn).apply
        setattr(fn, "_c_apply", a)
    return a


_DP = torch.Tensor.data_ptr
# tm_weights indices of TempME._encoder_params / _gate_params
_ENC_IDX = tuple(range(20)) + (26, 27)
_GATE_IDX = tuple(range(20, 26)) + (26, 27)
_VER = operator.attrgetter("_version")
_RG = operator.attrgetter("requires_grad")


class _FastState:
    """TempME._fast_state's derived objects for one weight / table version."""

    def __init__(self, wts, etab, nt, et, enc_grad, gate_grad, packed_key):
        self.wts, self.etab, self.nt, self.et = wts, etab, nt, et
        self.enc_grad, self.gate_grad, self.packed_key = enc_grad, gate_grad, packed_key
        self._bundles = {}

    def bundle(self, ex, which):
        """One tensor standing for the 22 encoder (or 8 gate) parameters in an eval call's autograd node:
        the concatenation of their flattened values, built under grad mode once per weight version (its
        CatBackward node -- no saved tensors -- routes a gradient of the bundle to every parameter), so
        the per-call node has a few inputs instead of 22 (Function.apply costs per input)."""
        b = self._bundles.get(which)
        if b is None:
            params = ex._encoder_params() if which == "enc" else ex._gate_params()
            with torch.enable_grad():
                b = self._bundles[which] = torch.cat([p.reshape(-1) for p in params])
        return b


class _DropinCtx:
    def __init__(self, h):
        self.h = h

    def __del__(self):
        try:
            L.lib().tm_dropin_free(self.h)
        except Exception:
            pass


def _flat_grads(grads, params):
    return torch.cat([(torch.zeros_like(p) if g is None else g).reshape(-1) for g, p in zip(grads, params)])


class _EvalEncoderBundleFn(torch.autograd.Function):
    """_EvalEncoderFn with the 22 encoder parameters behind one bundle tensor (TempME._param_bundle):
    backward returns the parameters' gradients flattened into the bundle's layout."""

    @staticmethod
    def forward(ctx, ex, args, out, bundle):
        ctx.ex, ctx.args = ex, args
        return out.detach()

    @staticmethod
    def backward(ctx, d_imp):
        a = ctx.args
        B, W = a[7], a[8]
        ctx.args = a[:3] + (a[3].reshape(B, W),
                            torch.from_numpy(a[4]).to(a[0].device) if isinstance(a[4], np.ndarray) else a[4]) + a[5:]
        d_imp = d_imp.reshape(-1)
        grads = _EvalEncoderFn.backward(ctx, d_imp)[3:]
        return None, None, None, _flat_grads(grads, ctx.ex._encoder_params())


class _EvalExplain3Fn(torch.autograd.Function):
    """retrieve_explanation(training=False) over the three sides with gradients enabled (_EvalExplainFn per
    side, the 8 gate parameters behind one bundle tensor): outputs the concatenated hop-1 / hop-2."""

    @staticmethod
    def forward(ctx, ex, args, imp_s, imp_t, imp_b, o1, o2, bundle):
        ctx.ex, ctx.args = ex, args
        ctx.save_for_backward(imp_s, imp_t, imp_b)
        return o1.detach(), o2.detach()

    @staticmethod
    def backward(ctx, g1, g2):
        ex = ctx.ex
        params = ex._gate_params()
        d_imps, gsum = [], None
        for s, imp in enumerate(ctx.saved_tensors):
            e3, t3, n1, x1, n2, x2, B, W, N = ctx.args[s]
            sub = _Ctx(ex, (e3, t3, n1, x1, n2, x2, B, W, N), imp)
            gs = _EvalExplainFn.backward(sub, g1[s * B:(s + 1) * B], g2[s * B:(s + 1) * B])
            d_imps.append(gs[2])
            pg = [torch.zeros_like(p) if g is None else g for g, p in zip(gs[5:], params)]
            gsum = pg if gsum is None else [a + b for a, b in zip(gsum, pg)]
        return (None, None, *[None if d is None else d.reshape(ctx.saved_tensors[s].shape) for s, d in enumerate(d_imps)],
                None, None, _flat_grads(gsum, params))


class _EvalExplain3RawFn(torch.autograd.Function):
    """The gathered maxima p of retrieve_edge_imp_node for the three sides, concatenated [3B*N | 3B*N^2]
    (tm_edge_importance_gf3_bern, eval-mode module), with gradients: backward recomputes each side through
    the HIP training kernels (gate + scatter-max, no dropout in eval mode) and differentiates p."""

    @staticmethod
    def forward(ctx, ex, args, imp_s, imp_t, imp_b, p, bundle):
        ctx.ex, ctx.args = ex, args
        ctx.save_for_backward(imp_s, imp_t, imp_b)
        return p.detach()

    @staticmethod
    def backward(ctx, gp):
        ex = ctx.ex
        params = ex._gate_params()
        d_imps, gsum = [], None
        B, N = ctx.args[0][4], ctx.args[0][6]
        g1, g2 = gp[:3 * B * N].view(3, B * N), gp[3 * B * N:].view(3, B * N * N)
        for s, imp in enumerate(ctx.saved_tensors):
            e3, t3, x1, x2, B, W, N = ctx.args[s]
            with torch.enable_grad():
                imp_ = imp.detach().reshape(-1).to(torch.float32).requires_grad_(True)
                a = (e3.contiguous(), t3.contiguous(), x1.contiguous(), x2.contiguous(), (None, None, 1.0, 1.0),
                     1, B, W, N)
                p, _ = _ExplainFn.apply(ex, a, imp_, *params)
                gs = torch.autograd.grad((p,), [imp_] + list(params), grad_outputs=(torch.cat([g1[s], g2[s]]),),
                                         allow_unused=True)
            d_imps.append(gs[0])
            pg = [torch.zeros_like(q) if g is None else g for g, q in zip(gs[1:], params)]
            gsum = pg if gsum is None else [a_ + b_ for a_, b_ in zip(gsum, pg)]
        return (None, None, *[d.reshape(ctx.saved_tensors[s].shape) for s, d in enumerate(d_imps)], None,
                _flat_grads(gsum, params))


class _Ctx:
    """A stand-in ctx for calling _EvalExplainFn.backward per side."""

    def __init__(self, ex, args, imp):
        self.ex, self.args, self.saved_tensors = ex, args, (imp,)


class _EvalExplainFn(torch.autograd.Function):
    """retrieve_edge_imp_node(training=False) with gradients enabled: forward = the eval kernels' hop-1 /
    hop-2 explanation; backward recomputes through explain_groups (HIP gate + scatter-max training kernels,
    Beta mean) and differentiates that."""

    @staticmethod
    def forward(ctx, ex, args, imp, o1, o2, *params):
        ctx.ex, ctx.args = ex, args
        ctx.save_for_backward(imp)
        return o1.detach(), o2.detach()

    @staticmethod
    def backward(ctx, g1, g2):
        (imp,) = ctx.saved_tensors
        e3, t3, n1, x1, n2, x2, B, W, N = ctx.args
        ex = ctx.ex
        params = ex._gate_params()
        with torch.enable_grad():
            imp_ = imp.detach().requires_grad_(True)
            if ex._hip_ok():
                e0, e1 = ex.explain_groups(imp_.reshape(1, B, W), e3, t3, n1, x1, n2, x2, 1, B, W, N, False)
            else:   # constructor variants without HIP training kernels: the torch formulation
                e0, e1 = ex._edge_imp_torch(([n1, n2], [x1, x2], None), imp_.reshape(B, W, 1), (None, e3, t3),
                                            False)
            gs = torch.autograd.grad((e0, e1), [imp_] + list(params),
                                     grad_outputs=(g1.reshape(e0.shape), g2.reshape(e1.shape)), allow_unused=True)
        return (None, None, gs[0], None, None, *gs[1:])


class _KLFn(torch.autograd.Function):
    """kl_loss of G groups summed: per-event shares and d/d prob from one tm_kl_loss launch."""

    @staticmethod
    def forward(ctx, prob, cat, null12, target):
        G, B, W = prob.shape
        dev = prob.device
        p = prob.detach().to(torch.float32).contiguous()
        c = cat.to(dev, torch.int32).contiguous()
        nv = null12.to(dev, torch.float32).contiguous()
        partial = torch.empty(max(G * B, 1), dtype=torch.float32, device=dev)
        dprob = torch.empty((G, B, W), dtype=torch.float32, device=dev)
        L.check(L.lib().tm_kl_loss(L.ptr(p), L.ptr(c), L.ptr(nv), float(target), G, B, W, L.ptr(partial),
                                   L.ptr(dprob), L.stream_ptr(dev)), "kl_loss")
        ctx.save_for_backward(dprob)
        return partial[:G * B].sum()

    @staticmethod
    def backward(ctx, g):
        (dprob,) = ctx.saved_tensors
        return dprob * g, None, None, None


class _BetaRsampleFn(torch.autograd.Function):
    """beta_sample(p, training=True) * pad (explainer_new.py:400-404, :420-430) with torch's own Dirichlet
    sampler and reparameterized gradient (torch._sample_dirichlet / torch._dirichlet_grad, the kernels
    Beta.rsample runs, same RNG stream) and the elementwise rest in one launch each way (tm_beta_params,
    tm_beta_rsample_bwd): bitwise the torch formulation, ~6 launches instead of ~25."""

    @staticmethod
    def forward(ctx, p, pad):
        dev = p.device
        n = p.numel()
        conc = torch.empty(n, 2, dtype=torch.float32, device=dev)
        total = torch.empty_like(conc)
        st = L.stream_ptr(dev)
        L.check(L.lib().tm_beta_params(L.ptr(p), n, L.ptr(conc), L.ptr(total), st), "beta_sample")
        x = torch._sample_dirichlet(conc)
        ctx.save_for_backward(p, pad, x, conc, total)
        return x[:, 0] * pad

    @staticmethod
    def backward(ctx, g):
        p, pad, x, conc, total = ctx.saved_tensors
        d = torch._dirichlet_grad(x, conc, total)
        g = g.contiguous()
        dp = torch.empty_like(p)
        L.check(L.lib().tm_beta_rsample_bwd(L.ptr(g), L.ptr(pad), L.ptr(x.contiguous()), L.ptr(d.contiguous()),
                                            L.ptr(p), p.numel(), L.ptr(dp), L.stream_ptr(p.device)), "beta_sample")
        return dp, None


class _ExplainFn(torch.autograd.Function):
    """retrieve_edge_imp_node's gate + scatter-max + gather (training) on the HIP kernels: p = [hop-1 | hop-2]
    maxima in one tensor, and (with the subgraph node ids in args) the padding mask (no gradient)."""

    @staticmethod
    def forward(ctx, ex, args, imp, *params):
        p, pad, bufs = ex._explain_fwd(args, imp)
        ctx.ex, ctx.args, ctx.bufs = ex, args, bufs
        ctx.save_for_backward(imp)
        if pad is not None:
            ctx.mark_non_differentiable(pad)
        return p, pad

    @staticmethod
    def backward(ctx, dp, _dpad):
        (imp,) = ctx.saved_tensors
        G, B, N = ctx.args[5], ctx.args[6], ctx.args[8]
        n1 = G * B * N
        dp = dp.contiguous()
        d_imp, grads = ctx.ex._explain_bwd(ctx.args, imp, ctx.bufs, dp[:n1], dp[n1:])
        ctx.bufs = None
        return (None, None, d_imp, *grads)
