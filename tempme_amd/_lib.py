"""ctypes binding of libtempme_hip.so (the C ABI in include/tempme.h).

The library is built in-tree (``tempme_amd/lib/libtempme_hip.so``, see
``__graft_entry__.build()``).  There is no fallback: if the library is missing or
no HIP device is visible, every entry point raises.

``import torch`` happens before the library is loaded so that its
``libamdhip64.so.7`` dependency binds to the HIP runtime torch already loaded
(one runtime per process: torch's streams and device pointers are then valid in
the library).
"""
import ctypes as C
import os
import types

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# TEMPME_LIB: an alternative in-tree build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("TEMPME_LIB") or os.path.join(_HERE, "lib", "libtempme_hip.so")

TM_OK = 0
TM_E_EDGE_NOT_IN_LIST = -1
TM_E_SHAPE = -2
TM_E_HIP = -3
TM_E_ARG = -4
TM_E_UNSUPPORTED = -5

SIDE_NONE, SIDE_SRC, SIDE_TGT, SIDE_BGD = 0, 1, 2, 3
SPLIT_TRAIN, SPLIT_TEST, SPLIT_NULL = 0, 1, 2
TM_DEBUG_FORCE_UNKEYED, TM_DEBUG_HOST_BUILD, TM_DEBUG_GRAPH_TIMING, TM_DEBUG_WALK_BLOCKS = 1, 2, 3, 4   # tm_debug_set (tests, A/B tools)
N_WEIGHTS = 28

# every symbol include/tempme.h declares
EXPORTS = (
    "tm_last_error", "tm_version", "tm_debug_set", "tm_set_host_threads", "tm_graph_build", "tm_graph_build_edges", "tm_graph_free", "tm_graph_info", "tm_graph_export",
    "tm_graph_strict_view",
    "tm_sample_khop", "tm_sample_walks", "tm_neg_sample", "tm_perm_keys", "tm_motif_hist", "tm_edge_counts",
    "tm_sample_events", "tm_gather_rows", "tm_weights_create", "tm_weights_create_ex", "tm_weights_pack", "tm_weights_variant", "tm_weights_set_node_zero", "tm_weights_version", "tm_weights_free",
    "tm_encoder_workspace_bytes",
    "tm_encoder_fwd", "tm_encoder_fwd_tab", "tm_encoder_train_supported", "tm_encoder_train_fwd", "tm_encoder_bwd", "tm_encoder_wgrad", "tm_wgrad",
    "tm_explain_train_fwd", "tm_explain_train_fwd_pad", "tm_explain_train_bwd", "tm_kl_loss", "tm_edge_importance", "tm_edge_gate_table",
    "tm_edge_table_cols", "tm_edge_tables", "tm_edge_feature_table", "tm_edge_importance_tab", "tm_tgn_attn_fwd", "tm_tgn_attn_bwd", "tm_gm_packed_floats", "tm_gm_pack", "tm_gm_embed", "tm_gm_embed_bwd_ok", "tm_gm_embed_bwd", "tm_gm_packed_a_floats", "tm_gm_pack_a", "tm_gm_fused_ok", "tm_dropin_create", "tm_dropin_free", "tm_dropin_forward", "tm_dropin_set_stream", "tm_dropin_gate_cache", "tm_dropin_gate_cache_clear", "tm_edge_importance_gf", "tm_edge_importance_gf3", "tm_edge_importance_gf3_bern",
    "tm_mask_least_important", "tm_profile_enable", "tm_profile_sync", "tm_profile_entry",
    "tm_beta_params", "tm_beta_rsample_bwd", "tm_adam_step", "tm_copy_many", "tm_host_register", "tm_host_unregister",
    "tm_stage_cast",
)


class TmRng(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("split", C.c_uint32), ("side", C.c_uint32)]


class TgnAttn(C.Structure):
    """tm_tgn_attn (include/tempme.h)."""
    _fields_ = [("rows", C.c_int32), ("n_ngh", C.c_int32), ("n_head", C.c_int32),
                ("d_node", C.c_int32), ("d_edge", C.c_int32), ("d_time", C.c_int32),
                ("node_rows", C.c_int32), ("edge_rows", C.c_int32), ("head_major_rows", C.c_int32),
                ("seg_rows", C.c_int32),
                ("temperature", C.c_float),
                ("node_tab", C.c_void_p), ("node_idx", C.c_void_p), ("edge_tab", C.c_void_p),
                ("edge_idx", C.c_void_p), ("dt", C.c_void_p), ("time_w", C.c_void_p), ("time_b", C.c_void_p),
                ("mask_node", C.c_void_p), ("ew", C.c_void_p), ("qf", C.c_void_p), ("err_flag", C.c_void_p)]


class GmEmbedArgs(C.Structure):
    """tm_gm_embed_args (include/tempme.h)."""
    _fields_ = [(n, C.c_int32) for n in ("R", "N", "C", "T", "D", "L", "HT", "HC")] + \
               [(n, C.c_void_p) for n in ("node", "nid", "eid", "cut", "ts", "ew", "edge_attr", "n_feat", "e_feat",
                                          "time_w", "time_b", "proj_w", "proj_b")] + \
               [("layer_table", C.c_void_p), ("x_mean", C.c_void_p), ("node_out", C.c_void_p)]


GRAD_IO_FIELDS = ("imp", "dlogit", "M2", "dM2", "M1d", "dM1", "X", "dY2", "H1d", "dH1", "O", "dP", "dQ", "dF",
                  "ev", "AB", "H", "dZ", "dlev", "g", "dt")


class EncoderGradIO(C.Structure):
    """tm_encoder_grad_io (include/tempme.h)."""
    _fields_ = [(n, C.c_void_p) for n in GRAD_IO_FIELDS]


EXPL_IO_FIELDS = ("X", "G1", "G2", "z", "gate", "d_gate", "dz", "dG2", "dG1", "g", "t")


class ExplainGradIO(C.Structure):
    """tm_explain_grad_io (include/tempme.h)."""
    _fields_ = [(n, C.c_void_p) for n in EXPL_IO_FIELDS]


class WgradJob(C.Structure):
    _fields_ = [("dy", C.c_void_p), ("x", C.c_void_p), ("ldy", C.c_int32), ("ldx", C.c_int32), ("O", C.c_int32),
                ("I", C.c_int32), ("R", C.c_int32)]


class GatherJob(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("row_bytes", C.c_int64), ("src_side_stride", C.c_int64),
                ("dst_side_stride", C.c_int64), ("src_rows", C.c_int64), ("sides", C.c_int32), ("reserved", C.c_int32)]


class CopyJob(C.Structure):
    """tm_copy_job (include/tempme.h)."""
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("n", C.c_int64)]


class StageJob(C.Structure):
    """tm_stage_job (include/tempme.h)."""
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("src_type", C.c_int32), ("dst_type", C.c_int32),
                ("ndim", C.c_int32), ("bound", C.c_int32), ("shape", C.c_int64 * 5), ("stride", C.c_int64 * 5)]


TM_I32, TM_F32, TM_I64, TM_F64 = 1, 2, 3, 4


class WgradTarget(C.Structure):
    _fields_ = [("w", C.c_void_p), ("b", C.c_void_p), ("first_job", C.c_int32), ("n_jobs", C.c_int32)]


class TempMEError(RuntimeError):
    pass


_lib = None
vp = C.c_void_p
i32, i64, u32, u64 = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64


def _sig(L):
    L.tm_last_error.restype = C.c_char_p
    L.tm_version.restype = C.c_int
    L.tm_debug_set.argtypes = [i32, i32]
    L.tm_set_host_threads.argtypes = [i32]
    L.tm_graph_build.argtypes = [i32, vp, vp, vp, vp, C.c_int, C.POINTER(vp)]
    L.tm_graph_build_edges.argtypes = [i32, i64, vp, vp, vp, vp, C.c_int, C.POINTER(vp)]
    L.tm_graph_free.argtypes = [vp]
    L.tm_graph_info.argtypes = [vp, C.POINTER(i32), C.POINTER(i64), C.POINTER(i32)]
    L.tm_graph_export.argtypes = [vp, vp, vp, vp, vp, vp]
    L.tm_graph_strict_view.argtypes = [vp, C.POINTER(vp)]
    L.tm_sample_khop.argtypes = [vp, TmRng, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.tm_sample_walks.argtypes = [vp, TmRng, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.tm_neg_sample.argtypes = [TmRng, vp, i64, vp, i32, i32, vp, vp]
    L.tm_perm_keys.argtypes = [u64, u32, i64, vp, vp]
    L.tm_motif_hist.argtypes = [vp, i64, i32, vp, vp, vp]
    L.tm_edge_counts.argtypes = [vp, i32, i32, vp, vp]
    L.tm_sample_events.argtypes = [vp, u64, u32, i32, i32, i32, vp, vp, vp, vp, vp, vp, i64] + [vp] * 15
    L.tm_weights_create.argtypes = [i32, i32, i32, C.c_int, C.POINTER(vp)]
    L.tm_weights_create_ex.argtypes = [i32, i32, i32, i32, C.c_int, C.POINTER(vp)]
    L.tm_weights_pack.argtypes = [vp, C.POINTER(vp), vp]
    L.tm_weights_variant.argtypes = [vp, i32, i32]
    L.tm_weights_set_node_zero.argtypes = [vp, i32]
    L.tm_weights_version.argtypes = [vp]
    L.tm_weights_version.restype = u64
    L.tm_weights_free.argtypes = [vp]
    L.tm_encoder_workspace_bytes.restype = i64
    L.tm_encoder_workspace_bytes.argtypes = [vp, i64]
    L.tm_encoder_fwd.argtypes = [vp, vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.tm_encoder_train_fwd.argtypes = [vp, vp, vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, C.c_float, vp, vp, vp]
    L.tm_encoder_bwd.argtypes = [vp, vp, vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, C.c_float, vp, vp,
                                 C.POINTER(EncoderGradIO), vp]
    L.tm_encoder_train_supported.argtypes = [i32, i32, i32, i32]
    L.tm_encoder_wgrad.argtypes = [vp, i32, i32, i32, C.POINTER(EncoderGradIO), vp, C.POINTER(vp), vp]
    L.tm_wgrad.argtypes = [C.POINTER(WgradJob), i32, C.POINTER(WgradTarget), i32, vp]
    L.tm_explain_train_fwd.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, C.c_float, C.c_float,
                                       C.POINTER(ExplainGradIO), vp, vp, vp]
    L.tm_explain_train_fwd_pad.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, C.c_float,
                                           C.c_float, C.POINTER(ExplainGradIO), vp, vp, vp, vp, vp, vp, vp]
    L.tm_explain_train_bwd.argtypes = [vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, C.c_float, C.c_float, vp, vp,
                                       C.POINTER(ExplainGradIO), vp, C.POINTER(vp), vp]
    L.tm_edge_importance.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.tm_edge_gate_table.argtypes = [vp, vp, vp, vp, vp]
    L.tm_gather_rows.argtypes = [C.POINTER(GatherJob), i32, vp, i64, vp, vp]
    L.tm_kl_loss.argtypes = [vp, vp, vp, C.c_float, i32, i32, i32, vp, vp, vp]
    L.tm_edge_table_cols.argtypes = [vp]
    L.tm_edge_tables.argtypes = [vp, vp, vp, vp, vp, vp]
    L.tm_edge_feature_table.argtypes = [vp, vp, i32, vp, vp]
    L.tm_encoder_fwd_tab.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.tm_edge_importance_tab.argtypes = [vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.tm_gm_packed_floats.restype = i64
    L.tm_gm_packed_floats.argtypes = [i32, i32]
    L.tm_gm_pack.argtypes = [vp, i32, i32, vp, vp]
    L.tm_gm_embed.argtypes = [C.POINTER(GmEmbedArgs), vp]
    L.tm_gm_embed_bwd_ok.argtypes = [i32, i32, i32, i32, i32]
    L.tm_gm_embed_bwd.argtypes = [C.POINTER(GmEmbedArgs), vp, vp, vp, vp]
    L.tm_gm_packed_a_floats.restype = i64
    L.tm_gm_packed_a_floats.argtypes = [i32, i32, i32, i32]
    L.tm_gm_pack_a.argtypes = [vp, i32, i32, i32, i32, vp, vp]
    L.tm_gm_fused_ok.argtypes = [i32, i32, i32, i32]
    L.tm_dropin_create.argtypes = [i32, C.POINTER(vp)]
    L.tm_dropin_free.restype = None
    L.tm_dropin_free.argtypes = [vp]
    L.tm_dropin_forward.argtypes = [vp, i32, i32, vp, vp, vp, vp, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.tm_dropin_set_stream.argtypes = [vp, i32, vp]
    L.tm_dropin_gate_cache.argtypes = [vp, i64]
    L.tm_dropin_gate_cache_clear.argtypes = [vp]
    L.tm_edge_importance_gf.argtypes = [vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.tm_edge_importance_gf3.argtypes = [i32, i32, i32] + [vp] * 24
    L.tm_edge_importance_gf3_bern.argtypes = [i32, i32, i32] + [vp] * 26
    L.tm_tgn_attn_fwd.argtypes = [C.POINTER(TgnAttn), vp, vp, vp]
    L.tm_tgn_attn_bwd.argtypes = [C.POINTER(TgnAttn), vp, vp, vp, vp, vp]
    L.tm_mask_least_important.argtypes = [vp, i32, i32, vp, i32, vp, vp, vp]
    L.tm_profile_enable.argtypes = [C.c_int]
    L.tm_beta_params.argtypes = [vp, i64, vp, vp, vp]
    f32 = C.c_float
    L.tm_adam_step.argtypes = [vp, vp, vp, vp, i64, f32, f32, f32, f32, f32, f32, vp, vp, i32, vp]
    L.tm_copy_many.argtypes = [C.POINTER(CopyJob), i32, vp]
    L.tm_host_register.argtypes = [vp, i64, C.POINTER(vp)]
    L.tm_host_unregister.argtypes = [vp]
    L.tm_stage_cast.argtypes = [vp, i32, vp]   # tm_stage_job rows (hoststage builds them as int64 words)
    L.tm_beta_rsample_bwd.argtypes = [vp, vp, vp, vp, vp, i64, vp, vp]
    L.tm_profile_entry.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.POINTER(i64)]
    for name in EXPORTS:
        if name not in ("tm_last_error", "tm_encoder_workspace_bytes"):
            getattr(L, name).restype = C.c_int


class _Lenient:
    """Attribute access on a CDLL that yields a throwaway object for symbols the library lacks."""

    def __init__(self, L):
        self.__dict__["_L"] = L

    def __getattr__(self, name):
        try:
            return getattr(self._L, name)
        except AttributeError:
            return types.SimpleNamespace()


def lib():
    """The loaded library; raises if it was not built (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"tempme_amd: HIP library not built ({LIB_PATH} missing); run __graft_entry__.build() "
                "or `make -C tempme_amd/csrc`")
        L = C.CDLL(LIB_PATH)
        # an A/B build (TEMPME_LIB) may predate newer entry points: their signatures are skipped, and a call
        # to one of them fails with AttributeError
        _sig(_Lenient(L) if os.environ.get("TEMPME_LIB") else L)
        _lib = L
        # the host-side graph builder's threads: this process's CPU share (the GPU box sets OMP_NUM_THREADS to it)
        fn = getattr(L, "tm_set_host_threads", None)
        if fn is not None:
            n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
            if n <= 0 and hasattr(os, "sched_getaffinity"):
                n = len(os.sched_getaffinity(0))
            fn(max(0, min(n, 64)))
    return _lib


def check(rc, what=""):
    """Map a TM_E_* code to the exception type the reference raises for the same condition."""
    if rc == TM_OK:
        return
    msg = lib().tm_last_error().decode(errors="replace")
    if rc == TM_E_EDGE_NOT_IN_LIST:
        raise IndexError(msg or f"{what}: e_idx not found in edge list")
    if rc == TM_E_SHAPE:
        raise AssertionError(msg or what)
    if rc in (TM_E_ARG,):
        raise ValueError(f"{what}: {msg}")
    if rc == TM_E_UNSUPPORTED:
        raise NotImplementedError(f"{what}: {msg}")
    raise TempMEError(f"{what}: {msg} (code {rc})")


def raise_device_error(code, what):
    """Device-side error flag (set by the kernels) -> reference exception."""
    if code == 0:
        return
    if code == TM_E_EDGE_NOT_IN_LIST:
        raise IndexError(f"{what}: e_idx not found in edge list of its node (utils/graph.py:134-135)")
    if code == TM_E_ARG:
        raise IndexError(f"{what}: node index out of range")
    raise TempMEError(f"{what}: device error {code}")


def ptr(t):
    """Raw device (or host) pointer of a torch tensor, None for None."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    """hipStream_t of the current stream of `device` (torch's raw accessor: no Stream object per call)."""
    if isinstance(device, torch.device) and device.index is not None:
        return C.c_void_p(torch._C._cuda_getCurrentRawStream(device.index))
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(device=None):
    """The torch.device the hot path runs on.  Fails loudly without a HIP GPU."""
    if not torch.cuda.is_available():
        raise RuntimeError("tempme_amd: no HIP device visible; the hot path has no CPU fallback")
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError(f"tempme_amd: device {device} is not a HIP device; the hot path has no CPU fallback")
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    return device


def profile_enable(on=True):
    check(lib().tm_profile_enable(1 if on else 0), "tm_profile_enable")


def profile_read():
    """{kernel name: (total_ms, launches)} recorded since profile_enable(True)."""
    n = lib().tm_profile_sync()
    if n < 0:
        check(n, "tm_profile_sync")
    out = {}
    for i in range(n):
        name, ms, cnt = C.c_char_p(), C.c_double(), i64()
        check(lib().tm_profile_entry(i, C.byref(name), C.byref(ms), C.byref(cnt)), "tm_profile_entry")
        out[name.value.decode()] = (ms.value, cnt.value)
    return out
