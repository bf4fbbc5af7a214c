"""Generate the committed golden vectors by running the REFERENCE itself.

Run once, in the build container only (it reads /root/reference, which does not
exist on the GPU box):

    python tests/golden/make_goldens.py

What it does
------------
* Imports the reference Python (read-only, from /root/reference) with the
  shims SURVEY.md §8(c) lists: ``numba.jit`` -> identity, ``torch_scatter.scatter``
  -> ``torch.scatter_reduce`` (fill-0-for-empty semantics), a stub ``turtle``,
  and an in-memory ``h5py`` stand-in that captures the datasets the reference
  writes (processed/data_preprocess.py:139-143, :393-404).
* Replaces ``np.random.randint`` / ``np.random.permutation`` by the keyed
  Philox contract of ``oracle/philox.py``.  The key of each draw is read from
  the reference's own call-site frames (loop index ``i`` of
  get_temporal_neighbor / get_next_step / get_final_step, the hop ``layer_i``
  of find_k_hop, the event loop ``k`` and the calling line of the
  pre_processing drivers), so the reference code runs unmodified.
* Drives the reference's own ``pre_processing`` (data_preprocess.py:99-145,
  extracted with ``ast`` because the module body runs the whole pipeline),
  ``marginal`` (:148-214), ``calculate_edge`` (:346-356),
  ``get_null_distribution`` (utils/null_model.py:124) and the ``TempME``
  explainer (models/explainer_new.py:103-453).

Only data (inputs and expected outputs) is written under tests/golden/.
"""
import ast
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

from oracle import philox as px  # noqa: E402

import torch  # noqa: E402

# ----------------------------------------------------------------------------- shims
numba = types.ModuleType("numba")


def _jit(*a, **k):
    if a and callable(a[0]) and not k:
        return a[0]
    return lambda f: f


numba.jit = _jit
sys.modules["numba"] = numba

tsc = types.ModuleType("torch_scatter")


def _scatter(src, index, dim=-1, out=None, dim_size=None, reduce="sum"):
    shape = list(src.shape)
    shape[dim] = dim_size
    base = torch.zeros(shape, dtype=src.dtype, device=src.device)
    red = {"max": "amax", "mean": "mean", "sum": "sum"}[reduce]
    return base.scatter_reduce(dim, index, src, red, include_self=False)


tsc.scatter = _scatter
sys.modules["torch_scatter"] = tsc
_turtle = types.ModuleType("turtle")
_turtle.pos = _turtle.position = None     # names imported (unused) by TGN/tgn.py:2, embedding_module.py:1
sys.modules["turtle"] = _turtle


class _FakeH5File:
    store = {}

    def __init__(self, name, mode="r"):
        self.name = os.path.basename(str(name))
        if "w" in mode:
            _FakeH5File.store[self.name] = {}

    def create_dataset(self, key, data):
        _FakeH5File.store[self.name][key] = np.array(data)

    def __getitem__(self, key):
        return _FakeH5File.store[self.name][key]

    def close(self):
        pass


h5 = types.ModuleType("h5py")
h5.File = _FakeH5File
sys.modules["h5py"] = h5

sys.path.insert(0, REF)

# ----------------------------------------------------------------------------- keyed RNG
CTX = {"seed": 0, "split": px.SPLIT_TEST, "event_base": 0, "side": px.SIDE_NONE, "batch": 1}
_orig_randint = np.random.randint
_orig_perm = np.random.permutation

# lines of the reference drivers that select the side of a sampling call
_DP_LINES = {112: px.SIDE_NONE, 114: px.SIDE_SRC, 118: px.SIDE_TGT, 122: px.SIDE_BGD,
             126: px.SIDE_SRC, 127: px.SIDE_TGT, 128: px.SIDE_BGD}          # data_preprocess.py
_NM_LINES = {106: px.SIDE_NONE, 107: px.SIDE_SRC, 108: px.SIDE_TGT, 109: px.SIDE_BGD,
             110: px.SIDE_SRC, 111: px.SIDE_TGT, 112: px.SIDE_BGD}          # null_model.py


def _driver_context(frame):
    """(event_base, side) from the enclosing reference pre_processing frame, else CTX."""
    f = frame
    while f is not None:
        if f.f_code.co_name == "pre_processing":
            fn = f.f_code.co_filename
            if fn.endswith("data_preprocess.py"):
                return f.f_locals["k"], _DP_LINES[f.f_lineno]
            if fn.endswith("null_model.py"):
                return f.f_locals["k"] * f.f_locals["batch_size"], _NM_LINES[f.f_lineno]
        f = f.f_back
    return CTX["event_base"], CTX["side"]


def keyed_randint(low, high=None, size=None, dtype=int):
    if high is None:
        low, high = 0, low
    assert low == 0
    f = sys._getframe(1)
    name = f.f_code.co_name
    base, side = _driver_context(f)
    seed, split = CTX["seed"], CTX["split"]
    if name == "get_temporal_neighbor":                       # graph.py:218
        fk = f.f_back
        assert fk.f_code.co_name == "find_k_hop"
        hop = fk.f_locals["layer_i"] + 1
        i, n = f.f_locals["i"], f.f_locals["num_neighbor"]
        rpe = n ** (hop - 1)
        out = px.draw(seed, split, side, hop, base + i // rpe, i % rpe, np.arange(size), high)
    elif name == "get_next_step":                             # graph.py:328
        i, deg = f.f_locals["i"], f.f_locals["degree"]
        out = px.draw(seed, split, side, px.STAGE_STEP2, base + i // deg, i % deg, np.arange(size), high)
    elif name == "get_final_step":                            # graph.py:380/420/457
        fw = f.f_back
        assert fw.f_code.co_name == "find_k_walks"
        w = fw.f_locals["degree"] * fw.f_locals["num_neighbors"]
        i = f.f_locals["i"]
        out = px.draw(seed, split, side, px.STAGE_STEP3, base + i // w, i % w, np.arange(size), high)
    elif name == "sample":                                    # batch_loader.py:40-41
        j = 1 if "src_index" in f.f_locals else 0
        out = px.draw(seed, split, px.SIDE_NONE, px.STAGE_NEG, base + np.arange(size), 0, j, high)
    else:
        raise RuntimeError(f"unexpected randint caller {name}")
    return np.asarray(out, dtype=np.int64)


def keyed_permutation(x):
    f = sys._getframe(1)
    assert f.f_code.co_name == "load_data_shuffle", f.f_code.co_name
    return px.keyed_permutation(int(x), CTX["seed"], px.SPLIT_NULL)


np.random.randint = keyed_randint
np.random.permutation = keyed_permutation

# ----------------------------------------------------------------------------- reference imports
from utils.graph import NeighborFinder  # noqa: E402
from utils.batch_loader import RandEdgeSampler, load_subgraph_margin, get_item, get_item_edge  # noqa: E402
import utils.null_model as ref_null  # noqa: E402


def load_data_preprocess_module():
    """data_preprocess.py minus its module-level pipeline (:364-420); line numbers kept."""
    path = os.path.join(REF, "processed", "data_preprocess.py")
    src = open(path).read()
    tree = ast.parse(src, path)
    keep = [n for n in tree.body if isinstance(n, (ast.Import, ast.ImportFrom, ast.FunctionDef))
            or (isinstance(n, ast.Assign) and n.targets[0].id in ("degree_dict", "data"))]
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {"__file__": path, "__name__": "data_preprocess_golden"}
    sys.path.insert(0, os.path.join(REF))
    exec(compile(mod, path, "exec"), ns)
    return ns


DP = load_data_preprocess_module()


def save_npz(name, **arrays):
    np.savez_compressed(os.path.join(HERE, name), **arrays)
    print("wrote", name, sum(a.size for a in arrays.values()), "elements")


# ----------------------------------------------------------------------------- cases
def build_finder(src, dst, eidx, ts, n_nodes):
    """The adjacency construction of temp_exp_main.py:135-144 / data_preprocess.py:59-63."""
    adj = [[] for _ in range(n_nodes)]
    for s, d, e, t in zip(src, dst, eidx, ts):
        adj[s].append((d, e, t))
        adj[d].append((s, e, t))
    return NeighborFinder(adj)


def run_pipeline(finder, sampler, src, dst, ts, eidx, n_deg, n_events, tag_name, split):
    """data_preprocess.pre_processing + marginal + calculate_edge on the first n_events."""
    CTX["split"] = split
    DP["ngh_finder"] = finder
    DP["NUM_NEIGHBORS"] = n_deg
    k = n_events + 1
    DP["pre_processing"](finder, sampler, src[:k], dst[:k], ts[:k], None if eidx is None else eidx[:k],
                         MODE=tag_name, data="golden")
    st = _FakeH5File.store[f"golden_{tag_name}.h5"]
    wsn, wtn, wbn = DP["marginal"](st["walks_src"], st["walks_tgt"], st["walks_bgd"])
    edge = DP["calculate_edge"](wsn, wtn, wbn)
    out = {k2: v for k2, v in st.items()}
    out.update(walks_src_new=wsn, walks_tgt_new=wtn, walks_bgd_new=wbn, edge=edge)
    return out


def pack_pipeline(out):
    """Store losslessly in narrow dtypes (all node/eid/count values are small ints,
    all ts are float32 values)."""
    res = {}
    for key, v in out.items():
        v = np.asarray(v)
        if key.startswith("subgraph"):
            n = v.shape[1] // 3
            res[key + "_node"] = v[:, :n].astype(np.int32)
            res[key + "_eid"] = v[:, n:2 * n].astype(np.int32)
            res[key + "_ts"] = v[:, 2 * n:].astype(np.float32)
            assert np.array_equal(res[key + "_ts"].astype(np.float64), v[:, 2 * n:])
        elif key in ("walks_src", "walks_tgt", "walks_bgd"):
            res[key + "_node"] = v[..., :6].astype(np.int32)
            res[key + "_eid"] = v[..., 6:9].astype(np.int32)
            res[key + "_ts"] = v[..., 9:12].astype(np.float32)
            res[key + "_anony"] = v[..., 12:15].astype(np.int32)
        elif key.endswith("_new"):
            res[key.replace("_new", "_cat")] = v[..., 12].astype(np.int32)
            res[key.replace("_new", "_marg")] = v[..., 13].astype(np.float64)
        elif key == "edge":
            res["edge"] = v.astype(np.int32)
            assert np.array_equal(res["edge"], v)
        elif key == "dst_fake":
            res["dst_fake"] = v.astype(np.int32)
    return res


def case_kats():
    out = {}
    # KAT-tie: node 1 adjacency ts [1,2,2,3,4,4,4], e = 1..7
    ts = [1., 2., 2., 3., 4., 4., 4.]
    src = [1] * 7
    dst = [2, 3, 4, 5, 6, 7, 8]
    eidx = list(range(1, 8))
    f = build_finder(src, dst, eidx, ts, 9)
    out["kat_tie"] = {
        "src": src, "dst": dst, "eidx": eidx, "ts": ts, "n_nodes": 9,
        "nodeedge2idx_1": {str(k): int(v) for k, v in f.nodeedge2idx[1].items()},
        "find_before_e7": len(f.find_before(1, 4.0, e_idx=7)[0]),
        "find_before_t4": len(f.find_before(1, 4.0)[0]),
        "find_before_t2p5": len(f.find_before(1, 2.5)[0]),
    }
    # KAT-leak: edges (1,2,1) (2,3,5) (2,4,9); root 1 cut 10 N=2 M=1
    src, dst, ts, eidx = [1, 2, 2], [2, 3, 4], [1., 5., 9.], [1, 2, 3]
    f = build_finder(src, dst, eidx, ts, 5)
    CTX.update(seed=0, split=px.SPLIT_TEST, event_base=0, side=px.SIDE_BGD)
    sub = f.find_k_hop(2, np.array([1]), np.array([10.]), 2, e_idx_l=None)
    walks = f.find_k_walks(2, np.array([1]), num_neighbors=1, subgraph_src=sub)
    out["kat_leak"] = {
        "src": src, "dst": dst, "eidx": eidx, "ts": ts, "n_nodes": 5, "seed": 0,
        "split": px.SPLIT_TEST, "side": px.SIDE_BGD, "N": 2, "M": 1,
        "hop1": [a.tolist() for a in (sub[0][0], sub[1][0], sub[2][0])],
        "hop2": [a.tolist() for a in (sub[0][1], sub[1][1], sub[2][1])],
        "walk_node": walks[0].tolist(), "walk_eid": walks[1].tolist(),
        "walk_ts": walks[2].tolist(), "walk_anony": walks[3].tolist(),
    }
    with open(os.path.join(HERE, "kats.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote kats.json")


def synth_small(seed=7, n_nodes=12, n_edges=240):
    """A tiny tie-heavy temporal graph: real node 0, self-loops, repeated pairs."""
    rng = np.random.RandomState(seed)
    src = rng.randint(0, n_nodes, n_edges)
    dst = rng.randint(0, n_nodes, n_edges)
    dst[5] = src[5]
    dst[77] = src[77]                                 # two self-loops
    ts = np.sort(rng.randint(0, 40, n_edges)).astype(np.float64)
    eidx = np.arange(1, n_edges + 1)
    return src, dst, ts, eidx


def case_synth_small():
    src, dst, ts, eidx = synth_small()
    n_nodes = int(max(src.max(), dst.max())) + 1
    finder = build_finder(src, dst, eidx, ts, n_nodes)
    sampler = RandEdgeSampler((src,), (dst,))
    res = {"src": src.astype(np.int32), "dst": dst.astype(np.int32), "ts": ts,
           "eidx": eidx.astype(np.int32)}
    # node-edge position table (the dict of get_ts2idx, graph.py:77-101)
    ne = []
    for u, d in finder.nodeedge2idx.items():
        for e, p in d.items():
            ne.append((u, e, p))
    res["nodeedge2idx"] = np.array(sorted(ne), dtype=np.int32)
    res["csr_node"] = finder.node_idx_l.astype(np.int32)
    res["csr_eid"] = finder.edge_idx_l.astype(np.int32)
    res["csr_ts"] = finder.node_ts_l.astype(np.float64)
    res["csr_off"] = finder.off_set_l.astype(np.int64)
    for n_deg in (5, 8):
        CTX.update(seed=11, event_base=0)
        out = run_pipeline(finder, sampler, src, dst, ts, eidx, n_deg, 24, f"small{n_deg}", px.SPLIT_TEST)
        for k2, v in pack_pipeline(out).items():
            res[f"N{n_deg}_{k2}"] = v
    # time-path k-hop for every row and a 3-hop call (find_k_hop, graph.py:233-262)
    CTX.update(seed=3, split=px.SPLIT_TRAIN, event_base=100, side=px.SIDE_BGD)
    roots = np.arange(n_nodes)
    cuts = np.linspace(0, 41, n_nodes)
    sub = finder.find_k_hop(3, roots, cuts, 4, e_idx_l=None)
    for h in range(3):
        res[f"khop3_node{h}"] = sub[0][h].astype(np.int32)
        res[f"khop3_eid{h}"] = sub[1][h].astype(np.int32)
        res[f"khop3_ts{h}"] = sub[2][h].astype(np.float32)
    save_npz("synth_small.npz", **res)


def uslegis_split(mode):
    """data_preprocess.load_data (the reference's own split code, :24-76)."""
    return DP["load_data"](mode=mode, data="uslegis_sampled")


def case_uslegis():
    res = {}
    for mode, split in (("train", px.SPLIT_TRAIN), ("test", px.SPLIT_TEST)):
        sampler, src, dst, ts, label, eidx, finder = uslegis_split(mode)
        res[f"{mode}_src"], res[f"{mode}_dst"] = src.astype(np.int32), dst.astype(np.int32)
        res[f"{mode}_ts"], res[f"{mode}_eidx"] = ts.astype(np.float64), eidx.astype(np.int32)
        res[f"{mode}_sampler_dst"] = sampler.dst_list.astype(np.int32)
        res[f"{mode}_sampler_src"] = sampler.src_list.astype(np.int32)
        for n_deg, n_ev in ((20, 32), (30, 12)):
            CTX.update(seed=0, event_base=0)
            out = run_pipeline(finder, sampler, src, dst, ts, eidx, n_deg, n_ev, f"{mode}{n_deg}", split)
            for k2, v in pack_pipeline(out).items():
                res[f"{mode}_N{n_deg}_{k2}"] = v
    save_npz("uslegis_pipeline.npz", **res)


def case_null():
    CTX.update(seed=0, split=px.SPLIT_NULL)
    d = ref_null.get_null_distribution("uslegis_sampled")
    with open(os.path.join(HERE, "null_uslegis.json"), "w") as fh:
        json.dump({"seed": 0, "data": "uslegis_sampled", "N": 30,
                   "dist": {str(k): float(v) for k, v in d.items()}}, fh, indent=1)
    print("wrote null_uslegis.json", d)
    return d


class _Base:
    """The four attributes TempME reads from its base model (explainer_new.py:107-108, :129-130)."""

    def __init__(self, n_feat, e_feat):
        self.n_feat_th = torch.from_numpy(n_feat.astype(np.float32))
        self.e_feat_th = torch.from_numpy(e_feat.astype(np.float32))
        self.node_raw_features = torch.nn.Embedding.from_pretrained(self.n_feat_th, padding_idx=0, freeze=True)
        self.edge_raw_features = torch.nn.Embedding.from_pretrained(self.e_feat_th, padding_idx=0, freeze=True)


USED_PREFIXES = ("event_conv.", "attention.W1.", "attention.W2.", "attention.MLP.", "MLP.",
                 "edge_dependency_gcn.", "time_encoder.")


def _pack_items(pipe, pre, n_deg, bsz, ts_key):
    """The first `bsz` events of a packed pipeline golden (keys `pre` + ...) through the reference's
    own H5 pack loader (data_preprocess.py:393-404 layout, batch_loader.py:120-242)."""
    st = {}
    for side in ("src", "tgt", "bgd"):
        for h in (0, 1):
            p = f"{pre}subgraph_{side}_{h}"
            st[f"subgraph_{side}_{h}"] = np.concatenate(
                [pipe[p + "_node"], pipe[p + "_eid"], pipe[p + "_ts"].astype(np.float64)], axis=1).astype(np.float64)
        p = f"{pre}walks_{side}"
        st[f"walks_{side}_new"] = np.concatenate(
            [pipe[p + "_node"], pipe[p + "_eid"], pipe[p + "_ts"].astype(np.float64),
             pipe[p + "_cat"][..., None], pipe[p + "_marg"][..., None]], axis=-1).astype(np.float64)
    st["dst_fake"] = pipe[f"{pre}dst_fake"].astype(np.float64)
    _FakeH5File.store["enc_pack"] = st

    class A:
        pass
    args = A()
    args.n_degree = n_deg
    pack = load_subgraph_margin(args, _FakeH5File("enc_pack"))
    edge = pipe[f"{pre}edge"].astype(np.float64)
    batch_idx = np.arange(bsz)
    items = get_item(pack, batch_idx)
    edges = get_item_edge(edge, batch_idx)
    ts_cut = pipe[ts_key][:bsz].astype(np.float64)
    return items, edges, ts_cut, batch_idx


def _enc_batch(n_deg=20, bsz=32):
    """The first `bsz` test events of uslegis_pipeline.npz as TempME receives them."""
    pipe = np.load(os.path.join(HERE, "uslegis_pipeline.npz"))
    items, edges, ts_cut, batch_idx = _pack_items(pipe, f"test_N{n_deg}_", n_deg, bsz, "test_ts")
    return pipe, items, edges, ts_cut, batch_idx


def _uslegis_feats():
    e_raw = np.load(os.path.join(REF, "processed", "ml_uslegis_sampled.npy"))
    n_raw = np.load(os.path.join(REF, "processed", "ml_uslegis_sampled_node.npy"))
    # the shipped edge table has 8832 rows for idx 1..8832 (sampling/sample_dataset.py:110-111);
    # pad one zero row so every idx is addressable
    e_pad = np.vstack([e_raw, np.zeros((1, e_raw.shape[1]))])
    rs = np.random.RandomState(5)
    return {
        "uslegis": (n_raw, e_pad, 0),
        "synth": (rs.uniform(0, 1, (n_raw.shape[0], 172)), rs.uniform(0, 1, (e_pad.shape[0], 32)), 1),
    }


def case_encoder():
    from models.explainer_new import TempME
    n_deg, bsz = 20, 32
    feats = _uslegis_feats()
    pipe, (sg_s, sg_t, sg_b, w_s, w_t, w_b, dst_fake), (e_s, e_t, e_b), ts_cut, batch_idx = _enc_batch(n_deg, bsz)
    res = {"ts_cut": ts_cut, "batch_idx": batch_idx}
    for name, (nf, ef, seed) in feats.items():
        torch.manual_seed(seed)
        CTX.update(seed=0, split=px.SPLIT_NULL)
        ex = TempME(_Base(nf, ef), base_model_type="tgn", data="uslegis_sampled", out_dim=40, hid_dim=64,
                    temp=0.07, if_cat_feature=True, dropout_p=0.1, device=torch.device("cpu"))
        ex.eval()
        with torch.no_grad():
            imp = [ex(w, ts_cut, e) for w, e in ((w_s, e_s), (w_t, e_t), (w_b, e_b))]
            expl = ex.retrieve_explanation(sg_s, imp[0], w_s, sg_t, imp[1], w_t, sg_b, imp[2], w_b, training=False)
            kl = [ex.kl_loss(p, w, target=0.3) for p, w in zip(imp, (w_s, w_t, w_b))]
        sd = {k: v.detach().numpy().astype(np.float32) for k, v in ex.state_dict().items()
              if k.startswith(USED_PREFIXES)}
        res[f"{name}_n_feat"] = nf.astype(np.float32)
        res[f"{name}_e_feat"] = ef.astype(np.float32)
        for k, v in sd.items():
            res[f"{name}_w_{k}"] = v
        for s, v in zip(("src", "tgt", "bgd"), imp):
            res[f"{name}_imp_{s}"] = v.numpy()
        res[f"{name}_expl0"] = expl[0].numpy()
        res[f"{name}_expl1"] = expl[1].numpy()
        res[f"{name}_kl"] = np.array([float(x) for x in kl])
        res[f"{name}_null"] = np.array([ex.null_model[k] for k in sorted(ex.null_model)])
        print(name, "imp mean", [float(v.mean()) for v in imp], "kl", [float(x) for x in kl])
    save_npz("encoder_uslegis.npz", **res)



def load_ref_function(relpath, name, **ns):
    """One FunctionDef of a reference module whose body cannot be imported (temp_exp_main.py
    parses argv and loads checkpoints at module level); line numbers kept."""
    path = os.path.join(REF, relpath)
    tree = ast.parse(open(path).read(), path)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name]
    ns.setdefault("__name__", "golden_" + name)
    exec(compile(ast.Module(body=fn, type_ignores=[]), path, "exec"), ns)
    return ns[name]


TGN_SEEDS = {"uslegis": 11, "synth": 12, "enron": 13}
TGN_RATIOS = [0.01, 0.02, 0.04, 0.06, 0.08, 0.10, 0.12, 0.14, 0.16, 0.18, 0.2, 0.22, 0.24, 0.26, 0.28, 0.30]
TGN_MSG_NODES = (3, 17, 42, 100, 101)


def tgn_perturbation(name, n_nodes, dim, raw_dim):
    """Memory state, last_update, TimeEncode bias and stored raw messages put on the random-init
    base model so that memory (tgn.py:104-108), the time-encoder bias and the message path of
    get_updated_memory (tgn.py:237-248) are all exercised.  Committed as data."""
    rng = np.random.default_rng(TGN_SEEDS[name])
    out = {
        "memory": rng.normal(0, 0.5, (n_nodes, dim)).astype(np.float32),
        "last_update": np.floor(rng.uniform(0, 10, n_nodes)).astype(np.float32),
        "time_bias": rng.normal(0, 0.5, dim).astype(np.float32),
        "msg_nodes": np.array(TGN_MSG_NODES, dtype=np.int64),
        # two messages per node; the "last" aggregator keeps the second (message_aggregator.py:40-46)
        "msg_raw": rng.normal(0, 1.0, (len(TGN_MSG_NODES), 2, raw_dim)).astype(np.float32),
        "msg_ts": np.floor(rng.uniform(0, 12, (len(TGN_MSG_NODES), 2))).astype(np.float32),
    }
    return out


def tgn_base(name, nf, ef, n_deg):
    """The seeded reference TGN of case_tgn with its committed perturbation applied."""
    from TGN.tgn import TGN
    torch.manual_seed(TGN_SEEDS[name])
    # learn_base.py:175-176 with its defaults (--n_layer 3, --n_head 2, --drop_out 0.5)
    base = TGN(nf, ef, n_neighbors=n_deg, device=torch.device("cpu"), n_layers=3, n_heads=2, dropout=0.5)
    base.forbidden_memory_update = True       # temp_exp_main.py:703-704
    base.eval()
    sd0 = {k: v.detach().clone() for k, v in base.state_dict().items()}
    dim = base.n_node_features
    raw_dim = 2 * dim + base.n_edge_features + dim
    pert = tgn_perturbation(name, base.n_nodes, dim, raw_dim)
    with torch.no_grad():
        base.memory.memory.data.copy_(torch.from_numpy(pert["memory"]))
        base.memory.last_update.data.copy_(torch.from_numpy(pert["last_update"]))
        base.time_encoder.w.bias.data.copy_(torch.from_numpy(pert["time_bias"]))
    for i, nd in enumerate(pert["msg_nodes"]):
        base.memory.messages[int(nd)] = [(torch.from_numpy(pert["msg_raw"][i, m]),
                                          torch.tensor(pert["msg_ts"][i, m])) for m in range(2)]
    return base, sd0, pert


def case_tgn():
    """Base TGN contrast (TGN/tgn.py:201-218) with and without TempME explanation weights, with
    explicit edge features (embedding_update_attr), and threshold_test (temp_exp_main.py:153-272)."""
    from sklearn.metrics import average_precision_score, roc_auc_score
    import math
    threshold_test = load_ref_function("temp_exp_main.py", "threshold_test", math=math, np=np, torch=torch,
                                       average_precision_score=average_precision_score,
                                       roc_auc_score=roc_auc_score)
    enc = np.load(os.path.join(HERE, "encoder_uslegis.npz"))
    n_deg, bsz = 20, 32
    pipe, (sg_s, sg_t, sg_b, _, _, _, dst_fake), _, ts_cut, _ = _enc_batch(n_deg, bsz)
    src, dst = pipe["test_src"][:bsz], pipe["test_dst"][:bsz]
    e_l = pipe["test_eidx"][:bsz]
    res = {}
    for name, (nf, ef, _) in _uslegis_feats().items():
        base, sd0, pert = tgn_base(name, nf, ef, n_deg)
        for k, v in sd0.items():
            v = v.double()
            res[f"{name}_sd_{k}"] = np.array([v.sum().item(), v.abs().sum().item(), (v * v).sum().item()])
        for k, v in pert.items():
            res[f"{name}_pert_{k}"] = v
        expl = [torch.from_numpy(enc[f"{name}_expl0"]), torch.from_numpy(enc[f"{name}_expl1"])]
        rng = np.random.default_rng(100 + TGN_SEEDS[name])
        ew_rand = [rng.uniform(0, 1, tuple(e.shape)).astype(np.float32) for e in expl]
        ew_rand[0][rng.uniform(0, 1, ew_rand[0].shape) < 0.2] = 0.0
        res[f"{name}_ew_rand0"], res[f"{name}_ew_rand1"] = ew_rand
        with torch.no_grad():
            upd_mem, _ = base.get_updated_memory(list(range(base.n_nodes)), base.memory.messages)
            res[f"{name}_updated_memory"] = upd_mem.numpy()
            pos_o, neg_o = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b)
            pos_e, neg_e = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b, explain_weights=expl)
            pos_r, neg_r = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b,
                                         explain_weights=[torch.from_numpy(x) for x in ew_rand])
        res[f"{name}_ori"] = torch.cat([pos_o, neg_o]).numpy()
        res[f"{name}_expl"] = torch.cat([pos_e, neg_e]).numpy()
        res[f"{name}_rand"] = torch.cat([pos_r, neg_r]).numpy()
        if name == "uslegis":
            ea = [x.numpy() for x in base.retrieve_edge_features(sg_s, sg_t, sg_b)]
            ea = [(x + rng.normal(0, 0.25, x.shape)).astype(np.float32) for x in ea]
            res[f"{name}_edge_attr0"], res[f"{name}_edge_attr1"] = ea
            with torch.no_grad():
                pos_a, neg_a = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b, explain_weights=expl,
                                             edge_attr=[torch.from_numpy(x) for x in ea])
            res[f"{name}_attr"] = torch.cat([pos_a, neg_a]).numpy()

        # threshold_test, capturing every masked-subgraph contrast it makes
        y_ori = torch.where(torch.cat([pos_o, neg_o]).sigmoid() > 0.5, 1., 0.).view(-1, 1)
        calls = []
        orig = base.contrast

        def capture(*a, **k):
            out = orig(*a, **k)
            calls.append((np.concatenate(a[5][0], axis=1) == 0, np.concatenate(a[6][0], axis=1) == 0,
                          np.concatenate(a[7][0], axis=1) == 0, torch.cat(out).numpy()))
            return out
        base.contrast = capture

        class A:
            pass
        args = A()
        args.ratios, args.base_type, args.n_degree, args.bs = TGN_RATIOS, "tgn", n_deg, bsz
        metrics = threshold_test(args, expl, base, src, dst, dst_fake, ts_cut, e_l, pos_o, neg_o, y_ori,
                                 sg_s, sg_t, sg_b)
        base.contrast = orig
        res[f"{name}_thr_metrics"] = np.array([float(m) for m in metrics])
        res[f"{name}_thr_logits"] = np.stack([c[3] for c in calls])
        res[f"{name}_thr_zero_bits"] = np.packbits(np.stack([np.concatenate(c[:3], axis=0) for c in calls]))
        print(name, "ori", float(res[f"{name}_ori"].mean()), "expl", float(res[f"{name}_expl"].mean()),
              "thr", res[f"{name}_thr_metrics"])
    res["ratios"] = np.array(TGN_RATIOS)
    save_npz("tgn_uslegis.npz", **res)


def case_train():
    """One deterministic iteration of the explainer training loop (temp_exp_main.py:584-632) with the
    reference TempME on the reference TGN: Explainer.eval() (dropout off) and if_bern=False (Beta mean),
    so loss, gradients and the Adam step are reproducible.  Stores the losses, every gradient that
    reaches the explainer and the parameter update of the Adam step."""
    from models.explainer_new import TempME
    n_deg, bsz = 20, 32
    pipe, (sg_s, sg_t, sg_b, w_s, w_t, w_b, dst_fake), (e_s, e_t, e_b), ts_cut, _ = _enc_batch(n_deg, bsz)
    src, dst = pipe["test_src"][:bsz], pipe["test_dst"][:bsz]
    e_l = pipe["test_eidx"][:bsz]
    res = {}
    for name, (nf, ef, seed) in _uslegis_feats().items():
        base, _, _ = tgn_base(name, nf, ef, n_deg)
        torch.manual_seed(seed)
        CTX.update(seed=0, split=px.SPLIT_NULL)
        ex = TempME(base, base_model_type="tgn", data="uslegis_sampled", out_dim=40, hid_dim=64, temp=0.07,
                    if_cat_feature=True, dropout_p=0.1, device=torch.device("cpu"))
        opt = torch.optim.Adam(ex.parameters(), lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0)
        criterion = torch.nn.BCEWithLogitsLoss()
        p0 = {k: v.detach().clone() for k, v in ex.named_parameters()}
        ex.eval()
        with torch.no_grad():
            pos_o, neg_o = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b)
            y_ori = torch.where(torch.cat([pos_o, neg_o], dim=0).sigmoid() > 0.5, 1., 0.).view(-1, 1)
        opt.zero_grad()
        g_s, g_t, g_b = ex(w_s, ts_cut, e_s), ex(w_t, ts_cut, e_t), ex(w_b, ts_cut, e_b)
        expl = ex.retrieve_explanation(sg_s, g_s, w_s, sg_t, g_t, w_t, sg_b, g_b, w_b, training=False)
        pos, neg = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b, explain_weights=expl)
        pred_loss = criterion(torch.cat([pos, neg], dim=0), y_ori)
        kl = ex.kl_loss(g_s, w_s, target=0.3) + ex.kl_loss(g_t, w_t, target=0.3) + ex.kl_loss(g_b, w_b, target=0.3)
        loss = pred_loss + 0.5 * kl
        loss.backward()
        opt.step()
        res[f"{name}_losses"] = np.array([loss.item(), pred_loss.item(), kl.item()])
        res[f"{name}_logits"] = torch.cat([pos, neg]).detach().numpy()
        n_grad = 0
        for k, v in ex.named_parameters():
            if v.grad is None:
                continue
            n_grad += v.numel()
            res[f"{name}_grad_{k}"] = v.grad.numpy().astype(np.float32)
            if name == "uslegis":
                res[f"{name}_upd_{k}"] = (v.detach() - p0[k]).numpy().astype(np.float32)
        print(name, "loss", res[f"{name}_losses"], "params with grad", n_grad)
    save_npz("train_uslegis.npz", **res)


# ----------------------------------------------------------------------------- Enron-scale case
ENRON = dict(n_nodes=184, n_edges=125235, alpha=1.2, de=32, dn=172, seed=0, node_feat="uniform")
ENRON_SETS = ((20, 100), (30, 32))          # (n_degree, events) of the test split
ENRON_VARIANTS = {"base": {}, "notg": dict(use_temporal_guidance=False),
                  "nodep": dict(use_dependency_aware_sampling=False), "h32": dict(hid_dim=32)}


def enron_graph():
    """Full-Enron-shaped synthetic graph of the bench (tempme_amd/workload.py enron_like: seeded
    numpy RandomState, so it is regenerated bit for bit from its parameters; a checksum is stored)."""
    from tempme_amd.workload import enron_like
    return enron_like(**ENRON)


def graph_checksum(g):
    return np.array([int(g["src"].sum()), int((g["src"] * g["dst"]).sum() % (1 << 61)), int(g["ts"].sum()),
                     float(g["e_feat"].astype(np.float64).sum()), float(g["n_feat"].astype(np.float64).sum())])


def _enron_load_data(g, mode):
    """The reference's own split code (data_preprocess.load_data, :24-76) on the synthetic graph: its
    pd.read_csv is pointed at an in-memory frame of the edges (the CSV layout of processed/ml_*.csv)."""
    import pandas
    df = pandas.DataFrame({"u": g["src"], "i": g["dst"], "ts": g["ts"], "label": g["label"], "idx": g["eidx"]})
    real = DP["pd"]
    DP["pd"] = types.SimpleNamespace(read_csv=lambda path, *a, **k: df if path.endswith("ml_enron_synth.csv")
                                     else real.read_csv(path, *a, **k))
    try:
        return DP["load_data"](mode=mode, data="enron_synth")
    finally:
        DP["pd"] = real


def _explain_outputs(ex, items, edges, ts_cut):
    """eval_one_epoch's scoring calls (temp_exp_main.py:446-452) plus the three kl_loss terms."""
    sg_s, sg_t, sg_b, w_s, w_t, w_b, _ = items
    e_s, e_t, e_b = edges
    with torch.no_grad():
        imp = [ex(w, ts_cut, e) for w, e in ((w_s, e_s), (w_t, e_t), (w_b, e_b))]
        expl = ex.retrieve_explanation(sg_s, imp[0], w_s, sg_t, imp[1], w_t, sg_b, imp[2], w_b, training=False)
        kl = [ex.kl_loss(p, w, target=0.3) for p, w in zip(imp, (w_s, w_t, w_b))]
    return imp, expl, kl


def _train_iteration(ex, base, src, dst, e_l, ts_cut, items, edges):
    """temp_exp_main.py:605-632 with Explainer.eval() and if_bern=False (see case_train)."""
    sg_s, sg_t, sg_b, w_s, w_t, w_b, dst_fake = items
    e_s, e_t, e_b = edges
    opt = torch.optim.Adam(ex.parameters(), lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0)
    criterion = torch.nn.BCEWithLogitsLoss()
    p0 = {k: v.detach().clone() for k, v in ex.named_parameters()}
    ex.eval()
    with torch.no_grad():
        pos_o, neg_o = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b)
        y_ori = torch.where(torch.cat([pos_o, neg_o], dim=0).sigmoid() > 0.5, 1., 0.).view(-1, 1)
    opt.zero_grad()
    g_s, g_t, g_b = ex(w_s, ts_cut, e_s), ex(w_t, ts_cut, e_t), ex(w_b, ts_cut, e_b)
    expl = ex.retrieve_explanation(sg_s, g_s, w_s, sg_t, g_t, w_t, sg_b, g_b, w_b, training=False)
    pos, neg = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b, explain_weights=expl)
    pred_loss = criterion(torch.cat([pos, neg], dim=0), y_ori)
    kl = ex.kl_loss(g_s, w_s, target=0.3) + ex.kl_loss(g_t, w_t, target=0.3) + ex.kl_loss(g_b, w_b, target=0.3)
    loss = pred_loss + 0.5 * kl
    loss.backward()
    opt.step()
    res = {"losses": np.array([loss.item(), pred_loss.item(), kl.item()]),
           "logits": torch.cat([pos, neg]).detach().numpy()}
    for k, v in ex.named_parameters():
        if v.grad is None:
            continue
        res[f"grad_{k}"] = v.grad.numpy().astype(np.float32)
        res[f"upd_{k}"] = (v.detach() - p0[k]).numpy().astype(np.float32)
    return res


def case_enron():
    """Bench-regime goldens: the full-Enron-shaped graph (V=184, E=125,235,
    ts in [0, 1e8)) through the reference's own load_data split, pre_processing, marginal and
    calculate_edge at N=20 and N=30; the reference TempME at Enron dims (de=32, dn=172) scoring those
    walks (forward x3, retrieve_explanation eval, kl_loss) for the default constructor and the
    use_temporal_guidance=False / use_dependency_aware_sampling=False / hid_dim=32 variants; and one
    deterministic training iteration on the reference TGN (as case_train)."""
    from models.explainer_new import TempME
    import time as _time
    g = enron_graph()
    t0 = _time.time()
    sampler, src, dst, ts, label, eidx, finder = _enron_load_data(g, "test")
    res = {"graph_checksum": graph_checksum(g), "graph_params": np.array(json.dumps(ENRON)),
           "test_src": src.astype(np.int32), "test_dst": dst.astype(np.int32), "test_ts": ts.astype(np.float64),
           "test_eidx": eidx.astype(np.int32), "test_sampler_dst": sampler.dst_list.astype(np.int32)}
    print("enron: load_data", round(_time.time() - t0, 1), "s; test events", len(src))
    for n_deg, n_ev in ENRON_SETS:
        t0 = _time.time()
        CTX.update(seed=0, event_base=0)
        out = run_pipeline(finder, sampler, src, dst, ts, eidx, n_deg, n_ev, f"enron{n_deg}", px.SPLIT_TEST)
        for k2, v in pack_pipeline(out).items():
            res[f"test_N{n_deg}_{k2}"] = v
        print(f"enron: N={n_deg} pipeline of {n_ev} events", round(_time.time() - t0, 1), "s")
    nf, ef = g["n_feat"], g["e_feat"]
    for n_deg, n_ev in ENRON_SETS:
        items, edges, ts_cut, _ = _pack_items(res, f"test_N{n_deg}_", n_deg, n_ev, "test_ts")
        for var, kw in ENRON_VARIANTS.items():
            if n_deg == 30 and var != "base":
                continue
            tag = f"N{n_deg}_{var}"
            torch.manual_seed(30 + len(tag))
            CTX.update(seed=0, split=px.SPLIT_NULL)
            ctor = dict(out_dim=40, hid_dim=64, temp=0.07, if_cat_feature=True, dropout_p=0.1,
                        device=torch.device("cpu"))
            ctor.update(kw)
            ex = TempME(_Base(nf, ef), base_model_type="tgn", data="uslegis_sampled", **ctor)
            ex.eval()
            imp, expl, kl = _explain_outputs(ex, items, edges, ts_cut)
            for k, v in ex.state_dict().items():
                if k.startswith(USED_PREFIXES):
                    res[f"{tag}_w_{k}"] = v.detach().numpy().astype(np.float32)
            for s, v in zip(("src", "tgt", "bgd"), imp):
                res[f"{tag}_imp_{s}"] = v.numpy()
            res[f"{tag}_expl0"], res[f"{tag}_expl1"] = expl[0].numpy(), expl[1].numpy()
            res[f"{tag}_kl"] = np.array([float(x) for x in kl])
            print("enron", tag, "imp mean", [round(float(v.mean()), 6) for v in imp], "kl", [float(x) for x in kl])
    res["null"] = np.array([v for _, v in sorted(ex.null_model.items())])
    # one training iteration on the reference TGN at N=20 (the Enron+TGN training config, a15)
    n_deg, n_ev = ENRON_SETS[0]
    items, edges, ts_cut, _ = _pack_items(res, f"test_N{n_deg}_", n_deg, n_ev, "test_ts")
    base, _, pert = tgn_base("enron", nf, ef, n_deg)
    for k, v in pert.items():
        res[f"train_pert_{k}"] = v
    torch.manual_seed(40)
    CTX.update(seed=0, split=px.SPLIT_NULL)
    ex = TempME(base, base_model_type="tgn", data="uslegis_sampled", out_dim=40, hid_dim=64, temp=0.07,
                if_cat_feature=True, dropout_p=0.1, device=torch.device("cpu"))
    for k, v in ex.state_dict().items():
        if k.startswith(USED_PREFIXES):
            res[f"train_w_{k}"] = v.detach().numpy().astype(np.float32)
    tr = _train_iteration(ex, base, src[:n_ev], dst[:n_ev], eidx[:n_ev], ts_cut, items, edges)
    for k, v in tr.items():
        res[f"train_{k}"] = v
    print("enron train loss", tr["losses"])
    save_npz("enron_goldens.npz", **res)


GM_SEEDS = {"uslegis": 21, "synth": 22}


def case_graphmixer():
    """Base GraphMixer contrast (GraphM/graphmixer.py:106-239) without / with the TempME hop-1
    explanation, with random weights, with explicit edge features, and threshold_test's graphmixer
    branch (temp_exp_main.py:186-206) with every masked contrast captured."""
    from GraphM.graphmixer import GraphMixer
    from sklearn.metrics import average_precision_score, roc_auc_score
    import math
    threshold_test = load_ref_function("temp_exp_main.py", "threshold_test", math=math, np=np, torch=torch,
                                       average_precision_score=average_precision_score,
                                       roc_auc_score=roc_auc_score)
    enc = np.load(os.path.join(HERE, "encoder_uslegis.npz"))
    n_deg, bsz = 20, 32
    pipe, (sg_s, sg_t, sg_b, _, _, _, dst_fake), _, ts_cut, _ = _enc_batch(n_deg, bsz)
    src, dst = pipe["test_src"][:bsz], pipe["test_dst"][:bsz]
    e_l = pipe["test_eidx"][:bsz]
    res = {}
    for name, (nf, ef, _) in _uslegis_feats().items():
        torch.manual_seed(GM_SEEDS[name])
        # learn_base.py:178-180 with its defaults (--n_layer 3, --drop_out 0.5)
        base = GraphMixer(nf, ef, n_neighbors=n_deg, device=torch.device("cpu"), num_tokens=n_deg, num_layers=3,
                          dropout=0.5)
        base.eval()
        for k, v in base.state_dict().items():
            v = v.detach().double()
            res[f"{name}_sd_{k}"] = np.array([v.sum().item(), v.abs().sum().item(), (v * v).sum().item()])
        expl = [torch.from_numpy(enc[f"{name}_expl0"])]
        rng = np.random.default_rng(200 + GM_SEEDS[name])
        ew_rand = rng.uniform(0, 1, tuple(expl[0].shape)).astype(np.float32)
        ew_rand[rng.uniform(0, 1, ew_rand.shape) < 0.2] = 0.0
        res[f"{name}_ew_rand"] = ew_rand
        with torch.no_grad():
            pos_o, neg_o = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b)
            pos_e, neg_e = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b, explain_weights=expl)
            pos_r, neg_r = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b,
                                         explain_weights=[torch.from_numpy(ew_rand)])
            ea = base.retrieve_edge_features(sg_s, sg_t, sg_b).numpy()
            ea = (ea + rng.normal(0, 0.25, ea.shape)).astype(np.float32)
            pos_a, neg_a = base.contrast(src, dst, dst_fake, ts_cut, e_l, sg_s, sg_t, sg_b, explain_weights=expl,
                                         edge_attr=torch.from_numpy(ea))
        res[f"{name}_edge_attr"] = ea
        for tag, (p, n) in (("ori", (pos_o, neg_o)), ("expl", (pos_e, neg_e)), ("rand", (pos_r, neg_r)),
                            ("attr", (pos_a, neg_a))):
            res[f"{name}_{tag}"] = torch.cat([p, n]).numpy()
        y_ori = torch.where(torch.cat([pos_o, neg_o]).sigmoid() > 0.5, 1., 0.).view(-1, 1)
        calls = []
        orig = base.contrast

        def capture(*a, **k):
            out = orig(*a, **k)
            calls.append((np.concatenate([a[5][0][0], a[6][0][0], a[7][0][0]], axis=0) == 0, torch.cat(out).numpy()))
            return out
        base.contrast = capture

        class A:
            pass
        args = A()
        args.ratios, args.base_type, args.n_degree, args.bs = TGN_RATIOS, "graphmixer", n_deg, bsz
        metrics = threshold_test(args, expl, base, src, dst, dst_fake, ts_cut, e_l, pos_o, neg_o, y_ori,
                                 sg_s, sg_t, sg_b)
        base.contrast = orig
        res[f"{name}_thr_metrics"] = np.array([float(m) for m in metrics])
        res[f"{name}_thr_logits"] = np.stack([c[1] for c in calls])
        res[f"{name}_thr_zero_bits"] = np.packbits(np.stack([c[0] for c in calls]))
        print(name, "ori", float(res[f"{name}_ori"].mean()), "expl", float(res[f"{name}_expl"].mean()),
              "thr", res[f"{name}_thr_metrics"])
    res["ratios"] = np.array(TGN_RATIOS)
    save_npz("graphmixer_uslegis.npz", **res)

if __name__ == "__main__":
    which = sys.argv[1:] or ["kats", "small", "uslegis", "null", "encoder", "tgn", "train", "graphmixer", "enron"]
    if "kats" in which:
        case_kats()
    if "small" in which:
        case_synth_small()
    if "uslegis" in which:
        case_uslegis()
    if "null" in which:
        case_null()
    if "encoder" in which:
        case_encoder()
    if "tgn" in which:
        case_tgn()
    if "train" in which:
        case_train()
    if "graphmixer" in which:
        case_graphmixer()
    if "enron" in which:
        case_enron()
