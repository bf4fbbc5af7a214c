"""tm_host_register / tm_stage_cast (csrc/stage.hip, tempme_amd/hoststage.py): the reference's host numpy views read
by the GPU in place and converted -- equal to numpy's astype (float64 / int64 -> int32 truncation toward zero,
float64 -> float32 round to nearest) for strided column views of large pack arrays; small or non-owning bases
are refused (the caller's pinned host-cast path serves them); a registration is made once per base."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_stage_cast_equals_numpy_astype():
    from tempme_amd import hoststage as H
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    w = rng.normal(0, 1e3, size=(2000, 60, 14))                     # walks_*_new rows: 6.7 MB float64
    w[:, :, :6] = np.trunc(w[:, :, :6])
    w[0, 0, 0] = -1.75                                               # truncation toward zero
    node = w[:, :, :6].astype(int)                                   # int64 owner (load_subgraph_margin)
    sub = rng.integers(0, 125000, size=(4000, 3 * 420)).astype(np.float64)   # subgraph_*_1: [E, 3 N^2] float64
    edge = rng.integers(0, 4, size=(3, 1000, 60, 3, 3)).astype(np.float64)   # np.load(..._edge.npy)
    rows = slice(100, 200)                                           # away from the arrays' partial first / last pages
    items = [(w[rows, :, 9:12], torch.float32), (w[rows, :, 6:9], torch.int32), (node[rows], torch.int32),
             (sub[rows, 0:400], torch.int32), (sub[rows, 400:800], torch.int32), (edge[1][rows], torch.float32),
             (w[rows, :, 13:14], torch.float32), (w[rows, :, 0], torch.int32)]
    st = torch.cuda.Stream()
    got = H.stage(dev, items, st)
    assert got is not None
    torch.cuda.synchronize()
    for (a, dt), x in zip(items, got):
        want = torch.from_numpy(np.ascontiguousarray(a.astype(np.int32 if dt == torch.int32 else np.float32)))
        assert x.dtype == dt and tuple(x.shape) == a.shape and x.is_contiguous()
        assert torch.equal(x.cpu(), want)
    # the bases are registered once: a second call reuses them
    n = len(H._REG.regs)
    again = H.stage(dev, items[:3], st)
    torch.cuda.synchronize()
    assert len(H._REG.regs) == n and torch.equal(again[0], got[0])


def test_window_bounds_and_staging_bound():
    """window_bounds = min / max of the view's columns over every row of its owning array (cached per layout);
    a staging bound clamps int32 ids into [0, bound) and leaves in-range ids unchanged."""
    from tempme_amd import hoststage as H
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(1)
    w = rng.integers(0, 5000, size=(3000, 60, 14)).astype(np.float64)      # 20 MB: registered
    w[2500, 7, 7] = 7777.0
    v = w[100:200, :, 6:9]
    assert H.window_bounds(v) == (w[:, :, 6:9].min(), w[:, :, 6:9].max())
    assert H.window_bounds(w[300:400, :, 6:9]) == H.window_bounds(v)           # same layout: cached
    assert H.window_bounds(w[100:200, :, 0:6]) == (w[:, :, 0:6].min(), w[:, :, 0:6].max())
    v[0, 0, 0] = 6000.0                                                          # out of a 5,000-row table
    v[0, 0, 1] = -3.0
    st = torch.cuda.Stream()
    got = H.stage(dev, [(v, torch.int32, 5000), (v, torch.int32)], st)
    torch.cuda.synchronize()
    want = np.ascontiguousarray(v.astype(np.int32))
    assert torch.equal(got[1].cpu(), torch.from_numpy(want))
    want[0, 0, 0], want[0, 0, 1] = 4999, 0
    assert torch.equal(got[0].cpu(), torch.from_numpy(want))


def test_stage_cpp_host_side_equals_python():
    """hoststage.stage on the current stream (the C++ per-view work of dropin_ext.stage_host) = the Python job
    builder on an explicit stream, bitwise, bounds included."""
    from tempme_amd import hoststage as H
    from tempme_amd.explainer import _dropin_ext
    if _dropin_ext() is None:
        pytest.skip("drop-in extension not built")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(2)
    w = rng.integers(-3, 9000, size=(2500, 60, 14)).astype(np.float64)
    e = rng.integers(0, 4, size=(3, 2500, 60, 3, 3)).astype(np.float64)
    node = w[:, :, :6].astype(np.int64)
    rows = slice(200, 300)
    items = [(node[rows], torch.int32, 5000), (w[rows, :, 6:9], torch.int32, 8000), (w[rows, :, 9:12], torch.float32),
             (w[rows, :, 12], torch.int32), (e[2][rows], torch.float32)]
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        a = H.stage(dev, items)
    b = H._stage_py(dev, items, st)
    torch.cuda.synchronize()
    assert a is not None and b is not None
    for x, y in zip(a, b):
        assert x.dtype == y.dtype and x.shape == y.shape and torch.equal(x, y)


def test_stage_refuses_what_it_cannot_read_in_place():
    from tempme_amd import hoststage as H
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    small = np.arange(1000, dtype=np.float64)                       # below MIN_BYTES (1 MB): the pinned host-cast path
    assert H.stage(dev, [(small[10:20], torch.float32)], st) is None
    big = np.zeros((1 << 20,), dtype=np.float64)
    assert H.stage(dev, [(big.astype(np.float16)[:10], torch.float32)], st) is None    # unsupported dtype
    assert H.stage(dev, [(big[:10], torch.float32), (small[:10], torch.float32)], st) is None   # one refusal: all


def test_host_pack_dropin_reads_pack_in_place(tmp_path):
    """The drop-in forward on host-pack views of large bases (the bench's host_pack leg shape) stages through
    tm_stage_cast (registered bases) and equals the same call on device tensors."""
    import tempme_amd as tm
    from tempme_amd import hoststage as H
    from tempme_amd import pack as P
    from tempme_amd.pipeline import ExplainPipeline
    from tempme_amd.workload import enron_like, split
    dev = torch.device("cuda", 0)
    g = enron_like(n_nodes=184, n_edges=60000, alpha=1.2, seed=4)
    (src, dst, ts, eidx), rows, pool = split(g)
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=4, split=tm.SPLIT_TEST)

    class Base:
        n_feat_th = torch.from_numpy(g["n_feat"])
        e_feat_th = torch.from_numpy(g["e_feat"])
        node_raw_features = torch.nn.Embedding.from_pretrained(n_feat_th, padding_idx=0, freeze=True)
        edge_raw_features = torch.nn.Embedding.from_pretrained(e_feat_th, padding_idx=0, freeze=True)

    torch.manual_seed(0)
    ex = tm.TempME(Base(), "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
                   null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).eval()
    N, B, E = 20, 100, 4000
    pipe = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), N, 3, B, seed=4)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:E], dtype=dt)).to(dev)  # noqa: E731
    imp, h1, h2 = [x.clone() for x in pipe.run(t(src, np.int32), t(dst, np.int32), t(ts, np.float64),
                                                t(eidx, np.int32), torch.arange(E, dtype=torch.int32, device=dev))]
    _, cat_d, edge = P.buffers_to_arrays(pipe.buf, E)

    class A:
        n_degree = N
    pk = P.load_subgraph_margin(A(), cat_d)
    cut = ts[:E].astype(np.float64)
    H._REG.clear()
    for b in (0, 13, 39):
        idx = np.arange(b * B, (b + 1) * B)
        sg_s, sg_t, sg_b, w_s, w_t, w_b, _ = P.get_item(pk, idx)
        e_s, e_t, e_b = P.get_item_edge(edge, idx)
        with torch.no_grad():
            i_s, i_t, i_b = ex(w_s, cut[idx], e_s), ex(w_t, cut[idx], e_t), ex(w_b, cut[idx], e_b)
            expl = ex.retrieve_explanation(sg_s, i_s, w_s, sg_t, i_t, w_t, sg_b, i_b, w_b, training=False)
        sl = slice(b * B, (b + 1) * B)
        for k, x in enumerate((i_s, i_t, i_b)):
            assert torch.equal(x[..., 0], imp[k][sl]), (b, k)
        assert torch.equal(expl[0], h1[:, sl].reshape(3 * B, N))
        assert torch.equal(expl[1], h2[:, sl].reshape(3 * B, N * N))
    # the walk / subgraph / edge bases went through the in-place path (at least the large ones)
    assert sum(1 for e in H._REG.regs.values() if e[3] is not None) >= 3
    # an edge id outside the edge table raises what the reference's embedding lookup raises (a small copy: the
    # per-call check of the pinned host-cast path)
    idx = np.arange(0, B)
    _, _, _, w_s, _, _, _ = P.get_item(pk, idx)
    e_s = P.get_item_edge(edge, idx)[0]
    bad = [np.array(x, copy=True) if isinstance(x, np.ndarray) else x for x in w_s]
    bad[1][0, 0, 0] = float(g["e_feat"].shape[0] + 5)
    with pytest.raises(IndexError):
        with torch.no_grad():
            ex(bad, cut[idx], e_s)
