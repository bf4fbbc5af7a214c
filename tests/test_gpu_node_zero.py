"""The walk kernel's zero-node-feature form (tm_weights_set_node_zero): with every node-feature bit zero,
event_gcn's two branches src + relu(tgt + event) and tgt + relu(src + event) (explainer_new.py:93-96) are the
same expression, so the kernel computes one, and the layers that read both branches (H = [U; U]) run as their
column-folded forms on U (pack-time fp64 sums, FoldLay KVZ / A1DZ / A1GZ: a re-association of the same sums).
Its outputs must equal the two-branch kernel's within the 1e-5 contract, the flag must follow the table (a
non-zero row turns it off), and tests/test_gpu_enron.py holds this form to the reference's own outputs (its
graphs have zero node features)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(node_feat, zero_spec):
    import tempme_amd as tm
    from tempme_amd.pipeline import ExplainPipeline
    from tempme_amd.workload import enron_like, split
    dev = torch.device("cuda", 0)
    g = enron_like(n_nodes=120, n_edges=6000, seed=11, node_feat=node_feat)
    (src, dst, ts, eidx), rows, pool = split(g)
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=3)

    class Base:
        n_feat_th = torch.from_numpy(g["n_feat"])
        e_feat_th = torch.from_numpy(g["e_feat"])
        node_raw_features = torch.nn.Embedding.from_pretrained(n_feat_th, padding_idx=0, freeze=True)
        edge_raw_features = torch.nn.Embedding.from_pretrained(e_feat_th, padding_idx=0, freeze=True)

    torch.manual_seed(0)
    ex = tm.TempME(Base(), "tgn", "enron", 40, 64, device=dev, null_model={k: 1 / 12 for k in range(1, 13)}).to(dev)
    ex = ex.eval()
    ex.node_zero_specialization = zero_spec
    B = 100
    pipe = ExplainPipeline(ex, f.graph, torch.from_numpy(pool), 20, 3, B, seed=3)
    n = (len(src) // B) * B
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[:n], dtype=dt)).to(dev)  # noqa: E731
    with torch.no_grad():
        imp, h1, h2 = pipe.run(t(src, np.int32), t(dst, np.int32), t(ts, np.float64), t(eidx, np.int32),
                               torch.arange(n, dtype=torch.int32, device=dev))
    torch.cuda.synchronize()
    pipe.check_errors()
    assert pipe.etab is not None, "the pipeline's table mode (where the zero-node form runs) is off"
    return ex, [x.clone() for x in (imp, h1, h2)]


def test_zero_node_form_equals_two_branch_form():
    ex, a = _run("zeros", True)
    assert ex._node_zero
    _, b = _run("zeros", False)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x.cpu().numpy(), y.cpu().numpy(), rtol=1e-5, atol=1e-6)
    assert not torch.equal(a[0], torch.zeros_like(a[0]))


def test_flag_follows_the_node_table():
    ex, _ = _run("uniform", True)
    assert not ex._node_zero              # non-zero rows: the two-branch kernel
    w = ex.node_raw_embed.weight
    with torch.no_grad():
        w.zero_()                          # in place: the tables' key holds the version counter
    ex.feature_tables()
    assert ex._node_zero
