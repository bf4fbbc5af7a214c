"""GPU parity of the explainer training step (temp_exp_main.py:584-632) against one
deterministic iteration of the reference (tests/golden/train_uslegis.npz, make_goldens.py case_train:
reference TempME on the reference TGN, Explainer.eval(), if_bern=False, Adam lr 1e-3): losses,
logits, every gradient that reaches the explainer (115,554 values at uslegis dims) and the Adam
update.  The stochastic configuration (dropout, Beta rsample) is checked for shape and finiteness."""
import os

import numpy as np
import pytest
import torch

import tgn_inputs as TI
from tests.encoder_inputs import SIDES, load as load_enc

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EX_SEEDS = {"uslegis": 0, "synth": 1}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    return torch.device("cuda", 0)


def _setup(case, dev):
    from tempme_amd import TempME
    from tempme_amd.train import Batch
    base = TI.build_model(case).to(dev)
    enc = load_enc(case)
    torch.manual_seed(EX_SEEDS[case])
    ex = TempME(base, "tgn", "uslegis_sampled", out_dim=40, hid_dim=64, temp=0.07, if_cat_feature=True,
                dropout_p=0.1, device=dev, null_model={k + 1: float(v) for k, v in enumerate(enc["null"])})
    missing, unexpected = ex.load_state_dict(enc["sd"], strict=False)
    assert not unexpected
    ex = ex.to(dev)
    d = TI.load_batch()
    walks = [(enc[s]["node"], enc[s]["eid"], enc[s]["ts"], enc[s]["cat"], enc[s]["marg"]) for s in SIDES]
    batch = Batch(d["src"], d["dst"], d["ts_cut"], d["e_idx"], d["fake"], [d["sg_" + s] for s in SIDES], walks,
                  [enc[s]["cnt"] for s in SIDES])
    opt = torch.optim.Adam(ex.parameters(), lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0)
    return base, ex, batch, opt


@pytest.mark.parametrize("case", ["uslegis", "synth"])
def test_train_step_matches_reference(dev, case):
    from tempme_amd.train import train_step
    g = np.load(os.path.join(G, "train_uslegis.npz"))
    base, ex, batch, opt = _setup(case, dev)
    p0 = {k: v.detach().clone() for k, v in ex.named_parameters()}
    ex.eval()
    out = train_step(ex, base, opt, batch, beta=0.5, prior_p=0.3, if_bern=False)
    got = np.array([out["loss"].item(), out["pred_loss"].item(), out["kl_loss"].item()])
    np.testing.assert_allclose(got, g[f"{case}_losses"], rtol=1e-5, atol=1e-6)
    logits = torch.cat([out["pos_logit"], out["neg_logit"]]).cpu().numpy()
    np.testing.assert_allclose(logits, g[f"{case}_logits"], atol=2e-5, rtol=1e-5)
    ref_keys = {k[len(case) + 6:] for k in g.files if k.startswith(f"{case}_grad_")}
    got_keys = {k for k, v in ex.named_parameters() if v.grad is not None}
    assert got_keys == ref_keys
    for k, v in ex.named_parameters():
        if k not in ref_keys:
            continue
        gr = g[f"{case}_grad_{k}"].astype(np.float64)
        ga = v.grad.detach().cpu().numpy().astype(np.float64)
        scale = np.abs(gr).max()
        assert np.linalg.norm(ga - gr) <= 2e-4 * np.linalg.norm(gr) + 1e-9, k
        assert np.abs(ga - gr).max() <= 1e-8 + 2e-4 * scale, k
        if f"{case}_upd_{k}" in g.files:
            upd = (v.detach() - p0[k]).cpu().numpy()
            ref = g[f"{case}_upd_{k}"]
            sure = np.abs(gr) > max(1e-3 * scale, 1e-7)      # Adam's first step is ~lr*sign(g)
            np.testing.assert_allclose(upd[sure], ref[sure], atol=2e-6, rtol=1e-3, err_msg=k)


@pytest.mark.parametrize("W", [60, 90])
def test_kl_loss_groups_matches_per_side(dev, W):
    """tm_kl_loss (three per-side kl_loss calls as one launch) = the torch formulation of kl_loss
    (explainer_new.py:432-448) summed over the sides: value and d/d prob within 1e-5, including
    probabilities clamped at 1e-6 / 1-1e-6 (zero gradient there), empty categories and W > 64."""
    from tempme_amd import TempME
    base = TI.build_model("uslegis").to(dev)
    torch.manual_seed(0)
    ex = TempME(base, "tgn", "uslegis_sampled", out_dim=40, hid_dim=64, device=dev,
                null_model={k: (k + 1.0) / 90 for k in range(1, 13)}).to(dev)
    gen = torch.Generator().manual_seed(W)
    G, B = 3, 37
    prob = torch.rand(G, B, W, generator=gen, dtype=torch.float64).float()
    prob[0, 0, :5] = 1.0            # sigmoid saturated: clamped
    prob[1, 2, :3] = 0.0
    cat = torch.randint(0, 9, (G, B, W), generator=gen, dtype=torch.int32)   # categories 9..11 empty
    p1 = prob.clone().to(dev).requires_grad_(True)
    p2 = prob.clone().to(dev).requires_grad_(True)
    a = ex.kl_loss_groups(p1, cat.to(dev), target=0.3)
    b = sum(ex._kl_loss_torch(p2[g].unsqueeze(-1), (None, None, None, cat[g].to(dev), None), target=0.3)
            for g in range(G))
    a.backward()
    b.backward()
    np.testing.assert_allclose(a.item(), b.item(), rtol=1e-5)
    np.testing.assert_allclose(p1.grad.cpu().numpy(), p2.grad.cpu().numpy(), rtol=1e-4, atol=1e-9)


def test_dropin_kl_loss_on_hip_matches_torch(dev):
    """TempME.kl_loss (the drop-in call, explainer_new.py:432-453) on a device tensor runs tm_kl_loss: value
    and gradient equal the torch formulation within 1e-5, for [B, W, 1] importances with host or device
    category arrays."""
    from tempme_amd import TempME
    base = TI.build_model("uslegis").to(dev)
    ex = TempME(base, "tgn", "uslegis_sampled", out_dim=40, hid_dim=64, device=dev,
                null_model={k: (k + 1.0) / 90 for k in range(1, 13)}).to(dev)
    gen = torch.Generator().manual_seed(3)
    B, W = 25, 60
    prob = torch.rand(B, W, 1, generator=gen)
    prob[0, :4] = 1.0
    cat = torch.randint(0, 12, (B, W, 1), generator=gen, dtype=torch.int32)
    for c in (cat.numpy().astype(np.float64), cat.to(dev)):
        p1 = prob.clone().to(dev).requires_grad_(True)
        p2 = prob.clone().to(dev).requires_grad_(True)
        a = ex.kl_loss(p1, (None, None, None, c, None), target=0.3)
        b = ex._kl_loss_torch(p2, (None, None, None, c, None), target=0.3)
        assert a.grad_fn is not None and "KLFn" in type(a.grad_fn).__name__, "the HIP kernel did not run"
        a.backward()
        b.backward()
        np.testing.assert_allclose(a.item(), b.item(), rtol=1e-5)
        np.testing.assert_allclose(p1.grad.cpu().numpy(), p2.grad.cpu().numpy(), rtol=1e-4, atol=1e-9)


def test_batch_from_pack_gather_equals_index_select(dev):
    """batch_from_pack's one-launch row gather (tm_gather_rows) = torch.index_select of every pack array."""
    import tempme_amd as tm
    from tempme_amd.preprocess import sample_events
    from tempme_amd.train import batch_from_pack
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=60, n_edges=2000, seed=8)
    (src, dst, ts, eidx), rows, pool = split(g, mode="train")
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=1, split=tm.SPLIT_TRAIN)
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    s_d, d_d, t_d, e_d = to(src, np.int32), to(dst, np.int32), to(ts, np.float64), to(eidx, np.int32)
    buf = sample_events(f.graph, 1, tm.SPLIT_TRAIN, 8, 3, s_d, d_d, t_d, e_d,
                        torch.arange(len(src), dtype=torch.int32, device=dev), to(pool, np.int32))
    r = torch.randperm(len(src) - 1, generator=torch.Generator().manual_seed(0))[:37].to(dev)
    b = batch_from_pack(buf, s_d, d_d, t_d, e_d, r)
    sel = lambda x, dim: x.index_select(dim, r)  # noqa: E731
    for got, want in zip(b.stacked, (sel(buf.node6, 1), sel(buf.eid3, 1), sel(buf.ts3, 1), sel(buf.cat, 1),
                                     sel(buf.cnt, 1))):
        assert torch.equal(got, want)
    for s in range(3):
        assert torch.equal(b.subgraphs[s][0][1], sel(buf.sub2_node, 1)[s])
        assert torch.equal(b.subgraphs[s][2][0], sel(buf.sub1_ts, 1)[s])
    for got, x in ((b.src, s_d), (b.dst, d_d), (b.ts, t_d), (b.e_idx, e_d), (b.fake, buf.dst_fake)):
        assert torch.equal(got, sel(x, 0))
    # a row outside the pack is not read; it flags the pack's error word (index_select would raise)
    assert int(buf.err.item()) == 0
    batch_from_pack(buf, s_d, d_d, t_d, e_d, torch.tensor([0, len(src) + 5], dtype=torch.int64, device=dev))
    from tempme_amd import _lib as L
    assert int(buf.err.item()) == L.TM_E_ARG


def test_stochastic_train_step_runs(dev):
    from tempme_amd.train import train_step
    base, ex, batch, opt = _setup("uslegis", dev)
    ex.train()
    before = {k: v.detach().clone() for k, v in ex.named_parameters()}
    out = train_step(ex, base, opt, batch, if_bern=True)
    assert torch.isfinite(out["loss"]).item()
    n_grad = sum(v.grad.numel() for v in ex.parameters() if v.grad is not None)
    assert n_grad == 115554
    changed = sum(int((v.detach() != before[k]).any()) for k, v in ex.named_parameters())
    assert changed > 0
    assert all(p.grad is None for p in base.parameters())


def test_graphed_step_equals_eager(dev):
    """GraphedTrainStep (the step captured as a HIP graph, replayed per batch) = eager train_step on the
    same batches from the same initial state (deterministic configuration: Explainer.eval(), Beta mean)."""
    import tempme_amd as tm
    from tempme_amd.preprocess import sample_events
    from tempme_amd.tgn import TGN
    from tempme_amd.train import GraphedTrainStep, batch_from_pack, train_step
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=80, n_edges=3000, seed=4)
    (src, dst, ts, eidx), rows, pool = split(g, mode="train")
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=2, split=tm.SPLIT_TRAIN)
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    s_d, d_d, t_d, e_d = to(src, np.int32), to(dst, np.int32), to(ts, np.float64), to(eidx, np.int32)
    buf = sample_events(f.graph, 2, tm.SPLIT_TRAIN, 10, 3, s_d, d_d, t_d, e_d,
                        torch.arange(len(src), dtype=torch.int32, device=dev), to(pool, np.int32))
    torch.manual_seed(3)
    base = TGN(g["n_feat"], g["e_feat"], n_neighbors=10, device=dev, n_layers=2, n_heads=2, dropout=0.1)
    base.forbidden_memory_update = True
    base = base.to(dev).eval()
    runs = []
    B = 40
    W = 30
    node6, eid3, ts3 = (buf.node6[0, :B].cpu().numpy(), buf.eid3[0, :B].cpu().numpy(), buf.ts3[0, :B].cpu().numpy())
    cat, cnt = buf.cat[0, :B].cpu().numpy(), buf.cnt[0, :B].cpu().numpy()
    cut = ts[:B].astype(np.float64)
    batches = [torch.arange(k * B, (k + 1) * B, device=dev) for k in range(4)]
    for graphed in (False, True):
        torch.manual_seed(5)
        ex = tm.TempME(base, "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
                       null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).eval()
        opt = torch.optim.Adam(ex.parameters(), lr=1e-3, capturable=graphed)
        losses = []
        if graphed:
            step = GraphedTrainStep(ex, base, opt, buf, s_d, d_d, t_d, e_d, batches[:1], if_bern=False)
            # the capture recorded the repack without running it: an eager call before the first replay repacks
            assert ex._packed_key is None
            for r in batches[1:]:
                losses.append(float(step(r)["loss"]))
        else:
            for r in batches:
                out = train_step(ex, base, opt, batch_from_pack(buf, s_d, d_d, t_d, e_d, r), if_bern=False)
                losses.append(float(out["loss"]))
            losses = losses[1:]
        runs.append((losses, {k: v.detach().clone() for k, v in ex.named_parameters()}))
    # step 1 after the shared warm-up step is the same computation; later steps drift apart only through
    # torch's atomic scatter/gather backward (nondeterministic summation order), which Adam's early
    # ~lr*sign(g) updates amplify for near-zero gradients -- a few lr units at most
    np.testing.assert_allclose(runs[1][0][0], runs[0][0][0], rtol=2e-5)
    np.testing.assert_allclose(runs[1][0], runs[0][0], rtol=2e-3)
    for k, v in runs[0][1].items():
        assert float((runs[1][1][k] - v).abs().max()) <= 5e-3, k
    # the replayed steps kept the encoder packs current: repacking from the parameters changes nothing
    w = tuple(torch.from_numpy(x).to(dev) for x in (node6, eid3, ts3, cat, cut, cnt))
    with torch.no_grad():
        a = ex.encoder_fwd(*w, 1, B, W).clone()
        ex.packed_weights(force=True)
        b = ex.encoder_fwd(*w, 1, B, W)
    assert torch.equal(a, b)


def test_run_steps_overlap_equals_serial(dev, monkeypatch):
    """train.run_steps (batch k+1's prepare_step issued while batch k's gradient all-reduce is in flight,
    i.e. before batch k's optimizer step) takes the same steps as the serial train_step loop
    (deterministic configuration, temp_exp_main.py:584-632).

    Well-posed form: every prepare_step output (the frozen base model's original predictions and y_ori)
    must be bitwise the serial loop's, and every overlapped step is taken from the serial run's parameters
    and Adam state (loaded right before the optimizer step), so each step's gradients are compared from
    identical parameters.  Comparing free-running trajectories instead is ill-posed: Adam's first steps move
    every parameter by ~lr * sign(g), near-zero gradients flip sign under torch's nondeterministic atomic
    summation, and the time encoder's basis_freq entries scale with dt ~ 1e8 (explainer_new.py:49-58), so a
    1e-3 change of one frequency rotates its cosine feature by ~1e5 rad and the trajectories decorrelate
    within two steps (tools/overlap_diag.py shows serial-vs-serial drifting as far)."""
    import tempme_amd as tm
    import tempme_amd.train as T
    from tempme_amd.preprocess import sample_events
    from tempme_amd.tgn import TGN
    from tempme_amd.workload import enron_like, split
    g = enron_like(n_nodes=80, n_edges=3000, seed=4)
    (src, dst, ts, eidx), rows, pool = split(g, mode="train")
    f = tm.NeighborFinder.from_edges(g["src"][rows], g["dst"][rows], g["eidx"][rows], g["ts"][rows], g["n_nodes"],
                                     device=dev, seed=2, split=tm.SPLIT_TRAIN)
    to = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    s_d, d_d, t_d, e_d = to(src, np.int32), to(dst, np.int32), to(ts, np.float64), to(eidx, np.int32)
    buf = sample_events(f.graph, 2, tm.SPLIT_TRAIN, 10, 3, s_d, d_d, t_d, e_d,
                        torch.arange(len(src), dtype=torch.int32, device=dev), to(pool, np.int32))
    torch.manual_seed(3)
    base = TGN(g["n_feat"], g["e_feat"], n_neighbors=10, device=dev, n_layers=2, n_heads=2, dropout=0.1)
    base.forbidden_memory_update = True
    base = base.to(dev).eval()
    B, K = 40, 4
    orig_prep = T.prepare_step

    def clone_state(opt):
        return {id(p): {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in st.items()}
                for p, st in opt.state.items()}

    class Rec:
        """grad_sync stand-in: at start() (after backward) records the step's gradients, parameters and Adam
        state; with ``serial`` given, finish() (after the next batch's prepare_step, right before the
        optimizer step) loads the serial run's parameters, gradients and Adam state of this step."""
        def __init__(self, ex, opt, serial=None):
            self.ex, self.opt, self.serial, self.steps = ex, opt, serial, []

        def start(self):
            ps = list(self.ex.parameters())
            self.steps.append(dict(grads=[p.grad.detach().clone() if p.grad is not None else None for p in ps],
                                   params=[p.detach().clone() for p in ps],
                                   state=[clone_state(self.opt).get(id(p)) for p in ps]))

        def finish(self):
            if self.serial is None:
                return
            ref = self.serial[len(self.steps) - 1]
            with torch.no_grad():
                for p, w, gr, st in zip(self.ex.parameters(), ref["params"], ref["grads"], ref["state"]):
                    p.copy_(w)
                    if gr is not None:
                        p.grad.copy_(gr)
                    if st is not None:
                        for k, v in st.items():
                            if torch.is_tensor(v):
                                self.opt.state[p][k].copy_(v)

    runs = []
    for overlap in (False, True):
        preps = []

        def rec_prep(bm, b):
            out = orig_prep(bm, b)
            preps.append(tuple(x.clone() for x in out[1:]))      # pos_out_ori, neg_out_ori, y_ori
            return out
        monkeypatch.setattr(T, "prepare_step", rec_prep)
        torch.manual_seed(5)
        ex = tm.TempME(base, "tgn", "enron", out_dim=40, hid_dim=64, device=dev,
                       null_model={k: 1.0 / 12 for k in range(1, 13)}).to(dev).eval()
        opt = torch.optim.Adam(ex.parameters(), lr=1e-3)
        rec = Rec(ex, opt, runs[0]["steps"] if overlap else None)
        batches = [T.batch_from_pack(buf, s_d, d_d, t_d, e_d, torch.arange(k * B, (k + 1) * B, device=dev))
                   for k in range(K)]
        if overlap:
            outs = T.run_steps(ex, base, opt, batches, overlap=True, if_bern=False, grad_sync=rec)
        else:
            outs = [T.train_step(ex, base, opt, b, if_bern=False, grad_sync=rec) for b in batches]
        torch.cuda.synchronize()
        runs.append(dict(losses=[float(o["loss"]) for o in outs], steps=rec.steps, preps=preps))
        monkeypatch.setattr(T, "prepare_step", orig_prep)
    ser, ovl = runs
    assert len(ser["preps"]) == len(ovl["preps"]) == K and len(ser["steps"]) == len(ovl["steps"]) == K
    for k in range(K):
        # the prepared inputs (issued before the previous batch's optimizer step) are the serial loop's
        for a, b in zip(ser["preps"][k], ovl["preps"][k]):
            assert torch.equal(a, b), k
        # every step ran from the serial run's parameters (loaded before the previous optimizer step)
        for a, b in zip(ser["steps"][k]["params"], ovl["steps"][k]["params"]):
            assert torch.equal(a, b), k
        np.testing.assert_allclose(ovl["losses"][k], ser["losses"][k], rtol=1e-5, err_msg=str(k))
        ga = torch.cat([x.reshape(-1) for x in ser["steps"][k]["grads"] if x is not None])
        gb = torch.cat([x.reshape(-1) for x in ovl["steps"][k]["grads"] if x is not None])
        assert float((ga - gb).norm()) <= 1e-5 * float(ga.norm()) + 1e-9, (k, float((ga - gb).norm()), float(ga.norm()))


@pytest.mark.parametrize("if_bern", [False, True])
def test_train_step_through_graphmixer_hip_equals_torch(dev, if_bern):
    """The explainer's training step with a GraphMixer base (temp_exp_main.py:605-632, base_type
    'graphmixer'): the explanation weights' gradient through tm_gm_embed_bwd gives the same losses and
    explainer gradients as the torch formulation of the frozen base under autograd (TEMPME_GM_TORCH=1),
    deterministic (Beta mean) and with rsample (same RNG state both times)."""
    from tests.test_graphmixer_oracle import build
    from tempme_amd.train import train_step
    _, ex, batch, opt = _setup("uslegis", dev)
    gm = build("uslegis").to(dev)
    p0 = {k: v.detach().clone() for k, v in ex.named_parameters()}
    res = {}
    for mode in ("hip", "torch"):
        with torch.no_grad():
            for k, v in ex.named_parameters():
                v.copy_(p0[k])
        opt.zero_grad(set_to_none=True)
        ex.eval()
        os.environ["TEMPME_GM_TORCH"] = "1" if mode == "torch" else "0"
        try:
            torch.manual_seed(123)
            out = train_step(ex, gm, opt, batch, beta=0.5, prior_p=0.3, if_bern=if_bern)
        finally:
            os.environ.pop("TEMPME_GM_TORCH", None)
        res[mode] = (out["loss"].item(), {k: v.grad.detach().clone() for k, v in ex.named_parameters()
                                          if v.grad is not None})
        if mode == "hip":
            assert getattr(gm, "_gmb_key", None) is not None, "the HIP explanation-weight backward did not run"
    (lh, gh), (lt, gt) = res["hip"], res["torch"]
    np.testing.assert_allclose(lh, lt, rtol=1e-5, atol=1e-6)
    assert gh.keys() == gt.keys() and len(gh) > 0
    for k in gh:
        d, n = float((gh[k] - gt[k]).norm()), float(gt[k].norm())
        assert d <= 1e-4 * n + 1e-9, (k, d, n)


def test_side_stream_prepare_equals_inline(dev):
    """train_step(side_stream=...) -- the base model's original-prediction contrast on a second stream,
    concurrent with the explainer's encoder and explanation, joined before the explained contrast -- takes
    the same step as the inline order: losses, y_ori and every explainer gradient (deterministic config)."""
    from tempme_amd.train import train_step
    res = []
    for side in (None, torch.cuda.Stream(device=dev)):
        base, ex, batch, opt = _setup("uslegis", dev)
        ex.eval()
        out = train_step(ex, base, opt, batch, beta=0.5, prior_p=0.3, if_bern=False, side_stream=side)
        torch.cuda.synchronize()
        res.append((out["loss"].item(), out["y_ori"].clone(),
                    {k: v.grad.detach().clone() for k, v in ex.named_parameters() if v.grad is not None}))
    (l0, y0, g0), (l1, y1, g1) = res
    np.testing.assert_allclose(l1, l0, rtol=1e-6)
    assert torch.equal(y0, y1)
    assert g0.keys() == g1.keys() and len(g0) > 0
    for k in g0:
        assert float((g0[k] - g1[k]).norm()) <= 1e-5 * float(g0[k].norm()) + 1e-9, k
