"""FusedAdam (tempme_amd/optim.py, csrc/optim.hip tm_adam_step): torch.optim.Adam's update (temp_exp_main.py:555,
:631-632) as one kernel over the explainer's flat fp32 bucket -- equal to torch.optim.Adam within fp32 rounding over
several steps (with and without weight decay, parameters that get no gradient untouched), replayable from a HIP
graph (the device step count advances per replay), state-dict round trip, and the explainer's training step at
Enron dims with FusedAdam against the reference's Adam update."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _nets(seed=0):
    torch.manual_seed(seed)
    a = torch.nn.Sequential(torch.nn.Linear(13, 37), torch.nn.ReLU(), torch.nn.Linear(37, 5),
                            torch.nn.Linear(3, 3)).cuda()            # the last layer never gets a gradient
    b = torch.nn.Sequential(torch.nn.Linear(13, 37), torch.nn.ReLU(), torch.nn.Linear(37, 5),
                            torch.nn.Linear(3, 3)).cuda()
    b.load_state_dict(a.state_dict())
    return a, b


def _loss(net, k):
    x = torch.randn(64, 13, generator=torch.Generator().manual_seed(100 + k)).cuda()
    return net[2](net[1](net[0](x))).pow(2).mean()


@pytest.mark.parametrize("wd", [0.0, 1e-2])
def test_fused_adam_equals_torch_adam(wd):
    from tempme_amd.optim import FusedAdam
    a, b = _nets()
    oa = torch.optim.Adam(a.parameters(), lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd)
    ob = FusedAdam(b.parameters(), lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd)
    p3 = b[3].weight.detach().clone()
    for k in range(6):
        for net, opt in ((a, oa), (b, ob)):
            opt.zero_grad()
            _loss(net, k).backward()
            opt.step()
        for (na, pa), (nb, pb) in zip(a.named_parameters(), b.named_parameters()):
            torch.testing.assert_close(pb, pa, rtol=1e-5, atol=1e-6, msg=f"step {k} {na}")
    assert float(ob.step_t.item()) == 6.0
    if wd == 0.0:
        assert torch.equal(b[3].weight, p3)          # no gradient reached it: it does not move (torch skips it)
    # the parameters, their gradients and the moments are views of the flat buckets
    assert all(p.grad.data_ptr() >= ob.flat_grad.data_ptr() for p in b.parameters() if p.grad is not None)
    assert b[3].weight.grad is None                  # not reached: torch's None, as torch.optim.Adam leaves it


def test_fused_adam_graph_replay_equals_eager():
    from tempme_amd.optim import FusedAdam
    a, b = _nets(1)
    oa = FusedAdam(a.parameters(), lr=5e-3)
    ob = FusedAdam(b.parameters(), lr=5e-3)
    for k in range(2):                               # eager warm-up on both
        for net, opt in ((a, oa), (b, ob)):
            opt.zero_grad()
            _loss(net, k).backward()
            opt.step()
    x = torch.randn(64, 13, generator=torch.Generator().manual_seed(7)).cuda()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ob.zero_grad()
        b[2](b[1](b[0](x))).pow(2).mean().backward()
        ob.step()
    torch.cuda.current_stream().wait_stream(s)
    oa.zero_grad()
    a[2](a[1](a[0](x))).pow(2).mean().backward()
    oa.step()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        ob.zero_grad()
        b[2](b[1](b[0](x))).pow(2).mean().backward()
        ob.step()
    for _ in range(3):                               # capture did not run the step; 3 replays = 3 eager steps
        gr.replay()
        oa.zero_grad()
        a[2](a[1](a[0](x))).pow(2).mean().backward()
        oa.step()
    torch.cuda.synchronize()
    assert float(ob.step_t.item()) == float(oa.step_t.item()) == 6.0
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)


def test_fused_adam_state_dict_round_trip():
    from tempme_amd.optim import FusedAdam
    a, b = _nets(2)
    oa = torch.optim.Adam(a.parameters(), lr=1e-2)
    for k in range(3):
        oa.zero_grad()
        _loss(a, k).backward()
        oa.step()
    b.load_state_dict(a.state_dict())
    ob = FusedAdam(b.parameters(), lr=1e-2)
    ob.load_state_dict(oa.state_dict())
    assert float(ob.step_t.item()) == 3.0
    for k in range(3, 5):
        for net, opt in ((a, oa), (b, ob)):
            opt.zero_grad()
            _loss(net, k).backward()
            opt.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pb, pa, rtol=1e-5, atol=1e-6)


def test_train_step_with_fused_adam_matches_reference_enron():
    """test_gpu_enron.py's one-iteration reference check (losses, every gradient, the Adam update) with the
    explainer's optimizer = FusedAdam: the update equals the reference's torch.optim.Adam update."""
    import enron_inputs as EI
    from tempme_amd import TempME
    from tempme_amd.optim import FusedAdam
    from tempme_amd.train import Batch, train_step
    dev = torch.device("cuda", 0)
    z = EI.golden()
    g = EI.graph(z)
    N, B = 20, EI.SETS[20]
    base = EI.build_tgn(z, g).to(dev)
    ex = TempME(base, "tgn", "enron", out_dim=40, hid_dim=64, temp=0.07, if_cat_feature=True, dropout_p=0.1,
                device=dev, null_model=EI.null(z))
    _, unexpected = ex.load_state_dict(EI.weights(z, "train"), strict=False)
    assert not unexpected
    ex = ex.to(dev)
    d = EI.walks(z, N)
    pre = f"test_N{N}_"
    sg = [tuple([z[pre + f"subgraph_{s}_{h}_{k}"][:B].astype(np.float64) for h in (0, 1)]
                for k in ("node", "eid", "ts")) for s in EI.SIDES]
    walks = [(d[s]["node"], d[s]["eid"], d[s]["ts"], d[s]["cat"], d[s]["marg"]) for s in EI.SIDES]
    batch = Batch(z["test_src"][:B].astype(np.int64), z["test_dst"][:B].astype(np.int64), d["ts_cut"],
                  z["test_eidx"][:B].astype(np.int64), z[pre + "dst_fake"][:B].astype(np.float64), sg, walks,
                  [d[s]["cnt"] for s in EI.SIDES])
    opt = FusedAdam(ex.parameters(), lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0)
    p0 = {k: v.detach().clone() for k, v in ex.named_parameters()}
    ex.eval()
    out = train_step(ex, base, opt, batch, beta=0.5, prior_p=0.3, if_bern=False)
    got = np.array([out["loss"].item(), out["pred_loss"].item(), out["kl_loss"].item()])
    np.testing.assert_allclose(got, z["train_losses"], rtol=1e-5, atol=1e-6)
    ref_keys = {k[len("train_grad_"):] for k in z.files if k.startswith("train_grad_")}
    for k, v in ex.named_parameters():
        upd = (v.detach() - p0[k]).cpu().numpy()
        if k not in ref_keys:
            # no gradient reaches it in the reference (its .grad stays None there): zero gradient, no update here
            assert v.grad is None or not v.grad.any(), k
            assert not upd.any(), k
            continue
        gr = z[f"train_grad_{k}"].astype(np.float64)
        ga = v.grad.detach().cpu().numpy().astype(np.float64)
        scale = np.abs(gr).max()
        assert np.linalg.norm(ga - gr) <= 2e-4 * np.linalg.norm(gr) + 1e-9, k
        sure = np.abs(gr) > max(1e-3 * scale, 1e-7)
        np.testing.assert_allclose(upd[sure], z[f"train_upd_{k}"][sure], atol=2e-6, rtol=1e-3, err_msg=k)
