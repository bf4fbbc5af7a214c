"""GPU checks of alternative forms of the training and GraphMixer paths, each against the oracle or the default
form (written in round 4, validated on the MI355X in round 5; the register-resident event_gcn training kernels,
now the default for hid_dim 64, are covered by tests/test_gpu_encoder_train.py):

* the padding mask from tm_explain_train_fwd_pad (the default): bitwise the torch mask;
* GraphedTrainStep(overlap_prepare=True): the graph with the base model's original contrast as a second branch =
  eager (the default, without the branch, is tests/test_gpu_train.py::test_graphed_step_equals_eager)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    return torch.device("cuda", 0)


def test_explain_pad_kernel_equals_torch_mask(dev, monkeypatch):
    from tempme_amd import TempME
    from tempme_amd import explainer as X
    from tests.test_gpu_explain_train import _Base
    rng = np.random.RandomState(5)
    G, B, N, de = 3, 9, 20, 32
    W, V, E = 3 * N, 50, 400
    n_feat = rng.uniform(0, 1, (V + 1, 172)).astype(np.float32)
    e_feat = rng.uniform(0, 1, (E + 1, de)).astype(np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    eid3 = t(rng.randint(0, E + 1, (G, B, W, 3)).astype(np.int32))
    ts3 = t(rng.uniform(0, 1e6, (G, B, W, 3)).astype(np.float32))
    s1e, s2e = t(rng.randint(0, E + 1, (G, B, N)).astype(np.int32)), t(rng.randint(0, E + 1, (G, B, N * N)).astype(np.int32))
    s1n, s2n = t(rng.randint(0, 3, (G, B, N)).astype(np.int32)), t(rng.randint(0, 3, (G, B, N * N)).astype(np.int32))
    imp_np = rng.uniform(0.05, 0.95, (G, B, W)).astype(np.float32)
    torch.manual_seed(9)
    ex = TempME(_Base(n_feat, e_feat), "tgn", "synth", 40, 64, device=dev,
                null_model={k: 1 / 12 for k in range(1, 13)}).to(dev).eval()
    ex.beta_sample = lambda prob, training: prob
    outs = []
    for on in (False, True):
        monkeypatch.setattr(X, "_EXPLAIN_PAD", on)
        imp = t(imp_np).requires_grad_(True)
        e1, e2 = ex.explain_groups(imp, eid3, ts3, s1n, s1e, s2n, s2e, G, B, W, N, True)
        (e1.sum() + 2 * e2.sum()).backward()
        outs.append((e1.detach().clone(), e2.detach().clone(), imp.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_graphed_step_with_prepare_branch_equals_eager(dev, monkeypatch):
    from tempme_amd import train as T
    from tests import test_gpu_train as TT
    orig = T.GraphedTrainStep.__init__

    def init(self, *a, **kw):
        kw.setdefault("overlap_prepare", True)
        orig(self, *a, **kw)
    monkeypatch.setattr(T.GraphedTrainStep, "__init__", init)
    TT.test_graphed_step_equals_eager(dev)
