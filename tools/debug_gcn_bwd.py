"""Diagnostic: tm_encoder_bwd's d lin_event rows (dlev) against the same quantity rebuilt in torch from the
kernel's own dZ (dlev = (dZ_s M0) [xt + L > 0] + (dZ_t M0) [xs + L > 0]) for one hid_dim; prints where
they differ."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")


def main(h):
    from tempme_amd import TempME
    from tempme_amd import _lib as L
    from test_gpu_encoder_train import _Base, _inputs
    dev = torch.device("cuda", 0)
    de, G, B, N = 32, 2, 9, 10
    n_feat, e_feat, node6, eid3, ts3, cat, cut, cnt = _inputs(de, G, B, N, seed=11 + h)
    W = 3 * N
    torch.manual_seed(5)
    ex = TempME(_Base(n_feat, e_feat), "tgn", "synth", 40, h, device=dev,
                null_model={k: 1 / 12 for k in range(1, 13)}).to(dev).eval()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    args = (t(node6), t(eid3), t(ts3), t(cat), t(cut).double(), t(cnt), G, B, W)
    out, ws = ex._train_fwd(args, None, 1.0)
    n = G * B * W
    R = 3 * n
    dn = ex.node_dim
    kev = de + 3 + dn
    KE, DN, KM = -(-kev // 16) * 16, -(-dn // 16) * 16, -(-ex.mlp_dim // 16) * 16
    e = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)  # noqa: E731
    b = dict(imp=None, dlogit=e(n), M2=e(n, h), dM2=e(n, h), M1d=e(n, KM), dM1=e(n, KM), X=e(n, KM), dY2=e(n, h),
             H1d=e(n, h), dH1=e(n, h), O=e(n, 2 * h), dP=e(n, 2 * h), dQ=e(2, n, 2 * h), dF=e(n, 3, 2 * h),
             ev=e(R, KE), AB=e(R, 2, DN), H=e(R, 2, h), dZ=e(R, 2, h), dlev=e(R, DN), g=e(R, DN), dt=e(R))
    io = L.EncoderGradIO(*[None if b[k] is None else b[k].data_ptr() for k in L.GRAD_IO_FIELDS])
    d_imp = torch.from_numpy(np.random.RandomState(4).uniform(-1, 1, n).astype(np.float32)).to(dev)
    nt, et = ex.feature_tables()
    L.check(L.lib().tm_encoder_bwd(ex.packed_weights(), L.ptr(nt), L.ptr(et), G, B, W, L.ptr(args[0]), L.ptr(args[1]),
                                   L.ptr(args[2]), L.ptr(args[3]), L.ptr(args[4]), L.ptr(args[5]), None, 1.0,
                                   L.ptr(ws), L.ptr(d_imp), L.C.byref(io), L.stream_ptr(dev)), "bwd")
    torch.cuda.synchronize()
    sd = ex.state_dict()
    Wev, bev = sd["event_conv.lin_event.weight"].float(), sd["event_conv.lin_event.bias"].float()
    M0 = sd["event_conv.MLP.0.weight"].float()
    ev = b["ev"][:, :kev]
    Lv = ev @ Wev.t() + bev
    n6 = args[0].reshape(-1, 3, 6).long()
    nf = torch.from_numpy(n_feat).to(dev)
    xs = nf[n6[:, :, [0, 2, 4]].reshape(-1)]
    xt = nf[n6[:, :, [1, 3, 5]].reshape(-1)]
    dZ = b["dZ"]
    ref = (dZ[:, 0] @ M0) * ((xt + Lv) > 0) + (dZ[:, 1] @ M0) * ((xs + Lv) > 0)
    got = b["dlev"][:, :dn]
    d = (got - ref).abs()
    print("h", h, "max |diff|", float(d.max()), "ref max", float(ref.abs().max()))
    bad = (d > 1e-5 * (1 + ref.abs().max())).nonzero()
    print("bad entries", bad.shape[0], "rows", torch.unique(bad[:, 0]).shape[0], "cols", torch.unique(bad[:, 1]).tolist()[:40])
    rows = torch.unique(bad[:, 0])
    print("row mod 32 of bad rows", torch.unique(rows % 32).tolist()[:40])
    # AB check (forward recompute)
    ab_ref_s = xs + torch.relu(xt + Lv)
    print("AB hs max diff", float((b["AB"][:, 0, :dn] - ab_ref_s).abs().max()))


if __name__ == "__main__":
    for h in [int(x) for x in sys.argv[1:]] or [128, 192]:
        main(h)
