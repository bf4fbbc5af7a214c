"""Debug: which host-staging call leaves a HIP error behind (checked with a tiny device round trip after each)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")


def probe(what):
    try:
        torch.zeros(1, device="cuda").cpu()
        torch.cuda.synchronize()
        print("ok  ", what, flush=True)
    except Exception as e:      # noqa: BLE001
        print("FAIL", what, repr(e)[:200], flush=True)
        sys.exit(1)


def main():
    import ctypes as C
    from tempme_amd import _lib as L
    from tempme_amd import hoststage as H
    dev = torch.device("cuda", 0)
    probe("start")
    big = np.zeros((1 << 20,), dtype=np.float64)
    d = C.c_void_p()
    rc = L.lib().tm_host_register(big.__array_interface__["data"][0], big.nbytes, C.byref(d))
    print("register rc", rc, hex(d.value or 0), L.lib().tm_last_error())
    probe("after register")
    st = torch.cuda.Stream()
    got = H.stage(dev, [(big[:10], torch.float32)], st)
    torch.cuda.synchronize()
    probe(f"after stage (got {got is not None})")
    rc = L.lib().tm_host_unregister(big.__array_interface__["data"][0])
    print("unregister rc", rc, L.lib().tm_last_error())
    probe("after unregister")
    w = np.random.default_rng(0).normal(size=(2000, 60, 14))
    x = H.stage(dev, [(w[:100, :, 9:12], torch.float32)], st)
    torch.cuda.synchronize()
    probe(f"after stage of w (got {x is not None})")
    H._REG.clear()
    probe("after clear")
    small = [np.random.default_rng(k).normal(size=(300, 600)) for k in range(6)]   # 1.4 MB heap arrays
    for k, a in enumerate(small):
        y = H.stage(dev, [(a[:10], torch.float32)], st)
        torch.cuda.synchronize()
        probe(f"heap array {k} staged={y is not None}")
    H._REG.clear()
    probe("after second clear")


if __name__ == "__main__":
    main()
