"""Time GraphMixer.contrast forward + d explanation-weight backward at BASELINE configs[4] shapes (de = dn = 172,
N = 30, 2 mixer layers) on the HIP path (tm_gm_embed + tm_gm_embed_bwd) and on the torch formulation under
autograd (TEMPME_GM_TORCH=1 semantics), and check the two gradients agree."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")


def main():
    from tempme_amd.graphmixer import GraphMixer
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    V, E, N, B, d = 9000, 200000, 30, 600, 172
    nf = rng.uniform(0, 1, (V, d)).astype(np.float32)
    ef = rng.uniform(0, 1, (E + 1, d)).astype(np.float32)
    nf[0] = ef[0] = 0
    torch.manual_seed(0)
    m = GraphMixer(nf, ef, n_neighbors=N, device=dev, num_tokens=N, num_layers=2, dropout=0.1).to(dev).eval()
    cut = np.floor(rng.uniform(5e7, 1e8, B))
    sgs = []
    for _ in range(3):
        node = rng.integers(1, V, (B, N))
        node[rng.uniform(size=node.shape) < 0.1] = 0
        eid = np.where(node > 0, rng.integers(1, E + 1, node.shape), 0)
        ts = np.where(node > 0, np.floor(cut[:, None] - rng.uniform(0, 5e7, node.shape)), 0.0)
        sgs.append(([torch.from_numpy(node.astype(np.float64)).to(dev), None],
                    [torch.from_numpy(eid.astype(np.float64)).to(dev), None], [torch.from_numpy(ts).to(dev), None]))
    src, dst, fake = (torch.from_numpy(rng.integers(1, V, B)).to(dev) for _ in range(3))
    cut_d = torch.from_numpy(cut).to(dev)
    ew0 = torch.from_numpy(rng.uniform(0, 1, (3 * B, N)).astype(np.float32)).to(dev)
    y = torch.cat([torch.ones(B, 1), torch.zeros(B, 1)]).to(dev)

    def step():
        ew = ew0.clone().requires_grad_(True)
        p, n = m.contrast(src, dst, fake, cut_d, None, *sgs, explain_weights=[ew])
        torch.nn.functional.binary_cross_entropy_with_logits(torch.cat([p, n]), y).backward()
        return ew.grad

    res = {}
    for mode in ("hip", "torch"):
        os.environ["TEMPME_GM_TORCH"] = "1" if mode == "torch" else "0"
        g = step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            g = step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        res[mode] = g.detach().clone()
        print("%-5s forward + d ew backward: %.2f ms per %d rows (%d events x 3 sides)" % (mode, dt * 1e3, 3 * B, B))
        if mode == "hip":
            from tempme_amd import _lib as L
            L.profile_enable(True)
            for _ in range(reps):
                step()
            prof = L.profile_read()
            L.profile_enable(False)
            for k, (ms, cnt) in sorted(prof.items()):
                print("  kernel %-16s %.3f ms per launch (%d launches)" % (k, ms / max(cnt, 1), cnt))
    err = float(torch.linalg.norm(res["hip"] - res["torch"]) / torch.linalg.norm(res["torch"]))
    print("relative difference of d ew, HIP vs torch formulation: %.2e" % err)


if __name__ == "__main__":
    main()
