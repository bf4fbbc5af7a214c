"""The threshold_test selection (tempme_amd/csrc/topk_select.h, run on the GPU by mask_least_kernel)
compiled for the host with g++ and checked against torch.topk(largest=False) on the CPU -- the op
temp_exp_main.py:166-168 calls -- including its tie order and NaN placement."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def host_select(tmp_path_factory):
    out = tmp_path_factory.mktemp("sel") / "libselect_host.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", os.path.join(HERE, "select_host.cpp"), "-o",
                    str(out)], check=True)
    lib = C.CDLL(str(out))
    lib.select_rows.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_void_p]

    def run(x, k):
        x = np.ascontiguousarray(x, dtype=np.float32)
        res = np.zeros((x.shape[0], k), np.int32)
        lib.select_rows(x.ctypes.data, x.shape[0], x.shape[1], k, res.ctypes.data)
        return res
    return run


@pytest.mark.parametrize("n", [3, 4, 7, 20, 100, 420, 930, 3000])
def test_selection_equals_cpu_topk(host_select, n):
    rng = np.random.default_rng(n)
    for k in sorted({1, 2, 3, max(1, n // 64), n // 3, n - 5, n - 1, n}):
        if not 1 <= k <= n:
            continue
        for levels in (6, 10 ** 6):          # tie-heavy and nearly tie-free rows
            x = (rng.integers(0, levels, (32, n)) / levels).astype(np.float32)
            if levels == 6:
                x[rng.uniform(size=x.shape) < 0.01] = np.nan
            got = np.sort(host_select(x, k), axis=1)
            ref = np.sort(torch.topk(torch.from_numpy(x), k=k, dim=-1, largest=False).indices.numpy(), axis=1)
            assert np.array_equal(got, ref), (n, k, levels)


def test_selection_golden_threshold_masks(host_select):
    """The masks threshold_test built in the golden run (tgn_uslegis.npz) from the golden explanation."""
    import math
    import tgn_inputs as TI
    g, d = TI.golden(), TI.load_batch()
    B, N = d["B"], d["N"]
    ne = N + N * N
    ratios = g["ratios"]
    for case in ("uslegis", "synth"):
        expl = TI.explanation(case)
        bits = np.unpackbits(g[f"{case}_thr_zero_bits"])[:len(ratios) * 3 * B * ne]
        bits = bits.reshape(len(ratios), 3 * B, ne).astype(bool)
        orig = np.concatenate([np.concatenate([d["sg_" + s][0][0], d["sg_" + s][0][1]], 1) for s in TI.SIDES]) == 0
        imp = torch.cat([expl[0], expl[1]], dim=1).numpy()
        for ri, r in enumerate(ratios):
            topk = min(max(math.ceil(r * ne), 1), ne)
            zero = orig.copy()
            np.put_along_axis(zero, host_select(imp, ne - topk), True, axis=-1)
            assert np.array_equal(zero, bits[ri]), (case, r)
