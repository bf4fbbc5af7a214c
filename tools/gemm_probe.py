"""Probe: fp32 GEMM times of the TGN contrast's shapes (training step, bs=100, N=20: layer 0 has R = 6000 rows)
in both orientations -- out = X W^T + b as torch.addmm (the module's call) and as (W X^T)^T (the library sees
M and N swapped and may pick a better-filled tile) -- each timed as a captured HIP graph of 20 calls, so the
host's launch cost is out of the figure."""
import torch

SHAPES = [  # (name, M, K, N): out[M, N] = X[M, K] @ W[N, K]^T (+ bias)
    ("fc G (fwd)", 6000, 752, 344), ("merger fc1", 6000, 516, 172), ("merger fc2", 6000, 172, 172),
    ("dz = dout G (bwd)", 6000, 344, 752), ("d fc1 (bwd)", 6000, 172, 516), ("d fc2 (bwd)", 6000, 172, 172),
    ("qf = query P^T", 6000, 344, 752), ("layer 1 fc G", 300, 752, 344)]


def graph_time(fn, it=20, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / it * 1e3)
    return best


def main():
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(0)
    for name, M, K, N in SHAPES:
        x = torch.randn(M, K, device=dev, generator=gen)
        w = torch.randn(N, K, device=dev, generator=gen)
        bias = torch.randn(N, device=dev, generator=gen)
        ref = torch.addmm(bias, x, w.t())
        alt = torch.addmm(bias[:, None], w, x.t()).t()
        err = float((ref - alt).abs().max())
        t1 = graph_time(lambda: torch.addmm(bias, x, w.t()))
        t2 = graph_time(lambda: torch.addmm(bias[:, None], w, x.t()))
        t3 = graph_time(lambda: torch.addmm(bias[:, None], w, x.t()).t().contiguous())
        fl = 2 * M * N * K / 1e6
        prev = torch.backends.cuda.preferred_blas_library()
        other = []
        for lib in ("hipblas", "ck"):
            try:
                torch.backends.cuda.preferred_blas_library(lib)
                t4 = graph_time(lambda: torch.addmm(bias, x, w.t()))
                err4 = float((torch.addmm(bias, x, w.t()) - ref).abs().max())
                other.append(f"{lib} {t4:7.1f} us ({fl / t4:5.1f}) diff {err4:.1e}")
            except Exception as e:      # noqa: BLE001
                other.append(f"{lib} failed: {str(e)[:60]}")
            finally:
                torch.backends.cuda.preferred_blas_library(prev)
        print(f"{name:20s} M={M} K={K} N={N}: addmm {t1:7.1f} us ({fl / t1:5.1f} TF/s) | swapped {t2:7.1f} us "
              f"({fl / t2:5.1f}) | swapped+copy {t3:7.1f} us | max diff {err:.2e} | " + " | ".join(other))


if __name__ == "__main__":
    main()
