"""Probe: fp32 GEMM times of the TGN contrast's shapes (training step, bs=100, N=20: layer 0 has R = 6000 rows)
under torch's BLAS back ends (hipBLASLt, rocBLAS) -- which library call the glue GEMMs should use."""
import torch

SHAPES = [  # (name, M, K, N): out[M, N] = X[M, K] @ W[N, K]^T (+ bias)
    ("fc G (fwd)", 6000, 752, 344), ("merger fc1", 6000, 516, 172), ("merger fc2", 6000, 172, 172),
    ("dz = dout G (bwd)", 6000, 344, 752), ("d fc1 (bwd)", 6000, 172, 516), ("d fc2 (bwd)", 6000, 172, 172),
    ("qf = query P^T", 6000, 344, 752), ("layer 1 fc G", 300, 752, 344)]


def bench(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for lib in ("hipblaslt", "rocblas", "default"):
        try:
            torch.backends.cuda.preferred_blas_library(lib if lib != "default" else "cublaslt")
        except Exception as exc:      # noqa: BLE001
            print(lib, "unavailable:", exc)
            continue
        for name, M, K, N in SHAPES:
            x = torch.randn(M, K, device=dev, generator=g)
            w = torch.randn(N, K, device=dev, generator=g)
            bias = torch.randn(N, device=dev, generator=g)
            us = bench(lambda: torch.addmm(bias, x, w.t()))
            tf = 2 * M * N * K / us / 1e6
            print(f"{lib:10s} {name:20s} M={M} K={K} N={N}: {us:8.1f} us  {tf:6.1f} TFLOP/s")


if __name__ == "__main__":
    main()
