#!/bin/bash
# One-GPU estimate of bench.py's strong scaling: the per-rank work of N = 1, 2, 4, 8 ranks (192 / N reference
# batches per step) timed on one GPU, in the mode bench.py runs each N in (N = 1: one step at a time; N > 1: 3 steps
# in flight with overlapping walk kernels) and, for comparison, the other mode; efficiency(N) ~ T(192) / (N * T(192 / N))
# before any inter-rank cost (there is no data-path collective)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for b in 192 96 48 24; do
  for mode in "s1:--streams 1" "s3o:--streams 3 --overlap-walk"; do
    n=${mode%%:*}; fl=${mode#*:}
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --batches $b $fl \
      > gpurun_out/strong_${n}_$b.log 2>&1 || exit $?
    echo "batches=$b $n $(grep -o '"value": [0-9.]*' gpurun_out/strong_${n}_$b.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/strong_${n}_$b.log | head -1) $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/strong_${n}_$b.log)" | tee -a gpurun_out/strong.txt
  done
done
