#!/bin/bash
# One-GPU estimate of bench.py's strong scaling: the per-rank work of N = 1, 2, 4, 8 ranks (192 / N reference
# batches per step) timed on one GPU; efficiency(N) ~ T(192) / (N * T(192 / N)) before any inter-rank cost
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for b in 192 96 48 24; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --batches $b > gpurun_out/strong_$b.log 2>&1 || exit $?
  echo "batches=$b auto-streams $(grep -o '"value": [0-9.]*' gpurun_out/strong_$b.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/strong_$b.log | head -1) $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/strong_$b.log)" | tee -a gpurun_out/strong.txt
done
# two steps in flight (PipelinedExplainer) at the 8-rank share
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --batches 24 --streams 2 > gpurun_out/strong_24s2.log 2>&1 || exit $?
echo "batches=24 streams=2 $(grep -o '"value": [0-9.]*' gpurun_out/strong_24s2.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/strong_24s2.log | head -1)" | tee -a gpurun_out/strong.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --batches 24 --streams 1 > gpurun_out/strong_24s1.log 2>&1 || exit $?
echo "batches=24 streams=1 $(grep -o '"value": [0-9.]*' gpurun_out/strong_24s1.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/strong_24s1.log | head -1)" | tee -a gpurun_out/strong.txt
