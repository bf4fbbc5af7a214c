#!/bin/bash
# Interleaved A/B of tempme_amd/lib/ab/*.so walk-kernel builds at the 8-rank share (24 batches) and the full step
# (192 batches): bench.py's walk_kernel average and step time, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  for so in tempme_amd/lib/ab/*.so; do
    n=$(basename "$so" .so)
    for b in 24 192; do
      TEMPME_LIB="$PWD/$so" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras \
        --batches $b --streams 1 > gpurun_out/tab_${n}_${b}_$r.log 2>&1 || exit $?
      echo "$n b=$b round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tab_${n}_${b}_$r.log | head -1) $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/tab_${n}_${b}_$r.log)" | tee -a gpurun_out/tail_ab.txt
    done
  done
done
