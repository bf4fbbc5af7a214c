#!/bin/bash
# walk_kernel persistent grid caps at the 8-rank share (24 batches) and the full step (192), two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  for cap in 0 480 450 416 384; do
    for b in 24 192; do
      timeout -k 10 200 python tools/walk_grid_ab.py $cap --steps 20 --warmup 3 --no-cpu-baseline --no-extras \
        --batches $b --streams 1 > gpurun_out/wg_${cap}_${b}_$r.log 2>&1 || exit $?
      echo "cap=$cap b=$b round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wg_${cap}_${b}_$r.log | head -1) $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/wg_${cap}_${b}_$r.log)" | tee -a gpurun_out/walk_grid_ab.txt
    done
  done
done
