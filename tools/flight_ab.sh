#!/bin/bash
# Steps in flight A/B at the 8-rank share (24 batches) and the full step: one stream, two streams with the encoders
# chained, two streams with overlapping walk kernels; two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  for b in 24 48 192; do
    for mode in "s1:--streams 1" "s2:--streams 2" "s2o:--streams 2 --overlap-walk" "s3o:--streams 3 --overlap-walk"; do
      n=${mode%%:*}; fl=${mode#*:}
      timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --batches $b $fl \
        > gpurun_out/fl_${n}_${b}_$r.log 2>&1 || exit $?
      echo "$n b=$b round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fl_${n}_${b}_$r.log | head -1) $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/fl_${n}_${b}_$r.log) $(grep -o '"events_kernel": {"avg_ms": [0-9.]*' gpurun_out/fl_${n}_${b}_$r.log)" | tee -a gpurun_out/flight_ab.txt
    done
  done
done
