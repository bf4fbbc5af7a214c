#!/bin/bash
# Interleaved A/B of tempme_amd/lib/ab/*.so builds on events_kernel: bench.py's events_kernel average at the
# full step (192 batches), three rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2 3; do
  for so in tempme_amd/lib/ab/*.so; do
    n=$(basename "$so" .so)
    TEMPME_LIB="$PWD/$so" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras \
      --streams 1 > gpurun_out/eab_${n}_$r.log 2>&1 || exit $?
    echo "$n round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/eab_${n}_$r.log | head -1) $(grep -o '"events_kernel": {"avg_ms": [0-9.]*' gpurun_out/eab_${n}_$r.log)" | tee -a gpurun_out/events_ab.txt
  done
done
