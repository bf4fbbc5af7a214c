#!/bin/bash
# A/B of walk-kernel edge-table variants (tempme_amd/lib/ab/*.so) against the plain mode, configs 1 and 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for c in 1 4; do
  for so in tempme_amd/lib/ab/*.so; do
    TEMPME_LIB="$PWD/$so" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $c > gpurun_out/etab.log 2>&1 || exit $?
    echo "config=$c $(basename $so) $(grep -o '"value": [0-9.]*' gpurun_out/etab.log) $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/etab.log) $(grep -o '"gate_table_kernel": {"avg_ms": [0-9.]*' gpurun_out/etab.log)" | tee -a gpurun_out/etab.txt
  done
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $c --no-edge-table > gpurun_out/etab.log 2>&1 || exit $?
  echo "config=$c plain $(grep -o '"value": [0-9.]*' gpurun_out/etab.log) $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/etab.log)" | tee -a gpurun_out/etab.txt
done; done
