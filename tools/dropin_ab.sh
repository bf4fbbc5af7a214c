#!/bin/bash
# Interleaved A/B of tempme_amd/lib/ab/*.so builds on the drop-in eval loop (tools/dropin_timing.py: free-running
# wall time per batch, GPU-bound time per batch), device pack, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  for so in tempme_amd/lib/ab/*.so; do
    n=$(basename "$so" .so)
    TEMPME_LIB="$PWD/$so" timeout -k 10 200 python tools/dropin_timing.py > gpurun_out/dab_${n}_$r.log 2>&1 || exit $?
    echo "$n round $r: $(grep -E 'free-running|GPU-bound' gpurun_out/dab_${n}_$r.log | tr '\n' ' ')" | tee -a gpurun_out/dropin_ab.txt
  done
done
