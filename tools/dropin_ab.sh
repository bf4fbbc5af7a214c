#!/bin/bash
# A/B of drop-in variants (tempme_amd/lib/ab/*.so, built by tools/ab_build.sh): tools/dropin_timing.py per
# variant (free-running, one batch alone, GPU-bound per batch), alternating rounds (DAB_ROUNDS, default 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in $(seq 1 "${DAB_ROUNDS:-2}"); do for so in tempme_amd/lib/ab/*.so; do
  n=$(basename "$so" .so)
  TEMPME_LIB="$PWD/$so" timeout -k 10 200 python tools/dropin_timing.py > gpurun_out/dab.log 2>&1 || exit $?
  echo "$n round $r: $(grep -E 'free-running|alone|GPU-bound' gpurun_out/dab.log | tr '\n' ' ')" | tee -a gpurun_out/dab.txt
done; done
