#!/bin/bash
# A/B of events_kernel variants (tempme_amd/lib/ab/*.so): the bench's sampling_roofline, three rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for so in tempme_amd/lib/ab/*.so; do
  TEMPME_LIB="$PWD/$so" timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras $EAB_ARGS > gpurun_out/eab.log 2>&1 || exit $?
  echo "$(basename $so) $(grep -o '"sampling_roofline": {[^}]*}' gpurun_out/eab.log | grep -o '"avg_ms": [0-9.]*\|"frac": [0-9.]*' | tr '\n' ' ') $(grep -o '"value": [0-9.]*' gpurun_out/eab.log)" | tee -a gpurun_out/eab.txt
done; done
