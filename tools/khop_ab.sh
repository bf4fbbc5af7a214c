#!/bin/bash
# A/B of khop2_kernel variants (tempme_amd/lib/ab/*.so): the bench's khop_roofline, two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for so in tempme_amd/lib/ab/*.so; do
  TEMPME_LIB="$PWD/$so" timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/kab.log 2>&1 || exit $?
  echo "$(basename $so) $(grep -o '"khop_roofline": {[^}]*}' gpurun_out/kab.log | grep -o '"avg_ms": [0-9.]*\|"frac": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/kab.txt
done; done
