#!/bin/bash
# A/B of training-kernel variants (tempme_amd/lib/ab/*.so) on bench_train.py, two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for so in tempme_amd/lib/ab/*.so; do
  TEMPME_LIB="$PWD/$so" timeout -k 10 300 python bench_train.py --steps 20 --warmup 2 > gpurun_out/tab.log 2>&1 || exit $?
  echo "$(basename $so) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tab.log)" | tee -a gpurun_out/tab.txt
done; done
