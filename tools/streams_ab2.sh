#!/bin/bash
# steps in flight (bench --streams 1|2) for every tempme_amd/lib/ab/*.so, two rounds; then a kernel trace
# of --streams 2 on the first library (does the next step's sampler overlap this step's walk kernel?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for so in tempme_amd/lib/ab/*.so; do for S in 1 2; do
  TEMPME_LIB="$PWD/$so" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --streams $S > gpurun_out/sab.log 2>&1 || exit $?
  echo "$(basename $so) S=$S round $r $(grep -o '"value": [0-9.]*' gpurun_out/sab.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sab.log)" | tee -a gpurun_out/sab.txt
done; done; done
so=$(ls tempme_amd/lib/ab/*.so | head -1)
TEMPME_LIB="$PWD/$so" timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/strace -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extras --streams 2 > gpurun_out/strace.log 2>&1
