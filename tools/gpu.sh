#!/bin/bash
# tools/gpu.sh <timeout_s> <steps...>: one gpurun call of tools/gpu_run.sh; clears the step logs first so a
# call that did not run (backoff, no box) cannot be mistaken for fresh results.
to=$1; shift
cd "$(dirname "$0")/.."
rm -rf gpurun_out/sab.txt gpurun_out/strace gpurun_out/wab.txt gpurun_out/steps.log gpurun_out/pytest_gpu.log gpurun_out/bench.log gpurun_out/ab.txt gpurun_out/stamps.txt
/usr/local/graft/bin/gpurun --timeout "$to" -- "./tools/gpu_run.sh $*" 2>&1 | grep "^\[gpurun\]" | grep -v "sending"
