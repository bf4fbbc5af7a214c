#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_graphmixer.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gm.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gm.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/bench_c4.log 2>&1; rc=$?
echo "rc=$rc"; tail -1 gpurun_out/bench_c4.log | grep -o '"value": [0-9.]*\|"gm_embed_kernel": {[^}]*}'
