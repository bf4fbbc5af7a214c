#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert|error" gpurun_out/$n.log | head -20; tail -5 gpurun_out/$n.log; exit $rc; fi; }
step pytest_gb 300 python -u -m pytest tests/test_gpu_graph_build.py -x -v --timeout 200 --timeout-method thread
step pytest_gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
TEMPME_GRAPH_TIMING=1 step graph_build 300 python tools/graph_build.py
