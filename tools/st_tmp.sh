#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_graphmixer.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gm.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|Mismatch|Max abs" gpurun_out/pytest_gm.log | head -30
