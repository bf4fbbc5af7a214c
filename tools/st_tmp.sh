#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|error" gpurun_out/$n.log | head; tail -5 gpurun_out/$n.log; exit $rc; fi; }
step pytest_gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-extras
step bench_c4 600 python bench.py --config 4 --no-cpu-baseline
