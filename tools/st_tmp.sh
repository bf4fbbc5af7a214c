#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_enron.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
rm -f gpurun_out/eab.txt; ./tools/events_ab.sh || exit $?
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS -d gpurun_out/ldsc -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/ldsc.log 2>&1
