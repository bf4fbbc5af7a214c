#!/bin/bash
# PMC passes for events_kernel only (short bench), plus the list of available counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pe$i -o run --output-format csv -- $B > gpurun_out/pe$i.log 2>&1
    echo "pass $i rc=$?"
done
