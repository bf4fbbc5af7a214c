#!/bin/bash
# SQ / LDS / MFMA PMC passes over a short bench (PMC_ARGS: extra bench flags, e.g. --config 4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras $PMC_ARGS"
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/sq$i -o run --output-format csv -- $B > gpurun_out/sq$i.log 2>&1 || exit $?
    echo "pass $i rc=$?"
done
