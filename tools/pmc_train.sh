#!/bin/bash
# PMC passes over the training bench (one counter group per run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python bench_train.py --steps 5 --warmup 1"
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAVES"; do
    i=$((i+1))
    timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pmct$i -o run --output-format csv -- $B > gpurun_out/pmct$i.log 2>&1 || exit $?
    echo "pass $i ok"
done
