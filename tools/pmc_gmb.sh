#!/bin/bash
# PMC passes over tools/gm_bwd_timing.py (configs[4] shapes): gm_bwd_kernel's MFMA / VALU / LDS / wait picture
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
i=0
for ctr in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pgm$i -o run --output-format csv -- \
        python tools/gm_bwd_timing.py > gpurun_out/pgm$i.log 2>&1
    rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
