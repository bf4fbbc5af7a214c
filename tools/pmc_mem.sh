#!/bin/bash
# PMC passes on the vector-memory pipeline (TA / TCP / TD) over a short bench: where the sampler's
# gathers queue (per-CU address unit, L1, L2 latency, TLB)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras $PMC_ARGS"
i=0
PASSES=${PASSES:-all}
for ctr in "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1)); [ "$PASSES" != all ] && [[ " $PASSES " != *" $i "* ]] && continue
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pm$i -o run --output-format csv -- $B > gpurun_out/pm$i.log 2>&1 || exit $?
    echo "pass $i rc=$?"
done
