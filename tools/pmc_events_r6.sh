#!/bin/bash
# Round-6 events_kernel re-diagnosis: address-unit (TA), data-return (TD) and VALU utilisation of the hop-1/2/3
# sampler on the current tree, one rocprofv3 --pmc pass per counter group (within the per-block limits), over a
# short default bench.  Counter names are checked against `rocprofv3 -L` first; a group with a missing name is
# skipped and said so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
grep -oE "\b(TA|TD|TCP|SQ|SQC|GRBM)_[A-Z0-9_]+" gpurun_out/counters.txt | sort -u > gpurun_out/counter_names.txt
i=0
for ctr in "TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE" \
           "TD_TD_BUSY_sum TD_BUSY_avr GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
           "TA_FLAT_READ_WAVEFRONTS_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
    have=""
    for c in $ctr; do
        base=${c%_sum}; base=${base%_avr}
        if grep -qx "$c" gpurun_out/counter_names.txt || grep -qx "$base" gpurun_out/counter_names.txt; then have="$have $c"; else echo "missing $c"; fi
    done
    i=$((i+1))
    [ -z "$have" ] && continue
    timeout -k 10 -s KILL 90 rocprofv3 --kernel-trace --pmc $have -d gpurun_out/pev$i -o run --output-format csv -- \
        python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/pev$i.log 2>&1
    rc=$?
    echo "pass $i [$have ] rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
exit 0
