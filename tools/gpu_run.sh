#!/bin/bash
# GPU-box driver for one gpurun call: each GPU step under its own timeout; stop at the first
# crash/abort/timeout (exit codes other than 0 = pass, 1 = test/assert failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
    local name=$1 to=$2; shift 2
    echo "=== $name: $*" | tee -a gpurun_out/steps.log
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
for s in "$@"; do
    case $s in
        tests) step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ;;
        f3) step pytest_f3 600 python -u -m pytest tests/test_gpu_encoder_train.py tests/test_gpu_explain_train.py tests/test_gpu_train.py tests/test_gpu_pack.py -x -v --timeout 300 -m gpu ;;
        tgn) step pytest_tgn 600 python -m pytest tests/test_gpu_tgn.py tests/test_gpu_train.py tests/test_gpu_graphmixer.py -x -q -m gpu ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        info) step info 60 bash -c 'nproc; cat /sys/fs/cgroup/cpu.max; python -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))"' ;;
        bench) step bench 600 python bench.py ;;
        bench1) step bench_c1 600 python bench.py --config 1 --no-cpu-baseline ;;
        benchq) step bench 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        prof) step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-extras ;;
        profx) step rocprof_x 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profx -o run --output-format csv -- python bench.py --no-cpu-baseline ;;
        prof4) step rocprof_c4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python bench.py --config 4 --no-cpu-baseline --no-extras ;;
        enron) step pytest_enron 900 python -u -m pytest tests/test_gpu_enron.py -v --timeout 300 --timeout-method thread ;;
        pmc1|pmc2|pmc4)  # PMC passes (one counter group per run) over a short bench of configs[1|2|4]
            c=${s#pmc}
            B="python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
            i=0
            for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                       "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU" \
                       "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" \
                       "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU"; do
                i=$((i+1))
                step pmc_c${c}_$i 400 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pmc_c${c}_$i -o run --output-format csv -- $B
            done ;;
        ablate)
            for ab in 0 1 2 4 7 0; do
                TEMPME_ABLATE=$ab step ablate$ab 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline
                grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/ablate$ab.log
            done ;;
        ab)  # interleaved A/B timing of every tempme_amd/lib/ab/*.so variant (two rounds)
            for r in 1 2; do
                for so in tempme_amd/lib/ab/*.so; do
                    n=$(basename "$so" .so)
                    TEMPME_LIB="$PWD/$so" step ab_${n}_$r 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
                    echo "$n round $r: $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/ab_${n}_$r.log) $(grep -o '"events_kernel": {"avg_ms": [0-9.]*' gpurun_out/ab_${n}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${n}_$r.log)" | tee -a gpurun_out/ab.txt
                done
            done ;;
        stamps)  # phase stamps of every -DTM_STAMPS build in tempme_amd/lib/ab_st/
            for so in tempme_amd/lib/ab_st/*.so; do
                n=$(basename "$so" .so)
                TEMPME_LIB="$PWD/$so" step stamps_$n 300 python tools/stamps.py
                { echo "== $n: $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/stamps_$n.log)"; grep -E "^(slot|walk) |clock|wave pass-loop" gpurun_out/stamps_$n.log; } | tee -a gpurun_out/stamps.txt
            done ;;
        dist2)  # multi-rank rehearsal on one GPU: bench.py starts its own 2 ranks (gloo barrier/max), both on cuda:0
            TEMPME_DIST_BACKEND=gloo step dist2 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline ;;
        proftrain) step rocprof_train 600 rocprofv3 --kernel-trace --stats -d gpurun_out/proftrain -o run --output-format csv -- python bench_train.py --steps 10 --warmup 2 ;;
        train) step bench_train 600 python bench_train.py --steps 10 --warmup 2 ;;
        train2)  # 2-rank rehearsal of the gradient all-reduce on one GPU (gloo)
            TEMPME_DIST_BACKEND=gloo step bench_train2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29512 bench_train.py --gpus 2 --steps 5 --warmup 1 ;;
        n30) step bench_n30 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --n-degree 30 ;;
        phases) step phases 300 python tools/train_phases.py ;;
        trainflags) step train_flags 1100 ./tools/train_flags_ab.sh ;;
        gmab) step gm_ab 900 ./tools/gm_ab.sh ;;
        gmbab) step gmb_ab 900 ./tools/gmb_ab.sh ;;
        gmbwd) step gm_bwd 300 python tools/gm_bwd_timing.py ;;
        trainops) step trainops 300 python tools/train_ops.py ;;
        gemmprobe) step gemm_probe 300 python tools/gemm_probe.py ;;
        c2) step bench_c2 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --config 2 ;;
        c4) step bench_c4 900 python bench.py --steps 5 --warmup 1 --config 4 ;;
        a3) step bench_a3 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --alpha 3.0 ;;
        dropint) step dropint 300 python tools/dropin_timing.py ;;
        dropinth) step dropinth 300 python tools/dropin_timing.py host ;;
        diag) step overlap_diag 300 python -u tools/overlap_diag.py ;;
        testsall) step pytest_gpu_all 1100 python -u -m pytest tests -q -m gpu -rfEs --timeout 300 --timeout-method thread ;;
        variants) step pytest_variants 600 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_enron.py -v -m gpu -rfEs --timeout 300 --timeout-method thread -k "variants or cpp_host" ;;
        tab) step tab 1100 ./tools/train_ab.sh ;;
        strong) step strong 900 ./tools/strong.sh ;;
        dab) step dab 900 ./tools/dropin_ab.sh ;;
        dropintrace) step dropintrace 300 rocprofv3 --kernel-trace -d gpurun_out/ditrace -o run --output-format csv -- python tools/dropin_timing.py && python tools/dropin_trace_summary.py > gpurun_out/dropin_trace.txt 2>&1 ;;
        dropinprof) TEMPME_DROPIN_PROFILE=1 step dropinprof 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
        abtests:*)  # the GPU suite against tempme_amd/lib/ab/<name>.so
            n=${s#abtests:}
            TEMPME_LIB="$PWD/tempme_amd/lib/ab/$n.so" step pytest_ab_$n 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ;;
        wab) step wab 1200 ./tools/walk_ab.sh ;;
        wabx) WAB_EXTRAS=" " step wab 1200 ./tools/walk_ab.sh ;;
        sab) step sab 1200 ./tools/streams_ab2.sh ;;
        k:*) kn=$(echo "${s#k:}" | tr -c 'A-Za-z0-9_\n' '_'); step "pytest_k_$kn" 600 python -u -m pytest tests -x -v -m gpu -rfEs --timeout 300 --timeout-method thread -k "${s#k:}" ;;
        micro:*) m=${s#micro:}; step micro_$m 200 ./micro/$m ;;   # a prebuilt micro-benchmark binary
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
