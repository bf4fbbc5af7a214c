#!/bin/bash
# GPU-box driver for one gpurun call: each GPU step under its own timeout; stop at the first
# crash/abort/timeout (exit codes other than 0 = pass, 1 = test/assert failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}" || exit 2
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
        tests) step pytest_gpu 900 python -m pytest tests -x -q -m gpu ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) step bench 600 python bench.py --steps 10 --warmup 2 ;;
        benchq) step bench 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        prof) step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
