#!/bin/bash
# bench_train.py under each round-4 opt-in training switch, interleaved, two rounds:
# ms_per_step per configuration into gpurun_out/train_flags.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # run <label> <env...> -- <extra args>
    local label=$1; shift
    local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 300 python bench_train.py --steps 10 --warmup 2 "$@" > gpurun_out/tf.log 2>&1 || exit $?
    echo "$label round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tf.log) $(grep -o '"value": [0-9.]*' gpurun_out/tf.log | head -1)" | tee -a gpurun_out/train_flags.txt
}
for r in 1 2; do
    run base X=0 --
    run nozn X=0 -- --no-node-zero
    run overlap X=0 -- --overlap-prepare
done
