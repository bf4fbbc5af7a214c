#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; if [ $rc -ne 0 ]; then tail -15 gpurun_out/$n.log; exit $rc; fi; }
step bench_train 600 python bench_train.py --steps 20 --warmup 3
TEMPME_DIST_BACKEND=gloo step bench_train2 600 python bench_train.py --gpus 2 --steps 5 --warmup 1
TEMPME_DIST_BACKEND=gloo step bench_dist2 600 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --no-extras
