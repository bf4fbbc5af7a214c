#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
TEMPME_LIB=$PWD/tempme_amd/lib/ab/stamps.so timeout -k 10 200 python tools/stamps.py > gpurun_out/st2.log 2>&1 || exit $?
PASSES="1 2 4 6" ./tools/pmc_mem.sh
