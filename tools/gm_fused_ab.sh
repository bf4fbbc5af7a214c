#!/bin/bash
# Build the gm_fused_kernel A/B pair for tools/gm_ab.sh: tempme_amd/lib/ab/gmf_base.so (default code) and
# gmf_tokpair.so (-DTM_GF_TOKPAIR=1: token mixing two channel tiles per iteration, branch-free), gmf_qg2.so
# (-DTM_GF_QG2=1: the projection's K loop over pairs of tiles, 22 instead of 24 at C = T = 172), gmf_both.so; then run
# `tools/gpu_run.sh` with a step that calls tools/gm_ab.sh (configs[4] bench per library, two rounds).
set -e
cd "$(dirname "$0")/.."
rm -f tempme_amd/lib/ab/*.so
EXTRA="" ./tools/ab_build.sh gmf_base tempme_amd/csrc/encoder.hip
EXTRA="-DTM_GF_TOKPAIR=1" ./tools/ab_build.sh gmf_tokpair tempme_amd/csrc/encoder.hip
EXTRA="-DTM_GF_QG2=1" ./tools/ab_build.sh gmf_qg2 tempme_amd/csrc/encoder.hip
EXTRA="-DTM_GF_TOKPAIR=1 -DTM_GF_QG2=1" ./tools/ab_build.sh gmf_both tempme_amd/csrc/encoder.hip
