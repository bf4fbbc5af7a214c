#!/bin/bash
# Build the GraphMixer A/B libraries for tools/gm_ab.sh (gm_fused_kernel knobs) and tools/gmb_ab.sh (gm_bwd_kernel
# phase ablations, TM_GMB_ABL bits: 1 = no per-channel token mixing, 2 = no channel-FFN GEMMs,
# 4 = no projection GEMM, 8 = no LayerNorm statistics / backward and per-token sums).  Sequential builds.
set -e
cd "$(dirname "$0")/.."
rm -f tempme_amd/lib/ab/gmf_*.so tempme_amd/lib/ab/gmb*.so
EXTRA="" ./tools/ab_build.sh gmf_base tempme_amd/csrc/encoder.hip
EXTRA="-DTM_GF_TOKPAIR=1" ./tools/ab_build.sh gmf_tokpair tempme_amd/csrc/encoder.hip
EXTRA="-DTM_GF_QG2=1" ./tools/ab_build.sh gmf_qg2 tempme_amd/csrc/encoder.hip
EXTRA="-DTM_GF_TOKPAIR=1 -DTM_GF_QG2=1" ./tools/ab_build.sh gmf_both tempme_amd/csrc/encoder.hip
for b in 0 1 2 4 8; do EXTRA="-DTM_GMB_ABL=$b" ./tools/ab_build.sh gmb$b tempme_amd/csrc/encoder.hip; done
