#!/bin/bash
# Build the GraphMixer A/B libraries for tools/gmb_ab.sh (gm_bwd_kernel phase ablations, TM_GMB_ABL bits: 1 = no token mixing, 2 = no channel-FFN GEMMs,
# 4 = no projection GEMM, 8 = no LayerNorm statistics / backward and per-token sums).  Sequential builds.
set -e
cd "$(dirname "$0")/.."
rm -f tempme_amd/lib/ab_gm/gmf_*.so tempme_amd/lib/ab_gm/gmb*.so
# the ablation hooks live in tools/patches/gm_bwd_ablation.patch: applied to a copy of graphmixer.hip
cp tempme_amd/csrc/graphmixer.hip /tmp/gm_abl.hip
patch -s /tmp/gm_abl.hip tools/patches/gm_bwd_ablation.patch
for b in 0 1 2 4 8; do GM=/tmp/gm_abl.hip EXTRA="-DTM_GMB_ABL=$b" ./tools/ab_build.sh gmb$b tempme_amd/csrc/encoder.hip; done
mkdir -p tempme_amd/lib/ab_gm && mv -f tempme_amd/lib/ab/gmb*.so tempme_amd/lib/ab_gm/
