#!/bin/bash
# gm_bwd_kernel phase ablations (tempme_amd/lib/ab_gm/gmb*.so, built with tools/ab_build.sh and
# EXTRA=-DTM_GMB_ABL=<bits>): forward + d ew timing at configs[4] shapes per variant, two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for so in tempme_amd/lib/ab_gm/gmb*.so; do
  n=$(basename "$so" .so)
  TEMPME_LIB="$PWD/$so" timeout -k 10 200 python tools/gm_bwd_timing.py > gpurun_out/gmb_$n.log 2>&1 || exit $?
  echo "$n round $r: $(grep -E 'hip |kernel gm_bwd' gpurun_out/gmb_$n.log | tr '\n' ' ')" | tee -a gpurun_out/gmb_ab.txt
done; done
