#!/bin/bash
# A/B of gm_embed_kernel variants (tempme_amd/lib/ab/*.so) on configs[4] + GraphMixer contrast: the
# kernel's average launch time and the bench value, two alternating rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for so in tempme_amd/lib/ab_gm/gmf_*.so; do
  TEMPME_LIB="$PWD/$so" timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/gab.log 2>&1 || exit $?
  python - "$so" <<'PY' | tee -a gpurun_out/gab.txt
import json, sys, os
d = json.loads([l for l in open("gpurun_out/gab.log") if l.startswith("{")][-1])
k = d["kernels"].get("gm_fused_kernel") or d["kernels"]["gm_embed_kernel"]
print(os.path.basename(sys.argv[1]), "gm_embed", k["avg_ms"], k["frac"], "value", d["value"])
PY
done; done
