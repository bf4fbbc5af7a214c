#!/bin/bash
# A/B of sampler variants (tempme_amd/lib/ab/*.so): events_kernel (sampling_roofline) and khop2_kernel
# (khop_roofline) average launch times and the bench value, two alternating rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for so in tempme_amd/lib/ab/*.so; do
  TEMPME_LIB="$PWD/$so" timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline $EAB_ARGS > gpurun_out/eab.log 2>&1 || exit $?
  python - "$so" <<'PY' | tee -a gpurun_out/eab.txt
import json, sys, os
d = json.loads([l for l in open("gpurun_out/eab.log") if l.startswith("{")][-1])
k = d.get("khop_roofline") or {}
print(os.path.basename(sys.argv[1]), "events", d["sampling_roofline"]["avg_ms"], d["sampling_roofline"]["frac"],
      "khop", k.get("avg_ms"), k.get("frac"), "value", d["value"])
PY
done; done
