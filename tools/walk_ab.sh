#!/bin/bash
# A/B of walk_kernel variants (tempme_amd/lib/ab/*.so, built by tools/ab_build.sh): walk_kernel average
# launch time, its executed fraction and the bench value, alternating rounds (WAB_ROUNDS, default 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in $(seq 1 "${WAB_ROUNDS:-2}"); do for so in tempme_amd/lib/ab/*.so; do
  TEMPME_LIB="$PWD/$so" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${WAB_EXTRAS:---no-extras} $WAB_ARGS > gpurun_out/wab.log 2>&1 || exit $?
  python - "$so" "$r" <<'PY' | tee -a gpurun_out/wab.txt
import json, sys, os
d = json.loads([l for l in open("gpurun_out/wab.log") if l.startswith("{")][-1])
k = d["kernels"]["walk_kernel"]
print(os.path.basename(sys.argv[1]), "round", sys.argv[2], "walk_kernel", k["avg_ms"], k["frac"],
      "events", d["kernels"]["events_kernel"]["avg_ms"], "explain_tab", d["kernels"].get("explain_tab_kernel", {}).get("avg_ms"), "khop", (d.get("khop_roofline") or {}).get("avg_ms"), "gate", d["kernels"].get("gate_table_kernel", {}).get("avg_ms"), "ms_per_step", d["ms_per_step"], "value", d["value"])
PY
done; done
