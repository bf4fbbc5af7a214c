#!/bin/bash
# A/B of training-kernel variants (tempme_amd/lib/ab/*.so) on bench_train.py, two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for so in tempme_amd/lib/ab/*.so; do
  TEMPME_LIB="$PWD/$so" timeout -k 10 300 python bench_train.py --steps 20 --warmup 2 > gpurun_out/tab.log 2>&1 || exit $?
  python - "$so" "$r" <<'PY' | tee -a gpurun_out/tab.txt
import json, sys, os
d = json.loads([l for l in open("gpurun_out/tab.log") if l.startswith("{")][-1])
k = d.get("kernels", {})
print(os.path.basename(sys.argv[1]), "round", sys.argv[2], "value", d["value"], "ms_per_step", d["ms_per_step"],
      {n: k[n]["avg_ms"] for n in ("wgrad_partial_kernel", "gcn_bwd_kernel", "head_bwd_kernel", "tgn_attn_fwd_kernel", "tgn_attn_bwd_kernel") if n in k})
PY
done; done
