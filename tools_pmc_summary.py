"""Summarise rocprofv3 --pmc CSV passes (gpurun_out/pmc*/run_counter_collection.csv) per kernel:
mean counter value per dispatch.  FETCH_SIZE/WRITE_SIZE are KB (rocprofv3); on gfx950 FETCH_SIZE
reads 1/2 of a wide coalesced stream's bytes (MI355X_MICROARCH.md §HBM) -- reported raw and x2."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "gpurun_out"
# --glob PAT: the pass directories (default pmc[0-9]* = the bench passes; tools_pmc_train.sh writes pmct*)
pat = sys.argv[sys.argv.index("--glob") + 1] if "--glob" in sys.argv else "pmc[0-9]*"
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{root}/{pat}/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in acc.items():
    if not k.startswith("tmk::"):
        continue
    out[k] = {c: sum(v) / len(v) for c, v in d.items()}
    x = out[k]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in x and "GRBM_GUI_ACTIVE" in x:
        x["mfma_busy_frac_est"] = x["SQ_VALU_MFMA_BUSY_CYCLES"] / (x["GRBM_GUI_ACTIVE"] * 4 * 256 / 8)
    if "TCC_HIT_sum" in x:
        x["l2_hit_rate"] = x["TCC_HIT_sum"] / max(1.0, x["TCC_HIT_sum"] + x["TCC_MISS_sum"])
    if "FETCH_SIZE" in x:
        x["hbm_read_bytes_x2"] = x["FETCH_SIZE"] * 1024 * 2
print(json.dumps(out, indent=1))
# --traffic FILE: per-launch HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM) keyed by
# the kernel names bench.py reports, read by bench.py for roofline.traffic
if "--traffic" in sys.argv:
    dest = sys.argv[sys.argv.index("--traffic") + 1]
    tr = {}
    for k, x in out.items():
        if "FETCH_SIZE" in x and "WRITE_SIZE" in x:
            short = k.replace("tmk::", "").split("<")[0]
            tr[short] = int(round(x["FETCH_SIZE"] * 1024 * 2 + x["WRITE_SIZE"] * 1024))
    with open(dest, "w") as fh:
        json.dump(tr, fh, indent=1)
    print("wrote", dest, tr)
