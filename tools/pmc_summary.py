"""Summarise rocprofv3 --pmc CSV passes (gpurun_out/<pass>/run_counter_collection.csv) per kernel INSTANCE
(full template arguments kept: events_kernel<true, 3> and the null model's events_kernel<true, 1> are
different kernels): mean counter value per dispatch and the dispatch count.  FETCH_SIZE/WRITE_SIZE are KB
(rocprofv3); on gfx950 FETCH_SIZE reads 1/2 of a wide coalesced stream's bytes (MI355X_MICROARCH.md §HBM)
-- reported raw and x2.

    python tools/pmc_summary.py gpurun_out --glob 'pmc_enron_*' [--out SUMMARY.json] [--traffic profiles/pmc_traffic_enron.json]

The summary JSON goes to --out (or stdout); every status message goes to stderr, so a redirected stdout
stays valid JSON.
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "gpurun_out"
pat = sys.argv[sys.argv.index("--glob") + 1] if "--glob" in sys.argv else "pmc[0-9]*"
# the names bench.py's HIP-event profiler uses for kernels whose symbol differs
BENCH_ALIAS = {"gate_reg_kernel": "gate_table_kernel", "gate_table_kernel": "gate_table_kernel"}

acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{root}/{pat}/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\((?!anonymous).*$", "", r["Kernel_Name"].replace("void ", "")).strip()
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in acc.items():
    if not k.startswith("tmk::"):
        continue
    out[k] = {c: sum(v) / len(v) for c, v in d.items()}
    x = out[k]
    x["dispatches"] = max(len(v) for v in d.values())
    if "SQ_VALU_MFMA_BUSY_CYCLES" in x and "GRBM_GUI_ACTIVE" in x:
        x["mfma_busy_frac_est"] = x["SQ_VALU_MFMA_BUSY_CYCLES"] / (x["GRBM_GUI_ACTIVE"] * 4 * 256 / 8)
    if "TCC_HIT_sum" in x:
        x["l2_hit_rate"] = x["TCC_HIT_sum"] / max(1.0, x["TCC_HIT_sum"] + x["TCC_MISS_sum"])
    if "FETCH_SIZE" in x:
        x["hbm_read_bytes_x2"] = x["FETCH_SIZE"] * 1024 * 2
    if "SQ_LDS_BANK_CONFLICT" in x and "SQ_INSTS_LDS" in x:
        x["lds_conflict_cycles_per_lds_inst"] = x["SQ_LDS_BANK_CONFLICT"] / max(1.0, x["SQ_INSTS_LDS"])
    if "SQ_WAIT_INST_ANY" in x and "SQ_WAVE_CYCLES" in x:
        x["wait_inst_any_per_wave_cycle"] = x["SQ_WAIT_INST_ANY"] / max(1.0, x["SQ_WAVE_CYCLES"])
if "--out" in sys.argv:
    with open(sys.argv[sys.argv.index("--out") + 1], "w") as fh:
        json.dump(out, fh, indent=1)
else:
    print(json.dumps(out, indent=1))
# --traffic FILE: per-launch HBM bytes (FETCH_SIZE x2 + WRITE_SIZE) of every instance, and for each name
# bench.py times the instance launched most often in this run (the bench kernel, not a one-off like the
# null model's), which bench.py reports as roofline.traffic for the config this PMC run measured
if "--traffic" in sys.argv:
    dest = sys.argv[sys.argv.index("--traffic") + 1]
    inst = {}
    for k, x in out.items():
        if "FETCH_SIZE" in x and "WRITE_SIZE" in x:
            inst[k] = {"bytes": int(round(x["FETCH_SIZE"] * 1024 * 2 + x["WRITE_SIZE"] * 1024)),
                       "dispatches": int(x["dispatches"])}
    by = {}
    for k, v in sorted(inst.items(), key=lambda kv: kv[1]["dispatches"]):
        short = k.replace("tmk::", "").split("<")[0]
        by[BENCH_ALIAS.get(short, short)] = v["bytes"]          # the most-dispatched instance wins
    with open(dest, "w") as fh:
        json.dump({"source": f"{root}/{pat}", "kernels": inst, "by_bench_name": by}, fh, indent=1)
    print("wrote", dest, by, file=sys.stderr)
