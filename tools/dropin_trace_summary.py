"""Summarise a rocprofv3 --kernel-trace CSV of tools/dropin_timing.py (gpu_run.sh step ``dropintrace``):
the GPU-bound phase (everything after the last torch spin kernel) as per-kernel launch counts and mean
durations, the batch period (explain_hash3_kernel start to start), and the timeline of one batch in the
middle of the phase (start / end relative to the previous batch's explanation kernel, queue id) -- which
launches sit on the batch's critical path."""
import csv
import glob
import sys
from collections import defaultdict


def load(path):
    with open(path, newline="") as f:
        rows = list(csv.DictReader(f))
    q = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    out = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get(q, "?")) for r in rows]
    out.sort()
    return out


def short(name, n=70):
    name = name.replace("tmk::", "")
    return name if len(name) <= n else name[:n] + "..."


def main(path):
    ks = load(path)
    spins = [i for i, k in enumerate(ks) if "spin_kernel" in k[2]]
    ph = ks[spins[-1] + 1:] if spins else ks
    stat = defaultdict(list)
    for s, e, n, _ in ph:
        stat[n].append(e - s)
    print("GPU-bound phase: %d kernels" % len(ph))
    for n, d in sorted(stat.items(), key=lambda kv: -sum(kv[1])):
        print("  %5d x %8.2f us  %s" % (len(d), sum(d) / len(d) / 1e3, short(n)))
    ex = [i for i, k in enumerate(ph) if "explain_hash3" in k[2]]
    if len(ex) < 3:
        return
    per = [(ph[ex[j + 1]][0] - ph[ex[j]][0]) / 1e3 for j in range(len(ex) - 1)]
    print("batch period (explain start to start): median %.2f us, min %.2f us over %d batches"
          % (sorted(per)[len(per) // 2], min(per), len(per)))
    j = len(ex) // 2
    t0 = ph[ex[j - 1]][0]
    print("one batch (times from the previous batch's explanation kernel start, us):")
    for s, e, n, q in ph[ex[j - 1]:ex[j] + 1]:
        print("  q%-4s %8.2f -> %8.2f  (%6.2f)  %s" % (q, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, short(n)))


if __name__ == "__main__":
    p = sys.argv[1] if len(sys.argv) > 1 else sorted(glob.glob("gpurun_out/ditrace/**/*kernel_trace.csv",
                                                               recursive=True))[-1]
    main(p)
