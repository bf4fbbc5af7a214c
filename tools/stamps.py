"""Debug: run bench.py once under a -DTM_STAMPS build (TEMPME_LIB=tempme_amd/lib/ab/<name>.so) and print
the average cycles per phase of events_kernel (per (event, side)) and of walk_kernel per pass type
(s_memtime deltas of lane 0)."""
import ctypes as C
import runpy
import sys

sys.argv = ["bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-extras"] + sys.argv[1:]
runpy.run_path("bench.py", run_name="__main__")
from tempme_amd import _lib  # noqa: E402

ev = (C.c_ulonglong * 16)()
if hasattr(_lib.lib(), "tm_debug_event_stamps"):   # sampler.hip built with -DTM_STAMPS too
    assert _lib.lib().tm_debug_event_stamps(ev) == 0
    n = max(1, ev[15])
    print("events_kernel n=%d" % ev[15], " ".join("%s=%.0f" % (nm, ev[k] / n) for k, nm in
                                                  enumerate(["hop1", "hop2_cuts", "hop2", "walks", "edge_counts"])))
    print("  walks:", " ".join("%s=%.0f" % (nm, ev[k] / n) for k, nm in
                               ((5, "clear+next_step"), (6, "final_loads"), (8, "final_filtered_counts"),
                                (9, "final_draw+kth"), (10, "final_rec"), (11, "final_ret"),
                                (12, "stores+hist+inserts"))))
buf = (C.c_ulonglong * 30)()
assert _lib.lib().tm_debug_stamps(buf) == 0
names = ["issue", "lin_event", "A/B", "g1", "relu", "next row", "folded gemms", "head/stash"]
for pt, pname in ((2, "slot p2"), (0, "walk p0"), (1, "walk p1")):
    row = buf[pt * 10:(pt + 1) * 10]
    n = max(1, row[8])
    print(pname, "n=%d" % row[8], " ".join("%s=%.0f" % (names[k], row[k] / n) for k in range(8)),
          "total=%.0f" % (sum(row[:8]) / n))
print("walk_kernel in-kernel clock %.3f GHz (s_memtime / s_memrealtime over each wave's pass loop)"
      % (0.1 * buf[9] / max(1, buf[19])))
print("walk_kernel mean wave pass-loop cycles %.0f over %d waves, %.1f us; max waves resident at once %d"
      % (buf[9] / max(1, buf[28]), buf[28], buf[19] / max(1, buf[28]) * 0.01, buf[29]))
