"""Debug: run bench.py once under a stamping walk_kernel build (TEMPME_LIB=.../stamp.so) and print the
average cycles per phase per pass type (s_memtime deltas of lane 0, blocks 512..1023)."""
import ctypes as C
import runpy
import sys

sys.argv = ["bench.py", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]
runpy.run_path("bench.py", run_name="__main__")
from tempme_amd import _lib  # noqa: E402

buf = (C.c_ulonglong * 30)()
assert _lib.lib().tm_debug_stamps(buf) == 0
names = ["issue", "xgen+ev_gemm", "A/B+gather", "g1", "g2+ep", "F ep", "W gemm", "head/stash"]
for pt, pname in ((2, "slot p2"), (0, "walk p0"), (1, "walk p1")):
    row = buf[pt * 10:(pt + 1) * 10]
    n = max(1, row[8])
    print(pname, "n=%d" % row[8], " ".join("%s=%.0f" % (names[k], row[k] / n) for k in range(8)),
          "total=%.0f" % (sum(row[:8]) / n))
