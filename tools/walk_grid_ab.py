"""A/B of the persistent walk kernel's grid size: run bench.py with the grid capped at ``cap`` workgroups (4 waves
each; 0 = the default one round of resident workgroups, 512 on MI355X) through tm_debug_set(TM_DEBUG_WALK_BLOCKS).

    python tools/walk_grid_ab.py CAP [bench.py arguments]"""
import runpy
import sys

sys.path.insert(0, ".")
from tempme_amd import _lib as L  # noqa: E402

cap = int(sys.argv[1])
L.check(L.lib().tm_debug_set(L.TM_DEBUG_WALK_BLOCKS, cap), "tm_debug_set")
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path("bench.py", run_name="__main__")
