"""Debug: run tests/test_gpu_hoststage.py's functions one by one with a device round trip after each (and after a
garbage collection), to find the call that leaves a HIP error behind."""
import gc
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")


def probe(what):
    try:
        torch.zeros(1, device="cuda").cpu()
        torch.cuda.synchronize()
        print("ok  ", what, flush=True)
    except Exception as e:      # noqa: BLE001
        print("FAIL", what, repr(e)[:200], flush=True)
        sys.exit(1)


import test_gpu_hoststage as T  # noqa: E402

probe("start")
T.test_stage_cast_equals_numpy_astype()
probe("test 1")
gc.collect()
probe("test 1 gc")
T.test_stage_refuses_what_it_cannot_read_in_place()
probe("test 2")
gc.collect()
probe("test 2 gc")
T.test_host_pack_dropin_reads_pack_in_place(None)
probe("test 3")
gc.collect()
probe("test 3 gc")
from tempme_amd import hoststage as H  # noqa: E402
print("registered", [(e[2], e[3] is not None) for e in H._REG.regs.values()])
