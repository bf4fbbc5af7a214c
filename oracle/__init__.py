"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the TempME explanation hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything under ``oracle/``; the product package ``tempme_amd``
never does (it fails loudly when its HIP library is missing).
"""
