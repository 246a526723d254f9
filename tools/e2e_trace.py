#!/usr/bin/env python3
"""One host-API call on the headline batch (bench.py's e2e leg: sa_align_batch from pageable host
buffers), warm, with SEQALIB_HOST_TIMING phases; run under rocprofv3 --kernel-trace
--memory-copy-trace to see where the call's time goes beyond the device-API step."""
import os
import sys
import time

os.environ.setdefault("SEQALIB_HOST_TIMING", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import seqalib_amd as sa  # noqa: E402

P, L = 10000, 4096
s1, o1, s2, o2 = sa.synth_dna_batch(10 ** 10, P, L, L, threads=16)
eng = sa.Engine(0)
sc = sa.ScoringSystem(-1, 1, -1)
out = eng.align_packed(sa.SA_SW, sc, s1, o1, s2, o2)
for k in range(3):
    t = time.perf_counter()
    out = eng.align_packed(sa.SA_SW, sc, s1, o1, s2, o2, out=out)
    print(f"call {k}: {(time.perf_counter() - t) * 1e3:.2f} ms", flush=True)
