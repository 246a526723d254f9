"""Host API (sa_align_batch) end-to-end phases on the headline batch: run with
SEQALIB_HOST_TIMING=1 to get the library's per-call phase line on stderr.
    SEQALIB_HOST_TIMING=1 python tools/host_api_timing.py [--pairs 10000] [--len 4096] [--reps 3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import seqalib_amd as sa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pairs", type=int, default=10000)
ap.add_argument("--len", type=int, default=4096)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
s1, o1, s2, o2 = sa.synth_dna_batch(3_000_000_000, a.pairs, a.len, a.len, threads=16)
eng = sa.Engine(0)
sc = sa.ScoringSystem(-1, 1, -1)
eng.align_packed(sa.SA_SW, sc, s1, o1, s2, o2)
for r in range(a.reps):
    t = time.perf_counter()
    res, ops = eng.align_packed(sa.SA_SW, sc, s1, o1, s2, o2)
    print(f"rep {r}: {1e3 * (time.perf_counter() - t):.2f} ms (python call incl. output allocation)", flush=True)
