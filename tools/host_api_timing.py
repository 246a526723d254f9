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
ap.add_argument("--chunks", default="", help="comma list of SEQALIB_HOST_CHUNKS values to sweep")
a = ap.parse_args()
s1, o1, s2, o2 = sa.synth_dna_batch(3_000_000_000, a.pairs, a.len, a.len, threads=16)
eng = sa.Engine(0)
sc = sa.ScoringSystem(-1, 1, -1)
out = eng.align_packed(sa.SA_SW, sc, s1, o1, s2, o2)
for G in ([int(x) for x in a.chunks.split(",")] if a.chunks else [0]):
    if G:
        os.environ["SEQALIB_HOST_CHUNKS"] = str(G)
    out = eng.align_packed(sa.SA_SW, sc, s1, o1, s2, o2, out=out)   # warm this chunking
    ms = []
    for r in range(a.reps):
        t = time.perf_counter()
        out = eng.align_packed(sa.SA_SW, sc, s1, o1, s2, o2, out=out)   # the caller's buffers, reused
        ms.append(1e3 * (time.perf_counter() - t))
    print(f"chunks {G or 'default'}: " + " ".join(f"{x:.2f}" for x in ms) + f" ms, best {min(ms):.2f}", flush=True)
