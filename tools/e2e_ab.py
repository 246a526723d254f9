#!/usr/bin/env python3
"""Host-API end to end (bench.py's e2e leg: sa_align_batch from pageable host buffers, headline
batch) under A/B switches read per call, alternating in one process:
    python3 tools/e2e_ab.py "base;SEQALIB_XFER2=0" [rounds] [calls]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import seqalib_amd as sa  # noqa: E402

variants = [v for v in sys.argv[1].split(";") if v]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 4
s1, o1, s2, o2 = sa.synth_dna_batch(10 ** 10, 10000, 4096, 4096, threads=16)
eng = sa.Engine(0)
sc = sa.ScoringSystem(-1, 1, -1)
out = eng.align_packed(sa.SA_SW, sc, s1, o1, s2, o2)
ref = (out[0].copy(), out[1].copy())
keys = {kv.split("=")[0] for v in variants if v != "base" for kv in v.split(",")}
for r in range(rounds):
    for v in variants:
        for k in keys:
            os.environ.pop(k, None)
        if v != "base":
            for kv in v.split(","):
                k, x = kv.split("=", 1)
                os.environ[k] = x
        ts = []
        for _ in range(calls):
            t = time.perf_counter()
            out = eng.align_packed(sa.SA_SW, sc, s1, o1, s2, o2, out=out)
            ts.append((time.perf_counter() - t) * 1e3)
        same = bool((out[0] == ref[0]).all() and (out[1] == ref[1]).all())
        print(json.dumps({"variant": v, "round": r, "ms": [round(x, 2) for x in ts], "min": round(min(ts), 2),
                          "median": round(sorted(ts)[len(ts) // 2], 2), "same": same}), flush=True)
