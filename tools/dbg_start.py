#!/usr/bin/env python3
"""Debugging aid: SW / LocalGotoh pairs through one plan (SEQALIB_PLAN) against the oracle, with
and without start-mode steps (SEQALIB_NO_START); prints the first mismatches.
    python3 tools/dbg_start.py sw 2,0 1500 24"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import seqalib_amd as sa
from util import oracle_align

algo_name, plan, L, count = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
A, args = (sa.SA_SW, (-1, 1, -1)) if algo_name == "sw" else (sa.SA_LOCAL_GOTOH, (-3, -1, 1, -1, True))
os.environ["SEQALIB_PLAN"] = plan
eng = sa.Engine(0)
pairs = [(sa.synth_dna(1000 + 2 * k, L), sa.synth_dna(1001 + 2 * k, L)) for k in range(count)]
exp = [oracle_align(A, args, a, b) for a, b in pairs]
for ns in (1, 0):
    if ns: os.environ["SEQALIB_NO_START"] = "1"
    else: os.environ.pop("SEQALIB_NO_START", None)
    res = eng.align(A, sa.ScoringSystem(*args), pairs)
    bad = []
    for k, (r, o) in enumerate(zip(res, exp)):
        got = (r.score, r.end_i, r.end_j, r.start_i, r.start_j)
        want = (o["score"], o["end_i"], o["end_j"], o["start_i"], o["start_j"])
        if got != want or r.ops != o["ops"]:
            d = next((i for i, (x, y) in enumerate(zip(r.ops, o["ops"])) if x != y), min(len(r.ops), len(o["ops"])))
            bad.append((k, got, want, len(r.ops), len(o["ops"]), d))
    print(f"no_start={ns} plan={eng.last_plan()} bad {len(bad)}/{count}")
    for b in bad[:6]:
        print("   pair %d got %s want %s nops %d/%d first op diff at %d" % b)
