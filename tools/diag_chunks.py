"""Diagnostic: host-API results vs the oracle for a ragged SPLIT batch under different host
chunkings / traceback flavours (which pairs differ, and how)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import seqalib_amd as sa
from util import oracle_align

algo = int(sys.argv[1]) if len(sys.argv) > 1 else 0
args = {0: (-1, 1, -1), 1: (-1, 2, -1), 2: (-3, -1, 1, -1, False), 3: (-3, -1, 1, -1, True)}[algo]
rng = np.random.default_rng(70 + algo)
pairs = []
for k in range(157):
    m = int(rng.integers(0, 500))
    a = sa.synth_dna(50_000 + 2 * k, m)
    b = sa.synth_mutate(a, k)[: int(rng.integers(0, 520))] if k % 3 else sa.synth_dna(50_001 + 2 * k, int(rng.integers(0, 500)))
    pairs.append((a, b))
eng = sa.Engine(0)
sc = sa.ScoringSystem(*args)
for env in ({"SEQALIB_HOST_CHUNKS": "1"}, {"SEQALIB_HOST_CHUNKS": "3"}, {"SEQALIB_HOST_CHUNKS": "3", "SEQALIB_TB": "wave"},
            {"SEQALIB_HOST_CHUNKS": "1", "SEQALIB_TB": "seg"}, {"SEQALIB_HOST_CHUNKS": "1", "SEQALIB_TB": "seg", "SEQALIB_T16": "0"}):
    for k in ("SEQALIB_HOST_CHUNKS", "SEQALIB_TB", "SEQALIB_T16"):
        os.environ.pop(k, None)
    os.environ.update(env)
    res = eng.align(algo, sc, pairs)
    bad = []
    for p, ((a, b), r) in enumerate(zip(pairs, res)):
        o = oracle_align(algo, args, a, b)
        got = (r.score, r.end_i, r.end_j, r.start_i, r.start_j, r.ops)
        exp = (o["score"], o["end_i"], o["end_j"], o["start_i"], o["start_j"], o["ops"])
        if got != exp:
            diff = next((i for i in range(min(len(r.ops), len(o["ops"]))) if r.ops[i] != o["ops"][i]), None)
            bad.append((p, len(a), len(b), got[:5], exp[:5], len(r.ops), len(o["ops"]), diff, r.flags))
    print(env, "plan", eng.last_plan(), "bad", len(bad), flush=True)
    for x in bad[:6]:
        print("   ", x, flush=True)
