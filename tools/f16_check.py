#!/usr/bin/env python3
"""Round 6 debugging aid: the f16 cell against the 16-bit cell (SEQALIB_SO2_F16=0) on ragged SW
batches, per plan: mismatching pairs, split by half (even / odd pair index) and band count."""
import os
import sys

import numpy as np

_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [_R, os.path.join(_R, "tests")]
import seqalib_amd as sa
from test_gpu_so import ragged_batch

eng = sa.Engine(0)
for plan in (None, "16,1"):
    for maxlen in (2000, 3000, 4096):
        if plan:
            os.environ["SEQALIB_PLAN"] = plan
        else:
            os.environ.pop("SEQALIB_PLAN", None)
        b = ragged_batch(90 + maxlen, 1100, maxlen)
        os.environ.pop("SEQALIB_SO2_F16", None)
        r1, _ = eng.align_packed(0, sa.ScoringSystem(-1, 1, -1), *b)
        r1 = r1.copy()
        p1 = eng.last_plan()
        os.environ["SEQALIB_SO2_F16"] = "0"
        r2, _ = eng.align_packed(0, sa.ScoringSystem(-1, 1, -1), *b)
        r2 = r2.copy()
        os.environ.pop("SEQALIB_SO2_F16", None)
        bad = np.nonzero((r1["score"] != r2["score"]) | (r1["end_i"] != r2["end_i"]) | (r1["end_j"] != r2["end_j"]))[0]
        m = np.diff(b[1])
        BAND = 64 * p1[1]
        bands = (m + BAND - 1) // BAND
        partner = np.where(np.arange(len(m)) % 2 == 1, np.roll(bands, 1), np.roll(bands, -1))
        print("   bad pairs whose partner has fewer bands:", int((partner[bad] < bands[bad]).sum()), "of", len(bad),
              "; such odd pairs in the batch:", int(((np.arange(len(m)) % 2 == 1) & (partner < bands)).sum()), flush=True)
        print(plan, maxlen, p1, "bad", len(bad), "odd", int((bad % 2).sum()), "m>2048", int((m[bad] > 2048).sum()),
              "m>1024", int((m[bad] > 1024).sum()), [(int(p), int(r1["score"][p]), int(r2["score"][p]), int(m[p])) for p in bad[:4]], flush=True)
