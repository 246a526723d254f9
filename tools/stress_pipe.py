#!/usr/bin/env python3
"""Debugging aid: the bench's pipelined device-API loop (two output sets, cross-call pipeline) on a
few-pairs (SPLIT) batch, every pair of every step checked against the oracle.
    python3 tools/stress_pipe.py PAIRS LEN ROUNDS [seed_base]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
import seqalib_amd as sa
from util import oracle_align

P, L, rounds = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
base = int(sys.argv[4]) if len(sys.argv) > 4 else 12345
args = (-1, 1, -1)
s1, o1, s2, o2 = sa.synth_dna_batch(base, P, L, L, threads=8)
dev = torch.device("cuda", 0)
t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
d1, do1, d2, do2 = t(s1), t(o1), t(s2), t(o2)
res = [torch.zeros(P * 32, dtype=torch.uint8, device=dev) for _ in range(2)]
ops = [torch.zeros(len(s1) + len(s2) + P, dtype=torch.uint8, device=dev) for _ in range(2)]
exp = [oracle_align(0, args, s1[o1[p]:o1[p + 1]].tobytes(), s2[o2[p]:o2[p + 1]].tobytes()) for p in range(P)]
eng = sa.Engine(0)
eng.set_pipeline(os.environ.get("NOPIPE") is None)
sc = sa.ScoringSystem(*args)
stream = torch.cuda.current_stream(dev).cuda_stream
nbad = 0
for rd in range(rounds):
    for k in range(2):
        eng.align_device(sa.SA_SW, sc, d1.data_ptr(), do1.data_ptr(), d2.data_ptr(), do2.data_ptr(), P, L, L,
                         res[k].data_ptr(), ops[k].data_ptr(), stream)
    eng.wait()
    torch.cuda.synchronize()
    for k in range(2):
        r = np.frombuffer(res[k].cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE)
        hops = ops[k].cpu().numpy()
        for p in range(P):
            off = int(o1[p] + o2[p]) + p
            got = (int(r["score"][p]), int(r["end_i"][p]), int(r["end_j"][p]), hops[off:off + int(r["nops"][p])].tobytes())
            e = exp[p]
            if got != (e["score"], e["end_i"], e["end_j"], e["ops"]) or r["flags"][p]:
                nbad += 1
                if nbad <= 8:
                    d = next((i for i, (x, y) in enumerate(zip(got[3], e["ops"])) if x != y), -1)
                    print(f"round {rd} set {k} pair {p}: got {got[:3]} nops {len(got[3])} flags {r['flags'][p]} "
                          f"want {(e['score'], e['end_i'], e['end_j'])} nops {len(e['ops'])} first op diff {d}", flush=True)
print(f"plan {eng.last_plan()}: {nbad} bad of {rounds * 2 * P}")
