"""Debug aid: HB / MM pairs through the byte path (16-bit sweeps on, SEQALIB_DC16 from the
environment) against the oracle -- prints the pairs whose score or op stream differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import seqalib_amd as sa  # noqa: E402
from util import oracle_align  # noqa: E402

eng = sa.Engine(0)
pairs = [(sa.synth_dna(300 + k, 200 + 37 * k), sa.synth_dna(400 + k, 180 + 29 * k)) for k in range(40)]
for algo, args in ((4, (-1, 2, -1)), (5, (-3, -1, 1, -1))):
    res = eng.align(algo, sa.ScoringSystem(*args), pairs)
    bad = []
    for k, ((a, b), r) in enumerate(zip(pairs, res)):
        o = oracle_align(algo, args, a, b)
        if (r.score, r.ops) != (o["score"], o["ops"]):
            bad.append((k, len(a), len(b), r.score, o["score"], r.ops == o["ops"]))
    print(f"algo {algo} DC16={os.environ.get('SEQALIB_DC16', '1')}: {len(bad)} bad of {len(pairs)}: {bad[:8]}")
