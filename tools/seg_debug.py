#!/usr/bin/env python3
"""Debugging aid for the segmented traceback (sa_traceback_seg.hip): align one long pair with
SEQALIB_TB=seg and SEQALIB_SEG_DUMP set, then follow the dumped exit records from the end cell
band by band next to the oracle's path (where it crosses each band's top row, how many ops it
emits inside the band).  Prints the first band where they disagree.

    python3 tools/seg_debug.py ALGO R M N [mutate]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import seqalib_amd as sa  # noqa: E402
from util import oracle_align  # noqa: E402

SC = {0: (-1, 1, -1), 1: (-1, 2, -1), 2: (-3, -1, 1, -1, True), 3: (-3, -1, 1, -1, True)}


def main():
    algo, R, m, n = (int(x) for x in sys.argv[1:5])
    mut = len(sys.argv) > 5
    a = sa.synth_dna(5, m)
    b = sa.synth_mutate(a, 3)[:n] if mut else sa.synth_dna(6, n)
    dump = os.path.join(ROOT, "gpurun_out", f"seg_dump_{algo}.bin")
    os.environ["SEQALIB_TB"] = "seg"
    os.environ["SEQALIB_PLAN"] = f"{R},0"
    os.environ["SEQALIB_SEG_DUMP"] = dump
    eng = sa.Engine()
    args = SC[algo]
    r = eng.align(algo, sa.ScoringSystem(*args), [(a, b)])[0]
    o = oracle_align(algo, args, a, b)
    print("gpu", r.score, r.end_i, r.end_j, r.start_i, r.start_j, len(r.ops))
    print("ora", o["score"], o["end_i"], o["end_j"], o["start_i"], o["start_j"], len(o["ops"]))
    raw = np.fromfile(dump, dtype=np.uint8)
    cnt, bands, rs, RR = np.frombuffer(raw[:32].tobytes(), dtype=np.uint64)
    rec = np.frombuffer(raw[32:].tobytes(), dtype=np.int32).reshape(-1, 4)
    fin = rec[cnt * bands * rs:]
    rec = rec[:cnt * bands * rs].reshape(cnt, bands, rs, 4)
    print("dump: cnt", cnt, "bands", bands, "rs", rs, "R", RR, "fin", fin[0])
    BR = 64 * R
    nst0 = 2 if algo >= 2 else 1
    W0 = int(rs - 1) // nst0
    body = rec[0, :-1, :W0 * nst0].reshape(int(bands) - 1, nst0, W0, 4)[:, :, :n + 1]
    nops = body[..., 2].astype(np.int64)
    waves = nops[..., : (n + 1) // 64 * 64].reshape(nops.shape[0], nst0, -1, 64)
    print(f"walk lengths: mean {nops.mean():.1f}, p99 {np.percentile(nops, 99):.0f}, max {nops.max()}; "
          f"per-wave max: mean {waves.max(axis=-1).mean():.1f}, max {waves.max()}")
    nst = 2 if algo >= 2 else 1
    W = int(rs - 1) // nst
    for bb in range(min(3, int(bands))):
        band = int(bands) - 2 - bb
        if band < 0:
            break
        for st in range(nst):
            rr = rec[0, band, st * W: st * W + n + 1]
            ex = (rr[:, 3] & 1) == 0
            print(f"band {band} st {st}: exits {int(ex.sum())}, exit rows {np.unique(rr[ex, 0])[:5]}, "
                  f"stop rows {np.unique(rr[~ex, 0])[:8]}, err {int(((rr[:, 3] & 16) != 0).sum())}")
        print("  samples", rec[0, band, [0, 1, n // 2, n, W, W + 1, W + n // 2, W + n]].tolist() if nst == 2 else rec[0, band, [0, 1, n // 2, n]].tolist())
    # oracle path crossings
    i, j = (o["end_i"], o["end_j"]) if algo in (0, 2) else (m, n)
    ops = o["ops"]
    cross = {}
    k0 = 0
    for k, op in enumerate(ops):
        c = chr(op)
        if c in "MSX":
            i -= 1; j -= 1
        elif c in "Uu":
            i -= 1
        elif c in "Ll":
            j -= 1
        if i % BR == 0 and i > 0 and c in "MSXUu":
            cross[i // BR] = (i, j, k + 1 - k0)
            k0 = k + 1
    be = ((o["end_i"] if algo in (0, 2) else m) - 1) // BR
    idx = rs - 1
    for cb in range(be, 0, -1):
        x = rec[0, cb, idx]
        e = cross.get(cb)
        print(f"band {cb}: rec i={x[0]} j={x[1]} nops={x[2]} w={x[3]:#x} | oracle {e}")
        if x[3] & 1:
            print("  stopped")
            break
        cj, cst = x[1], (x[3] >> 2) & 3
        if cj == 0 or cst == 2:
            cst = 0
        idx = cst * (int(rs - 1) // (2 if algo >= 2 else 1)) + cj
        if e is None or e[1] != x[1]:
            print("  DIVERGES here")
            break


if __name__ == "__main__":
    main()
