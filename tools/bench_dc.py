#!/usr/bin/env python3
"""Linear-space aligner batch timing: P pairs of L x L synthetic
DNA, inputs resident in HBM, sa_align_batch_device(SA_HIRSCHBERG or SA_MYERS_MILLER).  Reports
alignment-cell rate (m*n per pair / wall time; the linear-space methods sweep ~2*m*n cells) and,
when oracle/_ref is present, the reference's own aligner on a CPU sample.
    python3 tools/bench_dc.py --algo hb --pairs 1000 --len 4096
    python3 tools/bench_dc.py --algo mm --pairs 1000 --len 4096
"""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1000)
    ap.add_argument("--len", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cpu-pairs", type=int, default=4)
    ap.add_argument("--algo", choices=("hb", "mm"), default="hb")
    a = ap.parse_args()
    import torch
    import seqalib_amd as sa
    from util import oracle_align
    P, L = a.pairs, a.len
    s1, o1, s2, o2 = sa.synth_dna_batch(7 * 10 ** 9, P, L, L, threads=16)
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    d1, do1, d2, do2 = t(s1), t(o1), t(s2), t(o2)
    res = torch.zeros(P * 32, dtype=torch.uint8, device=dev)
    ops = torch.zeros(len(s1) + len(s2) + P, dtype=torch.uint8, device=dev)
    eng = sa.Engine(0)
    algo = sa.SA_HIRSCHBERG if a.algo == "hb" else sa.SA_MYERS_MILLER
    args = (-1, 2, -1) if a.algo == "hb" else (-3, -1, 1, -1, True)
    sc = sa.ScoringSystem(*args)
    run = lambda: eng.align_device(algo, sc, d1.data_ptr(), do1.data_ptr(), d2.data_ptr(), do2.data_ptr(),
                                   P, L, L, res.data_ptr(), ops.data_ptr(), 0)
    run(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    r = np.frombuffer(res.cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE)
    hops = ops.cpu().numpy()
    ok = 0
    for p in (0, P - 1):
        x, y = s1[o1[p]:o1[p + 1]].tobytes(), s2[o2[p]:o2[p + 1]].tobytes()
        o = oracle_align(algo, args, x, y)
        off = int(o1[p] + o2[p]) + p
        ok += int((int(r["score"][p]), hops[off:off + int(r["nops"][p])].tobytes()) == (o["score"], o["ops"]))
    name = "HirschbergSA" if a.algo == "hb" else "MyersMillerSA"
    line = {"metric": f"{name} alignment cells/s (m*n per pair)", "pairs": P, "len": L,
            "ms_per_batch": round(dt * 1e3, 2), "gcups": round(P * L * L / dt / 1e9, 1),
            "parity": f"{ok}/2 sampled pairs bit-exact vs oracle"}
    ref = os.path.join(ROOT, "oracle", "_ref", "libsaref.so")
    if os.path.exists(ref) and a.cpu_pairs:
        import ctypes as C
        Lr = C.CDLL(ref)
        class RefOut(C.Structure):
            _fields_ = [("score", C.c_int32), ("max_row", C.c_int32), ("max_col", C.c_int32), ("len", C.c_int32)]
        cap = 2 * L + 4
        bufs = [C.create_string_buffer(cap) for _ in range(3)]
        t0 = time.perf_counter()
        for p in range(a.cpu_pairs):
            x, y = s1[o1[p]:o1[p + 1]].tobytes(), s2[o2[p]:o2[p + 1]].tobytes()
            oo = RefOut()
            if a.algo == "hb":
                Lr.ref_align(4, 3, -1, 2, -1, 0, 1, 0, None, x, len(x), y, len(y), C.byref(oo), *bufs, cap)
            else:
                Lr.ref_align(5, 5, -3, -1, 1, -1, 1, 0, None, x, len(x), y, len(y), C.byref(oo), *bufs, cap)
        cdt = time.perf_counter() - t0
        line["cpu_reference_gcups_1thread"] = round(a.cpu_pairs * L * L / cdt / 1e9, 4)
        line["cpu_sample"] = (f"{a.cpu_pairs} pairs, reference {name}"
                              + (" (includes one NW score pass)" if a.algo == "hb" else "") + ", 1 thread")
    print(json.dumps(line))


if __name__ == "__main__":
    main()
