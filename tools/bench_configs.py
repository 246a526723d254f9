#!/usr/bin/env python3
"""Every BASELINE.json config that fits one MI355X, measured the same way as bench.py (inputs
resident in HBM, device API, fill + traceback per step), with a parity check and the reference
CPU path beside it.  One JSON line per config; tools/profile.sh-style evidence for DESIGN.md §2.5.

  config 2  1 x 4096^2 SW (-1,1,-1)              single pair: latency of one call
  config 3  10,000 x 1024^2 SW                   batch GCUPS (pipelined and serial)
  config 4  1 x 8192^2 LocalGotoh (-3,-1,1,-1,F)  single pair
  config 5  12,500 x 2048^2 SW                   the per-GPU shard of 100,000 pairs over 8 GPUs
  gotoh     10,000 x 1024^2 LocalGotoh / GlobalGotoh (-3,-1,1,-1,true): T16 affine vs int32 kernel
  drop-in   C++ SmithWatermanSA::getAlignments, 1,000 x 4096^2, end-to-end incl. std::list build

Seeds: config c uses base c x 1e9.  CPU figures come from oracle/_ref (the
reference compiled in place) when present, else they are omitted.
    python3 tools/bench_configs.py [--only 2,3,4,5,dropin]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "libsaref.so")


class RefOut(C.Structure):
    _fields_ = [("score", C.c_int32), ("max_row", C.c_int32), ("max_col", C.c_int32), ("len", C.c_int32)]


def ref_one(algo, args, a, b):
    """Time the reference's getAlignment on one pair (1 thread)."""
    L = C.CDLL(REF)
    n5 = len(args) == 5
    a0, a1, a2 = args[0], args[1], args[2]
    a3 = args[3] if n5 else 0
    allow = int(args[4]) if n5 else 1
    cap = len(a) + len(b) + 4
    bufs = [C.create_string_buffer(cap) for _ in range(3)]
    o = RefOut()
    t0 = time.perf_counter()
    rc = L.ref_align(algo, 5 if n5 else 3, a0, a1, a2, a3, allow, 1, None, a, len(a), b, len(b), C.byref(o),
                     *bufs, cap)
    dt = time.perf_counter() - t0
    assert rc == 0
    return dt, o.score


def ref_batch_sw(s1, o1, s2, o2, k, threads):
    L = C.CDLL(REF)
    vp = C.c_void_p
    L.ref_sw_batch.argtypes = [C.c_int] * 4 + [vp, vp, vp, vp, C.c_int, C.c_int, vp]
    sub1, sub2 = s1[: int(o1[k])].copy(), s2[: int(o2[k])].copy()
    so1, so2 = o1[: k + 1].copy(), o2[: k + 1].copy()
    out = np.zeros(k, dtype=np.int32)
    t0 = time.perf_counter()
    L.ref_sw_batch(-1, 1, -1, 1, sub1.ctypes.data, so1.ctypes.data, sub2.ctypes.data, so2.ctypes.data, k, threads,
                   out.ctypes.data)
    dt = time.perf_counter() - t0
    cells = float(np.sum((so1[1:] - so1[:-1]).astype(np.float64) * (so2[1:] - so2[:-1])))
    return cells / dt / 1e9, dt


class Runner:
    def __init__(self, sa, torch):
        self.sa, self.torch = sa, torch
        self.dev = torch.device("cuda", 0)
        self.eng = sa.Engine(0)
        self.stream = torch.cuda.current_stream(self.dev)

    def put(self, s1, o1, s2, o2):
        t = lambda x: self.torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(self.dev)
        n = len(o1) - 1
        outs = [(self.torch.zeros(n * 32, dtype=self.torch.uint8, device=self.dev),
                 self.torch.zeros(len(s1) + len(s2) + n, dtype=self.torch.uint8, device=self.dev)) for _ in range(2)]
        return [t(x) for x in (s1, o1, s2, o2)], outs, n

    def time_calls(self, algo, sc, dev_in, outs, n, m_max, n_max, steps, pipeline):
        d = dev_in
        self.eng.set_pipeline(pipeline)
        call = lambda k: self.eng.align_device(algo, sc, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                               d[3].data_ptr(), n, m_max, n_max, outs[k % 2][0].data_ptr(),
                                               outs[k % 2][1].data_ptr(), self.stream.cuda_stream)
        for k in range(2):
            call(k)
        self.eng.wait()
        self.torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            call(k)
        self.eng.wait()
        self.torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        self.eng.set_pipeline(False)
        fill_ms, tb_ms, _ = self.eng.last_timings()
        return dt, (steps - 1) % 2, fill_ms, tb_ms

    def results(self, outs, k):
        res = np.frombuffer(outs[k][0].cpu().numpy().tobytes(), dtype=self.sa.RESULT_DTYPE)
        return res, outs[k][1].cpu().numpy()


def parity(sa, algo, args, s1, o1, s2, o2, res, ops, idx):
    from util import oracle_align
    ok = 0
    for p in idx:
        a, b = s1[o1[p]:o1[p + 1]].tobytes(), s2[o2[p]:o2[p + 1]].tobytes()
        o = oracle_align(algo, args, a, b)
        off = int(o1[p] + o2[p]) + p
        got = (int(res["score"][p]), int(res["end_i"][p]), int(res["end_j"][p]),
               ops[off:off + int(res["nops"][p])].tobytes())
        ok += int(got == (o["score"], o["end_i"], o["end_j"], o["ops"]))
    return f"{ok}/{len(idx)} pairs bit-exact vs oracle (score, end cell, op stream)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="2,3,4,5,dropin")
    a = ap.parse_args()
    only = set(a.only.split(","))
    import torch
    import seqalib_amd as sa
    r = Runner(sa, torch)
    have_ref = os.path.exists(REF)

    if "2" in only:   # single 4096^2 SW pair
        s1, o1, s2, o2 = sa.synth_dna_batch(2 * 10 ** 9, 1, 4096, 4096)
        d, outs, n = r.put(s1, o1, s2, o2)
        sc = sa.ScoringSystem(-1, 1, -1)
        dt, k, fill_ms, tb_ms = r.time_calls(sa.SA_SW, sc, d, outs, n, 4096, 4096, 20, False)
        res, ops = r.results(outs, k)
        line = {"config": 2, "workload": "1 x 4096^2 SW (-1,1,-1)", "ms_per_call": round(dt * 1e3, 3),
                "gcups": round(4096 * 4096 / dt / 1e9, 1), "fill_ms": round(fill_ms, 3), "traceback_ms": round(tb_ms, 3),
                "plan": r.eng.last_plan(), "parity": parity(sa, 0, (-1, 1, -1), s1, o1, s2, o2, res, ops, [0])}
        if have_ref:
            cdt, _ = ref_one(0, (-1, 1, -1), s1.tobytes(), s2.tobytes())
            line["cpu_reference_ms_1thread"] = round(cdt * 1e3, 1)
        print(json.dumps(line), flush=True)

    if "3" in only:   # 10,000 x 1024^2 SW
        P = 10000
        s1, o1, s2, o2 = sa.synth_dna_batch(3 * 10 ** 9, P, 1024, 1024, threads=16)
        d, outs, n = r.put(s1, o1, s2, o2)
        sc = sa.ScoringSystem(-1, 1, -1)
        dtp, k, fill_ms, tb_ms = r.time_calls(sa.SA_SW, sc, d, outs, n, 1024, 1024, 10, True)
        dts, _, _, _ = r.time_calls(sa.SA_SW, sc, d, outs, n, 1024, 1024, 5, False)
        res, ops = r.results(outs, (5 - 1) % 2)
        cells = P * 1024 * 1024
        line = {"config": 3, "workload": "10,000 x 1024^2 SW (-1,1,-1)", "gcups": round(cells / dtp / 1e9, 1),
                "ms_per_step": round(dtp * 1e3, 2), "serial_ms_per_step": round(dts * 1e3, 2),
                "fill_ms": round(fill_ms, 2), "fill_gcups": round(cells / fill_ms / 1e6, 1),
                "traceback_ms": round(tb_ms, 2), "plan": r.eng.last_plan(),
                "parity": parity(sa, 0, (-1, 1, -1), s1, o1, s2, o2, res, ops, [0, P // 2, P - 1])}
        if have_ref:
            g, cdt = ref_batch_sw(s1, o1, s2, o2, 256, 16)
            line["cpu_reference_gcups"] = {"value": round(g, 3), "cores": 16, "sample": f"first 256 pairs, {cdt:.2f} s"}
        print(json.dumps(line), flush=True)
        del d, outs

    if "4" in only:   # single 8192^2 LocalGotoh pair: !allowMismatch (int32 kernel) and the
        # 4-argument ScoringSystem's allowMismatch = true (T16 affine kernel)
        s1, o1, s2, o2 = sa.synth_dna_batch(4 * 10 ** 9, 1, 8192, 8192)
        d, outs, n = r.put(s1, o1, s2, o2)
        for args in ((-3, -1, 1, -1, False), (-3, -1, 1, -1, True)):
            sc = sa.ScoringSystem(*args)
            dt, k, fill_ms, tb_ms = r.time_calls(sa.SA_LOCAL_GOTOH, sc, d, outs, n, 8192, 8192, 10, False)
            res, ops = r.results(outs, k)
            line = {"config": 4, "workload": f"1 x 8192^2 LocalGotoh ({','.join(str(x).lower() for x in args)})",
                    "ms_per_call": round(dt * 1e3, 3),
                    "gcups": round(8192 * 8192 / dt / 1e9, 1), "fill_ms": round(fill_ms, 3), "traceback_ms": round(tb_ms, 3),
                    "plan": r.eng.last_plan(), "parity": parity(sa, 2, args, s1, o1, s2, o2, res, ops, [0])}
            if have_ref:
                cdt, _ = ref_one(2, args, s1.tobytes(), s2.tobytes())
                line["cpu_reference_ms_1thread"] = round(cdt * 1e3, 1)
            print(json.dumps(line), flush=True)

    if "5" in only:   # per-GPU shard of 100,000 x 2048^2
        P = 12500
        s1, o1, s2, o2 = sa.synth_dna_batch(5 * 10 ** 9, P, 2048, 2048, threads=16)
        d, outs, n = r.put(s1, o1, s2, o2)
        sc = sa.ScoringSystem(-1, 1, -1)
        dtp, k, fill_ms, tb_ms = r.time_calls(sa.SA_SW, sc, d, outs, n, 2048, 2048, 6, True)
        res, ops = r.results(outs, k)
        cells = P * 2048 * 2048
        line = {"config": 5, "workload": "12,500 x 2048^2 SW (one GPU's shard of 100,000 over 8)",
                "gcups": round(cells / dtp / 1e9, 1), "ms_per_step": round(dtp * 1e3, 2), "fill_ms": round(fill_ms, 2),
                "fill_gcups": round(cells / fill_ms / 1e6, 1), "traceback_ms": round(tb_ms, 2), "plan": r.eng.last_plan(),
                "parity": parity(sa, 0, (-1, 1, -1), s1, o1, s2, o2, res, ops, [0, P - 1])}
        print(json.dumps(line), flush=True)
        del d, outs

    if "gotoh" in only:   # batched affine: T16 affine kernel vs the int32 kernel (SEQALIB_T16=0)
        P = 10000
        s1, o1, s2, o2 = sa.synth_dna_batch(6 * 10 ** 9, P, 1024, 1024, threads=16)
        d, outs, n = r.put(s1, o1, s2, o2)
        cells = P * 1024 * 1024
        for algo, name in ((sa.SA_LOCAL_GOTOH, "LocalGotoh"), (sa.SA_GLOBAL_GOTOH, "GlobalGotoh")):
            args = (-3, -1, 1, -1, True)
            sc = sa.ScoringSystem(*args)
            line = {"config": "gotoh", "workload": f"10,000 x 1024^2 {name} (-3,-1,1,-1,true)"}
            for kern, env in (("t16", "1"), ("int32", "0")):
                os.environ["SEQALIB_T16"] = env
                dtp, k, fill_ms, tb_ms = r.time_calls(algo, sc, d, outs, n, 1024, 1024, 6, True)
                res, ops = r.results(outs, k)
                line[kern] = {"gcups": round(cells / dtp / 1e9, 1), "ms_per_step": round(dtp * 1e3, 2),
                              "fill_ms": round(fill_ms, 2), "fill_gcups": round(cells / fill_ms / 1e6, 1),
                              "traceback_ms": round(tb_ms, 2), "plan": r.eng.last_plan(),
                              "parity": parity(sa, algo, args, s1, o1, s2, o2, res, ops, [0, P // 2, P - 1])}
            os.environ.pop("SEQALIB_T16")
            line["fill_speedup"] = round(line["int32"]["fill_ms"] / line["t16"]["fill_ms"], 2)
            print(json.dumps(line), flush=True)
        del d, outs

    if "dropin" in only:
        exe = os.path.join(ROOT, "tests", "cpp", "dropin_bench")
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp"), "dropin_bench"])
        out = subprocess.run([exe, "1000", "4096", "3"], capture_output=True, text=True, check=True).stdout
        print(out.strip(), flush=True)


if __name__ == "__main__":
    main()
