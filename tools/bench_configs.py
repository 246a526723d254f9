#!/usr/bin/env python3
"""BASELINE.json configs 2-5 on one MI355X, measured like bench.py's headline (inputs resident in
HBM, device API, fill + end cell + traceback per call), each with its oracle parity and the
reference CPU path (oracle/_ref, the reference compiled in place) beside it.  bench.py runs these
after its headline timed region and puts them in its JSON line under "configs"; run alone it prints
one JSON line per config.

  config 2  1 x 4096^2 SW (-1,1,-1)                    one pair: latency of one call; ref 1 thread
  config 3  10,000 x 1024^2 SW                         batch GCUPS; every pair's end cell vs oracle
  config 4  1 x 8192^2 LocalGotoh (-3,-1,1,-1,false)   one pair (and the 4-argument scoring's
                                                       allowMismatch = true); ref 1 thread
  config 5  12,500 x 2048^2 SW                         one GPU's shard of 100,000 pairs over 8
  nw/lg/gg  10,000 x 1024^2 NW (-1,2,-1), LocalGotoh / GlobalGotoh (-3,-1,1,-1,true): the score-only
            fill and the tagged one beside it, every pair vs the full-matrix oracle
  gotoh     10,000 x 1024^2 Local/GlobalGotoh          T16 affine vs int32 kernel (tuning, not in bench)

Seeds: config c uses base c x 1e9.  Reference semantics: SASmithWaterman.h:358-366
and SALocalGotoh.h:518-526 (getAlignment), include/Test.cpp:119-135.
    python3 tools/bench_configs.py [--only 2,3,4,5,gotoh]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "libsaref.so")
SW = (-1, 1, -1)


class RefOut(C.Structure):
    _fields_ = [("score", C.c_int32), ("max_row", C.c_int32), ("max_col", C.c_int32), ("len", C.c_int32)]


def ref_lib():
    L = C.CDLL(REF)
    L.ref_call_ns.restype = C.c_double
    L.ref_call_ns.argtypes = [C.c_int] * 6 + [C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_int]
    vp = C.c_void_p
    L.ref_sw_batch.argtypes = [C.c_int] * 4 + [vp, vp, vp, vp, C.c_int, C.c_int, vp]
    return L


def ref_one(algo, args, a, b):
    """The reference's getAlignment path on one pair, 1 thread (cacheAllMatches, computeScoreMatrix,
    buildResult, as ref_align drives it): seconds."""
    L = C.CDLL(REF)
    n5 = len(args) == 5
    a0, a1, a2 = args[0], args[1], args[2]
    a3 = args[3] if n5 else 0
    allow = int(args[4]) if n5 else (int(args[3]) if len(args) == 4 else 1)
    cap = len(a) + len(b) + 4
    bufs = [C.create_string_buffer(cap) for _ in range(3)]
    o = RefOut()
    t0 = time.perf_counter()
    rc = L.ref_align(algo, 5 if n5 else len(args), a0, a1, a2, a3, allow, 1, None, a, len(a), b, len(b), C.byref(o),
                     *bufs, cap)
    dt = time.perf_counter() - t0
    assert rc == 0
    return dt


def ref_batch_sw(s1, o1, s2, o2, k, threads):
    """The reference's SmithWatermanSA::getAlignment over the first k pairs on `threads` threads:
    (GCUPS, seconds)."""
    L = ref_lib()
    sub1, sub2 = s1[: int(o1[k])].copy(), s2[: int(o2[k])].copy()
    so1, so2 = o1[: k + 1].copy(), o2[: k + 1].copy()
    out = np.zeros(k, dtype=np.int32)
    t0 = time.perf_counter()
    L.ref_sw_batch(*SW, 1, sub1.ctypes.data, so1.ctypes.data, sub2.ctypes.data, so2.ctypes.data, k, threads,
                   out.ctypes.data)
    dt = time.perf_counter() - t0
    cells = float(np.sum((so1[1:] - so1[:-1]).astype(np.float64) * (so2[1:] - so2[:-1])))
    return cells / dt / 1e9, dt


class Runner:
    """Device buffers and timed device-API calls on one engine (the caller's)."""

    def __init__(self, sa, torch, eng, dev):
        self.sa, self.torch, self.eng, self.dev = sa, torch, eng, dev
        self.stream = torch.cuda.current_stream(dev)

    def put(self, s1, o1, s2, o2):
        t = lambda x: self.torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(self.dev)
        n = len(o1) - 1
        outs = [(self.torch.zeros(n * 32, dtype=self.torch.uint8, device=self.dev),
                 self.torch.zeros(len(s1) + len(s2) + n, dtype=self.torch.uint8, device=self.dev))
                for _ in range(self.sa.SA_PIPELINE_DEPTH)]
        return [t(x) for x in (s1, o1, s2, o2)], outs, n

    def time_calls(self, algo, sc, dev_in, outs, n, m_max, n_max, steps, pipeline):
        d = dev_in
        self.eng.set_pipeline(pipeline)
        call = lambda k: self.eng.align_device(algo, sc, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                               d[3].data_ptr(), n, m_max, n_max, outs[k % len(outs)][0].data_ptr(),
                                               outs[k % len(outs)][1].data_ptr(), self.stream.cuda_stream)
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
        fill_ms, tb_ms, _ = self.eng.last_timings()   # fill stream (fill + end cell), traceback stream
        try:
            self.fill_kernel_ms = self.eng.last_kernel_timings()[0]   # the fill kernel(s) alone
        except Exception:   # (SEQALIB_KERNEL_TIMING unset)
            self.fill_kernel_ms = None
        return dt, (steps - 1) % len(outs), fill_ms, tb_ms

    def fk(self):
        return {"fill_kernel_ms": round(self.fill_kernel_ms, 3) if self.fill_kernel_ms is not None else None}

    def results(self, outs, k):
        res = np.frombuffer(outs[k][0].cpu().numpy().tobytes(), dtype=self.sa.RESULT_DTYPE)
        return res, outs[k][1].cpu().numpy()


def parity_full(algo, args, s1, o1, s2, o2, res, ops, idx, threads):
    """Full results and op streams of pairs idx against the full-matrix oracle."""
    from util import oracle_batch, subset
    sub = subset(s1, o1, s2, o2, idx)
    ores, oops = oracle_batch(algo, args, *sub, threads=threads)
    ok = 0
    for q, p in enumerate(idx):
        off = int(o1[p] + o2[p]) + int(p)
        ooff = int(sub[1][q] + sub[3][q]) + q
        got = (int(res["score"][p]), int(res["end_i"][p]), int(res["end_j"][p]), int(res["start_i"][p]),
               int(res["start_j"][p]), ops[off:off + int(res["nops"][p])].tobytes())
        exp = (int(ores["score"][q]), int(ores["end_i"][q]), int(ores["end_j"][q]), int(ores["start_i"][q]),
               int(ores["start_j"][q]), oops[ooff:ooff + int(ores["nops"][q])].tobytes())
        ok += int(got == exp)
    return ok


def parity_sw_batch(s1, o1, s2, o2, res, ops, n_ops, threads, seed):
    """SW batch parity: every pair's (MaxScore, MaxRow, MaxCol) vs the linear-space oracle, every
    alignment re-scored, n_ops full op streams vs the full-matrix oracle."""
    from util import linear_rescore, oracle_sw_scores
    P = len(o1) - 1
    t0 = time.perf_counter()
    exp = oracle_sw_scores(SW, s1, o1, s2, o2, threads=threads)
    got = np.stack([res["score"][:P], res["end_i"][:P], res["end_j"][:P]], axis=1)
    ends_ok = int(np.count_nonzero((got == exp).all(axis=1)))
    rescore_ok = int(np.count_nonzero(linear_rescore(SW, res[:P], ops, o1, o2) == res["score"][:P]))
    idx = np.unique(np.concatenate([[0, P - 1], np.random.default_rng(seed).choice(P, max(0, n_ops - 2), replace=False)]))
    ops_ok = parity_full(0, SW, s1, o1, s2, o2, res, ops, idx, threads)
    return {"end_cells": f"{ends_ok}/{P}", "rescored": f"{rescore_ok}/{P}", "op_streams": f"{ops_ok}/{len(idx)}",
            "flagged": int(np.count_nonzero(res["flags"][:P])), "check_s": round(time.perf_counter() - t0, 1),
            "exact": ends_ok == P and rescore_ok == P and ops_ok == len(idx)}


def measure(sa, torch, eng, dev, only=("2", "3", "4", "5"), threads=16):
    """Configs 2-5: a list of dicts (one per measured workload)."""
    r = Runner(sa, torch, eng, dev)
    have_ref = os.path.exists(REF)
    out = []
    if "2" in only:   # single 4096^2 SW pair
        s1, o1, s2, o2 = sa.synth_dna_batch(2 * 10 ** 9, 1, 4096, 4096)
        d, outs, n = r.put(s1, o1, s2, o2)
        dt, k, fill_ms, tb_ms = r.time_calls(sa.SA_SW, sa.ScoringSystem(*SW), d, outs, n, 4096, 4096, 20, False)
        res, ops = r.results(outs, k)
        line = {"config": 2, "workload": "1 x 4096^2 SW (-1,1,-1)", "ms_per_call": round(dt * 1e3, 3),
                "gcups": round(4096 * 4096 / dt / 1e9, 1), "fill_ms": round(fill_ms, 3),
                "traceback_ms": round(tb_ms, 3), **r.fk(), "plan": list(eng.last_plan()),
                "parity": f"{parity_full(0, SW, s1, o1, s2, o2, res, ops, [0], 1)}/1 pair bit-exact "
                          "(score, end cell, start cell, op stream)"}
        if have_ref:
            cdt = ref_one(0, SW, s1.tobytes(), s2.tobytes())
            line["cpu_reference"] = {"ms": round(cdt * 1e3, 1), "cores": 1, "speedup": round(cdt / dt, 1)}
        out.append(line)
        del d, outs
    if "3" in only:   # 10,000 x 1024^2 SW
        P = 10000
        s1, o1, s2, o2 = sa.synth_dna_batch(3 * 10 ** 9, P, 1024, 1024, threads=threads)
        d, outs, n = r.put(s1, o1, s2, o2)
        sc = sa.ScoringSystem(*SW)
        dtp, k, fill_ms, tb_ms = r.time_calls(sa.SA_SW, sc, d, outs, n, 1024, 1024, 10, True)
        res, ops = r.results(outs, k)
        dts, _, _, _ = r.time_calls(sa.SA_SW, sc, d, outs, n, 1024, 1024, 5, False)
        cells = P * 1024 * 1024
        line = {"config": 3, "workload": "10,000 x 1024^2 SW (-1,1,-1)", "gcups": round(cells / dtp / 1e9, 1),
                "ms_per_step": round(dtp * 1e3, 3), "serial_ms_per_step": round(dts * 1e3, 3),
                "fill_ms": round(fill_ms, 3), "fill_gcups": round(cells / (r.fill_kernel_ms or fill_ms) / 1e6, 1),
                "traceback_ms": round(tb_ms, 3), **r.fk(), "plan": list(eng.last_plan()),
                "parity": parity_sw_batch(s1, o1, s2, o2, res, ops, 16, threads, 3)}
        if have_ref:
            g, cdt = ref_batch_sw(s1, o1, s2, o2, 32 * threads, threads)
            line["cpu_reference"] = {"gcups": round(g, 3), "cores": threads, "speedup": round(cells / dtp / 1e9 / g, 1),
                                     "sample": f"first {32 * threads} pairs, {cdt:.2f} s"}
        out.append(line)
        del d, outs
    if "4" in only:   # single 8192^2 LocalGotoh pair: BASELINE's !allowMismatch and allowMismatch = true
        s1, o1, s2, o2 = sa.synth_dna_batch(4 * 10 ** 9, 1, 8192, 8192)
        d, outs, n = r.put(s1, o1, s2, o2)
        for args in ((-3, -1, 1, -1, False), (-3, -1, 1, -1, True)):
            dt, k, fill_ms, tb_ms = r.time_calls(sa.SA_LOCAL_GOTOH, sa.ScoringSystem(*args), d, outs, n, 8192, 8192,
                                                 10, False)
            res, ops = r.results(outs, k)
            line = {"config": 4, "workload": f"1 x 8192^2 LocalGotoh ({','.join(str(x).lower() for x in args)})",
                    "ms_per_call": round(dt * 1e3, 3), "gcups": round(8192 * 8192 / dt / 1e9, 1),
                    "fill_ms": round(fill_ms, 3), "traceback_ms": round(tb_ms, 3), **r.fk(), "plan": list(eng.last_plan()),
                    "parity": f"{parity_full(2, args, s1, o1, s2, o2, res, ops, [0], 1)}/1 pair bit-exact "
                              "(score, end cell, start cell, op stream)"}
            if have_ref:
                cdt = ref_one(2, args, s1.tobytes(), s2.tobytes())
                line["cpu_reference"] = {"ms": round(cdt * 1e3, 1), "cores": 1, "speedup": round(cdt / dt, 1)}
            out.append(line)
        del d, outs
    if "5" in only:   # per-GPU shard of 100,000 x 2048^2
        P = 12500
        s1, o1, s2, o2 = sa.synth_dna_batch(5 * 10 ** 9, P, 2048, 2048, threads=threads)
        d, outs, n = r.put(s1, o1, s2, o2)
        dtp, k, fill_ms, tb_ms = r.time_calls(sa.SA_SW, sa.ScoringSystem(*SW), d, outs, n, 2048, 2048, 6, True)
        res, ops = r.results(outs, k)
        cells = P * 2048 * 2048
        line = {"config": 5, "workload": "12,500 x 2048^2 SW (one GPU's shard of 100,000 over 8)",
                "gcups": round(cells / dtp / 1e9, 1), "ms_per_step": round(dtp * 1e3, 3), "fill_ms": round(fill_ms, 3),
                "fill_gcups": round(cells / (r.fill_kernel_ms or fill_ms) / 1e6, 1), "traceback_ms": round(tb_ms, 3), **r.fk(),
                "plan": list(eng.last_plan()), "parity": parity_sw_batch(s1, o1, s2, o2, res, ops, 8, threads, 5)}
        if have_ref:
            g, cdt = ref_batch_sw(s1, o1, s2, o2, 8 * threads, threads)
            line["cpu_reference"] = {"gcups": round(g, 3), "cores": threads, "speedup": round(cells / dtp / 1e9 / g, 1),
                                     "sample": f"first {8 * threads} pairs, {cdt:.2f} s"}
        out.append(line)
        del d, outs
    for key, algo, name, args in (("nw", sa.SA_NW, "NeedlemanWunsch", (-1, 2, -1)),
                                  ("lg", sa.SA_LOCAL_GOTOH, "LocalGotoh", (-3, -1, 1, -1, True)),
                                  ("gg", sa.SA_GLOBAL_GOTOH, "GlobalGotoh", (-3, -1, 1, -1, True))):
        if key not in only:
            continue
        # 10,000 x 1024^2 batches of the other three aligners: the score-only fill (pipelined steps,
        # as the headline), the tagged-record fill beside it (SEQALIB_SO=0, serial calls), every
        # pair's full result and op stream against the full-matrix oracle, the reference beside it
        P = 10000
        s1, o1, s2, o2 = sa.synth_dna_batch(6 * 10 ** 9 + algo, P, 1024, 1024, threads=threads)
        d, outs, n = r.put(s1, o1, s2, o2)
        sc = sa.ScoringSystem(*args)
        cells = P * 1024 * 1024
        dtp, k, fill_ms, tb_ms = r.time_calls(algo, sc, d, outs, n, 1024, 1024, 10, True)
        fk_so = r.fill_kernel_ms
        plan = list(eng.last_plan_ex())
        res, ops = r.results(outs, k)
        os.environ["SEQALIB_SO"] = "0"
        try:
            dtt, _, _, _ = r.time_calls(algo, sc, d, outs, n, 1024, 1024, 3, False)
            fk_tag = r.fill_kernel_ms
        finally:
            os.environ.pop("SEQALIB_SO")
        t0 = time.perf_counter()
        ok = parity_full(algo, args, s1, o1, s2, o2, res, ops, np.arange(P), threads)
        line = {"config": key, "workload": f"10,000 x 1024^2 {name} ({','.join(str(x).lower() for x in args)})",
                "gcups": round(cells / dtp / 1e9, 1), "ms_per_step": round(dtp * 1e3, 3),
                "fill_ms": round(fill_ms, 3), "fill_gcups": round(cells / (fk_so or fill_ms) / 1e6, 1),
                "traceback_ms": round(tb_ms, 3), "fill_kernel_ms": round(fk_so, 3) if fk_so else None,
                "plan": plan, "records": "score-only" if plan[3] == sa.SA_RECORDS_SCORE_ONLY else "tagged",
                "tagged_fill_kernel_ms": round(fk_tag, 3) if fk_tag else None,
                "tagged_fill_gcups": round(cells / fk_tag / 1e6, 1) if fk_tag else None,
                "parity": {"pairs_bit_exact": f"{ok}/{P}", "what": "score, end cell, start cell and op stream of every "
                           "pair vs the full-matrix oracle", "check_s": round(time.perf_counter() - t0, 1),
                           "exact": ok == P}}
        if have_ref:
            from concurrent.futures import ThreadPoolExecutor
            ks = 16 * threads
            t0 = time.perf_counter()
            with ThreadPoolExecutor(threads) as ex:   # (ctypes releases the GIL)
                list(ex.map(lambda p: ref_one(algo, args, s1[o1[p]:o1[p + 1]].tobytes(), s2[o2[p]:o2[p + 1]].tobytes()),
                            range(ks)))
            cdt = time.perf_counter() - t0
            g = ks * 1024 * 1024 / cdt / 1e9
            line["cpu_reference"] = {"gcups": round(g, 3), "cores": threads, "speedup": round(cells / dtp / 1e9 / g, 1),
                                     "sample": f"first {ks} pairs, getAlignment per pair, {cdt:.2f} s"}
        out.append(line)
        del d, outs
    if "gotoh" in only:   # batched affine: T16 affine kernel vs the int32 kernel (SEQALIB_T16=0)
        P = 10000
        s1, o1, s2, o2 = sa.synth_dna_batch(6 * 10 ** 9, P, 1024, 1024, threads=threads)
        d, outs, n = r.put(s1, o1, s2, o2)
        cells = P * 1024 * 1024
        for algo, name in ((sa.SA_LOCAL_GOTOH, "LocalGotoh"), (sa.SA_GLOBAL_GOTOH, "GlobalGotoh")):
            args = (-3, -1, 1, -1, True)
            line = {"config": "gotoh", "workload": f"10,000 x 1024^2 {name} (-3,-1,1,-1,true)"}
            for kern, env in (("t16", "1"), ("int32", "0")):
                os.environ["SEQALIB_T16"] = env
                dtp, k, fill_ms, tb_ms = r.time_calls(algo, sa.ScoringSystem(*args), d, outs, n, 1024, 1024, 6, True)
                res, ops = r.results(outs, k)
                line[kern] = {"gcups": round(cells / dtp / 1e9, 1), "ms_per_step": round(dtp * 1e3, 2),
                              "fill_ms": round(fill_ms, 2), "fill_gcups": round(cells / (r.fill_kernel_ms or fill_ms) / 1e6, 1),
                              "traceback_ms": round(tb_ms, 2), "plan": list(eng.last_plan()),
                              "parity": f"{parity_full(algo, args, s1, o1, s2, o2, res, ops, [0, P // 2, P - 1], 3)}/3"}
            os.environ.pop("SEQALIB_T16")
            line["fill_speedup"] = round(line["int32"]["fill_ms"] / line["t16"]["fill_ms"], 2)
            out.append(line)
        del d, outs
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="2,3,4,5")
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import torch
    import seqalib_amd as sa
    eng = sa.Engine(0)
    for line in measure(sa, torch, eng, torch.device("cuda", 0), set(a.only.split(",")), a.threads):
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
