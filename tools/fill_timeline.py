#!/usr/bin/env python3
"""Schedule of the many-pairs score-only fill (debug build: `make stats`, tools/bin/libstats.so,
-DSA_TB_STATS): every workgroup's start / end (s_memrealtime, 100 MHz) and the SIMD it ran on
(HW_ID, XCC_ID).  Prints, per batch size, the kernel span, per-generation wave durations (waves
ordered by start; generation g = waves 4096 g .. 4096 g + 4095 at 4 waves per SIMD), and how many
waves a SIMD holds over time.  Not part of the product."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SEQALIB_HIP_LIB", os.path.join(ROOT, "tools", "bin", "libstats.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,10000,12288")
    ap.add_argument("--len", type=int, default=4096)
    a = ap.parse_args()
    import torch
    import seqalib_amd as sa
    L = sa.load_library()
    L.sa_debug_fill_stats_sw.argtypes = [C.c_void_p, C.c_int]
    dev = torch.device("cuda", 0)
    eng = sa.Engine(0)
    st = torch.cuda.current_stream(dev).cuda_stream
    sc = sa.ScoringSystem(-1, 1, -1)
    buf = np.zeros((32768, 3), dtype=np.uint64)
    for P in [int(x) for x in a.sizes.split(",") if x]:
        s1, o1, s2, o2 = sa.synth_dna_batch(10 ** 10, P, a.len, a.len, threads=16)
        t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
        d = [t(x) for x in (s1, o1, s2, o2)]
        res = torch.zeros(P * 32, dtype=torch.uint8, device=dev)
        ops = torch.zeros(len(s1) + len(s2) + P, dtype=torch.uint8, device=dev)
        for rep in range(2):
            L.sa_debug_fill_stats_sw(buf.ctypes.data, 1)
            eng.align_device(0, sc, *[x.data_ptr() for x in d], P, a.len, a.len, res.data_ptr(), ops.data_ptr(), st)
            torch.cuda.synchronize()
        L.sa_debug_fill_stats_sw(buf.ctypes.data, 0)
        # band units (score-only fills): one entry per (band, pair) unit, band-major
        _, _, W = eng.last_plan()
        units = min(32768, P * max(1, -(-a.len // (64 * eng.last_plan()[1]))))
        b = buf[:units].astype(np.int64)
        P = units
        t0, t1, hw = b[:, 0], b[:, 1], b[:, 2]
        ok = (t0 > 0) & (t1 >= t0)
        base = t0[ok].min()
        st_us, en_us = (t0 - base) / 100.0, (t1 - base) / 100.0
        dur = en_us - st_us
        order = np.argsort(st_us, kind="stable")
        gens = []
        for g in range(0, P, 4096):
            idx = order[g:g + 4096]
            gens.append({"gen": g // 4096, "waves": int(len(idx)), "start_us": [round(float(st_us[idx].min()), 1), round(float(st_us[idx].max()), 1)],
                         "dur_us_mean": round(float(dur[idx].mean()), 1), "dur_us_min": round(float(dur[idx].min()), 1),
                         "dur_us_max": round(float(dur[idx].max()), 1)})
        simd = ((hw >> 32) << 16) | ((hw >> 4) & 0xfff)   # XCC, SE/SH/CU/SIMD fields of HW_ID
        nsimd = len(np.unique(simd[ok]))
        # waves resident per SIMD over time (sampled every 100 us): mean over SIMDs
        span = float(en_us[ok].max())
        ts = np.arange(0.0, span, 100.0)
        res_mean = [round(float(((st_us[ok] <= t) & (en_us[ok] > t)).sum()) / nsimd, 2) for t in ts]
        print(json.dumps({"pairs": P, "valid": int(ok.sum()), "simds": int(nsimd), "span_us": round(span, 1),
                          "dur_us_mean": round(float(dur[ok].mean()), 1), "generations": gens,
                          "resident_waves_per_simd_every_100us": res_mean}), flush=True)


if __name__ == "__main__":
    main()
