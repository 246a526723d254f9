#!/usr/bin/env python3
"""Headline-fill A/B on one GPU (not part of the product): (1) fill-kernel time per pair against
the batch size (the launch tail: 4,096 single-wave workgroups are resident at 4 waves per SIMD);
(2) pipelined headline steps (bench.py's loop, device API, inputs in HBM) under A/B switches of
the engine (environment variables read per call), alternating so that every variant sees the same
box state.  Prints one JSON line per measurement."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402



def env_items(v):
    """'A=1,B=2,3' -> ['A=1', 'B=2,3']: a comma starts a new assignment only before KEY=."""
    out = []
    for part in v.split(","):
        if "=" in part or not out:
            out.append(part)
        else:
            out[-1] += "," + part
    return out

def batch(torch, dev, P, L, seed=10 ** 10, L1=None):
    import seqalib_amd as sa
    s1, o1, s2, o2 = sa.synth_dna_batch(seed, P, L1 or L, L, threads=16)
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    d = [t(x) for x in (s1, o1, s2, o2)]
    res = [torch.zeros(P * 32, dtype=torch.uint8, device=dev) for _ in range(sa.SA_PIPELINE_DEPTH)]
    ops = [torch.zeros(len(s1) + len(s2) + P, dtype=torch.uint8, device=dev) for _ in range(sa.SA_PIPELINE_DEPTH)]
    return d, res, ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,8192,10000,12288")
    ap.add_argument("--len", type=int, default=4096)
    ap.add_argument("--variants", default="base")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--algo", type=int, default=0, help="0 SW (-1,1,-1), 1 NW (-1,2,-1)")
    a = ap.parse_args()
    os.environ["SEQALIB_KERNEL_TIMING"] = "1"
    import torch
    import seqalib_amd as sa
    dev = torch.device("cuda", 0)
    eng = sa.Engine(0)
    st = torch.cuda.current_stream(dev).cuda_stream
    sc = sa.ScoringSystem(-1, 1, -1) if a.algo == 0 else sa.ScoringSystem(-1, 2, -1)
    L = a.len
    for spec in [x for x in a.sizes.split(",") if x]:
        P, m = (int(spec.split(":")[0]), int(spec.split(":")[1])) if ":" in spec else (int(spec), L)
        d, res, ops = batch(torch, dev, P, L, L1=m)
        best = 1e9
        for _ in range(3):
            eng.align_device(a.algo, sc, *[x.data_ptr() for x in d], P, m, L, res[0].data_ptr(), ops[0].data_ptr(), st)
            torch.cuda.synchronize()
            best = min(best, eng.last_kernel_timings()[0])
        print(json.dumps({"sweep": "fill_vs_pairs", "pairs": P, "m": m, "n": L, "fill_kernel_ms": round(best, 3),
                          "us_per_pair": round(best * 1e3 / P, 3), "gcups": round(P * m * L / best / 1e6, 1),
                          "plan": list(eng.last_plan())}), flush=True)
        del d, res, ops
        torch.cuda.empty_cache()
    P = 10000
    d, res, ops = batch(torch, dev, P, L)
    variants = [v for v in a.variants.split(";") if v]
    keys = sorted({kv.split("=")[0] for v in variants if v != "base" for kv in env_items(v)})
    eng.set_pipeline(True)
    for rnd in range(a.rounds):
        for v in variants:
            for k in keys:
                os.environ.pop(k, None)
            if v != "base":
                for kv in env_items(v):
                    k, x = kv.split("=", 1)
                    os.environ[k] = x
            for k in range(2):
                eng.align_device(a.algo, sc, *[x.data_ptr() for x in d], P, L, L, res[k % len(res)].data_ptr(), ops[k % len(ops)].data_ptr(), st)
            eng.wait()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.steps):
                eng.align_device(a.algo, sc, *[x.data_ptr() for x in d], P, L, L, res[k % len(res)].data_ptr(), ops[k % len(ops)].data_ptr(), st)
            eng.wait()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps * 1e3
            print(json.dumps({"sweep": "pipelined_step", "variant": v, "round": rnd, "ms_per_step": round(dt, 3),
                              "gcups": round(P * L * L / dt / 1e6, 1)}), flush=True)
    eng.set_pipeline(False)
    for k in keys:
        os.environ.pop(k, None)
    # parity of the last variant's output against a plain call
    r0 = np.frombuffer(res[(a.steps - 1) % len(res)].cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE).copy()
    eng.align_device(a.algo, sc, *[x.data_ptr() for x in d], P, L, L, res[0].data_ptr(), ops[0].data_ptr(), st)
    torch.cuda.synchronize()
    r1 = np.frombuffer(res[0].cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE)
    print(json.dumps({"check": "last pipelined variant == plain call", "equal": bool((r0 == r1).all())}), flush=True)


if __name__ == "__main__":
    main()
