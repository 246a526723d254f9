#!/usr/bin/env python3
"""Floor of the SPLIT plan for one pair (BASELINE configs 2 and 4).

A SPLIT fill runs B = m / (64 R) bands, one wave each; band b+1's lane 0 needs band b's lane 63 at
the same column, so the last band's last lane finishes after n + 64 B - 1 = n + m / R dependent
steps whatever the hand-off costs.  This measures the release build's step time t(R) of a lone
band (one pair of 64 R rows: the fill kernel's time at n and n / 2 columns, differenced so launch
and reduce drop out) and prints the floor (n + m / R) x t(R) beside the full pair's fill kernel.

    SEQALIB_KERNEL_TIMING=1 python3 tools/split_floor.py [--out profiles/split_floor_r06.json]
"""
import argparse
import json
import os
import sys

os.environ.setdefault("SEQALIB_KERNEL_TIMING", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import seqalib_amd as sa  # noqa: E402
from bench_configs import Runner  # noqa: E402

CASES = [("config 2: SW (-1,1,-1) 4096^2", sa.SA_SW, (-1, 1, -1), 4096, 2 * 10 ** 9),
         ("config 4: LocalGotoh (-3,-1,1,-1,false) 8192^2", sa.SA_LOCAL_GOTOH, (-3, -1, 1, -1, False), 8192, 4 * 10 ** 9)]


def fill_kernel_ms(r, algo, args, m, n, seed, plan):
    if plan:
        os.environ["SEQALIB_PLAN"] = plan
    else:
        os.environ.pop("SEQALIB_PLAN", None)
    s1, o1, s2, o2 = sa.synth_dna_batch(seed, 1, m, n)
    d, outs, cnt = r.put(s1, o1, s2, o2)
    r.time_calls(algo, sa.ScoringSystem(*args), d, outs, cnt, m, n, 20, False)
    plan_used = list(r.eng.last_plan())
    return r.fill_kernel_ms, plan_used


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = sa.Engine(0)
    r = Runner(sa, torch, eng, dev)
    rows = []
    for name, algo, args, n, seed in CASES:
        full_default, plan_default = fill_kernel_ms(r, algo, args, n, n, seed, None)
        for R in (1, 2, 4):
            t_full, _ = fill_kernel_ms(r, algo, args, 64 * R, n, seed + 1, f"{R},0")
            t_half, _ = fill_kernel_ms(r, algo, args, 64 * R, n // 2, seed + 1, f"{R},0")
            t_step_ns = (t_full - t_half) / (n // 2) * 1e6
            steps = n + n // R
            floor_ms = steps * t_step_ns / 1e6
            fk, plan = fill_kernel_ms(r, algo, args, n, n, seed, f"{R},0")
            row = {"case": name, "R": R, "bands": n // (64 * R), "lone_band_step_ns": round(t_step_ns, 1),
                   "critical_steps": steps, "floor_ms": round(floor_ms, 3), "fill_kernel_ms": round(fk, 3),
                   "fill_over_floor": round(fk / floor_ms, 3), "plan": plan}
            rows.append(row)
            print(json.dumps(row), flush=True)
        rows.append({"case": name, "default_plan": plan_default, "fill_kernel_ms": round(full_default, 3)})
        print(json.dumps(rows[-1]), flush=True)
    os.environ.pop("SEQALIB_PLAN", None)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"note": "tools/split_floor.py on one MI355X: floor (n + m/R) x lone-band step time vs the "
                               "SPLIT fill kernel (HIP events)", "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
