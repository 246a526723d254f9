#!/usr/bin/env python3
"""One headline step for profilers (rocprofv3 --pmc passes, tools/pmc_roofline.sh): the bench
workload (10,000 x 4096^2 SW (-1, 1, -1), seed base 1e10, inputs resident in HBM), --calls calls of
the device API without the cross-call pipeline.  No parity, configs or CPU legs (bench.py does
those); prints the last call's HIP-event fill / traceback times."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=10000)
    ap.add_argument("--len", type=int, default=4096)
    ap.add_argument("--calls", type=int, default=2)
    a = ap.parse_args()
    import torch
    import seqalib_amd as sa
    dev = torch.device("cuda", 0)
    s1, o1, s2, o2 = sa.synth_dna_batch(10 ** 10, a.pairs, a.len, a.len, threads=16)
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    d = [t(x) for x in (s1, o1, s2, o2)]
    res = torch.zeros(a.pairs * 32, dtype=torch.uint8, device=dev)
    ops = torch.zeros(len(s1) + len(s2) + a.pairs, dtype=torch.uint8, device=dev)
    eng = sa.Engine(0)
    st = torch.cuda.current_stream(dev)
    for _ in range(a.calls):
        eng.align_device(sa.SA_SW, sa.ScoringSystem(-1, 1, -1), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                         d[3].data_ptr(), a.pairs, a.len, a.len, res.data_ptr(), ops.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    print("fill_ms %.3f endcell+traceback_ms %.3f launches %d" % eng.last_timings(), "plan", eng.last_plan_ex())


if __name__ == "__main__":
    main()
