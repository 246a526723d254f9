"""Score-only quad traceback round statistics (debug build with -DSA_TB_STATS, `make stats` ->
tools/bin/libstats.so): per wave, rounds (block recomputes), walk-loop iterations, moves, and where
the wave's cycles go (recompute load wait, sub-step loop, the rest = walk).
    python3 tools/so4_stats.py [pairs=10000]"""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SEQALIB_HIP_LIB"] = os.path.join(ROOT, "tools", "bin", os.environ.get("SO4_STATS_LIB", "libstats.so"))
os.environ.setdefault("SEQALIB_KERNEL_TIMING", "1")
sys.path.insert(0, ROOT)
import numpy as np, torch
import seqalib_amd as sa
L = sa.load_library()
P, n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000, 4096
s1, o1, s2, o2 = sa.synth_dna_batch(10**10, P, n, n, threads=16)
dev = torch.device("cuda", 0)
t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
d1, do1, d2, do2 = t(s1), t(o1), t(s2), t(o2)
res = torch.zeros(P * 32, dtype=torch.uint8, device=dev); ops = torch.zeros(len(s1) + len(s2) + P, dtype=torch.uint8, device=dev)
eng = sa.Engine(0)
out = (C.c_ulonglong * 8)()
ec = (C.c_ulonglong * 8)()
for it in range(2):
    L.sa_debug_so4_stats(out, 1)
    L.sa_debug_ecso_stats(ec, 1)
    eng.align_device(0, sa.ScoringSystem(-1, 1, -1), d1.data_ptr(), do1.data_ptr(), d2.data_ptr(), do2.data_ptr(), P, n, n,
                     res.data_ptr(), ops.data_ptr(), 0)
    torch.cuda.synchronize()
    f, tb, _ = eng.last_timings()
    L.sa_debug_so4_stats(out, 1)
    L.sa_debug_ecso_stats(ec, 1)
    ep = max(ec[0], 1)
    kf, ks = eng.last_kernel_timings()
    print(f"end cell: {ks - kf:.3f} ms, {ec[0]} pairs, {ec[1] / ep:.1f} candidate lane blocks per pair, {ec[2]} dense fallbacks, "
          f"{ec[3] / ep:.0f} cycles per wave = to first scan load {ec[4] / ep:.0f} + first level {ec[5] / ep:.0f} + "
          f"second level {ec[6] / ep:.0f} + replay {(ec[3] - ec[4] - ec[5] - ec[6]) / ep:.0f}; longest wave {ec[7]}")
    rounds, iters, moves, cyc, wait, sub, nsub, waves = list(out)
    w = max(waves, 1)
    print(f"pairs {P} fill {f:.2f} ms tb {tb:.2f} ms | per wave: rounds {rounds / w:.0f} iters {iters / w:.0f} "
          f"moves/pair {moves / P:.0f} cycles {cyc / w:.0f} = load wait {wait / w:.0f} + sub-steps {sub / w:.0f} "
          f"({nsub / max(rounds, 1):.1f} per round, {sub / max(nsub, 1):.0f} cycles each) + walk/other "
          f"{(cyc - wait - sub) / w:.0f} ({(cyc - wait - sub) / max(iters, 1):.0f} cycles per iteration)")
