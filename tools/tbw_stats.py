"""Wave-traceback statistics (debug build: `make stats`, copied to tools/bin/libstats.so).
    python3 tools/tbw_stats.py [pairs=1] [len=4096]"""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SEQALIB_HIP_LIB"] = os.path.join(ROOT, "tools", "bin", "libstats.so")
sys.path.insert(0, ROOT)
import numpy as np, torch
import seqalib_amd as sa
L = sa.load_library()
P = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
s1, o1, s2, o2 = sa.synth_dna_batch(2 * 10**9, P, n, n, threads=16)
dev = torch.device("cuda", 0)
t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
d1, do1, d2, do2 = t(s1), t(o1), t(s2), t(o2)
res = torch.zeros(P * 32, dtype=torch.uint8, device=dev); ops = torch.zeros(len(s1) + len(s2) + P, dtype=torch.uint8, device=dev)
eng = sa.Engine(0)
out = (C.c_ulonglong * 8)()
for it in range(3):
    L.sa_debug_tbw_stats(out, 1)
    eng.align_device(0, sa.ScoringSystem(-1, 1, -1), d1.data_ptr(), do1.data_ptr(), d2.data_ptr(), do2.data_ptr(), P, n, n, res.data_ptr(), ops.data_ptr(), 0)
    torch.cuda.synchronize()
    f, tb, _ = eng.last_timings()
    L.sa_debug_tbw_stats(out, 1)
    win, dec, cyc, moves, waves, runs, runm = list(out)[:7]
    waves = max(waves, 1)
    print(f"pairs {P} fill {f:.3f} ms tb {tb:.3f} ms | per wave: windows {win/waves:.0f} decode ticks {dec/waves:.0f} "
          f"total ticks {cyc/waves:.0f} moves {moves/waves:.0f} walk ticks/move {(cyc-dec)/max(moves,1):.1f} "
          f"decode ticks/window {dec/max(win,1):.0f} runs {runs/waves:.0f} run moves {runm/waves:.0f}", flush=True)
