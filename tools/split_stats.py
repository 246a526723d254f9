"""Timeline of the few-pairs (SPLIT) fill: per band of one pair, when its workgroup started and
ended and how long it polled for the band above (debug build with -DSA_TB_STATS, `make stats`,
copied to tools/bin/libstats.so).  Times in microseconds (s_memrealtime, 100 MHz).
    python3 tools/split_stats.py [sw|lg] [R ...]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SEQALIB_HIP_LIB"] = os.path.join(ROOT, "tools", "bin", "libstats.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import seqalib_amd as sa  # noqa: E402

algo = sys.argv[1] if len(sys.argv) > 1 else "sw"
Rs = [int(x) for x in sys.argv[2:]] or [2, 4]
L = sa.load_library()
fn = getattr(L, f"sa_debug_split_stats_{algo}")
eng = sa.Engine(0)
if algo == "sw":
    A, args, n = sa.SA_SW, (-1, 1, -1), 4096
else:
    A, args, n = sa.SA_LOCAL_GOTOH, (-3, -1, 1, -1, False), 8192
pairs = [(sa.synth_dna(1, n), sa.synth_dna(2, n))]
out = (C.c_ulonglong * (4096 * 16))()
EV = ["post71", "pub_sees", "pub_stored", "poll_has8", "cmp_has", "cmp_start"]
for R in Rs:
    os.environ["SEQALIB_PLAN"] = f"{R},0"
    for rep in range(2):
        fn(out, 1)
        eng.align(A, sa.ScoringSystem(*args), pairs)
        f, tb, _ = eng.last_timings()
        fn(out, 0)
    allst = np.frombuffer(out, dtype=np.uint64)
    st = allst[:4096 * 4].reshape(4096, 4)
    ev = allst[4096 * 4:].reshape(4096, 12)
    keep = st[:, 0] > 0
    st, ev = st[keep], ev[keep]
    order = np.argsort(st[:, 0])
    st, ev = st[order], ev[order]
    t0 = st[:, 1].min()
    start = (st[:, 1] - t0) / 100.0
    end = (st[:, 2] - t0) / 100.0
    wait = st[:, 3] / 100.0
    busy = end - start
    lag = np.diff(start)
    steps = n + 63
    print(f"{algo} {n}^2 R={R}: fill {f * 1e3:.0f} us (HIP events), traceback {tb * 1e3:.0f} us, {len(st)} bands; "
          f"band busy {busy.mean():.0f} us (min {busy.min():.0f}), polled {wait.mean():.0f} us on average; "
          f"start lag per band {lag.mean():.2f} us (median {np.median(lag):.2f}); "
          f"last band ends {end.max():.0f} us; step {busy.min() / steps * 1e3:.1f} ns in the fastest band")
    for b in list(range(0, min(4, len(st)))) + list(range(max(4, len(st) - 3), len(st))):
        print(f"   band {b:3d}: start {start[b]:8.1f}  end {end[b]:8.1f}  busy {busy[b]:7.1f}  polled {wait[b]:7.1f}")
    # hand-off chain of the granule at column 2048 (kEvCol), band b-1 -> band b (us): producer
    # compute posts it -> its publisher sees the post -> has issued the stores -> consumer poller
    # has it -> consumer compute has it (after asking for it at [6])
    rel = lambda x: (x.astype(np.int64) - int(t0)) / 100.0
    hops = []
    for b in range(1, len(st)):
        p, c = ev[b - 1], ev[b]
        if p[0] and p[1] and p[2] and c[3] and c[4] and c[6]:
            hops.append([rel(p[1]) - rel(p[0]), rel(p[2]) - rel(p[1]), rel(c[3]) - rel(p[2]), rel(c[4]) - rel(c[3]),
                         rel(c[4]) - rel(c[6]), rel(c[4]) - rel(p[0])])
    e0 = ev[0]
    if e0[7] and e0[5] and e0[8]:
        ns = (int(e0[5]) - int(e0[7])) / 100.0 / 64 * 1e3
        sd = (int(e0[8]) - int(e0[5])) / 100.0 / 256 * 1e3
        print(f"   band 0: chunks 0-1 (non-steady) {ns:.1f} ns per step, chunks 2-9 (steady) {sd:.1f} ns per step")
    if hops:
        h = np.array(hops)
        print(f"   hand-off of the granule at column 2048, median us: publisher wake {np.median(h[:, 0]):.2f}, "
              f"store issue {np.median(h[:, 1]):.2f}, store -> poller {np.median(h[:, 2]):.2f}, poller -> compute "
              f"{np.median(h[:, 3]):.2f}; compute waited {np.median(h[:, 4]):.2f} (mean {h[:, 4].mean():.2f}); "
              f"post -> consumer has it {np.median(h[:, 5]):.2f} (min {h[:, 5].min():.2f}, max {h[:, 5].max():.2f})")
