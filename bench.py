#!/usr/bin/env python3
"""Benchmark: GCUPS of batched Smith-Waterman (linear gap) on MI355X — BASELINE.json's metric.

One "step" = one pass of the hot path (fill + traceback, i.e. getAlignment minus host list
assembly) over one batch of synthetic DNA pairs that is already resident in HBM.  Workload at
N=1 (north_star headline): 10,000 pairs of 4,096 x 4,096, ScoringSystem(-1, 1, -1) with
equal<char> — the same pairs the reference's SmithWatermanSA would see.

Multi-GPU: one process per GPU -- started by torch.distributed.run, or, when `--gpus N` is given
without a launcher, spawned by this script itself (spawn_ranks); rank r aligns its own 10,000-pair shard of a global
batch (pair p uses seeds base+2p+1 / base+2p+2), with no data-path collective (pairs are
independent); timing is barrier-bracketed (gloo, host memory: no RCCL anywhere) and the max over
ranks is reported.  scaling = weak.

Steps are pipelined (sa_set_pipeline; --no-pipeline turns it off): step k's traceback runs on
its own stream while step k+1's fill runs, with two workspace slots and two output buffer sets.
Every step's fill and traceback still lies inside the timed region (it ends with sa_wait + a
device synchronize); "serial_ms_per_step" reports the same step without overlap.

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "GCUPS (DP cell updates/s) on batched 4k×4k SW; bit-exact score match"
SEED_BASE = 10 ** 10          # workload "T" seed base (config id x 1e9 convention)
SCORING = (-1, 1, -1)         # SmithWatermanSA::getDefaultScoring (SASmithWaterman.h:352)
# The fill kernel is VALU-issue bound.  Its VALU instructions per cell come from an ISA count of
# the steady chunk loop (tools/issue_model.py -> ISSUE_MODEL).
ISSUE_MODEL = os.path.join(ROOT, "profiles", "issue_model_r06.json")
HBM_PEAK_GBPS = 8000.0
# VALU peak of the guide (/opt/skills/guides/MI355X_MICROARCH.md: 4 SIMD-32 per CU, a wave64 VALU
# instruction issues over 2 cycles, 2400 MHz max clock): 256 CU x 4 SIMD x 32 lanes x 2.4 GHz.
VALU_PEAK_TLANE = 256 * 4 * 32 * 2.4e9 / 1e12   # 78.64 T lane-instructions/s
SW_FLAG_BYTES_PER_CELL = 0.25  # 2 traceback bits per cell written to HBM


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=10000, help="pairs per GPU")
    ap.add_argument("--total-pairs", type=int, default=0,
                    help="strong scaling: a fixed global batch of this many pairs split over the ranks "
                         "(BASELINE config 5: --total-pairs 100000 --len 2048); 0 = --pairs per GPU (weak)")
    ap.add_argument("--len", type=int, default=4096, help="length of both sequences")
    ap.add_argument("--cpu-pairs", type=int, default=0,
                    help="CPU baseline sample, all-core leg (pairs; 0 = 64 per thread, ~10 s)")
    ap.add_argument("--cpu-pairs-1t", type=int, default=12, help="CPU baseline sample, 1-thread leg (pairs)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may use")
    ap.add_argument("--dropin-pairs", type=int, default=10000,
                    help="C++ drop-in end-to-end leg (tests/cpp/dropin_bench): pairs (0 = skip)")
    ap.add_argument("--dropin-reps", type=int, default=3)
    ap.add_argument("--e2e-steps", type=int, default=5,
                    help="host-API steps (H2D + fill + traceback + D2H of results and ops) timed after the run")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--out", default="", help="also write the JSON line to this file")
    ap.add_argument("--rank-out", default="",
                    help="directory: every rank writes rank<r>.json (its own time, shard and parity; tests)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run steps back to back without overlapping step k's traceback with step k+1's fill")
    ap.add_argument("--serial-steps", type=int, default=3,
                    help="after the timed run, also time this many non-pipelined steps (reported, not the value)")
    ap.add_argument("--configs", default="2,3,4,5,nw,lg,gg",
                    help="BASELINE.json configs measured after the headline (tools/bench_configs.py); '' = none")
    ap.add_argument("--parity-ops", type=int, default=16,
                    help="headline parity: full op streams checked against the full-matrix oracle "
                         "(every pair's end cell is always checked)")
    ap.add_argument("--latency-reps", type=int, default=200, help="drop-in single-call latency leg (0 = skip)")
    return ap.parse_args()


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE): start N rank processes of
    this script, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), as
    torch.distributed.run would.  This process touches no GPU and imports no torch: it only waits
    for the ranks (rank 0 prints the JSON line) and returns the first non-zero exit code; when one
    rank fails, the others are terminated instead of being left at a barrier."""
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # a line for N GPUs must come from N ranks: never report one rank's work as --gpus N
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} "
                         "(launch with torch.distributed.run --nproc-per-node N, or without a launcher)")
    import torch

    if world > 1:
        # pairs are independent: the data path has no collective at all; the timing barrier and
        # the max-over-ranks reduction go through gloo on host memory (no RCCL)
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if torch.cuda.is_available():
            torch.cuda.set_device(gpu_index(local))
        dist.init_process_group(backend="gloo")
    return world, rank, local


def gpu_index(local: int) -> int:
    """GPU of this rank: LOCAL_RANK, unless SEQALIB_BENCH_DEVICE pins every rank to one device
    (the multi-process test rehearses N ranks on a one-GPU box)."""
    return int(os.environ.get("SEQALIB_BENCH_DEVICE", local))


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_seed_base(rank: int, world: int, pairs_per_gpu: int) -> int:
    """Pair p of the global batch (world x P pairs) uses seeds SEED_BASE+2p+1 / +2p+2; rank r owns
    the contiguous slice seqalib_amd.multi.shard_range(r, world, world*P) — no exchange."""
    from seqalib_amd.multi import shard_range
    start, _ = shard_range(rank, world, world * pairs_per_gpu)
    return SEED_BASE + 2 * start


def rank_shard(rank: int, world: int, pairs_per_gpu: int, total_pairs: int, L: int):
    """(pairs, seed base, workload name) of this rank.  Weak scaling (total_pairs 0): every rank
    aligns pairs_per_gpu pairs of a world x pairs_per_gpu batch.  Strong scaling (BASELINE config 5,
    --total-pairs): the global batch is fixed and rank r aligns its contiguous slice
    (seqalib_amd.multi.shard_range).  Either way pair p of the global batch is seeded
    SEED_BASE + 2p + 1 / + 2, so the union of the shards is one batch whatever the rank count."""
    if total_pairs > 0:
        from seqalib_amd.multi import shard_range
        start, stop = shard_range(rank, world, total_pairs)
        return stop - start, SEED_BASE + 2 * start, f"sw_batch_{total_pairs}x{L}x{L}_strong"
    return pairs_per_gpu, shard_seed_base(rank, world, pairs_per_gpu), f"sw_batch_{pairs_per_gpu}x{L}x{L}"


def host_cores():
    """Cores this process may use: its CPU affinity, capped by the cgroup CPU quota (a GPU box
    shows the whole machine in os.cpu_count() but grants a share of it)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except Exception:
        pass
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cores": quota,
            "usable": min(aff, quota) if quota else aff}


def cpu_baseline(args, s1, o1, s2, o2, threads=None, pairs=None):
    """The reference (oracle/_ref, compiled from /root/reference) — or the oracle port if that is
    not built — on a bounded sample of the same pairs, on the host cores (all usable cores by
    default)."""
    hc = host_cores()
    threads = max(1, threads or args.cpu_threads or hc["usable"])
    k = min(pairs or args.cpu_pairs or 64 * threads, len(o1) - 1)
    sub1, sub2 = s1[: int(o1[k])].copy(), s2[: int(o2[k])].copy()
    so1, so2 = o1[: k + 1].copy(), o2[: k + 1].copy()
    cells = float(np.sum((so1[1:] - so1[:-1]).astype(np.float64) * (so2[1:] - so2[:-1])))
    ref = os.path.join(ROOT, "oracle", "_ref", "libsaref.so")
    out = np.zeros(k, dtype=np.int32)
    if os.path.exists(ref):
        L = C.CDLL(ref)
        vp = C.c_void_p
        L.ref_sw_batch.argtypes = [C.c_int] * 4 + [vp, vp, vp, vp, C.c_int, C.c_int, vp]
        t0 = time.perf_counter()
        L.ref_sw_batch(*SCORING, 1, sub1.ctypes.data, so1.ctypes.data, sub2.ctypes.data, so2.ctypes.data,
                       k, threads, out.ctypes.data)
        dt = time.perf_counter() - t0
        kind = "reference"
        what = "SmithWatermanSA<std::string,char,'-'>::getAlignment (unmodified reference headers, g++ -O2)"
    else:
        from util import OracleScoring, oracle_lib
        L = oracle_lib()
        sc = OracleScoring(SCORING[0], SCORING[1], SCORING[2], 0, 0, 1)
        t0 = time.perf_counter()
        L.oracle_sw_batch(C.byref(sc), sub1.ctypes.data, so1.ctypes.data, sub2.ctypes.data, so2.ctypes.data,
                          k, threads, out.ctypes.data)
        dt = time.perf_counter() - t0
        kind = "port"
        what = "oracle/sa_oracle.c SW (full-matrix restatement)"
    return {"value": round(cells / dt / 1e9, 4), "unit": "GCUPS", "cores": threads, "kind": kind,
            "nproc": hc["nproc"], "affinity": hc["affinity"], "cgroup_quota_cores": hc["cgroup_quota_cores"],
            "sample": f"first {k} pairs of this rank's batch ({args.len}x{args.len}), {what}, "
                      f"{threads} threads, {dt:.2f} s wall"}


def dropin_e2e(args):
    """The C++ drop-in exactly as a SeqALib user calls it (tests/cpp/dropin_bench.cpp:
    SmithWatermanSA<std::string, char, '-'>::getAlignments over host std::strings, symbol coding,
    host API (pinned chunked upload, fill, traceback, download) and every AlignedSequence's
    std::list), run as a child process after the timed region."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "cpp", "dropin_bench")
    if args.dropin_pairs <= 0 or not os.path.exists(exe):
        return None
    try:
        # SEQALIB_HOST_TIMING: the host phases of every getAlignments call on stderr (a few lines
        # per call), split per timed rep below
        env = dict(os.environ, SEQALIB_HOST_TIMING="1")
        r = subprocess.run([exe, str(args.dropin_pairs), str(args.len), str(args.dropin_reps)],
                           capture_output=True, text=True, timeout=300, check=True, env=env)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        d["phases_ms_each"] = dropin_phases(r.stderr)[1:]   # (the first call is the untimed warm-up)
        return d
    except Exception as e:   # reported, never fatal for the bench line
        return {"error": str(e)[:200]}


def dropin_phases(stderr: str):
    """Per getAlignments call, the host phases its SEQALIB_HOST_TIMING lines report (ms): symbol
    coding, match table + buffers, the GPU call (upload staging, waits, downloads, with the lists
    of landed ranges built beside it) and the lists left after it."""
    import re
    calls = []
    for line in stderr.splitlines():
        m = re.match(r"\[seqalib host\] (.+?)\s+([\d.]+) ms$", line)
        if m:
            name = m.group(1).strip()
            if name == "symbol coding":
                calls.append({})
            if calls:
                calls[-1][name] = float(m.group(2))
            continue
        m = re.search(r"\[seqalib host api\] \d+ pairs, \d+ chunks: ([\d.]+) ms = staging in ([\d.]+) \+ "
                      r"waiting ([\d.]+) \+ copies out ([\d.]+)", line)
        if m and calls:
            calls[-1].update({"api_total": float(m.group(1)), "api_staging_in": float(m.group(2)),
                              "api_waiting": float(m.group(3)), "api_copies_out": float(m.group(4))})
    return calls


def small_call_phases(stderr: str):
    """Host phases of the library's small-call path from its SEQALIB_HOST_TIMING lines
    ("... small-call kernel: T us = pinned buffer A + staging in B + launch C + kernel and sync D +
    copies out E"): the first call's, and the medians of the others."""
    import re
    names = ("total", "pinned_buffer", "staging_in", "launch", "kernel_and_sync", "copies_out")
    pat = re.compile(r"small-call kernel: ([\d.]+) us = pinned buffer ([\d.]+) \+ staging in ([\d.]+) \+ "
                     r"launch ([\d.]+) \+ kernel and sync ([\d.]+) \+ copies out ([\d.]+)")
    rows = [tuple(float(x) for x in m.groups()) for m in pat.finditer(stderr)]
    if not rows:
        return None
    rest = rows[1:] or rows
    med = [sorted(r[k] for r in rest)[len(rest) // 2] for k in range(len(names))]
    return {"first_call": dict(zip(names, rows[0])), "median": dict(zip(names, med)), "calls": len(rows)}


def dropin_latency(args):
    """Single-call latency of the C++ drop-in (tests/cpp/dropin_latency: getAlignment per call on
    test/Test.cpp's 11 x 8 NW pair and on one 1024^2 SW pair), beside the reference's own per-call
    time (oracle/_ref ref_call_ns: construct the aligner + getAlignment, as include/Test.cpp:98-107
    times it, 1 thread)."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "cpp", "dropin_latency")
    if args.latency_reps <= 0 or not os.path.exists(exe):
        return None
    try:
        out = subprocess.run([exe, str(args.latency_reps)], capture_output=True, text=True, timeout=300,
                             check=True).stdout
        d = json.loads(out.strip().splitlines()[-1])
        # host phases of the small call (a second run: printing them costs time per call)
        env = dict(os.environ, SEQALIB_HOST_TIMING="1")
        err = subprocess.run([exe, "100", "nw"], capture_output=True, text=True, timeout=300, check=True,
                             env=env).stderr
        d["nw_11x8"]["host_phases_us"] = small_call_phases(err)
    except Exception as e:   # reported, never fatal for the bench line
        return {"error": str(e)[:200]}
    ref = os.path.join(ROOT, "oracle", "_ref", "libsaref.so")
    if os.path.exists(ref):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from bench_configs import ref_lib
        import seqalib_amd as sa
        L = ref_lib()
        a, b = b"AAAGAATGCAT", b"AAACTCAT"
        d["nw_11x8"]["reference_us"] = round(L.ref_call_ns(1, 2, -1, 2, 0, 0, a, len(a), b, len(b), 20000) / 1e3, 3)
        x, y = sa.synth_dna(1_000_000_001, 1024), sa.synth_dna(1_000_000_002, 1024)
        d["sw_1024x1024"]["reference_us"] = round(L.ref_call_ns(0, 3, -1, 1, -1, 1, x, 1024, y, 1024, 5) / 1e3, 1)
        d["reference_basis"] = ("oracle/_ref ref_call_ns: SmithWatermanSA / NeedlemanWunschSA constructed + "
                                "getAlignment per call, 1 thread, mean")
    return d


def load_pmc(workload: str, label: str):
    """PMC figures of the shipped fill kernel (profiles/pmc_traffic.json, written by
    tools/pmc_roofline.py from separate rocprofv3 --pmc passes): HBM bytes per fill launch
    (FETCH_SIZE / WRITE_SIZE, gfx950-corrected) and the shader clock during the fill
    (GRBM_GUI_ACTIVE / 8 XCDs / duration).  Entries are keyed by workload and kernel label, so a
    record of another kernel is never reported for this one."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        e = json.load(open(path)).get(workload)
        return e if e is not None and e.get("label") == label else None
    except Exception:
        return None


def fill_streams(pairs: int, m: int, n: int, R: int, segs: int = 2):
    """Bytes the score-only SW fill moves per launch of `pairs` m x n pairs, stream by stream: every
    stream it writes and what it reads back or stages (sa_fill_impl.h BU / sa_fill_so2.hip; geometry
    of sa_layout.h)."""
    bands = -(-m // (64 * R))
    nch = (n + 63 + 31) // 32                       # chunks_per_band
    sg = max(1, min(segs, nch // 2))
    per = {
        "edge_stream": bands * nch * 32 * 64 * 2,          # 16 bits per lane-step, every step run
        "snapshots": bands * (nch - 1) * 64 * (R // 2 + 1) * 4,   # R/2 value words + the diagonal input
        "chunk_maxima": bands * nch * 64 * 4 + bands * nch * 4,  # per lane, and the wave's (snap_c)
        "band_rows": (bands - 1) * n * 4,                  # {tag, H} granules to the next band
        "segment_state": bands * (sg - 1) * (R + 1) * 64 * 4,
        "unit_words": bands * sg * 8,
        "result": 32,
        # reads: the hand-off words back (segment state, band rows) and the sequences each unit
        # stages (its band's Seq1 rows, its column range of Seq2 and the 64 columns before it)
        "read_segment_state": bands * (sg - 1) * (R + 1) * 64 * 4,
        "read_band_rows": (bands - 1) * n * 4,
        "read_sequences": sg * min(m, bands * 64 * R) + bands * (n + 64 * sg),
    }
    out = {k: v * pairs for k, v in per.items()}
    out["total"] = sum(out.values())
    return out


def f16_hi_exact(x: int) -> bool:
    """An f16 whose low byte is 0 holds x exactly (sa_api.hip f16_hi_exact)."""
    if not -2048 <= x <= 2048:
        return False
    h = np.array([x], np.float16)
    return int(h[0]) == x and (int(h.view(np.uint16)[0]) & 0xff) == 0


def issue_model(label: str):
    try:
        return json.load(open(ISSUE_MODEL))["kernels"][label]
    except Exception:
        return None


def gather_parity(par: dict, world: int):
    """Every rank's parity summary (gloo, host memory), in rank order."""
    if world == 1:
        return [par]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, par)
    return out


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    # HIP events around each fill kernel alone (sa_last_kernel_timings): the roofline's launch time
    os.environ.setdefault("SEQALIB_KERNEL_TIMING", "1")
    world, rank, local = dist_setup(args)
    import torch
    import seqalib_amd as sa

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (no CPU fallback)")
    gpu = gpu_index(local)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    Lq = args.len
    P, seed_base, workload = rank_shard(rank, world, args.pairs, args.total_pairs, Lq)

    s1, o1, s2, o2 = sa.synth_dna_batch(seed_base, P, Lq, Lq, threads=16)
    as_t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    d1, do1, d2, do2 = as_t(s1), as_t(o1), as_t(s2), as_t(o2)
    # SA_PIPELINE_DEPTH output sets: with the cross-call pipeline, step k's traceback still writes
    # its results while steps k+1 and k+2 fill, so those steps must not share result buffers
    NSET = sa.SA_PIPELINE_DEPTH
    d_res = [torch.zeros(P * 32, dtype=torch.uint8, device=dev) for _ in range(NSET)]
    d_ops = [torch.zeros(len(s1) + len(s2) + P, dtype=torch.uint8, device=dev) for _ in range(NSET)]
    eng = sa.Engine(gpu)
    scoring = sa.ScoringSystem(*SCORING)
    stream = torch.cuda.current_stream(dev)
    pipelined = not args.no_pipeline
    eng.set_pipeline(pipelined)

    def step(k):
        eng.align_device(sa.SA_SW, scoring, d1.data_ptr(), do1.data_ptr(), d2.data_ptr(), do2.data_ptr(), P, Lq, Lq,
                         d_res[k % NSET].data_ptr(), d_ops[k % NSET].data_ptr(), stream.cuda_stream)

    for k in range(args.warmup):
        step(k)
    eng.wait()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    eng.wait()                    # every step's fill AND traceback is inside the timed region
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    own = t1 - t0
    elapsed = max_over_ranks(own, world)
    fill_ms, tb_ms, launches = eng.last_timings()   # HIP events of the last step (fill stream / traceback stream)
    fill_kernel_ms, _ = eng.last_kernel_timings()    # the fill kernel alone (without the end-cell replay)
    last = (args.steps - 1) % NSET
    serial_ms = None
    if pipelined and args.serial_steps > 0:
        # the same steps without overlap, for reference (outside the timed region above)
        eng.set_pipeline(False)
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for k in range(args.serial_steps):
            step(last + 1 + NSET * k)   # another output set: keeps the checked one intact
        torch.cuda.synchronize()
        serial_ms = max_over_ranks(time.perf_counter() - ts, world) / args.serial_steps * 1e3
    kernel, plan_R, plan_W = eng.last_plan()
    fill_ms = max_over_ranks(fill_ms, world)
    fill_kernel_ms = max_over_ranks(fill_kernel_ms, world)
    # end to end through the host API (what the C++ drop-in does): sequences H2D, fill, end cell,
    # traceback, results + op streams D2H; outside the timed region
    e2e_ms, e2e_each = None, None
    if args.e2e_steps > 0:
        eng.set_pipeline(False)
        sc_ = sa.ScoringSystem(*SCORING)
        out = eng.align_packed(sa.SA_SW, sc_, s1, o1, s2, o2)   # warm the host-API buffers
        te = time.perf_counter()
        e2e_each = []
        for _ in range(args.e2e_steps):
            tc = time.perf_counter()
            out = eng.align_packed(sa.SA_SW, sc_, s1, o1, s2, o2, out=out)   # caller keeps its buffers
            e2e_each.append(round((time.perf_counter() - tc) * 1e3, 2))
        e2e_ms = max_over_ranks(time.perf_counter() - te, world) / args.e2e_steps * 1e3

    cells_rank = float(P) * Lq * Lq
    cells_job = float(args.total_pairs) * Lq * Lq if args.total_pairs > 0 else world * cells_rank
    value = cells_job * args.steps / elapsed / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    kernel, plan_R, plan_W, records = eng.last_plan_ex()

    # parity of this rank's batch, outside the timed region: every pair's (MaxScore, MaxRow, MaxCol)
    # against the linear-space oracle, every alignment re-scored to the reported maximum, and
    # --parity-ops full op streams against the full-matrix oracle (tools/bench_configs.py)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench_configs import parity_sw_batch
    res = np.frombuffer(d_res[last].cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE)
    ops = d_ops[last].cpu().numpy()
    cores = host_cores()["usable"]
    par = parity_sw_batch(s1, o1, s2, o2, res, ops, args.parity_ops, cores, 10)
    par_ranks = gather_parity(par, world)
    configs = None
    if rank == 0 and world == 1 and args.configs:
        from bench_configs import measure
        eng.set_pipeline(False)
        configs = measure(sa, torch, eng, dev, set(args.configs.split(",")), cores)

    if args.rank_out:
        os.makedirs(args.rank_out, exist_ok=True)
        with open(os.path.join(args.rank_out, f"rank{rank}.json"), "w") as f:
            json.dump({"rank": rank, "world": world, "own_s": own, "max_s": elapsed, "seed_base": seed_base, "pairs": P,
                       "parity": par, "flags": int(np.count_nonzero(res["flags"])), "plan": list(eng.last_plan())}, f)
    if rank != 0:
        return
    per_launch_cells = cells_rank  # one fill launch covers the whole batch when it fits HBM
    fill_s = fill_kernel_ms / 1e3 / max(launches, 1)   # one fill kernel launch (HIP events on its stream)
    t16 = kernel in (sa.SA_KERNEL_T16, sa.SA_KERNEL_T16_ENDCELL)
    endcell = kernel == sa.SA_KERNEL_T16_ENDCELL
    so = records == sa.SA_RECORDS_SCORE_ONLY
    # two pairs per wave (sa_fill_so2.hip) on the score-only SW plans at R = 16 / 32 unless SEQALIB_SO2=0
    so2 = so and plan_R in (16, 32) and os.environ.get("SEQALIB_SO2", "1") != "0"
    # the f16 cell (sa_fill_so2.hip FK) as the engine picks it (sa_api.hip so2_f16_scoring): SW at
    # an f16-exact match / mismatch unless SEQALIB_SO2_F16=0 (random DNA never turns it off)
    f16 = so2 and os.environ.get("SEQALIB_SO2_F16", "1") != "0" and all(f16_hi_exact(x) for x in (SCORING[1], SCORING[2]))
    label = f"sw_{'so2f' if f16 else 'so2' if so2 else 'so' if so else 't16c' if endcell else 't16' if t16 else 'int32'}_r{plan_R}"
    model = issue_model(label)
    fill_gcups = per_launch_cells / fill_s / 1e9
    # algorithmic HBM bytes per cell: score-only fill -- the edge stream (16 bits per lane-step =
    # 2/R B per cell), the end-cell snapshots ((R/2 + 1) words per lane per 32-step chunk) and the
    # chunk maxima (1 word per lane-chunk); tagged fill -- 2 record bits per cell + the snapshots
    snap = (plan_R // 2 + 1) * 4 / (32 * plan_R) if endcell else 0.0
    bytes_per_cell = (2.0 / plan_R + snap + 4 / (32 * plan_R)) if so else (SW_FLAG_BYTES_PER_CELL + snap)
    # every stream the score-only fill writes, per launch, from its geometry:
    # the streams above over the steps and chunks it really runs (n + 63 steps per band, snapshots
    # of all chunks but the last) plus the band rows, segment state, per-unit words and results
    # column segments per band unit as the engine picks them (sa_api.hip make_variant: two pairs per
    # wave up to kSo2Segs = 8 with at least 8 chunks each, kSoSegs = 2 otherwise; $SEQALIB_SO_SEGS overrides)
    nch_ = (Lq + 63 + 31) // 32
    segs = int(os.environ.get("SEQALIB_SO_SEGS", "0") or 0) or (max(2, min(8, nch_ // 8)) if so2 else 2)
    streams = fill_streams(P, Lq, Lq, plan_R, segs) if so else None
    if streams:
        bytes_per_cell = streams["total"] / per_launch_cells
    hbm_gbps = per_launch_cells * bytes_per_cell / fill_s / 1e9
    pmc = load_pmc(workload, label)
    kname = ("fill_so2_kernel<SW,R=%d,f16> (score-only, two pairs per wave in packed f16 halves, exact below 2048, "
             "band units, 4 waves/SIMD)" % plan_R if f16 else
             "fill_so2_kernel<SW,R=%d> (score-only T16, two pairs per wave in packed 16-bit halves, band units, "
             "4 waves/SIMD)" % plan_R if so2 else
             "fill_so_kernel<R=%d> (score-only T16, chunk-max end cell, 4 waves/SIMD)" % plan_R if so else
             f"fill_kernel<SW,R={plan_R},W={plan_W}," + ("T16 tagged int16 profile" if t16 else "int32 flags")
             + (",chunk-max end cell>" if endcell else ",KEYED>"))
    # achieved = fill cells/s x ISA-counted VALU instructions per cell of the steady loop (each lane
    # computes its own cells, so lane-instructions); peak = the guide's VALU issue peak at 2.4 GHz
    vpc = model["valu_per_cell"] if model else None
    # lane-element ops per cell: a packed 16-bit op (and the two-pair v_perm lookup) does two lanes'
    # work in a half-rate issue slot, so the VALU peak counts it twice (tools/issue_model.py)
    epc = model.get("valu_elem_per_cell", vpc) if model else None
    achieved = fill_gcups * epc / 1e3 if epc else None
    roof = {"bound": "valu", "achieved": round(achieved, 2) if achieved else None, "peak": round(VALU_PEAK_TLANE, 2),
            "unit": "T lane-ops/s", "frac": round(achieved / VALU_PEAK_TLANE, 4) if achieved else None,
            "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None}
    clk = pmc.get("clock_ghz") if pmc else None
    roof.update({"kernel": kname, "avg_launch_ms": round(fill_s * 1e3, 3),
                 "avg_launch_basis": "HIP events around the fill kernel on its stream, last timed step "
                                     "(sa_last_kernel_timings)",
                 "fill_gcups": round(fill_gcups, 1), "valu_per_cell": vpc, "valu_elem_per_cell": epc,
                 "valu_per_cell_basis": f"ISA count of the steady chunk loop (tools/issue_model.py, {os.path.relpath(ISSUE_MODEL, ROOT)})",
                 "peak_basis": "MI355X_MICROARCH.md: 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz (wave64 VALU op = 2 cycles)",
                 "clock_ghz_measured": clk,
                 "frac_at_measured_clock": round(achieved / (VALU_PEAK_TLANE * clk / 2.4), 4) if (achieved and clk) else None,
                 "pmc_source": pmc.get("source") if pmc else None,
                 "valu_per_cell_pmc": pmc.get("valu_wave_instr_per_cell") if pmc else None,
                 "pmc_kernel_ms": pmc.get("kernel_ms_per_pass") if pmc else None,
                 "bytes_per_cell": round(bytes_per_cell, 4), "hbm_achieved_GBps": round(hbm_gbps, 1),
                 "fill_streams_bytes_per_launch": streams,
                 "hbm_peak_GBps": HBM_PEAK_GBPS, "hbm_frac": round(hbm_gbps / HBM_PEAK_GBPS, 4)})
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "GCUPS", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2), "higher_is_better": True,
        "scaling": "strong" if args.total_pairs > 0 else "weak", "vs_baseline": None, "dtype": ("f16 (integer-exact below 2048)" if f16 else "int16") if t16 else "int32",
        "data": "synthetic DNA, std::mt19937_64 'ACGT'[g()&3], seeds base+2p+1/base+2p+2, resident in HBM",
        "config": {"workload": workload, "pairs_per_gpu": P, "total_pairs": args.total_pairs or world * P,
                   "m": Lq, "n": Lq, "algo": "SmithWatermanSA",
                   "scoring": list(SCORING), "match": "equal<char>", "parallelism": f"pair-shard x{world}"},
        "roofline": roof,
        "fill_ms": round(fill_ms, 2), "fill_kernel_ms": round(fill_kernel_ms, 2),
        "endcell_ms": round(fill_ms - fill_kernel_ms, 2), "traceback_ms": round(tb_ms, 2),
        "timings_basis": "HIP events of the last timed step: fill_ms = fill stream (fill kernel + end-cell "
                         "replay), traceback_ms = traceback stream after the fill stream",
        "records": "score-only fill + block-recompute traceback" if so else ("tagged" if t16 else "flags"),
        "e2e_ms_per_step": round(e2e_ms, 2) if e2e_ms else None,
        "e2e_ms_each": e2e_each if e2e_ms else None,
        "e2e_gcups": round(cells_job / (e2e_ms / 1e3) / 1e9, 1) if e2e_ms else None,
        "e2e_basis": "host API sa_align_batch from pageable host buffers, one call at a time (mean of e2e_steps "
                     "calls after one warm call), one chunk: upload of sequences + offsets in 16 MiB pieces, "
                     "A/C/G/T pieces packed to 2 bits on the host and unpacked on the device (host pass over "
                     "piece k+1 beside the H2D of piece k), fill, end cell, traceback, download of results and "
                     "2-bit op streams, expanded into the caller's (reused) buffers as pieces land",
        "pipelined": pipelined, "serial_ms_per_step": round(serial_ms, 2) if serial_ms else None,
        "parity": "; ".join(
            (f"rank {r}: " if world > 1 else "")
            + (f"{q['end_cells']} pairs' (MaxScore, MaxRow, MaxCol) bit-exact vs oracle; {q['rescored']} "
               f"alignments re-score to MaxScore; {q['op_streams']} full op streams bit-exact; {q['flagged']} flagged")
            for r, q in enumerate(par_ranks)),
        "parity_exact": all(q["exact"] for q in par_ranks),
        "parity_ranks": [{"rank": r, "exact": q["exact"], "end_cells": q["end_cells"], "op_streams": q["op_streams"]}
                         for r, q in enumerate(par_ranks)] if world > 1 else None,
        "configs": configs,
    }
    if world == 1:
        eng.L.sa_trim(eng.h)   # free this process's workspace for the children's
        line["dropin_e2e"] = dropin_e2e(args)
        line["dropin_single_call"] = dropin_latency(args)
    if world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args, s1, o1, s2, o2)
        line["cpu_baseline_1thread"] = cpu_baseline(args, s1, o1, s2, o2, threads=1, pairs=args.cpu_pairs_1t)
    else:
        line["cpu_baseline"] = None
    txt = json.dumps(line)
    print(txt, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
