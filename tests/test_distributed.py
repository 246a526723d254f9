"""CPU, world_size 2 over gloo: the multi-GPU path's sharding and timing reduction (bench.py,
seqalib_amd/multi.py).  Pairs are independent, so the union of the per-rank shards must be the
global batch, pair for pair, and each rank's results must equal a single-process run."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from seqalib_amd.multi import balanced_split, shard_range, slice_batch, static_split  # noqa: E402


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, P, L, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    import bench
    import seqalib_amd as sa
    from util import oracle_align
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    s1, o1, s2, o2 = sa.synth_dna_batch(bench.shard_seed_base(rank, world, P), P, L, L, threads=2)
    scores = []
    for p in range(P):
        o = oracle_align(0, (-1, 1, -1), s1[o1[p]:o1[p + 1]].tobytes(), s2[o2[p]:o2[p + 1]].tobytes())
        scores.append((o["score"], o["end_i"], o["end_j"], o["ops"]))
    gathered = [None] * world
    dist.all_gather_object(gathered, scores)
    t = bench.max_over_ranks(float(rank + 1) * 1.5, world)
    bench.barrier(world)
    if rank == 0:
        q.put((gathered, t))
    dist.destroy_process_group()


def test_two_rank_shards_reassemble_the_global_batch():
    import seqalib_amd as sa
    from util import oracle_align
    import bench
    world, P, L = 2, 6, 96
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, t = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == pytest.approx(3.0)   # max over ranks of (rank+1)*1.5
    # single-process reference run over the whole global batch
    s1, o1, s2, o2 = sa.synth_dna_batch(bench.SEED_BASE, world * P, L, L, threads=2)
    flat = [x for part in gathered for x in part]
    assert len(flat) == world * P
    for p in range(world * P):
        o = oracle_align(0, (-1, 1, -1), s1[o1[p]:o1[p + 1]].tobytes(), s2[o2[p]:o2[p + 1]].tobytes())
        assert flat[p] == (o["score"], o["end_i"], o["end_j"], o["ops"])


def test_strong_scaling_shards_tile_the_fixed_batch():
    """bench.py --total-pairs (BASELINE config 5, strong scaling): the ranks' slices of the fixed
    global batch are contiguous, cover it exactly, and regenerate its pairs byte for byte."""
    import seqalib_amd as sa
    import bench
    T, L = 7, 40
    s1, o1, s2, o2 = sa.synth_dna_batch(bench.SEED_BASE, T, L, L, threads=2)
    for world in (1, 2, 3, 8):
        got = []
        for rank in range(world):
            P, base, name = bench.rank_shard(rank, world, 10000, T, L)
            assert name == f"sw_batch_{T}x{L}x{L}_strong"
            if P == 0:
                continue
            a1, b1, a2, b2 = sa.synth_dna_batch(base, P, L, L, threads=2)
            got += [(a1[b1[p]:b1[p + 1]].tobytes(), a2[b2[p]:b2[p + 1]].tobytes()) for p in range(P)]
        assert got == [(s1[o1[p]:o1[p + 1]].tobytes(), s2[o2[p]:o2[p + 1]].tobytes()) for p in range(T)], world
    P, base, name = bench.rank_shard(1, 2, 6, 0, L)   # weak scaling: per-GPU pairs, as shard_seed_base
    assert (P, base, name) == (6, bench.shard_seed_base(1, 2, 6), f"sw_batch_6x{L}x{L}")


def test_static_and_balanced_splits():
    assert static_split(10, 4) == [(0, 2), (2, 5), (5, 7), (7, 10)]
    assert shard_range(1, 2, 20000) == (10000, 20000)
    cells = np.array([100, 1, 1, 1, 100, 1, 1, 100], dtype=float)
    r = balanced_split(cells, 3)
    assert r[0][0] == 0 and r[-1][1] == len(cells)
    assert all(a <= b for a, b in r) and all(r[k][1] == r[k + 1][0] for k in range(2))
    loads = [cells[a:b].sum() for a, b in r]
    assert max(loads) <= 2 * cells.sum() / 3
    assert balanced_split(np.zeros(0), 2) == [(0, 0), (0, 0)]


def test_slice_batch_rebases_offsets():
    import seqalib_amd as sa
    s1, o1, s2, o2 = sa.synth_dna_batch(5, 5, 10, 7, threads=1)
    a, oa, b, ob = slice_batch(s1, o1, s2, o2, 2, 4)
    assert list(oa) == [0, 10, 20] and list(ob) == [0, 7, 14]
    assert a.tobytes() == s1[20:40].tobytes() and b.tobytes() == s2[14:28].tobytes()


def _run_bench(args, env_extra, timeout=240):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=root, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_bench_refuses_world_size_mismatch():
    """A line for N GPUs must come from N ranks: --gpus 2 under a launcher's WORLD_SIZE=3 fails loudly."""
    r = _run_bench(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 2 but WORLD_SIZE=3" in r.stderr


def test_bench_gpus_n_spawns_n_ranks_without_launcher():
    """`bench.py --gpus 2` with no launcher starts two rank processes that rendezvous over gloo on
    127.0.0.1 (here, without a GPU, each rank then stops at the GPU check after the rendezvous)."""
    r = _run_bench(["--gpus", "2", "--steps", "1"], {"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode != 0
    assert r.stderr.count("bench.py needs a GPU") == 2, r.stderr[-2000:]
