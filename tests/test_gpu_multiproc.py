"""The multi-GPU launch path of bench.py on real HIP: one process per rank
started by torch.distributed.run, gloo only for the barrier and the max-over-ranks timing, every
rank aligning its own shard through the device API.  On a one-GPU box both ranks run on GPU 0
(SEQALIB_BENCH_DEVICE=0); the ranks are spawned as child processes (never an exec of this
process).  Checks: each rank's pairs bit-exact vs the oracle (every end cell, sampled op streams), distinct shards, and the
reported ms_per_step = the max over ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("length", [600, 1500])
def test_two_hip_ranks_gloo(tmp_path, length):
    steps = 3
    env = dict(os.environ, SEQALIB_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--pairs", "40", "--len",
           str(length), "--steps", str(steps), "--warmup", "1", "--no-cpu", "--e2e-steps", "0", "--serial-steps", "0",
           "--dropin-pairs", "0", "--rank-out", str(tmp_path), "--out", str(tmp_path / "line.json")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    ranks = [json.load(open(tmp_path / f"rank{k}.json")) for k in (0, 1)]
    for rr in ranks:
        assert rr["world"] == 2
        par = rr["parity"]
        assert par["exact"] and par["end_cells"] == "40/40" and rr["flags"] == 0, rr
    assert ranks[0]["seed_base"] != ranks[1]["seed_base"]
    slowest = max(rr["own_s"] for rr in ranks)
    for rr in ranks:
        assert abs(rr["max_s"] - slowest) < 1e-9
    line = json.loads(open(tmp_path / "line.json").read())
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert abs(line["ms_per_step"] - slowest / steps * 1e3) < 0.01
    assert line["value"] > 0


@pytest.mark.timeout(900)
def test_bench_gpus2_spawns_two_ranks(tmp_path):
    """`python3 bench.py --gpus 2 --steps 2 --warmup 1` exactly as the driver starts it for N = 2 --
    no launcher, no WORLD_SIZE -- must run two ranks (bench.py spawns them), each aligning its own
    10,000-pair shard of the 4096 x 4096 headline workload, and report n_gpus = 2, the max-over-ranks
    time and exact parity on both shards.  Both ranks share GPU 0 here (SEQALIB_BENCH_DEVICE=0)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(SEQALIB_BENCH_DEVICE="0")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--rank-out", str(tmp_path), "--out", str(tmp_path / "line.json")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=840)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 alone prints the line
    line = json.loads(lines[0])
    assert line == json.loads(open(tmp_path / "line.json").read())
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "pair-shard x2"
    assert line["config"]["workload"] == "sw_batch_10000x4096x4096"
    assert line["parity_exact"] is True
    assert [q["rank"] for q in line["parity_ranks"]] == [0, 1]
    for q in line["parity_ranks"]:
        assert q["exact"] and q["end_cells"] == "10000/10000", q
    ranks = [json.load(open(tmp_path / f"rank{k}.json")) for k in (0, 1)]
    assert [rr["world"] for rr in ranks] == [2, 2]
    assert ranks[0]["seed_base"] != ranks[1]["seed_base"]
    slowest = max(rr["own_s"] for rr in ranks)
    assert abs(line["ms_per_step"] - slowest / 2 * 1e3) < 0.01
    assert line["value"] == pytest.approx(2 * 10000 * 4096 * 4096 * 2 / slowest / 1e9, rel=1e-3)
