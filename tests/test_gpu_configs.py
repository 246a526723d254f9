"""GPU parity at the BASELINE.json configurations' full sizes.

Every check compares the HIP path (through the C ABI) with the pinned C oracle on the same seeded
inputs: (MaxScore, MaxRow, MaxCol) of whole batches or large samples with the linear-space oracle
(oracle_sw_score_batch, itself pinned to the reference's golden vectors in
tests/test_oracle_golden.py), full op streams of a sample with the full-matrix oracle, and the
size-independent properties on every pair (the alignment re-scores to the reported maximum and
consumes exactly end - start symbols of each sequence).  Reference semantics:
SASmithWaterman.h:89-117 (fill, last row-major maximum at :110) and :220-339 (traceback).
"""
import numpy as np
import pytest

import seqalib_amd as sa
from util import linear_rescore, oracle_batch, oracle_sw_scores, subset

pytestmark = pytest.mark.gpu
BATCH_KERNELS = True   # small host calls stay on the batch kernels (conftest.py)

SW = (-1, 1, -1)   # SmithWatermanSA::getDefaultScoring (SASmithWaterman.h:352)
THREADS = 16       # the GPU box's host share


def op_counts(res, ops, o1, o2, chars):
    """Per-pair count of the op bytes in `chars` (vectorised over the packed op buffer)."""
    n = len(res)
    starts = o1[:n].astype(np.int64) + o2[:n].astype(np.int64) + np.arange(n)
    sel = np.zeros(256, dtype=np.int64)
    for c in chars:
        sel[ord(c)] = 1
    csum = np.concatenate([[0], np.cumsum(sel[ops.astype(np.int64)])])
    return csum[starts + res["nops"].astype(np.int64)] - csum[starts]


def check_batch(engine, s1, o1, s2, o2, res, ops, score_sample, ops_sample, seed):
    n = len(o1) - 1
    assert (res["flags"] == 0).all()
    # properties on every pair
    assert (linear_rescore(SW, res, ops, o1, o2) == res["score"]).all()
    di = op_counts(res, ops, o1, o2, "MSUX")
    dj = op_counts(res, ops, o1, o2, "MSLX")
    assert (res["end_i"] - res["start_i"] == di).all()
    assert (res["end_j"] - res["start_j"] == dj).all()
    # score and end cell vs the linear-space oracle
    rng = np.random.default_rng(seed)
    idx = np.arange(n) if score_sample >= n else np.sort(rng.choice(n, score_sample, replace=False))
    sub = subset(s1, o1, s2, o2, idx)
    exp = oracle_sw_scores(SW, *sub, threads=THREADS)
    got = np.stack([res["score"][idx], res["end_i"][idx], res["end_j"][idx]], axis=1)
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert len(bad) == 0, [(int(idx[b]), got[b].tolist(), exp[b].tolist()) for b in bad[:5]]
    # full results and op streams vs the full-matrix oracle
    jdx = np.sort(rng.choice(n, min(ops_sample, n), replace=False))
    sub = subset(s1, o1, s2, o2, jdx)
    ores, oops = oracle_batch(0, SW, *sub, threads=THREADS)
    so1, so2 = sub[1], sub[3]
    for q, p in enumerate(jdx):
        off = int(o1[p] + o2[p]) + int(p)
        ooff = int(so1[q] + so2[q]) + q
        got = (int(res["score"][p]), int(res["end_i"][p]), int(res["end_j"][p]), int(res["start_i"][p]),
               int(res["start_j"][p]), ops[off:off + int(res["nops"][p])].tobytes())
        exp = (int(ores["score"][q]), int(ores["end_i"][q]), int(ores["end_j"][q]), int(ores["start_i"][q]),
               int(ores["start_j"][q]), oops[ooff:ooff + int(ores["nops"][q])].tobytes())
        assert got == exp, int(p)


def test_config3_batch_1024(engine):
    """Config 3: 10,000 independent 1024 x 1024 SW pairs on one GPU -- the T16 end-cell plan with
    R = 16 (one wave per pair, one band), every pair's score and end cell against the oracle."""
    s1, o1, s2, o2 = sa.synth_dna_batch(3_000_000_000, 10000, 1024, 1024, threads=THREADS)
    res, ops = engine.align_packed(0, sa.ScoringSystem(*SW), s1, o1, s2, o2)
    assert engine.last_plan() == (sa.SA_KERNEL_T16_ENDCELL, 16, 1)
    check_batch(engine, s1, o1, s2, o2, res, ops, score_sample=10000, ops_sample=256, seed=3)


def test_config5_shard_2048(engine):
    """Config 5's single-GPU shard: 12,500 of the 100,000 2048 x 2048 pairs (rank 0 of 8) -- the
    T16 end-cell plan with R = 32, 2,048 pairs' end cells and 64 pairs' op streams against the
    oracle, properties on all."""
    from seqalib_amd.multi import shard_range
    start, stop = shard_range(0, 8, 100000)
    assert (start, stop) == (0, 12500)
    s1, o1, s2, o2 = sa.synth_dna_batch(5_000_000_000 + 2 * start, stop - start, 2048, 2048, threads=THREADS)
    res, ops = engine.align_packed(0, sa.ScoringSystem(*SW), s1, o1, s2, o2)
    assert engine.last_plan() == (sa.SA_KERNEL_T16_ENDCELL, 32, 1)
    check_batch(engine, s1, o1, s2, o2, res, ops, score_sample=2048, ops_sample=64, seed=5)


def test_north_star_shape_1024x4096(engine):
    """North-star pair shape (4096 x 4096), 1,024 pairs in one launch: every end cell against the
    linear-space oracle, 128 pairs' op streams against the full-matrix oracle, on the shipped
    one-pair kernel (R = 32)."""
    s1, o1, s2, o2 = sa.synth_dna_batch(9_000_000_000, 1024, 4096, 4096, threads=THREADS)
    res, ops = engine.align_packed(0, sa.ScoringSystem(*SW), s1, o1, s2, o2)
    assert engine.last_plan() == (sa.SA_KERNEL_T16_ENDCELL, 32, 1)
    check_batch(engine, s1, o1, s2, o2, res, ops, score_sample=1024, ops_sample=128, seed=9)


def test_config2_single_pair_4096(engine):
    """Config 2: one 4096 x 4096 pair (the few-pairs plan), score, end cell and ops exact."""
    s1, o1, s2, o2 = sa.synth_dna_batch(2_000_000_000, 1, 4096, 4096)
    res, ops = engine.align_packed(0, sa.ScoringSystem(*SW), s1, o1, s2, o2)
    check_batch(engine, s1, o1, s2, o2, res, ops, score_sample=1, ops_sample=1, seed=2)
    # a related pair: the optimum spans the whole matrix
    a = sa.synth_dna(2_000_000_011, 4096)
    b = sa.synth_mutate(a, 7)[:4096]
    s1, o1, s2, o2 = sa.pack_pairs([(a, b)])
    res, ops = engine.align_packed(0, sa.ScoringSystem(*SW), s1, o1, s2, o2)
    assert res["score"][0] > 2000
    check_batch(engine, s1, o1, s2, o2, res, ops, score_sample=1, ops_sample=1, seed=2)


def _device_batches(torch, dev, specs):
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    out = []
    for seed, n, L in specs:
        s1, o1, s2, o2 = sa.synth_dna_batch(seed, n, L, L - 3)
        d = [t(x) for x in (s1, o1, s2, o2)]
        res = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
        ops = torch.zeros(len(s1) + len(s2) + n, dtype=torch.uint8, device=dev)
        out.append(((s1, o1, s2, o2), d, n, L, res, ops))
    return out


def _check_device_batches(engine, algo, sc, calls):
    for (h, d, n, L, res, ops) in calls:
        s1, o1, s2, o2 = h
        got = np.frombuffer(res.cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE)
        ref, ref_ops = engine.align_packed(algo, sc, s1, o1, s2, o2)
        for f in ("score", "end_i", "end_j", "start_i", "start_j", "nops", "flags"):
            assert (got[f] == ref[f]).all(), (algo, f)
        g_ops = ops.cpu().numpy()
        for p in range(n):
            off = int(o1[p] + o2[p]) + p
            k = int(ref["nops"][p])
            assert g_ops[off:off + k].tobytes() == ref_ops[off:off + k].tobytes(), (algo, p)


@pytest.mark.parametrize("algo", [0, 1, 2])
def test_pipeline_large_then_small_slots(engine, algo):
    """Pipelined calls alternate workspace slots: a large call on slot 0 followed by a small one
    on slot 1 must not touch the records slot 0's traceback is still reading (every buffer of a
    call lives inside its own slot)."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    sc = sa.ScoringSystem(*((-1, 1, -1) if algo < 2 else (-3, -1, 1, -1)))
    calls = _device_batches(torch, dev, [(41, 1200, 2048), (43, 1100, 256), (47, 1024, 1500), (53, 64, 300)])
    stream = torch.cuda.current_stream().cuda_stream
    engine.set_pipeline(True)
    try:
        for (h, d, n, L, res, ops) in calls:
            engine.align_device(algo, sc, *[x.data_ptr() for x in d], n, L, L, res.data_ptr(), ops.data_ptr(), stream)
        engine.wait()
    finally:
        engine.set_pipeline(False)
    torch.cuda.synchronize()
    _check_device_batches(engine, algo, sc, calls)


@pytest.mark.parametrize("algo", [0, 2])
def test_pipeline_multi_launch_call(engine, algo):
    """A pipelined call split into several launches by a small workspace limit: launch k+1's fill
    waits for launch k's traceback before it overwrites the shared records."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    sc = sa.ScoringSystem(*((-1, 1, -1) if algo < 2 else (-3, -1, 1, -1)))
    calls = _device_batches(torch, dev, [(61, 1500, 1024), (67, 1100, 900)])
    stream = torch.cuda.current_stream().cuda_stream
    engine.set_workspace_limit(64 << 20)   # ~ a few hundred pairs per launch
    engine.set_pipeline(True)
    try:
        for (h, d, n, L, res, ops) in calls:
            engine.align_device(algo, sc, *[x.data_ptr() for x in d], n, L, L, res.data_ptr(), ops.data_ptr(), stream)
            assert engine.last_timings()[2] > 1   # several launches
        engine.wait()
    finally:
        engine.set_pipeline(False)
        engine.set_workspace_limit(0)
    torch.cuda.synchronize()
    _check_device_batches(engine, algo, sc, calls)


def test_device_selects_int32_for_wide_alphabet(engine):
    """T16-eligible scoring but more than four symbols: the device picks the int32 kernel (the
    T16 launches return at once) and the results stay exact; DNA in the same context goes back to
    T16."""
    from util import oracle_align
    pairs = [(sa.synth_dna(800 + k, 700), sa.synth_dna(900 + k, 650)) for k in range(1100)]
    pairs[5] = (pairs[5][0][:100] + b"N" + pairs[5][0][101:], pairs[5][1])
    res = engine.align(0, sa.ScoringSystem(*SW), pairs)
    assert engine.last_plan()[0] == sa.SA_KERNEL_INT32
    for p in (0, 5, 1099):
        o = oracle_align(0, SW, *pairs[p])
        assert (res[p].score, res[p].end_i, res[p].end_j, res[p].ops) == (o["score"], o["end_i"], o["end_j"], o["ops"])
    pairs[5] = (sa.synth_dna(805, 700), pairs[5][1])
    res = engine.align(0, sa.ScoringSystem(*SW), pairs)
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16_ENDCELL
    o = oracle_align(0, SW, *pairs[5])
    assert (res[5].score, res[5].end_i, res[5].end_j, res[5].ops) == (o["score"], o["end_i"], o["end_j"], o["ops"])


def same_streams(res, ops, ref_ops, o1, o2):
    """Every pair's op stream (the first nops bytes of its slot) equal; the bytes past nops in a
    slot are unspecified (the device I/O buffers are reused between calls)."""
    n = len(res)
    starts = o1[:n].astype(np.int64) + o2[:n].astype(np.int64) + np.arange(n)
    for p in range(n):
        s, k = int(starts[p]), int(res["nops"][p])
        if ops[s:s + k].tobytes() != ref_ops[s:s + k].tobytes():
            return False
    return True


def test_multi_context_config5_shard_matches_single(engine):
    """sa_multi (two contexts on GPU 0 here; one per GPU on a node) over the config-5 shard
    returns byte for byte what one context returns; the ranges write in place, so there is no
    host gather step at all."""
    import time
    from seqalib_amd.multi import MultiEngine
    s1, o1, s2, o2 = sa.synth_dna_batch(5_000_000_000, 12500, 2048, 2048, threads=THREADS)
    sc = sa.ScoringSystem(*SW)
    t0 = time.perf_counter()
    ref, ref_ops = engine.align_packed(0, sc, s1, o1, s2, o2)
    t1 = time.perf_counter()
    me = MultiEngine([0, 0])
    try:
        me.align_packed(0, sc, s1, o1, s2, o2)          # warm the second context's workspace
        t2 = time.perf_counter()
        res, ops = me.align_packed(0, sc, s1, o1, s2, o2)
        t3 = time.perf_counter()
    finally:
        me.close()
    assert res.tobytes() == ref.tobytes()
    assert same_streams(res, ops, ref_ops, o1, o2)
    print(f"single context {1e3 * (t1 - t0):.1f} ms, two contexts on one GPU {1e3 * (t3 - t2):.1f} ms")


def test_multi_engine_four_contexts_stage_concurrently(engine, capfd, monkeypatch):
    """One process, four contexts (MultiEngine([0, 0, 0, 0]) -- four devices' host threads on the
    one-GPU box): results identical to a single context, and the host API's staging copies of the
    four contexts run side by side in the shared copy pool (SEQALIB_HOST_TIMING reports the most copy
    jobs ever in flight; one process-wide lock would keep it at 1)."""
    from seqalib_amd.multi import MultiEngine
    s1, o1, s2, o2 = sa.synth_dna_batch(8_100_000_000, 4096, 4096, 4096, threads=THREADS)
    sc = sa.ScoringSystem(*SW)
    ref, ref_ops = engine.align_packed(0, sc, s1, o1, s2, o2)
    me = MultiEngine([0, 0, 0, 0])
    try:
        me.align_packed(0, sc, s1, o1, s2, o2)   # warm the contexts' workspaces
        capfd.readouterr()
        monkeypatch.setenv("SEQALIB_HOST_TIMING", "1")
        res, ops = me.align_packed(0, sc, s1, o1, s2, o2)
        err = capfd.readouterr().err
    finally:
        me.close()
    assert res.tobytes() == ref.tobytes()
    assert same_streams(res, ops, ref_ops, o1, o2)
    lines = [ln for ln in err.splitlines() if ln.startswith("[seqalib host api]")]
    assert len(lines) == 4, err[-2000:]
    inflight = max(int(ln.split("max ")[1].split(" copy jobs")[0]) for ln in lines)
    print("\n".join(lines))
    assert inflight >= 2, lines


@pytest.mark.parametrize("algo,args", [(0, (-1, 1, -1)), (1, (-1, 2, -1)), (2, (-3, -1, 1, -1)),
                                       (3, (-3, -1, 1, -1, True))])
def test_host_chunks_with_distinct_small_alphabets(engine, monkeypatch, algo, args):
    """A host call cut into pipelined chunks (SEQALIB_HOST_CHUNKS) whose chunks are small enough for
    the host to decide each chunk's T16 alphabet, and whose alphabets differ (ACGT / ACGN / TWXY,
    <= 4 symbols each): every chunk must run with its OWN profile and symbol pack (each chunk has
    its own pinned profile slot; round-4 advisor finding), so every pair equals the oracle."""
    from util import oracle_batch
    rng = np.random.default_rng(100 + algo)
    pairs = []
    for alph in (b"ACGT", b"ACGN", b"TWXY"):
        sym = np.frombuffer(alph, dtype=np.uint8)
        for _ in range(700):   # equal cells per pair: the three chunks are exactly the three groups
            pairs.append((sym[rng.integers(0, 4, 24)].tobytes(), sym[rng.integers(0, 4, 20)].tobytes()))
    s1, o1, s2, o2 = sa.pack_pairs(pairs)
    monkeypatch.setenv("SEQALIB_HOST_CHUNKS", "3")
    res, ops = engine.align_packed(algo, sa.ScoringSystem(*args), s1, o1, s2, o2)
    ores, oops = oracle_batch(algo, args, s1, o1, s2, o2, threads=THREADS)
    for p in range(len(pairs)):
        off = int(o1[p] + o2[p]) + p
        got = (int(res["score"][p]), int(res["end_i"][p]), int(res["end_j"][p]), int(res["start_i"][p]),
               int(res["start_j"][p]), ops[off:off + int(res["nops"][p])].tobytes())
        exp = (int(ores["score"][p]), int(ores["end_i"][p]), int(ores["end_j"][p]), int(ores["start_i"][p]),
               int(ores["start_j"][p]), oops[off:off + int(ores["nops"][p])].tobytes())
        assert got == exp, (p, got, exp)
