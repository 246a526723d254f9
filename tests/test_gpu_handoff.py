"""Band-unit hand-offs of the score-only SW / NW fills (sa_fill_impl.h BU) and the int32 re-run of
flagged pairs, against the tagged path and the pinned oracle.

* The hand-off words (row granules, column-segment state, per-unit maxima) are {tag, value} words a
  consumer polls until the tag is its launch's.  They live in the context's hand-off buffer, which
  only these fills write and which is zeroed when allocated and when the 16-bit tag wraps
  (sa_api.hip next_hand_tag), so no stale word of an earlier call -- of any shape -- can carry the
  current tag.  The tests poison the shared workspace with words carrying the NEXT tag (what an
  earlier call's snapshots could hold; round 5 kept the hand-off words there) and drive the tag
  across its wrap.
* A consumer's wait is bounded (FillParams::wait_polls); an expired one flags the pair, which the
  int32 variant of the same call re-runs (SEQALIB_SO_WAIT_POLLS forces it here).
* Pipelined calls walk the int32 re-run before the T16 traceback (sa_api.hip tb_on_fill); the
  re-run pairs are handed over by flags (TbParams keep_redo / clear_redo), so they keep the int32
  result whatever the launch order -- pipelined device calls and chunked host calls alike.
Reference semantics: SASmithWaterman.h:89-117, :220-339; SANeedlemanWunsch.h (fill / traceback).
"""
import numpy as np
import pytest

import seqalib_amd as sa
from test_gpu_so import NW, SW, assert_same, check_vs_oracle, ragged_batch, run

pytestmark = pytest.mark.gpu
BATCH_KERNELS = True   # small host calls stay on the batch kernels (conftest.py)


def poison_word(tag_next: int, value: int = 0x0100) -> int:
    """A 32-bit {tag, value} word the next band-unit launch would accept as its own."""
    return ((tag_next & 0xffff) << 16) | (value & 0xffff)


@pytest.mark.parametrize("algo,scoring", [(0, SW), (1, NW)])
def test_poisoned_workspace_and_tag_wrap(engine, algo, scoring):
    """Before every score-only call the workspace is overwritten with words carrying the tag that
    call takes, and the tag runs across its wrap (65534 -> 65535 -> zeroed buffer -> 1 -> 2), with
    two shapes alternating: every result and op stream equals the tagged path's (computed first,
    on a clean workspace) and a sample the oracle's."""
    big = ragged_batch(501 + algo, 1100, 3000)
    small = ragged_batch(601 + algo, 1050, 1500)
    want = {id(b): run(engine, False, *b, scoring=scoring, algo=algo) for b in (big, small)}
    run(engine, True, *big, scoring=scoring, algo=algo)   # (the workspace at the larger shape)
    tag = 65533
    engine.test_hook(sa.SA_HOOK_HAND_TAG, tag)
    for k in range(5):
        b = (big, small)[k % 2]
        nxt = tag + 1 if tag < 65535 else 1
        engine.test_hook(sa.SA_HOOK_POISON_WS, poison_word(nxt))
        got = run(engine, True, *b, scoring=scoring, algo=algo)
        assert engine.last_plan_ex()[3] == sa.SA_RECORDS_SCORE_ONLY
        assert_same(got, want[id(b)], b[1], b[3])
        tag = nxt
    assert b is big
    check_vs_oracle(algo, scoring, got, big, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 200, 700, 1099])


@pytest.mark.parametrize("algo,scoring", [(0, SW), (1, NW)])
def test_fresh_context_after_other_shapes(algo, scoring):
    """A second context after calls of other shapes on a first one that was then destroyed (its
    buffers go back to the allocator): the new context's first score-only calls are exact."""
    first = sa.Engine(0)
    try:
        for maxlen, npairs in ((2500, 1030), (900, 1200)):
            run(first, True, *ragged_batch(700 + maxlen, npairs, maxlen), scoring=scoring, algo=algo)
    finally:
        first.close()
    second = sa.Engine(0)
    try:
        b = ragged_batch(801 + algo, 1100, 3000)
        got = run(second, True, *b, scoring=scoring, algo=algo)
        assert_same(got, run(second, False, *b, scoring=scoring, algo=algo), b[1], b[3])
    finally:
        second.close()


@pytest.mark.parametrize("algo,scoring", [(0, SW), (1, NW)])
def test_lost_producer_reruns_in_int32(engine, monkeypatch, algo, scoring):
    """Every band-unit wait gives up after one poll (SEQALIB_SO_WAIT_POLLS=1): units run on with
    whatever they read and flag their pair, the pair's final unit folds every unit's flag, and the
    int32 variant of the same call re-runs the pair -- results identical to the tagged path."""
    b = ragged_batch(901 + algo, 1100, 3000)
    want = run(engine, False, *b, scoring=scoring, algo=algo)
    monkeypatch.setenv("SEQALIB_SO_WAIT_POLLS", "1")
    got = run(engine, True, *b, scoring=scoring, algo=algo)
    assert engine.last_plan_ex()[3] == sa.SA_RECORDS_SCORE_ONLY
    assert_same(got, want, b[1], b[3])
    check_vs_oracle(algo, scoring, got, b, [0, 1, 2, 3, 8, 9, 10, 500, 1099])


def retry_batch():
    """Two pairs above SW's int16 headroom (identical 9,000-long sequences: score 9,000) among
    1,100 ordinary ones: the T16 fill flags them and the int32 variant re-runs them."""
    rng = np.random.default_rng(77)
    hot = sa.synth_dna(81_000, 9000)
    pairs = [(hot, hot), (hot[:8800], sa.synth_mutate(hot, 5)[:8900])]
    for k in range(1100):
        a = sa.synth_dna(82_000 + 2 * k, int(rng.integers(600, 1300)))
        b = sa.synth_mutate(a, k) if k % 3 == 0 else sa.synth_dna(82_001 + 2 * k, int(rng.integers(600, 1300)))
        pairs.append((a, b))
    return sa.pack_pairs(pairs)


def test_retry_pairs_pipelined_device_calls(engine):
    """The retry batch through sa_set_pipeline (three calls in flight, the int32 re-run walked on
    the fill stream before the T16 traceback): every call equals the unpipelined result, the hot
    pairs and a sample equal the oracle."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    s1, o1, s2, o2 = retry_batch()
    n = len(o1) - 1
    ref = run(engine, True, s1, o1, s2, o2)
    assert int(ref[0]["score"][0]) == 9000
    d = [t(x) for x in (s1, o1, s2, o2)]
    L1, L2 = int(np.diff(o1).max()), int(np.diff(o2).max())
    outs = [(torch.zeros(n * 32, dtype=torch.uint8, device=dev),
             torch.zeros(len(s1) + len(s2) + n, dtype=torch.uint8, device=dev)) for _ in range(3)]
    stream = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    engine.set_pipeline(True)
    try:
        for res, ops in outs:
            engine.align_device(0, sa.ScoringSystem(*SW), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                d[3].data_ptr(), n, L1, L2, res.data_ptr(), ops.data_ptr(), stream)
        engine.wait()
    finally:
        engine.set_pipeline(False)
    torch.cuda.synchronize()
    for res, ops in outs:
        got = (np.frombuffer(res.cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE).copy(), ops.cpu().numpy(), None)
        assert_same(got, ref, o1, o2)
    check_vs_oracle(0, SW, ref, (s1, o1, s2, o2), [0, 1, 2, 3, 50, 1101])


def test_retry_pairs_chunked_host_call(engine, monkeypatch):
    """The retry batch as a host call cut into 2 and 3 pipelined chunks (SEQALIB_HOST_CHUNKS): equal
    to the one-chunk call and, for the hot pairs and a sample, to the oracle."""
    b = retry_batch()
    one = run(engine, True, *b)
    for g in ("2", "3"):
        monkeypatch.setenv("SEQALIB_HOST_CHUNKS", g)
        assert_same(run(engine, True, *b), one, b[1], b[3])
    check_vs_oracle(0, SW, one, b, [0, 1, 2, 3, 600, 1101])
