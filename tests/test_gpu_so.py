"""Score-only Smith-Waterman fill + block-recompute traceback (sa_fill_impl.h SO,
seqalib_amd/csrc/sa_traceback_so.hip) against the tagged-record path and the pinned oracle.

The score-only fill stores no per-cell records; its traceback recomputes, block by block along the
path, the move tags the tagged fill would have stored, from the per-chunk snapshots and the edge
stream (each lane's last row per step).  Every test runs the same batch twice -- score-only (the
default for T16 SW batches of >= 1,024 pairs) and SEQALIB_SO=0 (tagged records, the round-3 path)
-- and requires every pair's result and op stream to be identical, then checks a sample against the
oracle (itself pinned to the reference's golden vectors, tests/test_oracle_golden.py).
Reference semantics: SASmithWaterman.h:89-117 (fill; last row-major maximum :110), :220-339
(traceback).
"""
import os

import numpy as np
import pytest

import seqalib_amd as sa
from util import linear_rescore, oracle_align, oracle_batch, oracle_sw_scores, subset

pytestmark = pytest.mark.gpu
BATCH_KERNELS = True   # small host calls stay on the batch kernels (conftest.py)

SW = (-1, 1, -1)   # SmithWatermanSA::getDefaultScoring (SASmithWaterman.h:352)
THREADS = 16
FIELDS = ("score", "end_i", "end_j", "start_i", "start_j", "nops", "flags")


def run(engine, so, *batch, scoring=SW, lut=None, tb="4", algo=0):
    """so: score-only fill (else SEQALIB_SO=0, tagged records); tb: SEQALIB_TB_SO, the score-only
    traceback with four lanes per pair ("4", default) or one ("1")."""
    old = {k: os.environ.get(k) for k in ("SEQALIB_SO", "SEQALIB_TB_SO")}
    os.environ["SEQALIB_SO"] = "1" if so else "0"
    os.environ["SEQALIB_TB_SO"] = tb
    try:
        res, ops = engine.align_packed(algo, sa.ScoringSystem(*scoring), *batch, lut=lut)
        plan = engine.last_plan()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    return res.copy(), ops.copy(), plan


def assert_same(a, b, o1, o2):
    ra, oa, _ = a
    rb, ob, _ = b
    for f in FIELDS:
        bad = np.nonzero(ra[f] != rb[f])[0]
        assert len(bad) == 0, (f, [(int(p), int(ra[f][p]), int(rb[f][p])) for p in bad[:5]])
    n = len(ra)
    starts = o1[:n].astype(np.int64) + o2[:n].astype(np.int64) + np.arange(n)
    for p in range(n):
        s, k = int(starts[p]), int(ra["nops"][p])
        if oa[s:s + k].tobytes() != ob[s:s + k].tobytes():
            raise AssertionError(f"op stream of pair {p} differs")


def ragged_batch(seed, npairs, maxlen):
    """Random DNA pairs of ragged lengths in [0, maxlen], with the edge shapes forced in, and one
    pair in four a mutated copy of its partner (long local paths that cross many blocks)."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    pairs = []
    fixed = [(maxlen, maxlen), (1, maxlen), (maxlen, 1), (0, 5), (5, 0), (63, 64), (64, 63), (65, 65),
             (maxlen, 33), (33, maxlen), (maxlen - 1, maxlen)]
    for p in range(npairs):
        if p < len(fixed):
            m, n = fixed[p]
        else:
            m, n = int(rng.integers(0, maxlen + 1)), int(rng.integers(0, maxlen + 1))
        a = acgt[rng.integers(0, 4, m)]
        if p % 4 == 3 and m > 0 and n > 0:
            b = a.copy()
            mut = rng.random(len(b)) < 0.08
            b[mut] = acgt[rng.integers(0, 4, int(mut.sum()))]
            keep = rng.random(len(b)) > 0.03              # deletions
            b = b[keep]
            ins = np.nonzero(rng.random(len(b)) < 0.03)[0]   # insertions
            b = np.insert(b, ins, acgt[rng.integers(0, 4, len(ins))])[:n]
        else:
            b = acgt[rng.integers(0, 4, n)]
        pairs.append((a.tobytes(), b.tobytes()))
    o1 = np.zeros(npairs + 1, np.uint64)
    o2 = np.zeros(npairs + 1, np.uint64)
    o1[1:] = np.cumsum([len(a) for a, _ in pairs])
    o2[1:] = np.cumsum([len(b) for _, b in pairs])
    s1 = np.frombuffer(b"".join(a for a, _ in pairs), np.uint8).copy()
    s2 = np.frombuffer(b"".join(b for _, b in pairs), np.uint8).copy()
    return s1, o1, s2, o2


@pytest.mark.parametrize("maxlen,R,tb", [(200, 4, "4"), (500, 8, "4"), (1000, 16, "4"), (2000, 32, "4"), (3000, 32, "4"),
                                         (200, 4, "1"), (3000, 32, "1")])
def test_so_ragged_matches_tagged_and_oracle(engine, maxlen, R, tb):
    """Ragged batches on every score-only plan (R = 4 .. 32, one and two bands), both score-only
    tracebacks: identical to the tagged path on every pair, and to the full-matrix oracle on a
    sample."""
    batch = ragged_batch(40 + maxlen, 1100, maxlen)
    so = run(engine, True, *batch, tb=tb)
    tg = run(engine, False, *batch)
    assert so[2] == (sa.SA_KERNEL_T16_ENDCELL, R, 1) and tg[2] == so[2]
    s1, o1, s2, o2 = batch
    assert (so[0]["flags"] == 0).all()
    assert_same(so, tg, o1, o2)
    nonempty = (np.diff(o1) > 0) & (np.diff(o2) > 0)   # (an empty pair keeps MaxScore = INT_MIN)
    assert (linear_rescore(SW, so[0], so[1], o1, o2) == so[0]["score"])[nonempty].all()
    idx = np.sort(np.random.default_rng(maxlen).choice(len(o1) - 1, 48, replace=False))
    idx = np.unique(np.concatenate([np.arange(11), idx]))
    sub = subset(s1, o1, s2, o2, idx)
    ores, oops = oracle_batch(0, SW, *sub, threads=THREADS)
    for q, p in enumerate(idx):
        off = int(o1[p] + o2[p]) + int(p)
        ooff = int(sub[1][q] + sub[3][q]) + q
        got = tuple(int(so[0][f][p]) for f in ("score", "end_i", "end_j", "start_i", "start_j"))
        exp = tuple(int(ores[f][q]) for f in ("score", "end_i", "end_j", "start_i", "start_j"))
        assert got == exp, (int(p), got, exp)
        assert so[1][off:off + int(so[0]["nops"][p])].tobytes() == oops[ooff:ooff + int(ores["nops"][q])].tobytes(), int(p)


@pytest.mark.parametrize("maxlen,R,npairs", [(1000, 16, 1101), (3000, 32, 1100)])
def test_so2_nw_matches_one_pair_per_wave(engine, monkeypatch, maxlen, R, npairs):
    """NeedlemanWunsch with two pairs per wave (fill_so2_kernel<SA_NW, R>) against one pair per wave
    (SEQALIB_SO2=0): identical results (H[m][n] of both pairs of every couple, taken at its one
    step) and op streams on ragged batches, an odd pair count; a sample against the oracle."""
    batch = ragged_batch(190 + maxlen, npairs, maxlen)
    s1, o1, s2, o2 = batch
    a = run(engine, True, *batch, scoring=NW, algo=1)
    monkeypatch.setenv("SEQALIB_SO2", "0")
    b = run(engine, True, *batch, scoring=NW, algo=1)
    monkeypatch.delenv("SEQALIB_SO2")
    assert a[2] == b[2] and a[2][1] == R
    assert (a[0]["flags"] == 0).all()
    assert_same(a, b, o1, o2)
    check_vs_oracle(1, NW, a, batch, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 500, npairs - 1])


@pytest.mark.parametrize("maxlen,R,npairs", [(1000, 16, 1101), (3000, 32, 1100)])
def test_so2_matches_one_pair_per_wave(engine, monkeypatch, maxlen, R, npairs):
    """Two pairs per wave (fill_so2_kernel, the default on the score-only SW plans at R = 16 / 32)
    against one pair per wave (SEQALIB_SO2=0) and against round 5's alphabet-scan launch
    (SEQALIB_SCAN_WG=256): identical results and op streams on ragged batches (an odd pair count
    leaves the last couple's second half empty); every end cell against the linear-space oracle."""
    batch = ragged_batch(90 + maxlen, npairs, maxlen)
    s1, o1, s2, o2 = batch
    a = run(engine, True, *batch)
    monkeypatch.setenv("SEQALIB_SO2", "0")
    b = run(engine, True, *batch)
    monkeypatch.delenv("SEQALIB_SO2")
    monkeypatch.setenv("SEQALIB_SCAN_WG", "256")
    c = run(engine, True, *batch)
    monkeypatch.delenv("SEQALIB_SCAN_WG")
    assert a[2] == (sa.SA_KERNEL_T16_ENDCELL, R, 1) and b[2] == a[2] and c[2] == a[2]
    assert (a[0]["flags"] == 0).all()
    assert_same(a, b, o1, o2)
    assert_same(a, c, o1, o2)
    exp = oracle_sw_scores(SW, s1, o1, s2, o2, threads=THREADS)
    got = np.stack([a[0]["score"], a[0]["end_i"], a[0]["end_j"]], axis=1)
    nonempty = (np.diff(o1) > 0) & (np.diff(o2) > 0)
    bad = np.nonzero((got != exp).any(axis=1) & nonempty)[0]
    assert len(bad) == 0, [(int(p), got[p].tolist(), exp[p].tolist()) for p in bad[:5]]


def test_so_scorings_and_lut(engine):
    """Other scorings (match 2, mismatch -3, gap -2; !AllowMismatch) and a non-identity match table
    on a 4-symbol alphabet (A~G, C~T): identical to the tagged path; a sample against the oracle."""
    batch = ragged_batch(7, 1030, 700)
    s1, o1, s2, o2 = batch
    lut = np.zeros((256, 256), np.uint8)
    for x in b"ACGT":
        lut[x, x] = 1
    for x, y in (b"AG", b"GA", b"CT", b"TC"):
        lut[x, y] = 1
    for scoring, lt in (((-2, 2, -3), None), ((-2, 1, -1, False), None), (SW, lut)):
        so = run(engine, True, *batch, scoring=scoring, lut=lt)
        tg = run(engine, False, *batch, scoring=scoring, lut=lt)
        assert so[2][0] == sa.SA_KERNEL_T16_ENDCELL, scoring
        assert_same(so, tg, o1, o2)
        for p in (0, 1, 2, 3, 11, 12, 13, 14, 15, 1029):
            a, b = s1[o1[p]:o1[p + 1]].tobytes(), s2[o2[p]:o2[p + 1]].tobytes()
            o = oracle_align(0, scoring, a, b, lut=lt)
            off = int(o1[p] + o2[p]) + p
            got = (int(so[0]["score"][p]), int(so[0]["end_i"][p]), int(so[0]["end_j"][p]),
                   so[1][off:off + int(so[0]["nops"][p])].tobytes())
            assert got == (o["score"], o["end_i"], o["end_j"], o["ops"]), (scoring, p)


def test_headline_batch_every_pair(engine):
    """The bench workload itself (bench.py: seed base 1e10, 10,000 x 4096^2, (-1, 1, -1),
    equal<char>): all 10,000 (MaxScore, MaxRow, MaxCol) against the linear-space oracle, 256 full op
    streams against the full-matrix oracle, every op stream identical to the tagged path."""
    s1, o1, s2, o2 = sa.synth_dna_batch(10 ** 10, 10000, 4096, 4096, threads=THREADS)
    so = run(engine, True, s1, o1, s2, o2)
    assert so[2] == (sa.SA_KERNEL_T16_ENDCELL, 32, 1)
    res, ops = so[0], so[1]
    assert (res["flags"] == 0).all()
    assert (linear_rescore(SW, res, ops, o1, o2) == res["score"]).all()
    exp = oracle_sw_scores(SW, s1, o1, s2, o2, threads=THREADS)
    got = np.stack([res["score"], res["end_i"], res["end_j"]], axis=1)
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert len(bad) == 0, [(int(b), got[b].tolist(), exp[b].tolist()) for b in bad[:5]]
    jdx = np.sort(np.random.default_rng(10).choice(10000, 256, replace=False))
    sub = subset(s1, o1, s2, o2, jdx)
    ores, oops = oracle_batch(0, SW, *sub, threads=THREADS)
    for q, p in enumerate(jdx):
        off = int(o1[p] + o2[p]) + int(p)
        ooff = int(sub[1][q] + sub[3][q]) + q
        assert (int(res["start_i"][p]), int(res["start_j"][p])) == (int(ores["start_i"][q]), int(ores["start_j"][q]))
        assert ops[off:off + int(res["nops"][p])].tobytes() == oops[ooff:ooff + int(ores["nops"][q])].tobytes(), int(p)
    tg = run(engine, False, s1, o1, s2, o2)
    assert_same(so, tg, o1, o2)


NW = (-1, 2, -1)   # NeedlemanWunschSA::getDefaultScoring (SANeedlemanWunsch.h:244-247)


def check_vs_oracle(algo, scoring, got, batch, idx, lut=None):
    """Full results and op streams of pairs idx against the full-matrix oracle."""
    s1, o1, s2, o2 = batch
    res, ops = got[0], got[1]
    for p in idx:
        a, b = s1[o1[p]:o1[p + 1]].tobytes(), s2[o2[p]:o2[p + 1]].tobytes()
        o = oracle_align(algo, scoring, a, b, lut=lut)
        off = int(o1[p] + o2[p]) + int(p)
        g = (int(res["score"][p]), int(res["end_i"][p]), int(res["end_j"][p]), int(res["start_i"][p]),
             int(res["start_j"][p]), ops[off:off + int(res["nops"][p])].tobytes())
        assert g == (o["score"], o["end_i"], o["end_j"], o["start_i"], o["start_j"], o["ops"]), (scoring, int(p))


@pytest.mark.parametrize("maxlen,R", [(200, 4), (500, 8), (1000, 16), (2000, 32), (3000, 32)])
def test_so_nw_ragged_matches_tagged_and_oracle(engine, maxlen, R):
    """Score-only NeedlemanWunsch (no records; the walk from (m, n) recomputes its blocks with the NW
    borders i * Gap / j * Gap and the fill's offset delta, then follows the border to (0, 0)):
    ragged batches on every plan, identical to the tagged path on every pair, a sample (and every
    edge shape, empty sides included) against the full-matrix oracle."""
    batch = ragged_batch(80 + maxlen, 1100, maxlen)
    so = run(engine, True, *batch, scoring=NW, algo=1)
    recs = engine.last_plan_ex()[3]
    tg = run(engine, False, *batch, scoring=NW, algo=1)
    assert so[2] == (sa.SA_KERNEL_T16, R, 1) and tg[2] == so[2]
    assert recs == sa.SA_RECORDS_SCORE_ONLY
    s1, o1, s2, o2 = batch
    assert (so[0]["flags"] == 0).all()
    assert_same(so, tg, o1, o2)
    assert (linear_rescore(NW, so[0], so[1], o1, o2) == so[0]["score"]).all()
    idx = np.unique(np.concatenate([np.arange(11), np.random.default_rng(maxlen).choice(len(o1) - 1, 40, replace=False)]))
    check_vs_oracle(1, NW, so, batch, idx)


def test_so_nw_scorings_and_lut(engine):
    """Score-only NW with other scorings -- the reference's 2-argument (Gap, Match) form
    (!AllowMismatch, test/Test.cpp's (-1, 2)), (-2, 1, -1, false), (-2, 2, -3) -- and a non-identity
    match table: identical to the tagged path, a sample against the oracle."""
    batch = ragged_batch(9, 1030, 700)
    lut = np.zeros((256, 256), np.uint8)
    for x in b"ACGT":
        lut[x, x] = 1
    for x, y in (b"AG", b"GA", b"CT", b"TC"):
        lut[x, y] = 1
    for scoring, lt in (((-1, 2), None), ((-2, 1, -1, False), None), ((-2, 2, -3), None), (NW, lut)):
        so = run(engine, True, *batch, scoring=scoring, lut=lt, algo=1)
        assert engine.last_plan_ex()[3] == sa.SA_RECORDS_SCORE_ONLY, scoring
        tg = run(engine, False, *batch, scoring=scoring, lut=lt, algo=1)
        assert_same(so, tg, batch[1], batch[3])
        check_vs_oracle(1, scoring, so, batch, [0, 1, 2, 3, 4, 5, 11, 12, 13, 14, 15, 1029], lut=lt)


def test_so_nw_batch_1024_every_pair(engine):
    """10,000 x 1024^2 NeedlemanWunsch (-1, 2, -1), the configs leg of bench.py: every pair's score
    re-scored from its op stream and consuming all of both sequences, 128 pairs against the oracle,
    every pair identical to the tagged path."""
    s1, o1, s2, o2 = sa.synth_dna_batch(6_000_000_000, 10000, 1024, 1024, threads=THREADS)
    so = run(engine, True, s1, o1, s2, o2, scoring=NW, algo=1)
    assert so[2] == (sa.SA_KERNEL_T16, 16, 1)
    res, ops = so[0], so[1]
    assert (res["flags"] == 0).all()
    assert (linear_rescore(NW, res, ops, o1, o2) == res["score"]).all()
    assert (res["start_i"] == 0).all() and (res["start_j"] == 0).all()
    assert (res["end_i"] == 1024).all() and (res["end_j"] == 1024).all()
    jdx = np.sort(np.random.default_rng(6).choice(10000, 128, replace=False))
    sub = subset(s1, o1, s2, o2, jdx)
    ores, oops = oracle_batch(1, NW, *sub, threads=THREADS)
    for q, p in enumerate(jdx):
        off = int(o1[p] + o2[p]) + int(p)
        ooff = int(sub[1][q] + sub[3][q]) + q
        assert int(res["score"][p]) == int(ores["score"][q]), int(p)
        assert ops[off:off + int(res["nops"][p])].tobytes() == oops[ooff:ooff + int(ores["nops"][q])].tobytes(), int(p)
    tg = run(engine, False, s1, o1, s2, o2, scoring=NW, algo=1)
    assert_same(so, tg, o1, o2)


LG_SIZE_HACK = {(314, 288), (60, 57), (61, 58)}   # SALocalGotoh.h:484-488 (parity unpinned there)
AFF = [(2, (-3, -1, 1, -1, True)), (2, (-3, -1, 1, -1, False)), (3, (-3, -1, 1, -1, True))]


@pytest.mark.parametrize("algo,scoring", AFF)
@pytest.mark.parametrize("maxlen,R", [(200, 4), (500, 8), (1000, 16), (2000, 16)])
def test_so_affine_ragged_matches_tagged_and_oracle(engine, algo, scoring, maxlen, R):
    """Score-only LocalGotoh / GlobalGotoh (the SO affine cell: A = Ix - GOE, B = Iy - GOE, 8 fast ops
    + v_bfe per cell, no records; the traceback recomputes its blocks with the tagged affine cell
    from the snapshots and the 32-bit edge stream): ragged batches on every plan (R = 4, 8, 16; one
    and two bands), identical to the tagged path on every pair, a sample and every edge shape against
    the full-matrix oracle."""
    batch = ragged_batch(120 + maxlen + algo, 1100, maxlen)
    so = run(engine, True, *batch, scoring=scoring, algo=algo)
    recs = engine.last_plan_ex()[3]
    tg = run(engine, False, *batch, scoring=scoring, algo=algo)
    kern = sa.SA_KERNEL_T16_ENDCELL if algo == 2 else sa.SA_KERNEL_T16
    assert so[2] == (kern, R, 1) and tg[2] == so[2]
    assert recs == sa.SA_RECORDS_SCORE_ONLY
    s1, o1, s2, o2 = batch
    assert ((so[0]["flags"] & np.uint32(0xffffffff ^ sa.SA_FLAG_SIZE_HACK)) == 0).all()
    assert_same(so, tg, o1, o2)
    idx = np.unique(np.concatenate([np.arange(11), np.random.default_rng(maxlen + algo).choice(len(o1) - 1, 40, replace=False)]))
    idx = [int(p) for p in idx if (int(o1[p + 1] - o1[p]), int(o2[p + 1] - o2[p])) not in LG_SIZE_HACK]
    check_vs_oracle(algo, scoring, so, batch, idx)


def test_so_affine_lut(engine):
    """Score-only Gotoh with a non-identity match table (A~G, C~T) and (-2, -1, 2, -1): identical to
    the tagged path, a sample against the oracle."""
    batch = ragged_batch(13, 1030, 700)
    lut = np.zeros((256, 256), np.uint8)
    for x in b"ACGT":
        lut[x, x] = 1
    for x, y in (b"AG", b"GA", b"CT", b"TC"):
        lut[x, y] = 1
    for algo in (2, 3):
        for scoring, lt in (((-2, -1, 2, -1, True), None), ((-3, -1, 1, -1, True), lut)):
            so = run(engine, True, *batch, scoring=scoring, lut=lt, algo=algo)
            assert engine.last_plan_ex()[3] == sa.SA_RECORDS_SCORE_ONLY, (algo, scoring)
            tg = run(engine, False, *batch, scoring=scoring, lut=lt, algo=algo)
            assert_same(so, tg, batch[1], batch[3])
            check_vs_oracle(algo, scoring, so, batch, [0, 1, 2, 3, 4, 5, 11, 12, 13, 14, 15, 1029], lut=lt)


@pytest.mark.parametrize("algo", [2, 3])
def test_so_affine_batch_1024(engine, algo):
    """10,000 x 1024^2 LocalGotoh / GlobalGotoh (-3, -1, 1, -1, true), the configs legs of bench.py:
    every pair identical to the tagged path, 96 pairs against the full-matrix oracle."""
    scoring = (-3, -1, 1, -1, True)
    s1, o1, s2, o2 = sa.synth_dna_batch(7_000_000_000 + algo, 10000, 1024, 1024, threads=THREADS)
    so = run(engine, True, s1, o1, s2, o2, scoring=scoring, algo=algo)
    assert so[2][1:] == (16, 1)
    assert (so[0]["flags"] == 0).all()
    jdx = np.sort(np.random.default_rng(algo).choice(10000, 96, replace=False))
    sub = subset(s1, o1, s2, o2, jdx)
    ores, oops = oracle_batch(algo, scoring, *sub, threads=THREADS)
    res, ops = so[0], so[1]
    for q, p in enumerate(jdx):
        off = int(o1[p] + o2[p]) + int(p)
        ooff = int(sub[1][q] + sub[3][q]) + q
        got = tuple(int(res[f][p]) for f in ("score", "end_i", "end_j", "start_i", "start_j"))
        exp = tuple(int(ores[f][q]) for f in ("score", "end_i", "end_j", "start_i", "start_j"))
        assert got == exp, (int(p), got, exp)
        assert ops[off:off + int(res["nops"][p])].tobytes() == oops[ooff:ooff + int(ores["nops"][q])].tobytes(), int(p)
    tg = run(engine, False, s1, o1, s2, o2, scoring=scoring, algo=algo)
    assert_same(so, tg, o1, o2)


def test_so_retry_pair_leaves_neighbours_intact(engine):
    """A score-only SW batch (R = 32 plan) with two pairs above the int16 headroom (identical
    9,000-long sequences: score 9,000) at the front: the int32 variant re-runs exactly those, and
    every other pair -- whose score-only edges and snapshots share the launch's workspace with
    the int32 records -- still equals the tagged path and the oracle."""
    rng = np.random.default_rng(77)
    hot = sa.synth_dna(81_000, 9000)
    pairs = [(hot, hot), (hot[:8800], sa.synth_mutate(hot, 5)[:8900])]
    for k in range(1100):
        a = sa.synth_dna(82_000 + 2 * k, int(rng.integers(600, 1300)))
        b = sa.synth_mutate(a, k) if k % 3 == 0 else sa.synth_dna(82_001 + 2 * k, int(rng.integers(600, 1300)))
        pairs.append((a, b))
    batch = sa.pack_pairs(pairs)
    so = run(engine, True, *batch)
    assert engine.last_plan_ex()[3] == sa.SA_RECORDS_SCORE_ONLY
    tg = run(engine, False, *batch)
    assert_same(so, tg, batch[1], batch[3])
    assert int(so[0]["score"][0]) == 9000
    check_vs_oracle(0, SW, so, batch, [0, 1, 2, 3, 4, 5, 50, 100, 500, 1000, 1101])


@pytest.mark.parametrize("algo,scoring", [(0, SW), (1, (-1, 2, -1))])
def test_so_column_segments_any_count(engine, monkeypatch, algo, scoring):
    """Column segments of the band units (SEQALIB_SO_SEGS; default kSoSegs = 2, two pairs per wave
    kSo2Segs = 8): the same ragged batch with 1, 2, 3, 5 and 8 segments per band (pairs with fewer
    chunks than 2 per segment use fewer) gives identical results and op streams, equal to the
    tagged path."""
    batch = ragged_batch(123 + algo, 1100, 3000)
    s1, o1, s2, o2 = batch
    monkeypatch.delenv("SEQALIB_SO_SEGS", raising=False)
    base = run(engine, True, *batch, scoring=scoring, algo=algo)
    assert engine.last_plan_ex()[3] == sa.SA_RECORDS_SCORE_ONLY
    for segs in ("1", "2", "3", "5", "8"):
        monkeypatch.setenv("SEQALIB_SO_SEGS", segs)
        assert_same(run(engine, True, *batch, scoring=scoring, algo=algo), base, o1, o2)
    monkeypatch.delenv("SEQALIB_SO_SEGS")
    assert_same(base, run(engine, False, *batch, scoring=scoring, algo=algo), o1, o2)


def identical_pairs_batch(seed, npairs, lengths, maxlen=2200):
    """Random pairs of ragged lengths with, first, identical pairs of the given lengths (SW score =
    length at (-1, 1, -1)): scores just below and above the f16 cell's retry threshold."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    pairs = []
    for p in range(npairs):
        if p < len(lengths):
            a = acgt[rng.integers(0, 4, lengths[p])]
            pairs.append((a.tobytes(), a.tobytes()))
        else:
            m, n = int(rng.integers(1, maxlen + 1)), int(rng.integers(1, maxlen + 1))
            pairs.append((acgt[rng.integers(0, 4, m)].tobytes(), acgt[rng.integers(0, 4, n)].tobytes()))
    o1 = np.zeros(npairs + 1, np.uint64)
    o2 = np.zeros(npairs + 1, np.uint64)
    o1[1:] = np.cumsum([len(a) for a, _ in pairs])
    o2[1:] = np.cumsum([len(b) for _, b in pairs])
    s1 = np.frombuffer(b"".join(a for a, _ in pairs), np.uint8).copy()
    s2 = np.frombuffer(b"".join(b for _, b in pairs), np.uint8).copy()
    return s1, o1, s2, o2


def test_so2_f16_threshold_pairs(engine, monkeypatch):
    """The f16 cell (fill_so2_kernel FK, exact below 2048) at its threshold: identical pairs scoring
    1,990 .. 3,000 among random ones -- the ones above the retry threshold re-run in int32 -- against
    the 16-bit integer cell (SEQALIB_SO2_F16=0) and the oracle; 10 flagged pairs of 1,100 leave the
    cell on (SA_HOOK_F16)."""
    engine.test_hook(sa.SA_HOOK_F16, 0)
    lengths = [1990, 1993, 1994, 1999, 2005, 2040, 2047, 2048, 2049, 2100, 2500, 3000]
    batch = identical_pairs_batch(5, 1100, lengths)
    s1, o1, s2, o2 = batch
    a = run(engine, True, *batch)
    monkeypatch.setenv("SEQALIB_SO2_F16", "0")
    b = run(engine, True, *batch)
    monkeypatch.delenv("SEQALIB_SO2_F16")
    assert (a[0]["flags"] == 0).all()
    assert [int(x) for x in a[0]["score"][:len(lengths)]] == lengths
    assert_same(a, b, o1, o2)
    check_vs_oracle(0, SW, a, batch, list(range(len(lengths))) + [500, 1099])
    run(engine, True, *batch)
    assert engine.test_hook(sa.SA_HOOK_F16, 2) == 0


def test_so2_f16_policy_high_identity(engine, monkeypatch):
    """A batch of near-identical 3,000-symbol pairs (scores ~2,800: every pair re-runs in int32 after
    the f16 cell) is exact, and its launch turns the f16 cell off for the context: the next call runs
    the 16-bit integer cell, with the same results."""
    engine.test_hook(sa.SA_HOOK_F16, 0)
    try:
        rng = np.random.default_rng(11)
        acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
        pairs = []
        for p in range(1030):
            a = acgt[rng.integers(0, 4, 3000)]
            b = a.copy()
            mut = rng.random(3000) < 0.02
            b[mut] = acgt[rng.integers(0, 4, int(mut.sum()))]
            pairs.append((a.tobytes(), b.tobytes()))
        o1 = np.arange(1031, dtype=np.uint64) * 3000
        o2 = o1.copy()
        s1 = np.frombuffer(b"".join(x for x, _ in pairs), np.uint8).copy()
        s2 = np.frombuffer(b"".join(y for _, y in pairs), np.uint8).copy()
        a = run(engine, True, s1, o1, s2, o2)
        assert (a[0]["flags"] == 0).all() and (a[0]["score"] > 2000).all()
        monkeypatch.setenv("SEQALIB_SO2_F16", "0")
        b = run(engine, True, s1, o1, s2, o2)
        monkeypatch.delenv("SEQALIB_SO2_F16")
        assert_same(a, b, o1, o2)
        assert engine.test_hook(sa.SA_HOOK_F16, 2) == 1
        c = run(engine, True, s1, o1, s2, o2)
        assert_same(a, c, o1, o2)
        check_vs_oracle(0, SW, a, (s1, o1, s2, o2), [0, 1, 515, 1029])
    finally:
        engine.test_hook(sa.SA_HOOK_F16, 0)
