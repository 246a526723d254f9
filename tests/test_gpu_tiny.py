"""GPU parity of the small-call path (sa_tiny.hip): host calls of at most 64 pairs with
m <= 256, n <= 1024 and m * n <= 32768 run as ONE kernel that fills each pair in one wave (int32
cells, flags in LDS) and walks its traceback in the same workgroup, reading and writing pinned
host memory.  The reference's canonical use is exactly such a call: one getAlignment() per pair
(include/Test.cpp:98-144, test/Test.cpp:44-45).

Bar: bit-exact against the C oracle (score, end cell, start cell, op stream and the three
alignment rows), on every scoring overload the batch tests use, DNA and wide alphabets, custom
match tables, empty sides and the size limits; and identical to the batch kernels
(SEQALIB_TINY=0) on the same calls.
"""
import numpy as np
import pytest

import seqalib_amd as sa
from util import named_lut, oracle_align

pytestmark = pytest.mark.gpu

SCORINGS = {0: [(-1, 1, -1), (-2, 1, -1, False), (-1, 2), (-3, 2, -2)],
            1: [(-1, 2, -1), (-1, 2), (-2, 1, -1, False)],
            2: [(-3, -1, 1, -1, False), (-3, -1, 1, -1, True), (-2, -1, 2, -1, True)],
            3: [(-3, -1, 1, -1, True), (-3, -1, 1, -1, False), (-5, -2, 3, -2, True)]}
LG_SIZE_HACK = {(314, 288), (60, 57), (61, 58)}   # SALocalGotoh.h:484-488 (NW on those sizes)


def rows_of(algo, a, b, r):
    return sa.expand_ops(algo if not (r.flags & sa.SA_FLAG_SIZE_HACK) else sa.SA_NW,
                         a.decode("latin-1"), b.decode("latin-1"), r).rows()


def check(engine, algo, args, pairs, match=None, expect_tiny=True):
    lut = named_lut(match)
    res = engine.align(algo, sa.ScoringSystem(*args), pairs, lut)
    if expect_tiny:
        assert engine.last_plan_ex()[0] == sa.SA_KERNEL_TINY
    for (a, b), r in zip(pairs, res):
        o = oracle_align(algo if not (r.flags & sa.SA_FLAG_SIZE_HACK) else sa.SA_NW, args, a, b, lut)
        assert o["rc"] == 0
        got = (r.score, r.end_i, r.end_j, r.start_i, r.start_j, r.ops)
        exp = (o["score"], o["end_i"], o["end_j"], o["start_i"], o["start_j"], o["ops"])
        assert got == exp, (algo, args, len(a), len(b))
        assert rows_of(algo, a, b, r) == o["rows"]
    return res


def small_pairs(seed, count, alphabet=b"ACGT", related=True):
    """count pairs within the small-call limits: thin, square and wide shapes, empty sides."""
    rng = np.random.default_rng(seed)
    sym = np.frombuffer(alphabet, dtype=np.uint8)
    pairs = []
    for k in range(count):
        kind = k % 6
        if kind == 0:
            m, n = int(rng.integers(0, 3)), int(rng.integers(0, 40))
        elif kind == 1:
            m, n = int(rng.integers(1, 65)), int(rng.integers(1, 65))
        elif kind == 2:
            m, n = int(rng.integers(65, 257)), int(rng.integers(1, 128))
        elif kind == 3:
            m, n = int(rng.integers(1, 32)), int(rng.integers(200, 1025))
        elif kind == 4:
            m, n = int(rng.integers(100, 181)), int(rng.integers(100, 181))
        else:
            m, n = int(rng.integers(0, 40)), int(rng.integers(0, 3))
        n = min(n, 32768 // max(m, 1))
        a = sym[rng.integers(0, len(sym), m)].tobytes()
        if related and k % 2 and m:
            b = bytearray(a[: n])
            for q in range(len(b)):
                if rng.random() < 0.15:
                    b[q] = int(sym[rng.integers(0, len(sym))])
            b = bytes(b) + sym[rng.integers(0, len(sym), max(0, n - len(b)))].tobytes()
        else:
            b = sym[rng.integers(0, len(sym), n)].tobytes()
        pairs.append((a, b))
    return pairs


def test_readme_known_answer_one_kernel(engine):
    """test/Test.cpp's pair through the small-call kernel: the README alignment and score 9."""
    r = check(engine, sa.SA_NW, (-1, 2), [(b"AAAGAATGCAT", b"AAACTCAT")])[0]
    assert sa.expand_ops(sa.SA_NW, "AAAGAATGCAT", "AAACTCAT", r).rows() == \
        ("AAA-GAATGCAT", "|||    | |||", "AAAC---T-CAT")
    assert r.score == 9
    assert engine.last_timings()[2] == 0   # no launch of the batch fill kernels


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_small_calls_vs_oracle(engine, algo):
    """Every scoring of the algorithm on 60 ragged DNA pairs (R = 4 rows per lane: m up to 256)
    and on 40 pairs of <= 64 rows (R = 1), one pair per call and whole batches."""
    for args in SCORINGS[algo]:
        pairs = [p for p in small_pairs(200 + algo, 60) if algo != 2 or (len(p[0]), len(p[1])) not in LG_SIZE_HACK]
        check(engine, algo, args, pairs)
        short = [(a[:64], b) for a, b in small_pairs(300 + algo, 40)]
        check(engine, algo, args, short)
        assert engine.last_plan()[1] == 1
        for p in pairs[:12]:
            check(engine, algo, args, [p])


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_small_calls_wide_alphabet_and_tables(engine, algo):
    """Byte alphabets beyond DNA (the int32 cells take any symbols) and custom match tables (the
    match-bit rows of the Seq1 symbols present, built on the host)."""
    args = SCORINGS[algo][0]
    check(engine, algo, args, small_pairs(400 + algo, 50, alphabet=bytes(range(33, 120))))
    check(engine, algo, args, small_pairs(500 + algo, 50, alphabet=b"ACGTN"), match="nwild")
    check(engine, algo, args, small_pairs(600 + algo, 50), match="purine")


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_small_call_limits(engine, algo):
    """The shape limits: 256 x 128, 32 x 1024, 181 x 181, 64 pairs; one row / one column; empty
    sides; and the first shapes past a limit go to the batch kernels with the same results."""
    args = SCORINGS[algo][1 % len(SCORINGS[algo])]
    edge = [(sa.synth_dna(1, 256), sa.synth_dna(2, 128)), (sa.synth_dna(3, 32), sa.synth_dna(4, 1024)),
            (sa.synth_dna(5, 181), sa.synth_mutate(sa.synth_dna(5, 181), 1)[:181]), (b"A", b"A"), (b"A", b"C"),
            (b"", b""), (b"", b"ACGT"), (b"ACGT", b""), (sa.synth_dna(6, 1), sa.synth_dna(7, 1024))]
    check(engine, algo, args, edge)
    check(engine, algo, args, small_pairs(700 + algo, 64))
    for past in ([(sa.synth_dna(8, 257), sa.synth_dna(9, 100))], [(sa.synth_dna(10, 20), sa.synth_dna(11, 1025))],
                 [(sa.synth_dna(12, 200), sa.synth_dna(13, 200))], small_pairs(800 + algo, 65)):
        check(engine, algo, args, past, expect_tiny=False)
        assert engine.last_plan_ex()[0] != sa.SA_KERNEL_TINY


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_small_calls_equal_batch_kernels(engine, algo, monkeypatch):
    """The same calls through the batch kernels (SEQALIB_TINY=0): identical results and ops."""
    pairs = [p for p in small_pairs(900 + algo, 64) if algo != 2 or (len(p[0]), len(p[1])) not in LG_SIZE_HACK]
    for args in SCORINGS[algo]:
        a = engine.align(algo, sa.ScoringSystem(*args), pairs)
        assert engine.last_plan_ex()[0] == sa.SA_KERNEL_TINY
        monkeypatch.setenv("SEQALIB_TINY", "0")
        b = engine.align(algo, sa.ScoringSystem(*args), pairs)
        assert engine.last_plan_ex()[0] != sa.SA_KERNEL_TINY
        monkeypatch.delenv("SEQALIB_TINY")
        for x, y in zip(a, b):
            assert (x.score, x.end_i, x.end_j, x.start_i, x.start_j, x.flags, x.ops) == \
                   (y.score, y.end_i, y.end_j, y.start_i, y.start_j, y.flags, y.ops)


def test_local_gotoh_size_hack_small(engine):
    """LocalGotoh's size hack (60 x 57 and 61 x 58 run NW, SALocalGotoh.h:484-488) inside a small
    call: the hack pairs go through their own NW small call and merge back."""
    pairs = [(sa.synth_dna(20, 60), sa.synth_dna(21, 57)), (sa.synth_dna(22, 50), sa.synth_dna(23, 40)),
             (sa.synth_dna(24, 61), sa.synth_dna(25, 58))]
    res = check(engine, 2, (-3, -1, 1, -1, True), pairs)
    assert [bool(r.flags & sa.SA_FLAG_SIZE_HACK) for r in res] == [True, False, True]
