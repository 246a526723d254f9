"""GPU parity of the generic-Ty path: sequences of arbitrary symbols
(here Python ints with thousands of distinct values, more than the 256 byte codes of the symbol
path) and arbitrary match predicates, aligned through sa_align_batch_bits (per-pair match
bitmaps = the reference's cacheAllMatches, SASmithWaterman.h:20-45, SequenceAlignment.h:143-147)
and compared bit-exactly with the oracle driven by the same match matrices."""
import numpy as np
import pytest

import seqalib_amd as sa
from util import oracle_align_matrix

pytestmark = pytest.mark.gpu

SCORINGS = {0: [(-1, 2, -1), (-2, 1, -1, False)], 1: [(-1, 2, -1), (-1, 2)],
            2: [(-3, -1, 2, -1), (-3, -1, 1, -1, False)], 3: [(-3, -1, 2, -1)],
            4: [(-1, 2, -1), (-2, 1, -1, False)], 5: [(-3, -1, 2, -1), (-3, -1, 1, -1, False)]}
PREDICATES = {"equal": None, "near": lambda x, y: abs(x - y) <= 2, "mod7": lambda x, y: x % 7 == y % 7}


def int_pairs(seed, count, lo, hi, vocab=5000):
    rng = np.random.default_rng(seed)
    pairs = []
    for k in range(count):
        m = int(rng.integers(lo, hi))
        a = [int(x) for x in rng.integers(0, vocab, m)]
        if k % 2:   # related: substitutions and indels
            b = []
            for x in a:
                r = rng.random()
                if r < 0.08:
                    b.append(int(rng.integers(0, vocab)))
                elif r < 0.11:
                    b.extend([x, int(rng.integers(0, vocab))])
                elif r < 0.14:
                    continue
                else:
                    b.append(x)
        else:
            b = [int(x) for x in rng.integers(0, vocab, int(rng.integers(lo, hi)))]
        pairs.append((a, b))
    return pairs


def matrix(a, b, match):
    if not a or not b:
        return np.zeros((len(a), len(b)), dtype=np.uint8)
    A = np.array(a)[:, None]
    B = np.array(b)[None, :]
    if match is None:
        return (A == B).astype(np.uint8)
    if match is PREDICATES["near"]:
        return (np.abs(A - B) <= 2).astype(np.uint8)
    return ((A % 7) == (B % 7)).astype(np.uint8)


def check(engine, algo, args, pairs, match):
    res = engine.align_generic(algo, sa.ScoringSystem(*args), pairs, match)
    for (a, b), r in zip(pairs, res):
        o = oracle_align_matrix(algo, args, matrix(a, b, match))
        assert o["rc"] == 0
        got = (r.score, r.end_i, r.end_j, r.start_i, r.start_j, r.ops)
        exp = (o["score"], o["end_i"], o["end_j"], o["start_i"], o["start_j"], o["ops"])
        assert got == exp, (algo, args, len(a), len(b))
        assert (r.flags & ~sa.SA_FLAG_SIZE_HACK) == 0


@pytest.mark.parametrize("algo", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("pred", list(PREDICATES))
def test_generic_ints_vs_oracle(engine, algo, pred):
    """Lists of ints, ~5000 distinct values per batch, few pairs (one wave per pair traceback);
    HirschbergSA / MyersMillerSA (4, 5) run their whole-wave and packed sweeps and their leaves on
    pair-local indices and the pairs' bitmaps (SAHirschberg.h:74, :90; SAMyersMiller.h:24-37)."""
    pairs = int_pairs(10 + algo, 24, 50, 700)
    pairs += [([], [1, 2, 3]), ([4], []), (list(range(1000, 1314)), list(range(1100, 1388)))]   # empty, size hack
    distinct = {x for a, b in pairs for x in a + b}
    assert len(distinct) > 1000
    for args in SCORINGS[algo]:
        check(engine, algo, args, pairs, PREDICATES[pred])


@pytest.mark.parametrize("algo", [0, 2])
def test_generic_many_pairs_and_single_long_pair(engine, algo):
    """The batch plans (>= 1024 pairs: one lane per pair traceback) and the multi-workgroup plan
    of a single long pair run the bitmap path too."""
    pairs = int_pairs(40 + algo, 1100, 20, 160, vocab=3000)
    check(engine, algo, SCORINGS[algo][0], pairs, PREDICATES["near"])
    big = int_pairs(50 + algo, 2, 1500, 1600, vocab=2000)[1:]
    check(engine, algo, SCORINGS[algo][0], big, None)


def test_generic_objects_unhashable(engine):
    """Unhashable symbols (lists) fall back to one predicate call per cell, as the reference's
    cacheAllMatches does."""
    a = [[k % 13, k % 5] for k in range(90)]
    b = [[k % 13, (k + 1) % 5] for k in range(70)]
    same_first = lambda x, y: x[0] == y[0]
    res = engine.align_generic(0, sa.ScoringSystem(-1, 2, -1), [(a, b)], same_first)[0]
    mt = np.array([[same_first(x, y) for y in b] for x in a], dtype=np.uint8)
    o = oracle_align_matrix(0, (-1, 2, -1), mt)
    assert (res.score, res.end_i, res.end_j, res.ops) == (o["score"], o["end_i"], o["end_j"], o["ops"])


def test_bits_path_equals_symbol_path(engine):
    """DNA through the bitmap path gives exactly what the byte-symbol path gives."""
    pairs = [(sa.synth_dna(300 + k, 200 + 37 * k), sa.synth_dna(400 + k, 180 + 29 * k)) for k in range(40)]
    for algo, args in ((0, (-1, 1, -1)), (1, (-1, 2, -1)), (2, (-3, -1, 1, -1)), (3, (-3, -1, 1, -1)),
                       (4, (-1, 2, -1)), (5, (-3, -1, 1, -1))):
        ref = engine.align(algo, sa.ScoringSystem(*args), pairs)
        got = engine.align_generic(algo, sa.ScoringSystem(*args), [(list(a), list(b)) for a, b in pairs])
        for r, g in zip(ref, got):
            assert (r.score, r.end_i, r.end_j, r.start_i, r.start_j, r.ops) == \
                   (g.score, g.end_i, g.end_j, g.start_i, g.start_j, g.ops)


@pytest.mark.parametrize("algo", [4, 5])
def test_generic_linear_space_batch(engine, algo):
    """HirschbergSA / MyersMillerSA over a batch of 300 wide-alphabet pairs up to 1,500 long
    (several device levels with R = 16 whole-wave sweeps, then packed sweeps and leaves), against
    the matrix-driven oracle."""
    pairs = int_pairs(60 + algo, 300, 10, 400, vocab=4000) + int_pairs(70 + algo, 4, 1200, 1500, vocab=4000)
    check(engine, algo, SCORINGS[algo][0], pairs, PREDICATES["near"])
