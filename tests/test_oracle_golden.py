"""CPU: the C restatement (oracle/sa_oracle.c) against golden vectors from the unmodified reference.

This pins the oracle that the GPU parity tests use on random inputs.  Each vector was produced
by oracle/_ref (the reference headers compiled in place) via tests/golden/make_golden.py.
"""
import pytest

from util import ALGOS, golden_sequences, load_golden, named_lut, oracle_align, rows_digest, sha

KAT = load_golden("kat.jsonl")
RND = load_golden("random.jsonl")
BIG = load_golden("large.jsonl")
HB = load_golden("hirschberg.jsonl")
MM = load_golden("myersmiller.jsonl")


def check(e):
    s1, s2 = golden_sequences(e)
    if "s1_sha" in e:
        assert sha(s1) == e["s1_sha"], "generator drift"
    if "s2_sha" in e:
        assert sha(s2) == e["s2_sha"], "generator drift"
    o = oracle_align(ALGOS[e["algo"]], e["scoring"], s1, s2, named_lut(e["match"]))
    assert o["rc"] == 0
    if e["score"] is not None:   # None: the reference exposes no score (MyersMillerSA)
        assert o["score"] == e["score"], e["id"]
    assert (o["end_i"], o["end_j"]) == (e["max_row"], e["max_col"]), e["id"]
    assert len(o["rows"][0]) == e["len"], e["id"]
    if "rows" in e:
        assert list(o["rows"]) == e["rows"], e["id"]
    else:
        assert rows_digest(*o["rows"]) == e["rows_sha"], e["id"]


def test_readme_known_answer():
    # README.md:28-37, test/Test.cpp:31-37: NW, ScoringSystem(-1,2), equal<char>
    o = oracle_align(1, (-1, 2), b"AAAGAATGCAT", b"AAACTCAT")
    assert o["rows"] == ("AAA-GAATGCAT", "|||    | |||", "AAAC---T-CAT")
    assert o["score"] == 9


@pytest.mark.parametrize("chunk", range(8))
def test_oracle_kat(chunk):
    for e in KAT[chunk::8]:
        check(e)


def test_oracle_hirschberg():
    """HirschbergSA restatement (SAHirschberg.h) vs the reference's own output."""
    assert len(HB) > 500
    for e in HB:
        check(e)


def test_oracle_myers_miller():
    """MyersMillerSA restatement (SAMyersMiller.h:43-420) vs the reference's own output."""
    assert len(MM) > 800
    for e in MM:
        check(e)


def test_oracle_random():
    for e in RND:
        check(e)


@pytest.mark.parametrize("e", BIG, ids=[e["id"] for e in BIG])
def test_oracle_large(e):
    check(e)


def _sw_equal_entries():
    return [e for e in KAT + RND + BIG if e["algo"] == "sw" and e["match"] in ("equal", None)]


def test_oracle_sw_score_batch_vs_golden():
    """The linear-space SW score/end-cell oracle (used to check whole north-star batches) against
    every SW golden vector with byte equality, batched as the GPU tests batch it."""
    import numpy as np
    from util import oracle_sw_scores, pack_bytes
    groups = {}
    for e in _sw_equal_entries():
        groups.setdefault(tuple(e["scoring"]), []).append(e)
    n = 0
    for args, es in groups.items():
        pairs = [golden_sequences(e) for e in es]
        s1, o1, s2, o2 = pack_bytes(pairs)
        out = oracle_sw_scores(args, s1, o1, s2, o2, threads=4)
        for e, row in zip(es, out):
            exp_score = e["score"] if e["m"] and e["n"] else -(2 ** 31)
            assert (int(row[0]), int(row[1]), int(row[2])) == (exp_score, e["max_row"], e["max_col"]), e["id"]
            n += 1
    assert n > 200


def test_oracle_sw_score_lanes_match_scalar():
    """The 8-lane (AVX2) form of the linear-space SW score oracle, taken for runs of 8 pairs of equal
    shape, returns exactly what the scalar form returns pair by pair (batches of one pair take the
    scalar form): random and related DNA, every scoring kind, shapes 1 x n, m x 1 and square."""
    import numpy as np
    from util import oracle_sw_scores, pack_bytes
    import seqalib_amd as sa
    for (m, n) in ((1, 37), (37, 1), (64, 64), (150, 97), (301, 300)):
        pairs = []
        for k in range(16):
            a = sa.synth_dna(7000 + 31 * k + m, m)
            b = sa.synth_mutate(a, k)[:n] if k % 3 == 0 else sa.synth_dna(8000 + 17 * k + n, n)
            b = (b + b"ACGT" * n)[:n]
            pairs.append((a, b))
        for args in ((-1, 1, -1), (-2, 2, -3), (-1, 2), (-2, 1, -1, False), (-1, 3, 1)):
            s1, o1, s2, o2 = pack_bytes(pairs)
            lanes = oracle_sw_scores(args, s1, o1, s2, o2, threads=2)
            for p, (a, b) in enumerate(pairs):
                one = oracle_sw_scores(args, *pack_bytes([(a, b)]), threads=1)
                assert np.array_equal(lanes[p], one[0]), (m, n, args, p)


def test_oracle_batch_matches_single():
    """oracle_batch (threaded, packed) returns exactly what oracle_align returns per pair."""
    import numpy as np
    from util import oracle_batch, pack_bytes
    import seqalib_amd as sa
    pairs = [(sa.synth_dna(40 + k, 50 + 13 * k), sa.synth_mutate(sa.synth_dna(40 + k, 50 + 13 * k), k))
             for k in range(24)] + [(b"", b"ACGT"), (b"A", b"")]
    for algo, args in ((0, (-1, 1, -1)), (1, (-1, 2, -1)), (2, (-3, -1, 1, -1)), (3, (-3, -1, 1, -1))):
        s1, o1, s2, o2 = pack_bytes(pairs)
        res, ops = oracle_batch(algo, args, s1, o1, s2, o2, threads=3)
        for p, (a, b) in enumerate(pairs):
            o = oracle_align(algo, args, a, b)
            off = int(o1[p] + o2[p]) + p
            got = (int(res["score"][p]), int(res["end_i"][p]), int(res["end_j"][p]), int(res["start_i"][p]),
                   int(res["start_j"][p]), ops[off:off + int(res["nops"][p])].tobytes())
            assert got == (o["score"], o["end_i"], o["end_j"], o["start_i"], o["start_j"], o["ops"]), (algo, p)


def test_oracle_matrix_form_matches_symbol_form():
    """oracle_align_matrix (generic Ty: an m x n match matrix) equals oracle_align on byte symbols
    whose match matrix it is, for every algorithm (HirschbergSA and MyersMillerSA included: their
    match is taken by position there), equality and a LUT."""
    import numpy as np
    from util import oracle_align_matrix
    import seqalib_amd as sa
    lut = named_lut("purine")
    pairs = [(sa.synth_dna(70 + k, 30 + 17 * k), sa.synth_mutate(sa.synth_dna(70 + k, 30 + 17 * k), k)) for k in range(10)]
    pairs += [(b"", b"ACG"), (b"A", b""), (b"A" * 314, b"C" * 288)]   # empty sides, LocalGotoh size hack
    for algo, args in ((0, (-1, 1, -1)), (0, (-2, 1, -1, False)), (1, (-1, 2, -1)), (1, (-1, 2)),
                       (2, (-3, -1, 1, -1)), (2, (-3, -1, 1, -1, False)), (3, (-3, -1, 1, -1)),
                       (4, (-1, 2, -1)), (4, (-2, 1, -1, False)), (5, (-3, -1, 2, -1)), (5, (-3, -1, 1, -1, False))):
        for table in (None, lut):
            for a, b in pairs:
                av = np.frombuffer(a, np.uint8) if a else np.zeros(0, np.uint8)
                bv = np.frombuffer(b, np.uint8) if b else np.zeros(0, np.uint8)
                mt = (av[:, None] == bv[None, :]) if table is None else table[av[:, None], bv[None, :]] != 0
                got = oracle_align_matrix(algo, args, mt.reshape(len(a), len(b)))
                exp = oracle_align(algo, args, a, b, table)
                assert got["rc"] == 0
                assert [got[k] for k in ("score", "end_i", "end_j", "start_i", "start_j", "ops")] == \
                       [exp[k] for k in ("score", "end_i", "end_j", "start_i", "start_j", "ops")], (algo, args, len(a))


def test_match_bitmaps_layout():
    """seqalib_amd.match_bitmaps packs bit (j % 32) of word [i * ceil(n/32) + j / 32] = match."""
    import numpy as np
    import seqalib_amd as sa
    rng = np.random.default_rng(1)
    pairs = [(list(rng.integers(0, 2000, 70)), list(rng.integers(0, 2000, 45))), ([], [1, 2]), ([3], list(range(33)))]
    near = lambda x, y: abs(int(x) - int(y)) <= 40
    for match in (None, near):
        off1, off2, bits, bits_off = sa.match_bitmaps(pairs, match)
        for p, (a, b) in enumerate(pairs):
            m, n = len(a), len(b)
            wn = (n + 31) // 32
            assert int(bits_off[p + 1] - bits_off[p]) == m * wn
            w = bits[int(bits_off[p]):int(bits_off[p + 1])].reshape(m, wn) if m and wn else np.zeros((m, wn), np.uint32)
            for i in range(m):
                for j in range(n):
                    exp = (a[i] == b[j]) if match is None else near(a[i], b[j])
                    assert bool((int(w[i, j // 32]) >> (j % 32)) & 1) == bool(exp)


def test_match_bitmaps_type_sensitive_predicate():
    """Symbols that hash and compare equal but differ in type (1, 1.0, True) are not merged: a
    MatchFnTy that tells them apart gets the per-cell answers the reference's cacheAllMatches
    would record."""
    import numpy as np
    import seqalib_amd as sa
    a = [1, 1.0, True, 2]
    b = [True, 1, 1.0, 2.0]
    same = lambda x, y: x == y and type(x) is type(y)
    off1, off2, bits, bits_off = sa.match_bitmaps([(a, b)], same)
    w = int(bits[0]), int(bits[1]), int(bits[2]), int(bits[3])
    for i in range(4):
        for j in range(4):
            assert bool((w[i] >> j) & 1) == same(a[i], b[j]), (i, j)
