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
