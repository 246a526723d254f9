"""GPU: the C++ header-only drop-in (include/seqalib/) used exactly like the reference's API.

* tests/cpp/dropin_driver — SmithWatermanSA / NeedlemanWunschSA / LocalGotohSA / GlobalGotohSA
  <std::string, char, '-'> over every literal golden vector; printed alignments must equal the
  reference's.
* tests/cpp/dropin_types — the same source compiled against the unmodified reference in the
  build container produced tests/golden/dropin_types.ref.txt; the drop-in build must print the
  identical text (std::vector<int> + predicate, ArrayView + StaticFuncs::useNW/bridgeNW, batch,
  SmithWaterman member persistence on empty input).
* tests/cpp/dropin_wide — std::vector<int> with ~2,000 distinct values (more than the 256 byte
  codes), equality / a "within 1" predicate, all four aligners: the drop-in takes the
  match-bitmap path and must print what the reference build printed (dropin_wide.ref.txt).
* tests/cpp/dropin_bridge — anchor gaps of three sequence pairs bridged with NW: the reference
  build calls StaticFuncs::bridgeNW per window (tests/golden/dropin_bridge.ref.txt); the
  drop-in build sends every window through StaticFuncs::bridgeNWBatch in one GPU pass.
"""
import os
import subprocess

import pytest

from util import GOLDEN, ROOT, load_golden, scoring_fields

pytestmark = pytest.mark.gpu
CPP = os.path.join(ROOT, "tests", "cpp")


@pytest.fixture(scope="module")
def binaries():
    subprocess.check_call(["make", "-s", "-C", CPP])
    return (os.path.join(CPP, "dropin_driver"), os.path.join(CPP, "dropin_types"),
            os.path.join(CPP, "dropin_bridge"), os.path.join(CPP, "dropin_wide"))


def case_line(e):
    args = e["scoring"]
    nargs = len(args)
    if nargs == 4 and not isinstance(args[3], bool):
        nargs = 5
    a = list(args) + [0] * (5 - len(args))
    if nargs == 2:
        a0, a1, a2, a3, allow = a[0], a[1], 0, 0, 0
    elif nargs in (3, 4):
        a0, a1, a2, a3, allow = a[0], a[1], a[2], 0, int(args[3]) if nargs == 4 else 1
    else:
        a0, a1, a2, a3, allow = a[0], a[1], a[2], a[3], int(args[4]) if len(args) == 5 else 1
    return f"{e['algo']} {nargs} {a0} {a1} {a2} {a3} {allow} {e['match']} {e['s1'] or '.'} {e['s2'] or '.'}"


def test_driver_matches_reference_vectors(binaries, engine):
    entries = [e for src in ("kat.jsonl", "random.jsonl", "hirschberg.jsonl", "myersmiller.jsonl") for e in load_golden(src)
               if isinstance(e["s1"], str) and isinstance(e["s2"], str) and e["match"] in ("equal", "null", "purine")
               and "rows" in e]
    assert len(entries) > 2000
    inp = "\n".join(case_line(e) for e in entries) + "\n"
    out = subprocess.run([binaries[0]], input=inp, capture_output=True, text=True, timeout=600, check=True).stdout
    lines = out.split("\n")
    for e, line in zip(entries, lines):
        r0, bars, r1, score = line.split("\t")
        assert [r0, bars, r1] == e["rows"], e["id"]
        if e["score"] is not None:
            assert int(score) == e["score"], e["id"]


def test_generic_types_match_reference_build(binaries, engine):
    ref = open(os.path.join(GOLDEN, "dropin_types.ref.txt")).read()
    out = subprocess.run([binaries[1]], capture_output=True, text=True, timeout=300, check=True).stdout
    assert out == ref


def test_batched_bridging_matches_reference_bridgeNW(binaries, engine):
    ref = open(os.path.join(GOLDEN, "dropin_bridge.ref.txt")).read()
    out = subprocess.run([binaries[2]], capture_output=True, text=True, timeout=300, check=True).stdout
    assert out == ref


def test_wide_alphabet_matches_reference_build(binaries, engine):
    ref = open(os.path.join(GOLDEN, "dropin_wide.ref.txt")).read()
    out = subprocess.run([binaries[3]], capture_output=True, text=True, timeout=300, check=True).stdout
    assert out == ref


def test_types_over_two_contexts_matches_reference_build(binaries, engine):
    """SEQALIB_DEVICES=0,0: the C++ drop-in spreads its batches over two contexts (sa_multi);
    the printed output is unchanged."""
    ref = open(os.path.join(GOLDEN, "dropin_types.ref.txt")).read()
    env = dict(os.environ, SEQALIB_DEVICES="0,0")
    out = subprocess.run([binaries[1]], capture_output=True, text=True, timeout=300, check=True, env=env).stdout
    assert out == ref


def _fnv(s: str) -> int:
    h = 1469598103934665603
    for c in s.encode("latin-1"):
        h = ((h ^ c) * 1099511628211) & (2 ** 64 - 1)
    return h


@pytest.mark.parametrize("algo,code,args", [("sw", 0, (-1, 1, -1)), ("nw", 1, (-1, 2, -1)), ("lg", 2, (-3, -1, 1, -1))])
def test_chunked_batch_lists_match_oracle(binaries, engine, algo, code, args):
    """tests/cpp/dropin_chunks: 4,500 pairs through getAlignments(), aligned as three chunks of one
    sa_align_batch_cb call whose lists are built while later chunks run (SequenceAlignment.h run;
    LocalGotoh lands as one range after its size-hack split): every pair's printAlignment rows
    must equal the full-matrix oracle's (getAlignment incl. forceGlobal for the local modes)."""
    import numpy as np
    import seqalib_amd as sa
    from util import oracle_batch, pack_bytes
    P = 4500
    env = dict(os.environ, SEQALIB_LIST_CHUNK_PAIRS="2048")   # (chunking is opt-in since round 6)
    out = subprocess.run([os.path.join(CPP, "dropin_chunks"), str(P), algo], capture_output=True, text=True,
                         timeout=240, check=True, env=env).stdout.split()
    assert len(out) == P
    pairs = []
    for p in range(P):
        m, n = 40 + (37 * p) % 260, 30 + (53 * p) % 270
        a = sa.synth_dna(7_000_000_000 + 2 * p + 1, m)
        b = bytearray(sa.synth_dna(7_000_000_000 + 2 * p + 2, n))
        if p % 3 == 0:
            for k in range(min(m, n)):
                if k % 11 != 5:
                    b[k] = a[k]
        pairs.append((a, bytes(b)))
    s1, o1, s2, o2 = pack_bytes(pairs)
    res, ops = oracle_batch(code, args, s1, o1, s2, o2, threads=16)
    bad = []
    for p, (a, b) in enumerate(pairs):
        off = int(o1[p] + o2[p]) + p
        r = sa.PairResult(int(res["score"][p]), int(res["end_i"][p]), int(res["end_j"][p]), int(res["start_i"][p]),
                          int(res["start_j"][p]), 0, ops[off:off + int(res["nops"][p])].tobytes())
        hack = code == 2 and (len(a), len(b)) in ((314, 288), (60, 57), (61, 58))   # SALocalGotoh.h:484-488
        rows = sa.expand_ops(sa.SA_NW if hack else code, a.decode("latin-1"), b.decode("latin-1"), r).rows()
        if int(out[p], 16) != _fnv("\n".join(rows)):
            bad.append(p)
    assert not bad, (len(bad), bad[:10])
