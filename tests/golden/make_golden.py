#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the UNMODIFIED reference.

Runs ONLY in the build container, where /root/reference exists: `make ref` compiles
oracle/ref_harness.cpp against /root/reference/include into oracle/_ref/libsaref.so; this script
drives it through ctypes and writes JSON-lines fixtures (inputs + expected outputs — data, no
reference source).  Usage:  python tests/golden/make_golden.py

Corpus:
  * the README / test/Test.cpp known answer (NW, ScoringSystem(-1,2), AAAGAATGCAT / AAACTCAT);
  * the pairs written (commented) in include/Test.cpp:36-79 and test/Test.cpp:28-29, under every
    algorithm x scoring variant x match function (equal<char>, nullptr where defined, and two
    custom predicates);
  * seeded random DNA (std::mt19937_64, "ACGT"[g() & 3]) at 1 .. 8192 and mutated relatives;
  * edge shapes: empty sequences, single symbols, long-thin matrices.
Reference paths that are undefined are not recorded: SmithWaterman with a
nullptr match fn, the LocalGotoh size-hack sizes, Gotoh default constructors.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from util import REF_SO, MT64, named_lut, py_dna, py_mutate, rows_digest, scoring_fields, sha  # noqa: E402

FULL_ROWS_MAX = 400   # store the alignment strings verbatim up to this length, else a digest


class RefOut(C.Structure):
    _fields_ = [("score", C.c_int32), ("max_row", C.c_int32), ("max_col", C.c_int32), ("len", C.c_int32)]


def ref_lib():
    L = C.CDLL(REF_SO)
    vp = C.c_void_p
    L.ref_align.argtypes = [C.c_int] * 8 + [vp, vp, C.c_int, vp, C.c_int, C.POINTER(RefOut), vp, vp, vp, C.c_int]
    L.ref_align.restype = C.c_int
    L.ref_gen_dna.argtypes = [C.c_uint64, C.c_int, vp]
    L.ref_gen_dna.restype = None
    return L


L = None


def ref_dna(seed: int, n: int) -> bytes:
    buf = C.create_string_buffer(n + 1)
    L.ref_gen_dna(seed, n, buf)
    return buf.raw[:n]


def ref_align(algo: int, args, match: str, s1: bytes, s2: bytes):
    nargs = len(args)
    if nargs == 4 and not isinstance(args[3], bool):
        nargs = 5
    a = list(args) + [0] * (5 - len(args))
    if nargs == 2:
        a0, a1, a2, a3, allow = a[0], a[1], 0, 0, 0
    elif nargs in (3, 4):
        a0, a1, a2, a3, allow = a[0], a[1], a[2], 0, int(a[3]) if nargs == 4 else 1
    else:
        a0, a1, a2, a3 = a[0], a[1], a[2], a[3]
        allow = int(args[4]) if len(args) == 5 else 1
    mode = {"null": 0, "equal": 1}.get(match, 2)
    lut = named_lut(match)
    lut_p = lut.ctypes.data if lut is not None else None
    cap = len(s1) + len(s2) + 4
    r0, bars, r1 = C.create_string_buffer(cap), C.create_string_buffer(cap), C.create_string_buffer(cap)
    o = RefOut()
    rc = L.ref_align(algo, nargs, a0, a1, a2, a3, allow, mode, lut_p, s1, len(s1), s2, len(s2), C.byref(o),
                     r0, bars, r1, cap)
    assert rc == 0
    k = o.len
    return o.score, o.max_row, o.max_col, (r0.raw[:k].decode("latin-1"), bars.raw[:k].decode("latin-1"),
                                           r1.raw[:k].decode("latin-1"))


ALGO = {"sw": 0, "nw": 1, "lg": 2, "gg": 3, "hb": 4, "mm": 5}
LINEAR = [(-1, 2), (-1, 1, -1), (-1, 2, -1), (-2, 1, -1, False), (-3, 2, -2), (-1, 1, -1, False)]
AFFINE = [(-3, -1, 1, -1, False), (-3, -1, 1, -1, True), (-2, -1, 2, -1, True), (-5, -2, 3, -2, True),
          (0, -1, 1, -1, True), (-4, -1, 2, -3, False)]

# include/Test.cpp:36-79 (the authors' manual corpus) and test/Test.cpp:28-29
TEST_CPP_PAIRS = [
    ("AATCG", "AACG"),
    ("AGGATCGGCTAGAGCTAGAGCTAGCTAGTAGC", "GAGATCGGCGGATTACAGGCTATCGA"),
    ("AAAAAAAAAAAAAAAGGGGGGGGGGGGGGGGGGGGTTTTTTTTTTTTTTTTTTCCCCCCCCCCCCCCCCCAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA",
     "AAAAAAAAAAAAAAAGGGGGGGGGGGGGGGGGGGGTTTTTTTTTTTTTTTTTTCCCCCCCCCCCCCCCCCAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA"),
    ("AAAAGGGGTTTTCCCC", "AAAAGGGGTTTTCCCC"),
    ("AAAGGGTTTCCC", "AAAGGGTTTCCC"),
    ("AAAA", "AAAA"),
    ("CTGAAGCGG", "CTCAAGCGTAGTCC"),
    ("AGTAC", "AAG"),
    ("GGTCGCGACTACGTGAGCTAGGGCTCCGGACTGGGCTGTATAGTCGAGTC", "TGATCTCGCCCCGACAACTGCAAACCCCAACTTATTTAGATAACATGGTTTACAGG"),
    ("AGGGGGGGGTTTTCAAAAGCTCTTCGCATGCGCATAGGCTTAGGAGTCGAGGATCGGCGGCATATTAAGAGAGGGCGGCGCCCATATATTAGGCGCGCGCGATTATATTATAATATATATATTAATCGGGCGCTATGCGC",
     "AGGTCTCCGGCATGAGCTAGCGGCGAGTTATAGCGCGTTTCAAAAGCTCTTCGCATGCGCATAGGCTTAGGAGTCGAGGATCGGCGGCATATTAAGAGAGGGCGGCAGGCTTGGAAAAAGGCTCTGAGATGCGAGAATAGAGGAGAG"),
    ("ACGGTTGC", "AGCGTC"),
    ("AGTC", "GACT"),
    ("AAGG", "AAGG"),
    ("AAGGGGGCAACCCAATTGTCAAAA", "AAGTTGGCGGCCCAAGCTGCGAAA"),
    ("AAAGGGTTTCCCAAGGTTCCAGTC", "AAAGGGTTTCCCAAGGCTCCAGTC"),
    ("CGAA", "CGA"),
    ("AGCTTCAGGCTGA", "AGCTGGATCGATCGATG"),
    ("AGCTCGATCAA", "GCAACCGATCGA"),
    ("AAAGAATGCAT", "AAACTCAT"),
    ("AA", "A"),
    ("AATCGG", "AACGGT"),
    ("A", "A"), ("A", "C"), ("ACGT", "TGCA"),
]


def seq_of(spec) -> bytes:
    if isinstance(spec, str):
        return spec.encode()
    if spec["kind"] == "dna":
        return ref_dna(spec["seed"], spec["len"])
    if spec["kind"] == "mut":
        return py_mutate(seq_of(spec["src"]), spec["seed"])
    if spec["kind"] == "withN":
        b = bytearray(seq_of(spec["src"]))
        for p in range(spec["phase"], len(b), spec["every"]):
            b[p] = ord("N")
        return bytes(b)
    if spec["kind"] == "lower":
        b = bytearray(seq_of(spec["src"]))
        for p in range(spec["phase"], len(b), spec["every"]):
            b[p] = ord(chr(b[p]).lower())
        return bytes(b)
    raise ValueError(spec)


def record(out, tag, algo, args, match, s1spec, s2spec):
    s1, s2 = seq_of(s1spec), seq_of(s2spec)
    score, mr, mc, rows = ref_align(ALGO[algo], args, match, s1, s2)
    e = {"id": f"{tag}/{algo}/{'_'.join(str(int(x)) for x in args)}/{match}", "algo": algo, "scoring": list(args),
         "match": match, "s1": s1spec, "s2": s2spec, "m": len(s1), "n": len(s2), "score": score,
         "max_row": mr, "max_col": mc, "len": len(rows[0])}
    if algo == "mm":
        e["score"] = None   # MyersMillerSA exposes no score (SAMyersMiller.h:412-420)
    if not isinstance(s1spec, str):
        e["s1_sha"] = sha(s1)
    if not isinstance(s2spec, str):
        e["s2_sha"] = sha(s2)
    if len(rows[0]) <= FULL_ROWS_MAX:
        e["rows"] = list(rows)
    else:
        e["rows_sha"] = rows_digest(*rows)
    out.append(e)


def lg_hack(m, n):
    return (m, n) in ((314, 288), (60, 57), (61, 58))


def hirschberg_vectors():
    """HirschbergSA (SAHirschberg.h) vectors: KAT pairs x linear scorings x match fns, random and
    mutated DNA up to 2k, empty and length-1 edges (the NW base case :119-126)."""
    hb = []
    for pi, (a, b) in enumerate(TEST_CPP_PAIRS):
        for sc in LINEAR:
            for mt in ("equal", "null", "purine"):
                record(hb, f"testcpp{pi}", "hb", sc, mt, a, b)
                if a != b:
                    record(hb, f"testcpp{pi}r", "hb", sc, mt, b, a)
    for a, b in (("", "ACGT"), ("ACGT", ""), ("", ""), ("A", "ACGTTGCA"), ("ACGTTGCA", "A"), ("A", "C"),
                 ("AC", "CA"), ("ACGT" * 8, "TGCA" * 8)):
        for sc in ((-1, 2), (-1, 2, -1), (-2, 1, -1, False)):
            record(hb, "edge", "hb", sc, "equal", a, b)
    for k, (m, n) in enumerate(((17, 23), (64, 64), (65, 63), (128, 97), (255, 300), (513, 511), (1000, 1024),
                                (2048, 2048))):
        s1 = {"kind": "dna", "seed": 3_000_000_001 + 2 * k, "len": m}
        s2 = {"kind": "dna", "seed": 3_000_000_002 + 2 * k, "len": n}
        for sc in ((-1, 2, -1), (-1, 1, -1), (-2, 1, -1, False)):
            record(hb, f"rnd{m}x{n}", "hb", sc, "equal", s1, s2)
        src = {"kind": "dna", "seed": 3_100_000_000 + k, "len": m}
        record(hb, f"mut{m}", "hb", (-1, 2, -1), "equal", src, {"kind": "mut", "src": src, "seed": 11 + k})
        record(hb, f"mutP{m}", "hb", (-1, 2, -1), "purine", src, {"kind": "mut", "src": src, "seed": 11 + k})
    return hb


def mm_vectors():
    """MyersMillerSA (SAMyersMiller.h) vectors: KAT pairs x affine scorings x match fns, random
    and mutated DNA up to 2k, empty and length-1 edges (the M == 1 / N == 0 / M == 0 cases
    :57-160 and both midpoint types :358-395)."""
    mm = []
    for pi, (a, b) in enumerate(TEST_CPP_PAIRS):
        for sc in AFFINE:
            for mt in ("equal", "null", "purine"):
                record(mm, f"testcpp{pi}", "mm", sc, mt, a, b)
                if a != b:
                    record(mm, f"testcpp{pi}r", "mm", sc, mt, b, a)
    for a, b in (("", "ACGT"), ("ACGT", ""), ("", ""), ("A", "ACGTTGCA"), ("ACGTTGCA", "A"), ("A", "C"),
                 ("C", "AGT"), ("AC", "CA"), ("AC", "GGGG"), ("ACGT" * 8, "TGCA" * 8), ("A" * 40, "A" * 3),
                 ("A" * 3, "A" * 40), ("ACGTACGT" * 12, "T"), ("G", "ACGTACGT" * 12)):
        for sc in ((-3, -1, 1, -1, False), (-3, -1, 1, -1, True), (-1, -2, 2, -1, True), (0, -1, 1, -1, True),
                   (-4, -1, 2, -3, False)):
            record(mm, "edge", "mm", sc, "equal", a, b)
    for k, (m, n) in enumerate(((17, 23), (64, 64), (65, 63), (128, 97), (200, 3), (3, 200), (255, 300),
                                (513, 511), (1000, 1024), (2048, 2048))):
        s1 = {"kind": "dna", "seed": 3_200_000_001 + 2 * k, "len": m}
        s2 = {"kind": "dna", "seed": 3_200_000_002 + 2 * k, "len": n}
        for sc in ((-3, -1, 1, -1, True), (-2, -1, 2, -1, True), (-3, -1, 1, -1, False), (-5, -2, 3, -2, True)):
            record(mm, f"rnd{m}x{n}", "mm", sc, "equal", s1, s2)
        src = {"kind": "dna", "seed": 3_300_000_000 + k, "len": m}
        record(mm, f"mut{m}", "mm", (-3, -1, 2, -1, True), "equal", src, {"kind": "mut", "src": src, "seed": 21 + k})
        record(mm, f"mutP{m}", "mm", (-3, -1, 2, -1, True), "purine", src,
               {"kind": "mut", "src": src, "seed": 21 + k})
    return mm


def main():
    global L
    if not os.path.exists(REF_SO):
        sys.exit("oracle/_ref/libsaref.so missing: run `make ref` (needs /root/reference)")
    L = ref_lib()
    if "--only-mm" in sys.argv:
        rows = mm_vectors()
        with open(os.path.join(HERE, "myersmiller.jsonl"), "w") as f:
            for e in rows:
                f.write(json.dumps(e, separators=(",", ":")) + "\n")
        print(f"myersmiller.jsonl: {len(rows)} vectors")
        return
    if "--only-hirschberg" in sys.argv:
        rows = hirschberg_vectors()
        with open(os.path.join(HERE, "hirschberg.jsonl"), "w") as f:
            for e in rows:
                f.write(json.dumps(e, separators=(",", ":")) + "\n")
        print(f"hirschberg.jsonl: {len(rows)} vectors")
        return
    # pin the pure-Python generators to std::mt19937_64 before using them
    for seed, n in ((1, 1000), (2, 333), (1_000_000_001, 64)):
        assert py_dna(seed, n) == ref_dna(seed, n), "MT64 restatement disagrees with std::mt19937_64"

    kat = []
    # README.md:28-37 / test/Test.cpp:31-37 known answer
    record(kat, "readme", "nw", (-1, 2), "equal", "AAAGAATGCAT", "AAACTCAT")
    record(kat, "readme_default", "nw", (-1, 2, -1), "null", "AAAGAATGCAT", "AAACTCAT")
    for pi, (a, b) in enumerate(TEST_CPP_PAIRS):
        for algo in ("sw", "nw"):
            for sc in LINEAR:
                matches = ["equal", "purine"] + (["null"] if algo == "nw" else [])
                for mt in matches:
                    record(kat, f"testcpp{pi}", algo, sc, mt, a, b)
                    if a != b:
                        record(kat, f"testcpp{pi}r", algo, sc, mt, b, a)
        if lg_hack(len(a), len(b)):
            continue
        for algo in ("lg", "gg"):
            for sc in AFFINE:
                for mt in ("equal", "null", "purine"):
                    record(kat, f"testcpp{pi}", algo, sc, mt, a, b)
                    if a != b:
                        record(kat, f"testcpp{pi}r", algo, sc, mt, b, a)

    rnd = []
    shapes = [(1, 1), (1, 7), (9, 1), (2, 3), (31, 33), (63, 64), (64, 63), (65, 129), (100, 37), (127, 128),
              (255, 256), (256, 255), (257, 1000), (1000, 257), (1023, 1025), (300, 5000), (5000, 300),
              (20000, 150), (150, 20000)]
    base = 7_000_000_000
    for k, (m, n) in enumerate(shapes):
        s1 = {"kind": "dna", "seed": base + 2 * k + 1, "len": m}
        s2 = {"kind": "dna", "seed": base + 2 * k + 2, "len": n}
        for algo, scs in (("sw", [(-1, 1, -1), (-2, 1, -1, False), (-3, 2, -2)]), ("nw", [(-1, 2), (-1, 2, -1)]),
                          ("lg", [(-3, -1, 1, -1, False), (-2, -1, 2, -1, True)]),
                          ("gg", [(-3, -1, 1, -1, True), (-3, -1, 1, -1, False)])):
            if algo == "lg" and lg_hack(m, n):
                continue
            for sc in scs:
                record(rnd, f"rnd{m}x{n}", algo, sc, "equal", s1, s2)
    # mutated relatives (long tracebacks), custom match fns on larger inputs
    for k, (m, seedm) in enumerate(((700, 11), (2000, 12), (3000, 13))):
        src = {"kind": "dna", "seed": base + 100 + k, "len": m}
        rel = {"kind": "mut", "src": src, "seed": seedm}
        for algo, sc in (("sw", (-1, 1, -1)), ("nw", (-1, 2, -1)), ("lg", (-3, -1, 1, -1, True)),
                         ("gg", (-3, -1, 1, -1, True)), ("sw", (-2, 1, -1, False)), ("lg", (-3, -1, 1, -1, False))):
            record(rnd, f"mut{m}", algo, sc, "equal", src, rel)
        withn = {"kind": "withN", "src": rel, "every": 7, "phase": 3}
        for algo, sc in (("sw", (-1, 1, -1)), ("nw", (-1, 2, -1)), ("lg", (-3, -1, 1, -1, True)),
                         ("gg", (-3, -1, 1, -1, True))):
            record(rnd, f"mutN{m}", algo, sc, "nwild", src, withn)
            record(rnd, f"mutP{m}", algo, sc, "purine", src, rel)
        low = {"kind": "lower", "src": rel, "every": 5, "phase": 1}
        record(rnd, f"mutC{m}", "sw", (-1, 1, -1), "caseless", src, low)
        record(rnd, f"mutC{m}", "gg", (-3, -1, 1, -1, True), "caseless", low, src)
    # edge shapes
    for algo, sc in (("sw", (-1, 1, -1)), ("nw", (-1, 2, -1)), ("gg", (-3, -1, 1, -1, True)),
                     ("lg", (-3, -1, 1, -1, True))):
        for a, b in (("", "ACGT"), ("ACGT", ""), ("", "")):
            record(rnd, "empty", algo, sc, "equal", a, b)

    big = []
    # SURVEY.md §8(c) probed values: seeds 1 and 2, SW default scoring + equal<char>
    for n in (1024, 2048, 4096, 8192):
        record(big, f"probe{n}", "sw", (-1, 1, -1), "equal", {"kind": "dna", "seed": 1, "len": n},
               {"kind": "dna", "seed": 2, "len": n})
    for allow in (False, True):
        record(big, "probe8192", "lg", (-3, -1, 1, -1, allow), "equal", {"kind": "dna", "seed": 1, "len": 8192},
               {"kind": "dna", "seed": 2, "len": 8192})
    record(big, "probe4096", "nw", (-1, 2, -1), "equal", {"kind": "dna", "seed": 1, "len": 4096},
           {"kind": "dna", "seed": 2, "len": 4096})
    record(big, "probe4096", "gg", (-3, -1, 1, -1, True), "equal", {"kind": "dna", "seed": 1, "len": 4096},
           {"kind": "dna", "seed": 2, "len": 4096})
    src = {"kind": "dna", "seed": 99, "len": 4096}
    record(big, "mut4096", "sw", (-1, 1, -1), "equal", src, {"kind": "mut", "src": src, "seed": 5})
    record(big, "mut4096", "lg", (-3, -1, 1, -1, True), "equal", src, {"kind": "mut", "src": src, "seed": 5})

    for name, rows in (("kat.jsonl", kat), ("random.jsonl", rnd), ("large.jsonl", big),
                       ("hirschberg.jsonl", hirschberg_vectors()), ("myersmiller.jsonl", mm_vectors())):
        with open(os.path.join(HERE, name), "w") as f:
            for e in rows:
                f.write(json.dumps(e, separators=(",", ":")) + "\n")
        print(f"{name}: {len(rows)} vectors")

    # generator pins: sha of lib-generated sequences must equal std::mt19937_64's
    pins = [{"seed": s, "len": n, "sha": sha(ref_dna(s, n))} for s, n in
            ((1, 1024), (2, 4096), (12345, 1), (2_000_000_001, 4096), (2_000_000_002, 4096), (0, 100))]
    with open(os.path.join(HERE, "dna_pins.json"), "w") as f:
        json.dump(pins, f, indent=1)
    print("dna_pins.json:", len(pins))


if __name__ == "__main__":
    main()
