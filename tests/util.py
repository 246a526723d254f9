"""Test helpers: the CPU checkers (oracle/) and shared input generators.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use the oracle, and only as
the checker (see oracle/sa_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
from typing import Optional, Tuple

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libsaref.so")

ALGOS = {"sw": 0, "nw": 1, "lg": 2, "gg": 3, "hb": 4, "mm": 5}


# ------------------------------------------------------------------ std::mt19937_64 (pure Python)
class MT64:
    """std::mt19937_64 ([rand.predef]); used to pin the C generators on small inputs."""
    N, M = 312, 156

    def __init__(self, seed: int):
        self.s = [0] * self.N
        self.s[0] = seed & 0xFFFFFFFFFFFFFFFF
        for i in range(1, self.N):
            p = self.s[i - 1]
            self.s[i] = (6364136223846793005 * (p ^ (p >> 62)) + i) & 0xFFFFFFFFFFFFFFFF
        self.i = self.N

    def __call__(self) -> int:
        if self.i >= self.N:
            UM, LM, A = 0xFFFFFFFF80000000, 0x7FFFFFFF, 0xB5026F5AA96619E9
            s = self.s
            for k in range(self.N):
                x = (s[k] & UM) | (s[(k + 1) % self.N] & LM)
                s[k] = s[(k + self.M) % self.N] ^ (x >> 1) ^ (A if x & 1 else 0)
            self.i = 0
        x = self.s[self.i]
        self.i += 1
        x ^= (x >> 29) & 0x5555555555555555
        x ^= (x << 17) & 0x71D67FFFEDA60000
        x ^= (x << 37) & 0xFFF7EEE000000000
        x ^= x >> 43
        return x & 0xFFFFFFFFFFFFFFFF


def py_dna(seed: int, n: int) -> bytes:
    g = MT64(seed)
    return bytes(b"ACGT"[g() & 3] for _ in range(n))


def py_mutate(src: bytes, seed: int) -> bytes:
    g = MT64(seed)
    out = bytearray()
    for c in src:
        r = g() % 100
        if r < 10:
            out.append(b"ACGT"[g() & 3])
        elif r < 12:
            out.append(b"ACGT"[g() & 3])
            out.append(c)
        elif r < 14:
            pass
        else:
            out.append(c)
    return bytes(out)


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()[:32]


def rows_digest(r0: str, bars: str, r1: str) -> str:
    return sha((r0 + "\n" + bars + "\n" + r1).encode("latin-1"))


# ----------------------------------------------------------------------- named match tables
def named_lut(name: Optional[str]) -> Optional[np.ndarray]:
    """Custom MatchFnTy predicates used by the golden corpus, as 256x256 tables."""
    if name in (None, "equal", "null"):
        return None
    lut = np.zeros((256, 256), dtype=np.uint8)
    if name == "purine":       # purine~purine, pyrimidine~pyrimidine
        cls = {ord("A"): 0, ord("G"): 0, ord("C"): 1, ord("T"): 1}
        for a in range(256):
            for b in range(256):
                lut[a, b] = 1 if (a in cls and b in cls and cls[a] == cls[b]) or a == b else 0
    elif name == "nwild":      # 'N' matches anything, otherwise equality
        for a in range(256):
            for b in range(256):
                lut[a, b] = 1 if a == b or a == ord("N") or b == ord("N") else 0
    elif name == "caseless":   # case-insensitive
        for a in range(256):
            for b in range(256):
                lut[a, b] = 1 if chr(a).upper() == chr(b).upper() else 0
    else:
        raise ValueError(name)
    return lut


# --------------------------------------------------------------------------- oracle (C)
class OracleScoring(C.Structure):
    _fields_ = [("gap", C.c_int32), ("match", C.c_int32), ("mismatch", C.c_int32),
                ("gap_open", C.c_int32), ("gap_extend", C.c_int32), ("allow_mismatch", C.c_int32)]


class OracleResult(C.Structure):
    _fields_ = [("score", C.c_int32), ("end_i", C.c_int32), ("end_j", C.c_int32), ("start_i", C.c_int32),
                ("start_j", C.c_int32), ("nops", C.c_int32), ("len", C.c_int32)]


_oracle = None


def oracle_lib():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError("oracle not built: run `make oracle`")
        L = C.CDLL(ORACLE_SO)
        vp = C.c_void_p
        L.oracle_align.argtypes = [C.c_int, C.POINTER(OracleScoring), vp, C.c_int, vp, C.c_int, vp,
                                   C.POINTER(OracleResult), vp, C.c_int, vp, vp, vp, C.c_int]
        L.oracle_align.restype = C.c_int
        L.oracle_sw_batch.argtypes = [C.POINTER(OracleScoring), vp, vp, vp, vp, C.c_int, C.c_int, vp]
        L.oracle_sw_batch.restype = C.c_int
        L.oracle_batch.argtypes = [C.c_int, C.POINTER(OracleScoring), vp, vp, vp, vp, C.c_int, C.c_int, vp, vp]
        L.oracle_batch.restype = C.c_int
        L.oracle_sw_score_batch.argtypes = [C.POINTER(OracleScoring), vp, vp, vp, vp, C.c_int, C.c_int, vp]
        L.oracle_sw_score_batch.restype = C.c_int
        L.oracle_align_matrix.argtypes = [C.c_int, C.POINTER(OracleScoring), C.c_int, C.c_int, vp,
                                          C.POINTER(OracleResult), vp, C.c_int]
        L.oracle_align_matrix.restype = C.c_int
        _oracle = L
    return _oracle


def scoring_fields(args) -> Tuple[int, int, int, int, int, int]:
    """(gap, match, mismatch, gap_open, gap_extend, allow) for a ScoringSystem argument tuple."""
    a = list(args)
    if len(a) == 2:
        return a[0], a[1], -(2 ** 31), 0, 0, 0
    if len(a) == 3 or (len(a) == 4 and isinstance(a[3], bool)):
        return a[0], a[1], a[2], 0, 0, int(a[3]) if len(a) == 4 else 1
    allow = int(a[4]) if len(a) == 5 else 1
    return 0, a[2], a[3], a[0], a[1], allow


def oracle_align(algo: int, args, s1: bytes, s2: bytes, lut: Optional[np.ndarray] = None):
    """Run the C restatement; returns dict(score, end_i, end_j, start_i, start_j, ops, rows, rc)."""
    L = oracle_lib()
    g, ma, mi, go, ge, al = scoring_fields(args)
    if not al:
        mi = -(2 ** 31)
    sc = OracleScoring(g, ma, mi, go, ge, al)
    m, n = len(s1), len(s2)
    cap = m + n + 4
    ops = C.create_string_buffer(cap)
    r0, bars, r1 = C.create_string_buffer(cap), C.create_string_buffer(cap), C.create_string_buffer(cap)
    res = OracleResult()
    lut_p = None
    if lut is not None:
        lut = np.ascontiguousarray(lut, dtype=np.uint8).reshape(65536)
        lut_p = lut.ctypes.data
    b1 = C.create_string_buffer(s1, m + 1)
    b2 = C.create_string_buffer(s2, n + 1)
    rc = L.oracle_align(algo, C.byref(sc), b1, m, b2, n, lut_p, C.byref(res), ops, cap, r0, bars, r1, cap)
    k = res.len
    return dict(rc=rc, score=res.score, end_i=res.end_i, end_j=res.end_j, start_i=res.start_i,
                start_j=res.start_j, ops=ops.raw[: res.nops],
                rows=(r0.raw[:k].decode("latin-1"), bars.raw[:k].decode("latin-1"), r1.raw[:k].decode("latin-1")))


ORACLE_RESULT_DTYPE = np.dtype([("score", "<i4"), ("end_i", "<i4"), ("end_j", "<i4"), ("start_i", "<i4"),
                                 ("start_j", "<i4"), ("nops", "<i4"), ("len", "<i4")])


def _oracle_sc(args):
    g, ma, mi, go, ge, al = scoring_fields(args)
    if not al:
        mi = -(2 ** 31)
    return OracleScoring(g, ma, mi, go, ge, al)


def oracle_batch(algo: int, args, s1, o1, s2, o2, threads: int = 16):
    """Full oracle results (ORACLE_RESULT_DTYPE) and op streams (pair p at o1[p]+o2[p]+p) of a
    packed batch, byte-equality match fn, on `threads` host threads."""
    L = oracle_lib()
    n = len(o1) - 1
    s1 = np.ascontiguousarray(s1, dtype=np.uint8)
    s2 = np.ascontiguousarray(s2, dtype=np.uint8)
    o1 = np.ascontiguousarray(o1, dtype=np.uint64)
    o2 = np.ascontiguousarray(o2, dtype=np.uint64)
    res = np.zeros(n, dtype=ORACLE_RESULT_DTYPE)
    ops = np.zeros(int(o1[-1] + o2[-1]) + n + 1, dtype=np.uint8)
    sc = _oracle_sc(args)
    rc = L.oracle_batch(algo, C.byref(sc), s1.ctypes.data, o1.ctypes.data, s2.ctypes.data, o2.ctypes.data, n,
                        threads, res.ctypes.data, ops.ctypes.data)
    assert rc == 0, rc
    return res, ops


def oracle_sw_scores(args, s1, o1, s2, o2, threads: int = 16):
    """(MaxScore, MaxRow, MaxCol) per pair of a packed SW batch, linear-space oracle: (n, 3) int32."""
    L = oracle_lib()
    n = len(o1) - 1
    s1 = np.ascontiguousarray(s1, dtype=np.uint8)
    s2 = np.ascontiguousarray(s2, dtype=np.uint8)
    o1 = np.ascontiguousarray(o1, dtype=np.uint64)
    o2 = np.ascontiguousarray(o2, dtype=np.uint64)
    out = np.zeros((n, 3), dtype=np.int32)
    sc = _oracle_sc(args)
    rc = L.oracle_sw_score_batch(C.byref(sc), s1.ctypes.data, o1.ctypes.data, s2.ctypes.data, o2.ctypes.data,
                                 n, threads, out.ctypes.data)
    assert rc == 0, rc
    return out


def pack_bytes(pairs):
    """Packed batch (s1, o1, s2, o2) of (bytes, bytes) pairs, no library needed."""
    o1 = np.zeros(len(pairs) + 1, dtype=np.uint64)
    o2 = np.zeros(len(pairs) + 1, dtype=np.uint64)
    o1[1:] = np.cumsum([len(a) for a, _ in pairs])
    o2[1:] = np.cumsum([len(b) for _, b in pairs])
    s1 = np.frombuffer(b"".join(a for a, _ in pairs) + b"\0", dtype=np.uint8)[:-1].copy()
    s2 = np.frombuffer(b"".join(b for _, b in pairs) + b"\0", dtype=np.uint8)[:-1].copy()
    return s1, o1, s2, o2


def oracle_align_matrix(algo: int, args, mt: np.ndarray):
    """The oracle driven by an m x n match matrix (generic Ty): dict(score, end_i, end_j, start_i,
    start_j, ops, rc)."""
    L = oracle_lib()
    m, n = mt.shape
    mt = np.ascontiguousarray(mt, dtype=np.uint8)
    sc = _oracle_sc(args)
    cap = m + n + 4
    ops = C.create_string_buffer(cap)
    res = OracleResult()
    rc = L.oracle_align_matrix(algo, C.byref(sc), m, n, mt.ctypes.data if mt.size else None, C.byref(res), ops, cap)
    return dict(rc=rc, score=res.score, end_i=res.end_i, end_j=res.end_j, start_i=res.start_i,
                start_j=res.start_j, ops=ops.raw[: res.nops])


def subset(s1, o1, s2, o2, idx):
    """Pack pairs idx of a packed batch into a new packed batch."""
    a = [s1[int(o1[p]):int(o1[p + 1])] for p in idx]
    b = [s2[int(o2[p]):int(o2[p + 1])] for p in idx]
    ro1 = np.zeros(len(idx) + 1, dtype=np.uint64)
    ro2 = np.zeros(len(idx) + 1, dtype=np.uint64)
    ro1[1:] = np.cumsum([len(x) for x in a])
    ro2[1:] = np.cumsum([len(x) for x in b])
    cat = lambda xs: np.concatenate(xs).astype(np.uint8) if xs else np.zeros(0, np.uint8)
    return cat(a), ro1, cat(b), ro2


def linear_rescore(args, res, ops, o1, o2):
    """Vectorised re-score of every emitted linear-gap alignment: #M*match + #S*mismatch +
    (#U + #L)*gap per pair (ops of pair p at o1[p]+o2[p]+p, res['nops'][p] of them)."""
    g, ma, mi, _, _, _ = scoring_fields(args)
    val = np.zeros(256, dtype=np.int64)
    val[ord("M")], val[ord("S")], val[ord("U")], val[ord("L")] = ma, mi, g, g
    n = len(res)
    starts = (o1[:n].astype(np.int64) + o2[:n].astype(np.int64) + np.arange(n))
    nops = res["nops"].astype(np.int64)
    contrib = val[ops.astype(np.int64)]
    csum = np.concatenate([[0], np.cumsum(contrib)])
    return csum[starts + nops] - csum[starts]


# ------------------------------------------------------------------------------ fixtures
def load_golden(name: str):
    path = os.path.join(GOLDEN, name)
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


def golden_sequences(entry) -> Tuple[bytes, bytes]:
    """Materialise an entry's sequences (literal, or regenerated from its generator spec)."""
    def one(spec):
        if isinstance(spec, str):
            return spec.encode("latin-1")
        kind = spec["kind"]
        if kind == "dna":
            from seqalib_amd import synth_dna
            return synth_dna(spec["seed"], spec["len"])
        if kind == "mut":
            from seqalib_amd import synth_mutate
            return synth_mutate(one(spec["src"]), spec["seed"])
        if kind == "withN":   # every k-th symbol replaced by N
            b = bytearray(one(spec["src"]))
            for p in range(spec["phase"], len(b), spec["every"]):
                b[p] = ord("N")
            return bytes(b)
        if kind == "lower":   # every k-th symbol lower-cased
            b = bytearray(one(spec["src"]))
            for p in range(spec["phase"], len(b), spec["every"]):
                b[p] = ord(chr(b[p]).lower())
            return bytes(b)
        raise ValueError(kind)
    return one(entry["s1"]), one(entry["s2"])
