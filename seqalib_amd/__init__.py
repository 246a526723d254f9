"""seqalib_amd — MI355X (gfx950) pairwise sequence alignment behind the SeqALib API.

Python view of the engine in ``seqalib_amd/lib/libseqalib_hip.so`` (C ABI:
``include/seqalib_hip.h``).  The C++ drop-in for the reference's header-only API lives in
``include/seqalib/SequenceAlignment.h``; this module mirrors the same surface for tests, the
benchmark and Python users:

* :class:`ScoringSystem` — the three constructor overloads of the reference
  (``include/SequenceAlignment.h:92-118``), with the same "which fields are meaningful" rules.
* :class:`SmithWatermanSA`, :class:`NeedlemanWunschSA`, :class:`LocalGotohSA`,
  :class:`GlobalGotohSA` — ``getAlignment(seq1, seq2)`` returns an :class:`AlignedSequence`
  exactly like the reference's (``SASmithWaterman.h:358-366`` etc.); ``getAlignments`` aligns a
  batch in one GPU pass.
* :class:`Engine` — the batch C ABI (host or device-resident buffers).

There is no CPU fallback: if the HIP library is missing or no GPU is present, calls fail with
:class:`SeqalibError`.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Callable, Iterable, List, Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "SA_SW", "SA_NW", "SA_LOCAL_GOTOH", "SA_GLOBAL_GOTOH", "ALGO_NAMES",
    "SeqalibError", "ScoringSystem", "Entry", "AlignedSequence", "PairResult", "Engine",
    "SmithWatermanSA", "NeedlemanWunschSA", "LocalGotohSA", "GlobalGotohSA", "HirschbergSA", "MyersMillerSA",
    "load_library", "library_path", "expand_ops", "synth_dna", "synth_mutate", "synth_dna_batch",
    "SA_FLAG_DIVERGED", "SA_FLAG_BAD_SHAPE", "SA_FLAG_SIZE_HACK", "SA_FLAG_TIMEOUT",
]

SA_SW, SA_NW, SA_LOCAL_GOTOH, SA_GLOBAL_GOTOH, SA_HIRSCHBERG, SA_MYERS_MILLER = 0, 1, 2, 3, 4, 5
ALGO_NAMES = {SA_SW: "sw", SA_NW: "nw", SA_LOCAL_GOTOH: "local_gotoh", SA_GLOBAL_GOTOH: "global_gotoh",
              SA_HIRSCHBERG: "hirschberg", SA_MYERS_MILLER: "myers_miller"}
SA_FLAG_DIVERGED, SA_FLAG_BAD_SHAPE, SA_FLAG_SIZE_HACK, SA_FLAG_TIMEOUT = 1, 2, 4, 8
SA_KERNEL_INT32, SA_KERNEL_T16, SA_KERNEL_T16_ENDCELL, SA_KERNEL_TINY = 0, 1, 2, 3
SA_PIPELINE_DEPTH = 2   # pipelined device calls that may run at once (distinct output buffers)
SA_RECORDS_FLAGS, SA_RECORDS_TAGS, SA_RECORDS_SCORE_ONLY = 0, 1, 2
SA_HOOK_HAND_TAG, SA_HOOK_POISON_WS, SA_HOOK_F16 = 1, 2, 3   # sa_test_hook (tests only)
INT32_MIN = -(2 ** 31)

_HERE = os.path.dirname(os.path.abspath(__file__))


class SeqalibError(RuntimeError):
    pass


class _Scoring(C.Structure):
    _fields_ = [("gap", C.c_int32), ("match", C.c_int32), ("mismatch", C.c_int32),
                ("gap_open", C.c_int32), ("gap_extend", C.c_int32), ("allow_mismatch", C.c_int32)]


class _Result(C.Structure):
    _fields_ = [("score", C.c_int32), ("end_i", C.c_int32), ("end_j", C.c_int32),
                ("start_i", C.c_int32), ("start_j", C.c_int32), ("nops", C.c_uint32),
                ("flags", C.c_uint32), ("reserved", C.c_uint32)]


RESULT_DTYPE = np.dtype([("score", "<i4"), ("end_i", "<i4"), ("end_j", "<i4"), ("start_i", "<i4"),
                         ("start_j", "<i4"), ("nops", "<u4"), ("flags", "<u4"), ("reserved", "<u4")])
assert RESULT_DTYPE.itemsize == C.sizeof(_Result) == 32

_lib = None


def library_path() -> str:
    return os.environ.get("SEQALIB_HIP_LIB", os.path.join(_HERE, "lib", "libseqalib_hip.so"))


def _share_hip_runtime_with_torch():
    """PyTorch-ROCm wheels bundle their own libamdhip64 (same soname as /opt/rocm's).  Two HIP
    runtimes in one process cannot both own the device, so when torch is installed we bind the
    engine to torch's copy (loaded RTLD_GLOBAL by path, without importing torch); a later
    ``import torch`` then maps the very same file.  SEQALIB_HIP_RUNTIME=system disables this."""
    if os.environ.get("SEQALIB_HIP_RUNTIME", "torch") != "torch":
        return
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.submodule_search_locations:
        return
    hip = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(hip):
        C.CDLL(hip, mode=C.RTLD_GLOBAL)


def load_library():
    """Load libseqalib_hip.so (built in-tree by ``make`` / ``__graft_entry__.build()``)."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise SeqalibError(f"HIP engine not built: {path} missing (run `make` or __graft_entry__.build())")
    _share_hip_runtime_with_torch()
    L = C.CDLL(path)
    vp, u8p, u64p, i32p = C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.POINTER(C.c_int)
    L.sa_version.restype = C.c_int
    L.sa_device_count.argtypes = [i32p]
    L.sa_status_string.restype = C.c_char_p
    L.sa_status_string.argtypes = [C.c_int]
    L.sa_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.sa_destroy.argtypes = [vp]
    L.sa_destroy.restype = None
    L.sa_last_error.argtypes = [vp]
    L.sa_last_error.restype = C.c_char_p
    L.sa_set_workspace_limit.argtypes = [vp, C.c_uint64]
    L.sa_trim.argtypes = [vp]
    L.sa_align_batch.argtypes = [vp, C.c_int, C.POINTER(_Scoring), vp, vp, vp, vp, C.c_uint32, vp, vp, vp,
                                 C.c_uint64]
    L.sa_multi_create.argtypes = [vp, C.c_int, C.POINTER(vp)]
    L.sa_multi_destroy.argtypes = [vp]
    L.sa_multi_destroy.restype = None
    L.sa_multi_last_error.argtypes = [vp]
    L.sa_multi_last_error.restype = C.c_char_p
    L.sa_multi_align_batch.argtypes = [vp, C.c_int, C.POINTER(_Scoring), vp, vp, vp, vp, C.c_uint32, vp, vp, vp,
                                       C.c_uint64]
    L.sa_align_batch_bits.argtypes = [vp, C.c_int, C.POINTER(_Scoring), vp, vp, C.c_uint32, vp, vp, vp, vp,
                                      C.c_uint64]
    L.sa_align_batch_device.argtypes = [vp, C.c_int, C.POINTER(_Scoring), vp, vp, vp, vp, C.c_uint32,
                                        C.c_uint32, C.c_uint32, vp, vp, vp, vp]
    L.sa_last_timings.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(C.c_float), i32p]
    L.sa_last_kernel_timings.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    L.sa_plan_query.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, i32p, i32p, u64p, u64p]
    L.sa_plan_query_ex.argtypes = [C.c_int, C.POINTER(_Scoring), C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                   i32p, i32p, i32p, u64p]
    L.sa_last_plan.argtypes = [vp, i32p, i32p, i32p]
    L.sa_last_plan_ex.argtypes = [vp, i32p, i32p, i32p, i32p]
    L.sa_set_pipeline.argtypes = [vp, C.c_int]
    L.sa_wait.argtypes = [vp]
    L.sa_test_hook.argtypes = [vp, C.c_int, C.c_uint64]
    L.sa_synth_dna.argtypes = [C.c_uint64, C.c_uint32, vp]
    L.sa_synth_mutate.argtypes = [vp, C.c_uint32, C.c_uint64, vp, C.c_uint32, C.POINTER(C.c_uint32)]
    L.sa_synth_dna_batch.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp, vp, C.c_int]
    for fn in ("sa_set_workspace_limit", "sa_trim", "sa_align_batch", "sa_align_batch_bits", "sa_align_batch_device",
               "sa_multi_create", "sa_multi_align_batch",
               "sa_last_timings", "sa_last_kernel_timings", "sa_last_plan", "sa_last_plan_ex", "sa_plan_query", "sa_plan_query_ex", "sa_synth_dna", "sa_synth_mutate", "sa_synth_dna_batch",
               "sa_create", "sa_device_count", "sa_set_pipeline", "sa_wait", "sa_test_hook"):
        getattr(L, fn).restype = C.c_int
    if L.sa_version() != 1:
        raise SeqalibError("libseqalib_hip ABI version mismatch")
    _lib = L
    return L


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


# ----------------------------------------------------------------------------------- scoring
class ScoringSystem:
    """Mirror of the reference's ScoringSystem (include/SequenceAlignment.h:82-131).

    * ``ScoringSystem(gap, match)``                        -> Mismatch = INT_MIN, AllowMismatch = False
    * ``ScoringSystem(gap, match, mismatch[, allow: bool])``
    * ``ScoringSystem(gap_open, gap_extend, match, mismatch[, allow])`` — four ints pick this
      overload, as in C++.
    Fields the chosen overload leaves uninitialised in the reference are 0 here.
    """

    def __init__(self, *args):
        self.gap = self.match = self.mismatch = self.gap_open = self.gap_extend = 0
        self.allow_mismatch = True
        if len(args) == 2:
            self.gap, self.match = args
            self.mismatch, self.allow_mismatch = INT32_MIN, False
            self.nargs = 2
        elif len(args) == 3 or (len(args) == 4 and isinstance(args[3], bool)):
            self.gap, self.match, self.mismatch = args[:3]
            self.allow_mismatch = bool(args[3]) if len(args) == 4 else True
            self.nargs = len(args)
        elif len(args) in (4, 5):
            self.gap_open, self.gap_extend, self.match, self.mismatch = args[:4]
            self.allow_mismatch = bool(args[4]) if len(args) == 5 else True
            self.nargs = 5
        else:
            raise TypeError("ScoringSystem takes 2, 3, 4 or 5 arguments")

    def getAllowMismatch(self): return self.allow_mismatch
    def getMismatchPenalty(self): return self.mismatch
    def getGapPenalty(self): return self.gap
    def getMatchProfit(self): return self.match
    def getGapOpenPenalty(self): return self.gap_open
    def getGapExtendPenalty(self): return self.gap_extend

    def _c(self) -> _Scoring:
        return _Scoring(self.gap, self.match, self.mismatch, self.gap_open, self.gap_extend,
                        1 if self.allow_mismatch else 0)

    def args(self) -> tuple:
        if self.nargs == 2:
            return (self.gap, self.match)
        if self.nargs in (3, 4):
            return (self.gap, self.match, self.mismatch) + ((self.allow_mismatch,) if self.nargs == 4 else ())
        return (self.gap_open, self.gap_extend, self.match, self.mismatch, self.allow_mismatch)

    def __repr__(self):
        return f"ScoringSystem{self.args()}"


# --------------------------------------------------------------------------------- results
@dataclass
class Entry:
    """AlignedSequence::Entry (include/SequenceAlignment.h:17-53)."""
    first: object
    second: object
    is_match: bool

    def get(self, index: int):
        assert index in (0, 1), "Index out of bounds!"
        return self.first if index == 0 else self.second

    def match(self) -> bool:
        return self.is_match

    def mismatch(self) -> bool:
        return not self.is_match


class AlignedSequence:
    """AlignedSequence<Ty, Blank> (include/SequenceAlignment.h:13-80): an ordered list of Entry."""

    def __init__(self, entries: Optional[List[Entry]] = None, blank="-"):
        self.Data: List[Entry] = entries or []
        self.blank = blank

    def __iter__(self):
        return iter(self.Data)

    def __len__(self):
        return len(self.Data)

    def rows(self) -> Tuple[str, str, str]:
        """The three lines the reference's printAlignment prints (include/Test.cpp:10-31)."""
        r0 = "".join(str(e.first) for e in self.Data)
        bars = "".join("|" if e.is_match else " " for e in self.Data)
        r1 = "".join(str(e.second) for e in self.Data)
        return r0, bars, r1


@dataclass
class PairResult:
    score: int
    end_i: int
    end_j: int
    start_i: int
    start_j: int
    flags: int
    ops: bytes   # traceback order


def expand_ops(algo: int, s1: Sequence, s2: Sequence, r: PairResult, blank="-",
               match_fn: Optional[Callable] = None) -> AlignedSequence:
    """Host half of buildResult: op stream -> Entry list, plus forceGlobal for the local modes
    (SequenceAligner::forceGlobal, include/SequenceAlignment.h:156-189)."""
    local: List[Entry] = []
    i, j = r.end_i, r.end_j
    for op in r.ops:
        c = chr(op)
        if c in "MS":
            local.append(Entry(s1[i - 1], s2[j - 1], c == "M"))
            i -= 1; j -= 1
        elif c == "X":
            local.append(Entry(s1[i - 1], blank, False))
            local.append(Entry(blank, s2[j - 1], False))
            i -= 1; j -= 1
        elif c in "Uu":
            local.append(Entry(s1[i - 1], blank, False))
            if c == "U":
                i -= 1
        elif c in "Ll":
            local.append(Entry(blank, s2[j - 1], False))
            if c == "L":
                j -= 1
        else:
            raise SeqalibError(f"bad op {op!r}")
    local.reverse()   # push_front order -> forward order
    if r.flags & SA_FLAG_SIZE_HACK or algo in (SA_NW, SA_GLOBAL_GOTOH, SA_HIRSCHBERG, SA_MYERS_MILLER):
        return AlignedSequence(local, blank)
    idx1, idx2, end1, end2 = r.start_i, r.start_j, r.end_i, r.end_j
    front = [Entry(s1[k], blank, False) for k in range(idx1)] + [Entry(blank, s2[k], False) for k in range(idx2)]
    back = [Entry(s1[k], blank, False) for k in range(end1, len(s1))] + \
           [Entry(blank, s2[k], False) for k in range(end2, len(s2))]
    return AlignedSequence(front + local + back, blank)


# ---------------------------------------------------------------------------------- engine
def _as_bytes(s) -> bytes:
    if isinstance(s, (bytes, bytearray)):
        return bytes(s)
    if isinstance(s, str):
        return s.encode("latin-1")
    if isinstance(s, np.ndarray) and s.dtype == np.uint8:
        return s.tobytes()
    raise TypeError("sequences must be str, bytes or uint8 arrays (use the symbol mapping for other types)")


def pack_pairs(pairs: Sequence[Tuple[object, object]]):
    """Concatenate pairs into (seq1, off1, seq2, off2) uint8/uint64 arrays."""
    b1 = [_as_bytes(a) for a, _ in pairs]
    b2 = [_as_bytes(b) for _, b in pairs]
    off1 = np.zeros(len(pairs) + 1, dtype=np.uint64)
    off2 = np.zeros(len(pairs) + 1, dtype=np.uint64)
    off1[1:] = np.cumsum([len(x) for x in b1]) if b1 else []
    off2[1:] = np.cumsum([len(x) for x in b2]) if b2 else []
    s1 = np.frombuffer(b"".join(b1), dtype=np.uint8).copy() if b1 else np.zeros(0, np.uint8)
    s2 = np.frombuffer(b"".join(b2), dtype=np.uint8).copy() if b2 else np.zeros(0, np.uint8)
    return s1, off1, s2, off2


def lut_from_fn(fn: Callable[[str, str], bool], alphabet1: Iterable[int], alphabet2: Iterable[int]) -> np.ndarray:
    """256x256 match table from a predicate over characters (the reference's MatchFnTy)."""
    lut = np.zeros((256, 256), dtype=np.uint8)
    for a in alphabet1:
        for b in alphabet2:
            lut[a, b] = 1 if fn(chr(a), chr(b)) else 0
    return lut


def match_bitmaps(pairs: Sequence[Tuple[Sequence, Sequence]], match: Optional[Callable] = None):
    """The generic-Ty input of sa_align_batch_bits for pairs of sequences of ANY symbols (lists or
    tuples of ints, objects, ...): length offsets and per-pair m x n match bitmaps, i.e. the
    reference's cacheAllMatches (SASmithWaterman.h:20-45) packed to bits.  match(a, b) is the
    MatchFnTy; None means equality (the reference's nullptr match fn).  Hashable symbols are coded
    first (by type and value, so 1, 1.0 and True stay distinct), and the predicate runs once per
    distinct (a, b) pair of a pair's sequences."""
    n_p = len(pairs)
    off1 = np.zeros(n_p + 1, dtype=np.uint64)
    off2 = np.zeros(n_p + 1, dtype=np.uint64)
    bits_off = np.zeros(n_p + 1, dtype=np.uint64)
    chunks = []
    for p, (a, b) in enumerate(pairs):
        m, n = len(a), len(b)
        off1[p + 1] = off1[p] + m
        off2[p + 1] = off2[p] + n
        wn = (n + 31) // 32
        if m and n:
            try:
                ua = {}
                c1 = np.fromiter((ua.setdefault((type(x), x), len(ua)) for x in a), dtype=np.int64, count=m)
                ub = {}
                c2 = np.fromiter((ub.setdefault((type(x), x), len(ub)) for x in b), dtype=np.int64, count=n)
                va, vb = [k[1] for k in ua], [k[1] for k in ub]
                if match is None:
                    tab = np.array([[x == y for y in vb] for x in va], dtype=bool)
                else:
                    tab = np.array([[bool(match(x, y)) for y in vb] for x in va], dtype=bool)
                mm = tab[c1][:, c2]
            except TypeError:   # unhashable symbols: evaluate every cell, as the reference does
                f = (lambda x, y: x == y) if match is None else match
                mm = np.array([[bool(f(x, y)) for y in b] for x in a], dtype=bool)
            packed = np.packbits(mm, axis=1, bitorder="little")
            row = np.zeros((m, 4 * wn), dtype=np.uint8)
            row[:, :packed.shape[1]] = packed
            chunks.append(row.reshape(-1).view("<u4"))
        bits_off[p + 1] = bits_off[p] + m * wn
    bits = np.concatenate(chunks) if chunks else np.zeros(1, dtype=np.uint32)
    return off1, off2, np.ascontiguousarray(bits, dtype=np.uint32), bits_off


class Engine:
    """One context per GPU (sa_create).  Not thread-safe; use one Engine per host thread."""

    def __init__(self, device: int = 0):
        self.L = load_library()
        h = C.c_void_p()
        rc = self.L.sa_create(device, C.byref(h))
        if rc != 0:
            raise SeqalibError(f"sa_create({device}) failed: {self.L.sa_last_error(None).decode()}")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            self.L.sa_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self.L.sa_last_error(self.h).decode()
            raise SeqalibError(f"{what}: {self.L.sa_status_string(rc).decode()} ({msg})")

    def set_workspace_limit(self, nbytes: int):
        self._check(self.L.sa_set_workspace_limit(self.h, nbytes), "sa_set_workspace_limit")

    def align_packed(self, algo: int, scoring: ScoringSystem, s1: np.ndarray, off1: np.ndarray,
                     s2: np.ndarray, off2: np.ndarray, lut: Optional[np.ndarray] = None, out=None):
        """Host-buffer batch (sa_align_batch).  Returns (results structured array, ops uint8 array).
        out: optional (results, ops) arrays of a previous call with the same shapes, reused as the
        output buffers (a caller that keeps its buffers avoids re-faulting ~m+n bytes per pair)."""
        npairs = len(off1) - 1
        s1 = np.ascontiguousarray(s1, dtype=np.uint8)
        s2 = np.ascontiguousarray(s2, dtype=np.uint8)
        off1 = np.ascontiguousarray(off1, dtype=np.uint64)
        off2 = np.ascontiguousarray(off2, dtype=np.uint64)
        ops_cap = int(off1[-1] + off2[-1]) + npairs + 1
        if out is not None and out[0].base is not None and len(out[0].base) == max(npairs, 1) \
                and out[0].base.dtype == RESULT_DTYPE and out[1].dtype == np.uint8 and len(out[1]) == ops_cap \
                and out[1].flags.c_contiguous and out[1].flags.writeable:
            res, ops = out[0].base, out[1]
        else:
            res = np.zeros(max(npairs, 1), dtype=RESULT_DTYPE)
            ops = np.zeros(ops_cap, dtype=np.uint8)
        lut_p = 0
        if lut is not None:
            lut = np.ascontiguousarray(lut, dtype=np.uint8).reshape(65536)
            lut_p = _ptr(lut)
        sc = scoring._c()
        rc = self.L.sa_align_batch(self.h, algo, C.byref(sc), _ptr(s1), _ptr(off1), _ptr(s2), _ptr(off2),
                                   npairs, lut_p, _ptr(res), _ptr(ops), ops_cap)
        self._check(rc, "sa_align_batch")
        return res[:npairs], ops

    def align_bits(self, algo: int, scoring: ScoringSystem, off1: np.ndarray, off2: np.ndarray, bits: np.ndarray,
                   bits_off: np.ndarray):
        """Generic-Ty batch (sa_align_batch_bits) from match_bitmaps(): (results, ops)."""
        npairs = len(off1) - 1
        off1 = np.ascontiguousarray(off1, dtype=np.uint64)
        off2 = np.ascontiguousarray(off2, dtype=np.uint64)
        bits = np.ascontiguousarray(bits, dtype=np.uint32)
        bits_off = np.ascontiguousarray(bits_off, dtype=np.uint64)
        res = np.zeros(max(npairs, 1), dtype=RESULT_DTYPE)
        ops_cap = int(off1[-1] + off2[-1]) + npairs + 1
        ops = np.zeros(ops_cap, dtype=np.uint8)
        sc = scoring._c()
        rc = self.L.sa_align_batch_bits(self.h, algo, C.byref(sc), _ptr(off1), _ptr(off2), npairs, _ptr(bits),
                                        _ptr(bits_off), _ptr(res), _ptr(ops), ops_cap)
        self._check(rc, "sa_align_batch_bits")
        return res[:npairs], ops

    def align_generic(self, algo: int, scoring: ScoringSystem, pairs: Sequence[Tuple[Sequence, Sequence]],
                      match: Optional[Callable] = None) -> List[PairResult]:
        """Align pairs of sequences of any symbol type with any match predicate (the reference's
        templated ContainerType / Ty / MatchFnTy): the symbols stay on the host, the GPU gets the
        match bitmaps.  Expand with expand_ops(algo, a, b, r, blank=...)."""
        off1, off2, bits, bits_off = match_bitmaps(pairs, match)
        res, ops = self.align_bits(algo, scoring, off1, off2, bits, bits_off)
        out = []
        for p in range(len(pairs)):
            o = int(off1[p] + off2[p]) + p
            r = res[p]
            out.append(PairResult(int(r["score"]), int(r["end_i"]), int(r["end_j"]), int(r["start_i"]),
                                  int(r["start_j"]), int(r["flags"]), ops[o:o + int(r["nops"])].tobytes()))
        return out

    def align(self, algo: int, scoring: ScoringSystem, pairs: Sequence[Tuple[object, object]],
              lut: Optional[np.ndarray] = None) -> List[PairResult]:
        s1, off1, s2, off2 = pack_pairs(pairs)
        res, ops = self.align_packed(algo, scoring, s1, off1, s2, off2, lut)
        out = []
        for p in range(len(pairs)):
            o = int(off1[p] + off2[p]) + p
            r = res[p]
            out.append(PairResult(int(r["score"]), int(r["end_i"]), int(r["end_j"]), int(r["start_i"]),
                                  int(r["start_j"]), int(r["flags"]), ops[o:o + int(r["nops"])].tobytes()))
        return out

    def align_device(self, algo: int, scoring: ScoringSystem, d_s1: int, d_off1: int, d_s2: int, d_off2: int,
                     npairs: int, max_m: int, max_n: int, d_res: int, d_ops: int, stream: int = 0,
                     d_lut: int = 0):
        """Device-resident batch (sa_align_batch_device); pointers are device addresses."""
        sc = scoring._c()
        rc = self.L.sa_align_batch_device(self.h, algo, C.byref(sc), d_s1, d_off1, d_s2, d_off2, npairs, max_m,
                                          max_n, d_lut or None, d_res, d_ops, stream or None)
        self._check(rc, "sa_align_batch_device")

    def set_pipeline(self, enable: bool):
        """Overlap consecutive align_device calls (sa_set_pipeline); results need wait()."""
        self._check(self.L.sa_set_pipeline(self.h, 1 if enable else 0), "sa_set_pipeline")

    def test_hook(self, hook: int, value: int) -> int:
        """Tests only (sa_test_hook): SA_HOOK_HAND_TAG / SA_HOOK_POISON_WS / SA_HOOK_F16 (value 2:
        returns 1 when the context turned the f16 cell off)."""
        rc = self.L.sa_test_hook(self.h, hook, value)
        if rc > 0:
            return rc
        self._check(rc, "sa_test_hook")
        return 0

    def wait(self):
        """Wait for all pipelined align_device work (sa_wait)."""
        self._check(self.L.sa_wait(self.h), "sa_wait")

    def last_timings(self) -> Tuple[float, float, int]:
        f, t, n = C.c_float(), C.c_float(), C.c_int()
        self._check(self.L.sa_last_timings(self.h, C.byref(f), C.byref(t), C.byref(n)), "sa_last_timings")
        return f.value, t.value, n.value

    def last_kernel_timings(self) -> Tuple[float, float]:
        """(fill kernels alone, fill stream = fill + end-cell replay) of the last call, ms; the call
        must have run with $SEQALIB_KERNEL_TIMING set."""
        f, s = C.c_float(), C.c_float()
        self._check(self.L.sa_last_kernel_timings(self.h, C.byref(f), C.byref(s)), "sa_last_kernel_timings")
        return f.value, s.value


    def last_plan_ex(self) -> Tuple[int, int, int, int]:
        """last_plan() plus the records the fill stored (SA_RECORDS_FLAGS / _TAGS / _SCORE_ONLY)."""
        k, R, W, rec = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        self._check(self.L.sa_last_plan_ex(self.h, C.byref(k), C.byref(R), C.byref(W), C.byref(rec)), "sa_last_plan_ex")
        return k.value, R.value, W.value, rec.value

    def last_plan(self) -> Tuple[int, int, int]:
        """(kernel, R, W) of the last call: kernel is SA_KERNEL_INT32, SA_KERNEL_T16,
        or SA_KERNEL_T16_ENDCELL; W = 0 for the multi-workgroup plan (one single-wave workgroup per
        band of 64*R rows)."""
        k, R, W = C.c_int(), C.c_int(), C.c_int()
        self._check(self.L.sa_last_plan(self.h, C.byref(k), C.byref(R), C.byref(W)), "sa_last_plan")
        return k.value, R.value, W.value


def plan_query(algo: int, max_m: int, max_n: int, npairs: int):
    L = load_library()
    R, W = C.c_int(), C.c_int()
    db, rb = C.c_uint64(), C.c_uint64()
    rc = L.sa_plan_query(algo, max_m, max_n, npairs, C.byref(R), C.byref(W), C.byref(db), C.byref(rb))
    if rc:
        raise SeqalibError("sa_plan_query failed")
    return R.value, W.value, db.value, rb.value


def plan_query_ex(algo: int, scoring: "ScoringSystem", max_m: int, max_n: int, npairs: int, nsym: int = 4):
    """(kernel, R, W, workspace bytes per pair) the engine selects for a batch with `nsym`
    distinct symbols under `scoring` (sa_plan_query_ex)."""
    L = load_library()
    k, R, W, ws = C.c_int(), C.c_int(), C.c_int(), C.c_uint64()
    sc = scoring._c()
    rc = L.sa_plan_query_ex(algo, C.byref(sc), max_m, max_n, npairs, nsym, C.byref(k), C.byref(R), C.byref(W),
                            C.byref(ws))
    if rc:
        raise SeqalibError("sa_plan_query_ex failed")
    return k.value, R.value, W.value, ws.value


# ------------------------------------------------------------------- synthetic inputs (host)
def synth_dna(seed: int, length: int) -> bytes:
    L = load_library()
    out = np.zeros(length, dtype=np.uint8)
    if L.sa_synth_dna(seed, length, _ptr(out)):
        raise SeqalibError("sa_synth_dna failed")
    return out.tobytes()


def synth_mutate(src: bytes, seed: int) -> bytes:
    L = load_library()
    a = np.frombuffer(src, dtype=np.uint8).copy()
    cap = 2 * len(src) + 16
    out = np.zeros(cap, dtype=np.uint8)
    n = C.c_uint32()
    if L.sa_synth_mutate(_ptr(a), len(src), seed, _ptr(out), cap, C.byref(n)):
        raise SeqalibError("sa_synth_mutate failed")
    return out[: n.value].tobytes()


def synth_dna_batch(base: int, npairs: int, len1: int, len2: int, threads: int = 8):
    L = load_library()
    s1 = np.zeros(npairs * len1, dtype=np.uint8)
    s2 = np.zeros(npairs * len2, dtype=np.uint8)
    o1 = np.zeros(npairs + 1, dtype=np.uint64)
    o2 = np.zeros(npairs + 1, dtype=np.uint64)
    if L.sa_synth_dna_batch(base, npairs, len1, len2, _ptr(s1), _ptr(o1), _ptr(s2), _ptr(o2), threads):
        raise SeqalibError("sa_synth_dna_batch failed")
    return s1, o1, s2, o2


# ------------------------------------------------------------- reference-shaped aligners
_engines = {}


def _engine(device: int = 0) -> Engine:
    e = _engines.get(device)
    if e is None:
        e = _engines[device] = Engine(device)
    return e


class _Aligner:
    ALGO = SA_SW

    def __init__(self, scoring: Optional[ScoringSystem] = None, match=None, device: int = 0, blank="-"):
        self.scoring = scoring if scoring is not None else self.getDefaultScoring()
        self.match_fn = match
        self.device = device
        self.blank = blank
        self.last: Optional[PairResult] = None

    @staticmethod
    def getDefaultScoring() -> ScoringSystem:
        return ScoringSystem(-1, 2, -1)

    def getScoring(self):
        return self.scoring

    def getMatchOperation(self):
        return self.match_fn

    def _lut(self, pairs):
        if self.match_fn is None:
            return None
        al1 = sorted({c for a, _ in pairs for c in _as_bytes(a)})
        al2 = sorted({c for _, b in pairs for c in _as_bytes(b)})
        return lut_from_fn(self.match_fn, al1, al2)

    def getAlignments(self, pairs: Sequence[Tuple[object, object]]) -> List[AlignedSequence]:
        eng = _engine(self.device)
        res = eng.align(self.ALGO, self.scoring, pairs, self._lut(pairs))
        out = []
        for (a, b), r in zip(pairs, res):
            if r.flags & SA_FLAG_DIVERGED:
                raise SeqalibError("the reference traceback does not terminate for this scoring")
            if r.flags & SA_FLAG_TIMEOUT:
                raise SeqalibError("device hand-off timed out; result invalid")
            out.append(expand_ops(self.ALGO if not (r.flags & SA_FLAG_SIZE_HACK) else SA_NW,
                                  a, b, r, self.blank))
        self.last = res[-1] if res else None
        return out

    def getAlignment(self, seq1, seq2) -> AlignedSequence:
        return self.getAlignments([(seq1, seq2)])[0]

    def getScore(self) -> Optional[int]:
        return None if self.last is None else self.last.score


class SmithWatermanSA(_Aligner):
    ALGO = SA_SW

    @staticmethod
    def getDefaultScoring():
        return ScoringSystem(-1, 1, -1)   # SASmithWaterman.h:352


class NeedlemanWunschSA(_Aligner):
    ALGO = SA_NW


class LocalGotohSA(_Aligner):
    ALGO = SA_LOCAL_GOTOH


class HirschbergSA(_Aligner):
    """HirschbergSA (SAHirschberg.h): linear-space NW with the reference's own split/tie rules.
    Default scoring is NeedlemanWunschSA's (-1, 2, -1) (:166-167)."""
    ALGO = SA_HIRSCHBERG


class GlobalGotohSA(_Aligner):
    ALGO = SA_GLOBAL_GOTOH


class MyersMillerSA(_Aligner):
    """MyersMillerSA (SAMyersMiller.h): linear-space affine global alignment with the reference's
    own midpoint/tie rules and base cases.  Default scoring (-1, 2, -1) (:406) leaves the affine
    terms unset in the reference; pass a 4/5-argument ScoringSystem."""
    ALGO = SA_MYERS_MILLER

    @staticmethod
    def getDefaultScoring():
        return ScoringSystem(-1, 2, -1)
