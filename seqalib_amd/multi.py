"""Multi-GPU batching: pairs are independent, so a batch is split statically across GPUs with no
collective on the data path.

Two ways to use several GPUs of one node:
* one process per GPU (torchrun; what bench.py does): rank r takes the contiguous slice
  :func:`shard_range` of the global batch; only the timing is reduced across ranks;
* one process, persistent HIP contexts on several GPUs: :class:`MultiEngine` /
  :func:`align_multi_gpu` (native sa_multi_*: one host thread per device, results in place).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import RESULT_DTYPE, ScoringSystem


def static_split(npairs: int, parts: int) -> List[Tuple[int, int]]:
    """Contiguous [start, end) ranges of near-equal pair counts: GPU g gets [g*P/G, (g+1)*P/G)."""
    return [(g * npairs // parts, (g + 1) * npairs // parts) for g in range(parts)]


def balanced_split(cells: np.ndarray, parts: int) -> List[Tuple[int, int]]:
    """Contiguous ranges with near-equal sum of m*n (for ragged batches)."""
    cells = np.asarray(cells, dtype=np.float64)
    if len(cells) == 0:
        return [(0, 0)] * parts
    csum = np.concatenate([[0.0], np.cumsum(cells)])
    total = csum[-1]
    cuts = [0]
    for g in range(1, parts):
        cuts.append(int(np.searchsorted(csum, total * g / parts, side="left")))
    cuts.append(len(cells))
    cuts = np.maximum.accumulate(np.array(cuts))
    return [(int(cuts[g]), int(cuts[g + 1])) for g in range(parts)]


def shard_range(rank: int, world: int, npairs_global: int) -> Tuple[int, int]:
    return static_split(npairs_global, world)[rank]


def slice_batch(s1, o1, s2, o2, start: int, end: int):
    """Sub-batch [start, end) with offsets re-based to 0."""
    a, b = int(o1[start]), int(o1[end])
    c, d = int(o2[start]), int(o2[end])
    return (s1[a:b], (o1[start:end + 1] - o1[start]).astype(np.uint64),
            s2[c:d], (o2[start:end + 1] - o2[start]).astype(np.uint64))


class MultiEngine:
    """Several GPUs behind one handle (sa_multi_*): one persistent HIP context per listed device
    (a device may repeat), a batch cut into contiguous pair ranges of near-equal sum of m*n and
    aligned concurrently, one native host thread per device.  Results and op streams land in
    place, laid out exactly as a single sa_align_batch returns them -- no gather."""

    def __init__(self, devices: Sequence[int]):
        from . import _Scoring, load_library  # noqa: F401
        import ctypes as C
        self.L = load_library()
        self.devices = list(devices)
        arr = (C.c_int * len(self.devices))(*self.devices)
        h = C.c_void_p()
        rc = self.L.sa_multi_create(arr, len(self.devices), C.byref(h))
        if rc:
            raise RuntimeError(f"sa_multi_create: {self.L.sa_multi_last_error(None).decode()}")
        self.h = h

    def align_packed(self, algo: int, scoring: ScoringSystem, s1, o1, s2, o2, lut: Optional[np.ndarray] = None):
        import ctypes as C
        from . import _ptr
        npairs = len(o1) - 1
        s1 = np.ascontiguousarray(s1, dtype=np.uint8)
        s2 = np.ascontiguousarray(s2, dtype=np.uint8)
        o1 = np.ascontiguousarray(o1, dtype=np.uint64)
        o2 = np.ascontiguousarray(o2, dtype=np.uint64)
        res = np.zeros(max(npairs, 1), dtype=RESULT_DTYPE)
        cap = int(o1[-1] + o2[-1]) + npairs + 1
        ops = np.zeros(cap, dtype=np.uint8)
        lut_p = 0
        if lut is not None:
            lut = np.ascontiguousarray(lut, dtype=np.uint8).reshape(65536)
            lut_p = _ptr(lut)
        sc = scoring._c()
        rc = self.L.sa_multi_align_batch(self.h, algo, C.byref(sc), _ptr(s1), _ptr(o1), _ptr(s2), _ptr(o2), npairs,
                                         lut_p or None, _ptr(res), _ptr(ops), cap)
        if rc:
            raise RuntimeError(f"sa_multi_align_batch: {self.L.sa_multi_last_error(self.h).decode()}")
        return res[:npairs], ops

    def close(self):
        if self.h:
            self.L.sa_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_multi_cache: dict = {}


def _close_cached():
    for eng in _multi_cache.values():
        eng.close()
    _multi_cache.clear()


import atexit  # noqa: E402

atexit.register(_close_cached)


def align_multi_gpu(algo: int, scoring: ScoringSystem, s1: np.ndarray, o1: np.ndarray, s2: np.ndarray,
                    o2: np.ndarray, devices: Sequence[int], lut: Optional[np.ndarray] = None):
    """Align a batch on several GPUs of this node (a cached MultiEngine per device list).  Returns
    (results, ops) laid out exactly as a single-GPU sa_align_batch would return them."""
    key = tuple(devices)
    eng = _multi_cache.get(key)
    if eng is None:
        eng = _multi_cache[key] = MultiEngine(devices)
    return eng.align_packed(algo, scoring, s1, o1, s2, o2, lut)
