"""Multi-GPU batching: pairs are independent, so a batch is split statically across GPUs with no
collective on the data path.

Two ways to use several GPUs of one node:
* one process per GPU (torchrun; what bench.py does): rank r takes the contiguous slice
  :func:`shard_range` of the global batch; only the timing is reduced across ranks;
* one process, one host thread + HIP context per GPU: :func:`align_multi_gpu`.
"""
from __future__ import annotations

import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import RESULT_DTYPE, Engine, ScoringSystem


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


def align_multi_gpu(algo: int, scoring: ScoringSystem, s1: np.ndarray, o1: np.ndarray, s2: np.ndarray,
                    o2: np.ndarray, devices: Sequence[int], lut: Optional[np.ndarray] = None,
                    balance: str = "cells"):
    """Align a batch on several GPUs (one host thread and HIP context each).  Returns
    (results, ops) laid out exactly as a single-GPU sa_align_batch would return them."""
    npairs = len(o1) - 1
    if balance == "cells":
        cells = (o1[1:] - o1[:-1]).astype(np.float64) * (o2[1:] - o2[:-1]).astype(np.float64)
        ranges = balanced_split(cells, len(devices))
    else:
        ranges = static_split(npairs, len(devices))
    results = np.zeros(npairs, dtype=RESULT_DTYPE)
    ops = np.zeros(int(o1[-1] + o2[-1]) + npairs + 1, dtype=np.uint8)
    errors: List[BaseException] = []

    def work(dev: int, start: int, end: int):
        try:
            if end <= start:
                return
            eng = Engine(dev)
            a, oa, b, ob = slice_batch(s1, o1, s2, o2, start, end)
            res, sub_ops = eng.align_packed(algo, scoring, a, oa, b, ob, lut)
            results[start:end] = res
            for k in range(end - start):
                p = start + k
                src = int(oa[k] + ob[k]) + k
                dst = int(o1[p] + o2[p]) + p
                nops = int(res["nops"][k])
                ops[dst:dst + nops] = sub_ops[src:src + nops]
            eng.close()
        except BaseException as e:  # surfaced to the caller below
            errors.append(e)

    threads = [threading.Thread(target=work, args=(d, r0, r1)) for d, (r0, r1) in zip(devices, ranges)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return results, ops
