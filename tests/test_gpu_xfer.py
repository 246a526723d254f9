"""2-bit transfers of the host API (seqalib_amd/csrc/sa_codec.cpp, sa_api.hip align_host): sequence
pieces of A / C / G / T travel packed and are unpacked on the device, other pieces as bytes; op
streams come down packed (M, S / X, U, L) unless a call holds another letter.  Every result and op
stream must equal the byte transfers' ($SEQALIB_XFER2=0) and a sample the oracle's.
Reference semantics: SASmithWaterman.h:358-366 (getAlignment), SANeedlemanWunsch.h:256-264,
SALocalGotoh.h:518-526.
"""
import numpy as np
import pytest

import seqalib_amd as sa
from test_gpu_so import NW, SW, assert_same, check_vs_oracle, ragged_batch

pytestmark = pytest.mark.gpu
BATCH_KERNELS = True   # small host calls stay on the batch kernels (conftest.py)
LG = (-3, -1, 1, -1, True)


def host_call(engine, monkeypatch, xfer2, algo, scoring, batch):
    if xfer2:
        monkeypatch.delenv("SEQALIB_XFER2", raising=False)
    else:
        monkeypatch.setenv("SEQALIB_XFER2", "0")
    res, ops = engine.align_packed(algo, sa.ScoringSystem(*scoring), *batch)
    monkeypatch.delenv("SEQALIB_XFER2", raising=False)
    return res.copy(), ops.copy(), engine.last_plan()


def test_two_pieces_each_way(engine, monkeypatch):
    """4,500 x 4096^2 SW: 18.4 MB per sequence buffer (two 16 MiB pieces each), 2-bit both ways
    against bytes both ways; the pairs at the piece boundary and a sample against the oracle."""
    s1, o1, s2, o2 = sa.synth_dna_batch(77 * 10 ** 8, 4500, 4096, 4096, threads=16)
    a = host_call(engine, monkeypatch, True, 0, SW, (s1, o1, s2, o2))
    b = host_call(engine, monkeypatch, False, 0, SW, (s1, o1, s2, o2))
    assert (a[0]["flags"] == 0).all()
    assert_same(a, b, o1, o2)
    edge = int(np.searchsorted(o1, 16 << 20)) - 1   # the pair across seq1's piece boundary
    check_vs_oracle(0, SW, a, (s1, o1, s2, o2), [0, edge, edge + 1, 4499])


@pytest.mark.parametrize("algo,scoring", [(0, SW), (1, NW), (2, LG)])
def test_non_acgt_pieces_go_as_bytes(engine, monkeypatch, algo, scoring):
    """A batch whose seq1 holds lowercase and N symbols (a piece that cannot pack) and whose seq2 is
    plain DNA (packs): identical to byte transfers, and to the oracle on a sample."""
    s1, o1, s2, o2 = ragged_batch(900 + algo, 1500, 2000)
    s1 = s1.copy()
    rng = np.random.default_rng(algo)
    s1[rng.choice(len(s1), 50, replace=False)] = ord("N")
    s1[rng.choice(len(s1), 50, replace=False)] = ord("a")
    batch = (s1, o1, s2, o2)
    a = host_call(engine, monkeypatch, True, algo, scoring, batch)
    b = host_call(engine, monkeypatch, False, algo, scoring, batch)
    assert_same(a, b, o1, o2)
    check_vs_oracle(algo, scoring, a, batch, [0, 1, 2, 3, 11, 700, 1499])


@pytest.mark.parametrize("algo,scoring", [(1, NW), (2, LG)])
def test_packed_ops_other_algorithms(engine, monkeypatch, algo, scoring):
    """NW and LocalGotoh op streams come down 2-bit too (one piece each way)."""
    batch = ragged_batch(950 + algo, 1200, 2000)
    a = host_call(engine, monkeypatch, True, algo, scoring, batch)
    b = host_call(engine, monkeypatch, False, algo, scoring, batch)
    assert_same(a, b, batch[1], batch[3])
    check_vs_oracle(algo, scoring, a, batch, [0, 5, 600, 1199])
