"""GPU robustness paths: no API returns an invalid pair with SA_OK.

* SPLIT plans (few long pairs, one single-wave workgroup per band) wait for the band above with
  a bounded poll; a pair whose wait expired (SA_FLAG_TIMEOUT) is re-run, in the same call, by the
  single-workgroup fallback launch (run_device, sa_api.hip) -- host API and device API alike.
* the band-parallel traceback (sa_traceback_seg.hip) guards every walk; when a guard fires or no
  band records the end of the walk, the wave walker re-walks the pair (SA_FLAG_RECOVERED, exact).
* calls on one context from different streams are ordered (shared workspace and DC buffers).
Faults are injected with test-only environment switches (SEQALIB_SPLIT_WAIT_TICKS,
SEQALIB_SPLIT_FALLBACK, SEQALIB_SEG_INJECT)."""
import numpy as np
import pytest

import seqalib_amd as sa
from test_gpu_parity import SCORINGS, compare_with_oracle, sc_obj
from util import oracle_align

pytestmark = pytest.mark.gpu
BATCH_KERNELS = True   # small host calls stay on the batch kernels (conftest.py)
SA_FLAG_RECOVERED = 16


def long_pairs(seed, count=3, lo=900, hi=2600):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(count):
        a = sa.synth_dna(seed * 100 + 2 * k, int(rng.integers(lo, hi)))
        b = sa.synth_mutate(a, seed + k) if k % 2 == 0 else sa.synth_dna(seed * 100 + 2 * k + 1, int(rng.integers(lo, hi)))
        out.append((a, b))
    return out


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_split_timeout_rerun_host_api(engine, algo, monkeypatch):
    """Every SPLIT band wait expires at once (SEQALIB_SPLIT_WAIT_TICKS=0): without the fallback
    the pairs come back flagged SA_FLAG_TIMEOUT (the injection works); with it, the same call
    returns every pair exact and unflagged."""
    pairs = long_pairs(11 + algo)
    args = SCORINGS[algo][0]
    monkeypatch.setenv("SEQALIB_PLAN", "2,0")
    monkeypatch.setenv("SEQALIB_SPLIT_WAIT_TICKS", "0")
    monkeypatch.setenv("SEQALIB_SPLIT_FALLBACK", "0")
    res = engine.align(algo, sc_obj(args), pairs)
    assert any(r.flags & sa.SA_FLAG_TIMEOUT for r in res)
    monkeypatch.delenv("SEQALIB_SPLIT_FALLBACK")
    for args in SCORINGS[algo][:2]:
        compare_with_oracle(engine, algo, args, pairs)
        assert engine.last_plan()[2] == 0   # the SPLIT plan was the one enqueued
        res = engine.align(algo, sc_obj(args), pairs)
        assert all(r.flags == 0 for r in res), [r.flags for r in res]


@pytest.mark.parametrize("algo", [0, 2])
def test_split_timeout_rerun_device_api(engine, algo, monkeypatch):
    """The device API (asynchronous, results stay in HBM) re-runs timed-out pairs itself too."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    pairs = long_pairs(31 + algo, count=4)
    s1, o1, s2, o2 = sa.pack_pairs(pairs)
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    d = [t(x) for x in (s1, o1, s2, o2)]
    n = len(pairs)
    res = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
    ops = torch.zeros(len(s1) + len(s2) + n, dtype=torch.uint8, device=dev)
    mm = max(len(a) for a, _ in pairs)
    nn = max(len(b) for _, b in pairs)
    args = SCORINGS[algo][0]
    monkeypatch.setenv("SEQALIB_SPLIT_WAIT_TICKS", "0")
    stream = torch.cuda.current_stream().cuda_stream
    engine.align_device(algo, sc_obj(args), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), n, mm,
                        nn, res.data_ptr(), ops.data_ptr(), stream)
    torch.cuda.synchronize()
    got = np.frombuffer(res.cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE)
    g_ops = ops.cpu().numpy()
    assert engine.last_plan()[2] == 0
    for p, (a, b) in enumerate(pairs):
        o = oracle_align(algo, args, a, b)
        r = got[p]
        assert int(r["flags"]) == 0
        off = int(o1[p] + o2[p]) + p
        assert (int(r["score"]), int(r["end_i"]), int(r["end_j"]), int(r["start_i"]), int(r["start_j"])) == \
               (o["score"], o["end_i"], o["end_j"], o["start_i"], o["start_j"])
        assert g_ops[off:off + int(r["nops"])].tobytes() == o["ops"]


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_segmented_traceback_guard_recovers(engine, algo, monkeypatch):
    """Corrupted exit records (SEQALIB_SEG_INJECT=1 overwrites them between the exit-map and the
    emit kernels): no band can chain the walk, so the wave walker re-walks those pairs -- every
    result exact, the re-walked ones flagged SA_FLAG_RECOVERED; none is fabricated."""
    pairs = long_pairs(51 + algo, count=4, lo=1200, hi=2400)
    monkeypatch.setenv("SEQALIB_PLAN", "2,0")
    monkeypatch.setenv("SEQALIB_TB", "seg")
    monkeypatch.setenv("SEQALIB_SEG_INJECT", "1")
    args = SCORINGS[algo][0]
    compare_with_oracle(engine, algo, args, pairs)
    res = engine.align(algo, sc_obj(args), pairs)
    assert any(r.flags & SA_FLAG_RECOVERED for r in res)
    assert all((r.flags & ~SA_FLAG_RECOVERED) == 0 for r in res)
    monkeypatch.delenv("SEQALIB_SEG_INJECT")
    res = engine.align(algo, sc_obj(args), pairs)
    assert all(r.flags == 0 for r in res)


@pytest.mark.parametrize("algo", [4, 5, 0])
def test_calls_on_two_streams_are_ordered(engine, algo):
    """Two device-API calls on one context from two different streams, back to back with no host
    wait: the second waits for the first (they share the workspace / DC buffers), and
    both equal the host API."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    args = (-1, 2, -1) if algo != 5 else (-3, -1, 2, -1)
    sc = sc_obj(args)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    calls = []
    for k in range(2):
        L = (700, 400)[k]
        s1, o1, s2, o2 = sa.synth_dna_batch(1300 + 7 * k, 300 - 100 * k, L, L - 13)
        d = [t(x) for x in (s1, o1, s2, o2)]
        n = len(o1) - 1
        res = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
        ops = torch.zeros(len(s1) + len(s2) + n, dtype=torch.uint8, device=dev)
        calls.append(((s1, o1, s2, o2), d, n, L, res, ops))
    torch.cuda.synchronize()
    for (h, d, n, L, res, ops), st in zip(calls, streams):
        engine.align_device(algo, sc, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), n, L, L,
                            res.data_ptr(), ops.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    for (h, d, n, L, res, ops) in calls:
        s1, o1, s2, o2 = h
        got = np.frombuffer(res.cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE)
        ref, ref_ops = engine.align_packed(algo, sc, s1, o1, s2, o2)
        for f in ("score", "end_i", "end_j", "start_i", "start_j", "nops", "flags"):
            assert (got[f] == ref[f]).all(), (algo, f)
        g_ops = ops.cpu().numpy()
        for p in range(n):
            off = int(o1[p] + o2[p]) + p
            assert g_ops[off:off + int(ref["nops"][p])].tobytes() == ref_ops[off:off + int(ref["nops"][p])].tobytes()


def test_multi_handle_linear_space(engine):
    """HirschbergSA / MyersMillerSA through the multi-device handle (two contexts on GPU 0): each
    context has its own DC buffers, results equal one context's."""
    from seqalib_amd.multi import MultiEngine
    pairs = [(sa.synth_dna(1700 + k, 150 + 23 * k), sa.synth_dna(1800 + k, 170 + 19 * k)) for k in range(30)]
    s1, o1, s2, o2 = sa.pack_pairs(pairs)
    me = MultiEngine([0, 0])
    try:
        for algo, args in ((4, (-1, 2, -1)), (5, (-3, -1, 2, -1))):
            for _ in range(2):
                got, gops = me.align_packed(algo, sc_obj(args), s1, o1, s2, o2)
                ref, rops = engine.align_packed(algo, sc_obj(args), s1, o1, s2, o2)
                for f in ("score", "nops", "flags"):
                    assert (got[f] == ref[f]).all()
                for p in range(len(pairs)):   # (bytes past nops in a slot are unspecified)
                    off, k = int(o1[p] + o2[p]) + p, int(ref["nops"][p])
                    assert gops[off:off + k].tobytes() == rops[off:off + k].tobytes()
    finally:
        me.close()


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_host_api_chunked_pipeline(engine, algo, monkeypatch):
    """The host API cuts big batches into pair ranges and pipelines them (upload of range g+1 and
    download of g-1 under the kernels of g, sa_api.hip align_host).  Forced to 1, 3 and 5 ranges
    on a ragged batch (LUT and equality): identical results and op streams."""
    rng = np.random.default_rng(70 + algo)
    pairs = []
    for k in range(157):
        m = int(rng.integers(0, 500))
        a = sa.synth_dna(50_000 + 2 * k, m)
        b = sa.synth_mutate(a, k)[: int(rng.integers(0, 520))] if k % 3 else sa.synth_dna(50_001 + 2 * k, int(rng.integers(0, 500)))
        pairs.append((a, b))
    s1, o1, s2, o2 = sa.pack_pairs(pairs)
    args = SCORINGS[algo][0]
    out = {}
    for g in ("1", "3", "5"):
        monkeypatch.setenv("SEQALIB_HOST_CHUNKS", g)
        for lut in (None, "purine"):
            from util import named_lut
            out[(g, lut)] = engine.align_packed(algo, sc_obj(args), s1, o1, s2, o2, named_lut(lut))
    for lut in (None, "purine"):
        r1, p1 = out[("1", lut)]
        for g in ("3", "5"):
            r, q = out[(g, lut)]
            assert r.tobytes() == r1.tobytes(), (g, lut)
            for p in range(len(pairs)):   # (bytes past a pair's nops are unspecified)
                off = int(o1[p] + o2[p]) + p
                assert q[off:off + int(r["nops"][p])].tobytes() == p1[off:off + int(r1["nops"][p])].tobytes(), (g, lut, p)
    monkeypatch.setenv("SEQALIB_HOST_CHUNKS", "3")
    compare_with_oracle(engine, algo, args, pairs)
