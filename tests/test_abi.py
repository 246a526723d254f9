"""CPU: the C-ABI library loads, exports every symbol include/seqalib_hip.h declares, its host-only
entry points (planner, synthetic inputs) behave, and the traceback layout math is consistent.
No GPU compute is called here."""
import ctypes as C
import json
import os
import re

import numpy as np
import pytest

import seqalib_amd as sa
from util import GOLDEN, ROOT, py_dna, py_mutate, sha

HEADER = os.path.join(ROOT, "include", "seqalib_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sa_[a-z_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    L = sa.load_library()
    syms = declared_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert L.sa_version() == 1


def test_status_strings():
    L = sa.load_library()
    for code in (0, -1, -2, -3, -4, -5):
        assert L.sa_status_string(code)


def test_no_gpu_fails_loudly():
    """Without a device the engine must refuse (no silent CPU fallback)."""
    L = sa.load_library()
    n = C.c_int(0)
    L.sa_device_count(C.byref(n))
    if n.value > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(sa.SeqalibError):
        sa.Engine(0)


def test_scoring_overloads_mirror_reference():
    s = sa.ScoringSystem(-1, 2)
    assert (s.gap, s.match, s.mismatch, s.allow_mismatch) == (-1, 2, -(2 ** 31), False)
    s = sa.ScoringSystem(-2, 1, -1, False)
    assert (s.gap, s.match, s.mismatch, s.allow_mismatch) == (-2, 1, -1, False)
    s = sa.ScoringSystem(-3, -1, 1, -1)       # four ints -> the affine overload, as in C++
    assert (s.gap_open, s.gap_extend, s.match, s.mismatch, s.allow_mismatch) == (-3, -1, 1, -1, True)
    s = sa.ScoringSystem(-3, -1, 1, -1, False)
    assert s.allow_mismatch is False


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
@pytest.mark.parametrize("shape", [(1, 1, 1), (1024, 1024, 10000), (4096, 4096, 10000), (4096, 4096, 1),
                                   (8192, 8192, 1), (2048, 2048, 12500), (100, 37, 5), (20000, 150, 3)])
def test_plan_and_layout(algo, shape):
    m, n, npairs = shape
    R, W, dir_bytes, row_bytes = sa.plan_query(algo, m, n, npairs)
    assert R in (2, 4, 8, 16) and 1 <= W <= 16
    bands = -(-m // (64 * R))
    assert W <= max(bands, 1)
    bpc = 4 if (algo >= 2 or R <= 2) else 2   # sa_layout.h record_bpc: padded at R <= 2
    if R == 1:
        bpc = 8
    steps_pad = -(-(n + 63) // 32) * 32
    assert dir_bytes == bands * steps_pad * 64 * R * bpc // 8
    assert row_bytes == (2 if algo >= 2 else 1) * max(n, 1) * 4


def test_headline_plan_fits_hbm():
    # north-star batch: 10,000 pairs of 4096 x 4096 SW (DNA, default scoring).  The shipped plan is
    # the T16 end-cell kernel, one wave per pair, R = 32; the int32 plan is the fallback.
    sw = sa.ScoringSystem(-1, 1, -1)
    kernel, R, W, ws = sa.plan_query_ex(0, sw, 4096, 4096, 10000, nsym=4)
    assert (kernel, R, W) == (sa.SA_KERNEL_T16_ENDCELL, 32, 1)
    # both variants are provisioned (the choice is made on the device): dirs + row buffers +
    # snapshots of the larger one; the pipelined context keeps two slots per pair of a launch
    steps_pad = -(-(4096 + 63) // 32) * 32
    t16_dirs = 2 * steps_pad * 64 * 8
    assert ws >= t16_dirs
    assert 2 * 10000 * ws + 2 * 4096 < 0.5 * 288e9, ws   # one launch, both slots, well inside HBM
    R32, W32, dir_bytes, row_bytes = sa.plan_query(0, 4096, 4096, 10000)
    assert (R32, W32) == (16, 1)
    assert 10000 * (dir_bytes + row_bytes) < 64e9
    # more than four symbols: the int32 kernel
    assert sa.plan_query_ex(0, sw, 4096, 4096, 10000, nsym=5)[:3] == (sa.SA_KERNEL_INT32, 16, 1)


@pytest.mark.parametrize("m,n,npairs,plan", [
    (1024, 1024, 10000, (sa.SA_KERNEL_T16_ENDCELL, 16, 1)),    # config 3
    (2048, 2048, 12500, (sa.SA_KERNEL_T16_ENDCELL, 32, 1)),    # config 5 shard (1 of 8 GPUs)
    (4096, 4096, 1, None),                                      # config 2: few pairs
])
def test_config_plans(m, n, npairs, plan):
    sw = sa.ScoringSystem(-1, 1, -1)
    got = sa.plan_query_ex(0, sw, m, n, npairs, nsym=4)
    if plan is not None:
        assert got[:3] == plan
    assert got[3] * npairs * 2 < 0.5 * 288e9


def test_plan_t16_eligibility_by_scoring():
    # NW at its default scoring (-1, 2, -1): H in [-4096, 8192] on 4096^2 fits int16 as 4*(H - delta);
    # on 8192^2 the range is 24,577 wide -> int32
    assert sa.plan_query_ex(1, sa.ScoringSystem(-1, 2, -1), 4096, 4096, 10000)[0] == sa.SA_KERNEL_T16
    assert sa.plan_query_ex(1, sa.ScoringSystem(-1, 2, -1), 8192, 8192, 10000)[0] == sa.SA_KERNEL_INT32
    assert sa.plan_query_ex(1, sa.ScoringSystem(-1, 1, -1), 4096, 4096, 10000)[0] == sa.SA_KERNEL_T16
    # SW: any size with n < 65535 (pairs whose maximum passes the int16 headroom re-run on int32)
    assert sa.plan_query_ex(0, sa.ScoringSystem(-1, 1, -1), 8192, 8192, 10000)[0] == sa.SA_KERNEL_T16_ENDCELL
    assert sa.plan_query_ex(0, sa.ScoringSystem(-1, 1, -1), 8192, 70000, 10000)[0] == sa.SA_KERNEL_INT32
    # gap 0: the clamped up term needs gap < 0
    assert sa.plan_query_ex(0, sa.ScoringSystem(0, 1, -1), 1024, 1024, 10000)[0] == sa.SA_KERNEL_INT32
    # affine (T16 affine kernel): LocalGotoh at any size (retry above the int16 headroom),
    # GlobalGotoh while the affine path bounds fit 8*(V - delta); no mismatches allowed -> T16 too
    # (mismatch' = 2 (GO + GE) - 1 never wins, like the reference's INT_MIN), unless mismatch'
    # leaves the int8 profile
    aff = sa.ScoringSystem(-3, -1, 1, -1)
    assert sa.plan_query_ex(2, aff, 1024, 1024, 10000)[:3] == (sa.SA_KERNEL_T16_ENDCELL, 16, 1)
    assert sa.plan_query_ex(2, aff, 8192, 8192, 10000)[0] == sa.SA_KERNEL_T16_ENDCELL
    assert sa.plan_query_ex(3, aff, 2048, 2048, 10000)[:3] == (sa.SA_KERNEL_T16, 16, 1)
    # 4096^2 exceeds the a-priori width: the screened T16 kernel on batch plans (per-pair
    # composition cap, int32 re-run above it), int32 for a single pair (SPLIT plan)
    assert sa.plan_query_ex(3, aff, 4096, 4096, 10000)[0] == sa.SA_KERNEL_T16
    assert sa.plan_query_ex(3, aff, 4096, 4096, 1)[0] == sa.SA_KERNEL_INT32
    assert sa.plan_query_ex(3, aff, 16384, 16384, 10000)[0] == sa.SA_KERNEL_INT32   # cap below k / 2
    assert sa.plan_query_ex(2, sa.ScoringSystem(-3, -1, 1, -1, False), 1024, 1024, 10000)[0] == sa.SA_KERNEL_T16_ENDCELL
    assert sa.plan_query_ex(2, sa.ScoringSystem(-3, -1, 1, -1, False), 8192, 8192, 1)[0] == sa.SA_KERNEL_T16_ENDCELL
    assert sa.plan_query_ex(2, sa.ScoringSystem(-9, -1, 1, -1, False), 1024, 1024, 10000)[0] == sa.SA_KERNEL_INT32
    assert sa.plan_query_ex(0, sa.ScoringSystem(-2, 1, -1, False), 1024, 1024, 10000)[0] == sa.SA_KERNEL_T16_ENDCELL
    assert sa.plan_query_ex(1, sa.ScoringSystem(-1, 2), 1024, 1024, 10000)[0] == sa.SA_KERNEL_T16
    assert sa.plan_query_ex(0, sa.ScoringSystem(-20, 1, -1, False), 1024, 1024, 10000)[0] == sa.SA_KERNEL_INT32
    assert sa.plan_query_ex(2, sa.ScoringSystem(-3, 0, 1, -1), 1024, 1024, 10000)[0] == sa.SA_KERNEL_INT32
    assert sa.plan_query_ex(2, aff, 1024, 1024, 10000, nsym=5)[0] == sa.SA_KERNEL_INT32


def cell_byte(R, bpc, max_n, i, j, tagged=False):
    """Python restatement of sa_layout.h cell_byte (independent check of the layout)."""
    bps = R * bpc // 8
    spp = 1 if bps >= 16 else 16 // bps
    pps = bps // 16 if bps > 16 else 1
    steps_pad = -(-(max_n + 63) // 32) * 32
    band_stride = steps_pad * 64 * bps
    ii = i - 1
    b, rem = divmod(ii, 64 * R)
    t, r = divmod(rem, R)
    s = (j - 1) + t
    rb = R * bpc
    wb = min(rb, 32)
    rpw = wb // bpc
    word = r // rpw
    if tagged == 2:   # two-pair kernel: 8 rows per 16-bit half, first row highest
        lowbit = 16 * ((r % 16) // 8) + 2 * (7 - r % 8)
    else:
        lowbit = bpc * (r % rpw) if tagged else wb - bpc * (r % rpw + 1)
    byte_in_rec = word * 4 + lowbit // 8
    half = byte_in_rec // 16
    packet = (s // spp) * pps + half
    return b * band_stride + packet * 1024 + t * 16 + (s % spp) * bps + byte_in_rec % 16, lowbit % 8


@pytest.mark.parametrize("R,bpc,tagged", [(16, 2, 2), (32, 2, 2), (4, 2, False), (8, 2, False), (16, 2, False), (4, 4, False),
                                          (8, 4, False), (16, 4, False), (4, 2, True), (8, 2, True),
                                          (16, 2, True), (1, 8, False), (1, 8, True), (2, 4, False),
                                          (2, 4, True), (2, 8, True), (4, 8, True), (8, 8, True),
                                          (16, 8, True)])
def test_flag_layout_is_a_bijection(R, bpc, tagged):
    """Every cell of a band gets its own bits, records pack exactly R*bpc bits per lane-step."""
    max_n = 70
    m = 64 * R * 2
    seen = set()
    for i in range(1, m + 1):
        for j in range(1, max_n + 1):
            off, sh = cell_byte(R, bpc, max_n, i, j, tagged)
            for k in range(bpc):
                bit = (off, sh + k)
                assert sh + k < 8
                assert bit not in seen
                seen.add(bit)
    assert len(seen) == m * max_n * bpc


def test_synth_matches_std_mt19937_64():
    pins = json.load(open(os.path.join(GOLDEN, "dna_pins.json")))
    for p in pins:
        assert sha(sa.synth_dna(p["seed"], p["len"])) == p["sha"], p
    assert sa.synth_dna(7, 300) == py_dna(7, 300)


def test_synth_mutate_and_batch():
    src = sa.synth_dna(42, 500)
    assert sa.synth_mutate(src, 9) == py_mutate(src, 9)
    s1, o1, s2, o2 = sa.synth_dna_batch(3_000_000_000, 5, 64, 80, threads=3)
    assert list(o1) == [64 * k for k in range(6)] and list(o2) == [80 * k for k in range(6)]
    for p in range(5):
        assert s1[o1[p]:o1[p + 1]].tobytes() == sa.synth_dna(3_000_000_000 + 2 * p + 1, 64)
        assert s2[o2[p]:o2[p + 1]].tobytes() == sa.synth_dna(3_000_000_000 + 2 * p + 2, 80)


def test_expand_ops_matches_oracle_strings():
    """Host-side list assembly + forceGlobal (Python) reproduces the oracle's strings from its ops."""
    from util import oracle_align
    for algo, args, a, b in [(0, (-1, 1, -1), b"AGGATCGGCTAGAGCTAG", b"GAGATCGGCGGATTACAGG"),
                             (1, (-1, 2), b"AAAGAATGCAT", b"AAACTCAT"),
                             (2, (-3, -1, 1, -1, True), b"CTGAAGCGGTTAGC", b"CTCAAGCGTAGTCC"),
                             (3, (-3, -1, 1, -1, False), b"AGCTTCAGGCTGA", b"AGCTGGATCGATCGATG")]:
        o = oracle_align(algo, args, a, b)
        r = sa.PairResult(o["score"], o["end_i"], o["end_j"], o["start_i"], o["start_j"], 0, o["ops"])
        got = sa.expand_ops(algo, a.decode(), b.decode(), r).rows()
        assert got == o["rows"]


def test_transfer_codec_round_trips(tmp_path):
    """The host API's 2-bit transfer codecs (seqalib_amd/csrc/sa_codec.cpp), both packing paths
    (scalar and AVX2), against a byte-by-byte restatement (tests/cpp/codec_test.cpp): every length
    0..300 and large ones, every byte value at every position (only A / C / G / T pack), and the
    op-letter expansion."""
    import subprocess
    exe = str(tmp_path / "codec_test")
    subprocess.run(["g++", "-O2", "-std=c++17", "-DSA_CODEC_TEST", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "codec_test.cpp"),
                    os.path.join(ROOT, "seqalib_amd", "csrc", "sa_codec.cpp")], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True)
    assert out.stdout.strip() == "ok"
