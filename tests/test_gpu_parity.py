"""GPU parity: the HIP path (through the C ABI) against the golden vectors of the unmodified
reference and against the pinned C oracle on seeded random inputs.

Bar: bit-exact — score, end cell (MaxRow, MaxCol), and the three alignment strings.
All tests run in one process on one HIP context (tests/conftest.py `engine`).
"""
import collections

import numpy as np
import pytest

import seqalib_amd as sa
from util import ALGOS, golden_sequences, load_golden, named_lut, oracle_align, rows_digest

pytestmark = pytest.mark.gpu
BATCH_KERNELS = True   # small host calls stay on the batch kernels (conftest.py)


def sc_obj(args):
    return sa.ScoringSystem(*args)


def run_group(engine, algo, args, match, pairs):
    lut = named_lut(match)
    res = engine.align(algo, sc_obj(args), pairs, lut)
    return res


def rows_of(algo, a, b, r):
    return sa.expand_ops(algo if not (r.flags & sa.SA_FLAG_SIZE_HACK) else sa.SA_NW,
                         a.decode("latin-1"), b.decode("latin-1"), r).rows()


def check_golden(engine, entries):
    groups = collections.defaultdict(list)
    for e in entries:
        groups[(e["algo"], tuple(e["scoring"]), e["match"])].append(e)
    n = 0
    for (algo, args, match), es in groups.items():
        pairs = [golden_sequences(e) for e in es]
        res = run_group(engine, ALGOS[algo], args, match, pairs)
        for e, (a, b), r in zip(es, pairs, res):
            assert (r.flags & (sa.SA_FLAG_DIVERGED | sa.SA_FLAG_BAD_SHAPE)) == 0, e["id"]
            if e["score"] is not None:   # None: the reference exposes no score (MyersMillerSA)
                assert r.score == e["score"], e["id"]
            assert (r.end_i, r.end_j) == (e["max_row"], e["max_col"]), e["id"]
            rows = rows_of(ALGOS[algo], a, b, r)
            assert len(rows[0]) == e["len"], e["id"]
            if "rows" in e:
                assert list(rows) == e["rows"], e["id"]
            else:
                assert rows_digest(*rows) == e["rows_sha"], e["id"]
            n += 1
    return n


def test_readme_known_answer(engine):
    r = engine.align(sa.SA_NW, sa.ScoringSystem(-1, 2), [(b"AAAGAATGCAT", b"AAACTCAT")])[0]
    rows = sa.expand_ops(sa.SA_NW, "AAAGAATGCAT", "AAACTCAT", r).rows()
    assert rows == ("AAA-GAATGCAT", "|||    | |||", "AAAC---T-CAT")
    assert r.score == 9


def test_golden_kat(engine):
    assert check_golden(engine, load_golden("kat.jsonl")) > 2000


def test_golden_random(engine):
    assert check_golden(engine, load_golden("random.jsonl")) > 200


def test_golden_small_calls(engine, monkeypatch):
    """The known-answer and random vectors of the unmodified reference, one getAlignment() per
    pair as its tests call it: every pair within the small-call limits is its own host call on
    the small-call kernel (sa_tiny.hip)."""
    monkeypatch.setenv("SEQALIB_TINY", "1")
    n = 0
    for name in ("kat.jsonl", "random.jsonl"):
        for e in load_golden(name):
            if ALGOS[e["algo"]] > 3:
                continue
            a, b = golden_sequences(e)
            if len(a) > 256 or len(b) > 1024 or len(a) * len(b) > 32768:
                continue
            n += check_golden(engine, [e])
            assert engine.last_plan()[0] == sa.SA_KERNEL_TINY, e["id"]
    assert n > 1000


def test_golden_hirschberg(engine):
    """HirschbergSA (SAHirschberg.h) vectors of the unmodified reference: device levels (pairs
    taller than 12 rows, packed and whole-wave sweeps), per-thread leaves, NW base cases, empty /
    length-1 edges."""
    assert check_golden(engine, load_golden("hirschberg.jsonl")) > 800


@pytest.mark.parametrize("args,match", [((-1, 2, -1), None), ((-2, 1, -1, False), None), ((-1, 2), "purine"),
                                        ((-3, 2, -2), "nwild")])
def test_hirschberg_batch_vs_oracle(engine, args, match):
    rng = np.random.default_rng(11)
    pairs = []
    for k in range(120):
        m = int(rng.integers(0, 900)) if k % 4 else int(rng.integers(0, 4))
        n = int(rng.integers(0, 900)) if k % 5 else int(rng.integers(0, 4))
        a = sa.synth_dna(70_000 + 2 * k, m)
        b = sa.synth_mutate(a, k)[:n] if k % 2 else sa.synth_dna(70_001 + 2 * k, n)
        if match == "nwild":
            b = bytes(ord("N") if (x % 7 == 3) else c for x, c in enumerate(b))
        pairs.append((a, b))
    pairs.append((sa.synth_dna(5, 3000), sa.synth_dna(6, 2500)))
    compare_with_oracle(engine, sa.SA_HIRSCHBERG, args, pairs, match)


def test_golden_myers_miller(engine):
    """MyersMillerSA (SAMyersMiller.h) vectors of the unmodified reference: device levels (pairs
    taller than 12 rows), per-thread leaves, both midpoint types, M == 1 / N == 0 / M == 0 base
    cases, empty edges."""
    assert check_golden(engine, load_golden("myersmiller.jsonl")) > 850


@pytest.mark.parametrize("args,match", [((-3, -1, 1, -1, True), None), ((-3, -1, 1, -1, False), None),
                                        ((-2, -1, 2, -1, True), "purine"), ((-5, -2, 3, -2, True), "nwild"),
                                        ((0, -1, 1, -1, True), None)])
def test_myers_miller_batch_vs_oracle(engine, args, match):
    """Ragged batch vs the oracle, score included (the oracle's top-call optimum)."""
    rng = np.random.default_rng(13)
    pairs = []
    for k in range(120):
        m = int(rng.integers(0, 900)) if k % 4 else int(rng.integers(0, 4))
        n = int(rng.integers(0, 900)) if k % 5 else int(rng.integers(0, 4))
        a = sa.synth_dna(80_000 + 2 * k, m)
        b = sa.synth_mutate(a, k)[:n] if k % 2 else sa.synth_dna(80_001 + 2 * k, n)
        if match == "nwild":
            b = bytes(ord("N") if (x % 7 == 3) else c for x, c in enumerate(b))
        pairs.append((a, b))
    pairs.append((sa.synth_dna(7, 3000), sa.synth_dna(8, 2500)))
    pairs.append((sa.synth_dna(9, 5000), sa.synth_dna(10, 7)))     # tall and thin: levels with n tiny
    pairs.append((sa.synth_dna(11, 40), sa.synth_dna(12, 3000)))   # short and wide: leaf in global rows
    compare_with_oracle(engine, sa.SA_MYERS_MILLER, args, pairs, match)


@pytest.mark.parametrize("algo,args", [(sa.SA_HIRSCHBERG, (-1, 2, -1)), (sa.SA_MYERS_MILLER, (-3, -1, 1, -1, True))])
@pytest.mark.parametrize("park", ["1", "0"])
def test_dc16_handoff_row_every_register(engine, monkeypatch, algo, args, park):
    """16-bit whole-wave sweeps with R = 16 (a level whose longest sweep has 513..1024 rows): the
    steady chunks hand on register (m - 1) % 16 of lane (m - 1) % 1024 / 16 in the last band (and
    register 15 of lane 63 in the others), parked in LDS (SEQALIB_DC16_PARK=1, default) or stored
    per step (0).  Top-level sweep heights 550 .. 1000 cover every register index; round 3's park
    variant sent indices >= 7 to register 7.  (R = 32 and several bands: the
    3000 x 2500 and 5000 x 7 pairs of the batch tests above.)"""
    monkeypatch.setenv("SEQALIB_DC16_PARK", park)
    pairs = []
    for k in range(32):
        m, n = 1100 + 29 * k, 1000 + 23 * k
        a = sa.synth_dna(90_000 + 2 * k, m)
        b = sa.synth_mutate(a, k)[:n] if k % 2 else sa.synth_dna(90_001 + 2 * k, n)
        pairs.append((a, b))
    compare_with_oracle(engine, algo, args, pairs, None)


def test_golden_large(engine):
    assert check_golden(engine, load_golden("large.jsonl")) == 10


@pytest.mark.parametrize("algo", ["hb", "mm"])
@pytest.mark.parametrize("leaf,seg", [(6, "1"), (24, "0"), (24, "1"), (100, "1")])
def test_dc_level_loop_variants_vs_oracle(engine, monkeypatch, algo, leaf, seg):
    """Device-resident level loop (sa_dc.hip) under other leaf thresholds and with the packed
    16/32-lane sweeps on or off: more levels (leaf 6: packed sweeps of <= 16 rows, 3-row leaves),
    fewer (leaf 100: leaves past the LDS tile, global scratch), ragged and empty pairs."""
    monkeypatch.setenv("SEQALIB_HB_LEAF" if algo == "hb" else "SEQALIB_MM_LEAF", str(leaf))
    monkeypatch.setenv("SEQALIB_DC_SEG", seg)
    rng = np.random.default_rng(17 + leaf)
    pairs = []
    for k in range(60):
        m = int(rng.integers(0, 700)) if k % 6 else int(rng.integers(0, 3))
        n = int(rng.integers(0, 700)) if k % 7 else int(rng.integers(0, 3))
        a = sa.synth_dna(90_000 + 2 * k, m)
        b = sa.synth_mutate(a, k)[:n] if k % 2 else sa.synth_dna(90_001 + 2 * k, n)
        pairs.append((a, b))
    pairs.append((sa.synth_dna(13, 2000), sa.synth_dna(14, 150)))   # wide leaves / thin levels
    if algo == "hb":
        compare_with_oracle(engine, sa.SA_HIRSCHBERG, (-1, 2, -1), pairs)
    else:
        compare_with_oracle(engine, sa.SA_MYERS_MILLER, (-3, -1, 1, -1, True), pairs)


@pytest.mark.parametrize("algo", ["hb", "mm"])
def test_dc_int32_sweeps_grid_stride(engine, algo):
    """Five-symbol batch (N wildcards): the int32 whole-wave sweeps run beside the 16-bit two-per-
    wave kernel, on a grid capped at kDcSkipGrid (sa_dc.h) blocks, each block looping over the
    level's sweeps -- 2500 pairs give levels of more than 8192 sweeps."""
    pairs = []
    for k in range(2500):
        m, n = 180 + k % 97, 170 + (k * 7) % 113
        a = sa.synth_dna(120_000 + 2 * k, m)
        b = sa.synth_mutate(a, k)[:n] if k % 2 else sa.synth_dna(120_001 + 2 * k, n)
        b = bytes(ord("N") if (x % 11 == 5) else c for x, c in enumerate(b))
        pairs.append((a, b))
    if algo == "hb":
        compare_with_oracle(engine, sa.SA_HIRSCHBERG, (-3, 2, -2), pairs, "nwild")
    else:
        compare_with_oracle(engine, sa.SA_MYERS_MILLER, (-5, -2, 3, -2, True), pairs, "nwild")


def compare_with_oracle(engine, algo, args, pairs, match=None):
    lut = named_lut(match)
    res = engine.align(algo, sc_obj(args), pairs, lut)
    for (a, b), r in zip(pairs, res):
        o = oracle_align(algo, args, a, b, lut)
        assert o["rc"] == 0
        got = (r.score, r.end_i, r.end_j, r.start_i, r.start_j, r.ops)
        exp = (o["score"], o["end_i"], o["end_j"], o["start_i"], o["start_j"], o["ops"])
        assert got == exp, (algo, args, len(a), len(b))
        assert rows_of(algo, a, b, r) == o["rows"]


SCORINGS = {0: [(-1, 1, -1), (-2, 1, -1, False), (-1, 2), (-3, 2, -2)],
            1: [(-1, 2, -1), (-1, 2), (-2, 1, -1, False)],
            2: [(-3, -1, 1, -1, False), (-3, -1, 1, -1, True), (-2, -1, 2, -1, True)],
            3: [(-3, -1, 1, -1, True), (-3, -1, 1, -1, False), (-5, -2, 3, -2, True)]}


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_ragged_batch_vs_oracle(engine, algo):
    """One batch with many different shapes (slots padded to the batch max)."""
    rng = np.random.default_rng(100 + algo)
    pairs = []
    for k in range(60):
        m = int(rng.integers(0, 700)) if k % 7 else int(rng.integers(1, 5))
        n = int(rng.integers(0, 700)) if k % 5 else int(rng.integers(1, 5))
        a = sa.synth_dna(10_000 + 2 * k, m)
        b = sa.synth_mutate(a, 50 + k)[:n] if k % 3 == 0 else sa.synth_dna(10_001 + 2 * k, n)
        if algo == 2 and (len(a), len(b)) in ((314, 288), (60, 57), (61, 58)):
            continue
        pairs.append((a, b))
    for args in SCORINGS[algo]:
        compare_with_oracle(engine, algo, args, pairs)


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_many_pairs_plan_vs_oracle(engine, algo):
    """>= 1024 pairs selects the one-wave many-pairs plan (bands back to back through the row
    buffer; T16 for DNA SW/NW/Gotoh with allow-mismatch, int32 otherwise)."""
    pairs = []
    for k in range(1100):
        m, n = 150 + (k % 37), 140 + (k % 53)
        a = sa.synth_dna(20_000 + 2 * k, m)
        b = sa.synth_mutate(a, k)[:n] if k % 2 else sa.synth_dna(20_001 + 2 * k, n)
        pairs.append((a, b))
    compare_with_oracle(engine, algo, SCORINGS[algo][0], pairs)


@pytest.mark.parametrize("algo,tall", [(0, False), (0, True), (1, False), (2, False), (3, False)])
def test_many_pairs_unstaged_seq2_vs_oracle(engine, algo, tall, monkeypatch):
    """The many-pairs plans with Seq2 read from global memory per chunk instead of staged in LDS
    (what a batch with max_n > kMaxStagedSeq2 = 48 KiB takes; $SEQALIB_STAGE_SEQ2=0 forces it):
    SW runs the score-only fill, at R = 4 and (tall) R = 32."""
    monkeypatch.setenv("SEQALIB_STAGE_SEQ2", "0")
    pairs = []
    for k in range(1100):
        m, n = (2100 + (k % 29), 120 + (k % 31)) if tall else (150 + (k % 37), 140 + (k % 53))
        a = sa.synth_dna(40_000 + 2 * k, m)
        b = sa.synth_mutate(a, k)[:n] if k % 2 else sa.synth_dna(40_001 + 2 * k, n)
        pairs.append((a, b))
    compare_with_oracle(engine, algo, SCORINGS[algo][0], pairs)


@pytest.mark.parametrize("lp", ["4", "8"])
@pytest.mark.parametrize("tall", [False, True])
def test_so_traceback_lanes_per_pair_vs_oracle(engine, lp, tall, monkeypatch):
    """Score-only traceback (traceback_so4_kernel) at 4 and 8 lanes per pair ($SEQALIB_TB_LP; the
    default is 8 at R = 32, 4 below): R = 16 and (tall) R = 32 many-pairs batches, every op stream
    against the full-matrix oracle."""
    monkeypatch.setenv("SEQALIB_TB_LP", lp)
    pairs = []
    for k in range(1100):
        m, n = (2050 + (k % 41), 150 + (k % 37)) if tall else (600 + (k % 43), 300 + (k % 29))
        a = sa.synth_dna(50_000 + 2 * k, m)
        b = sa.synth_mutate(a, k)[:n] if k % 2 else sa.synth_dna(50_001 + 2 * k, n)
        pairs.append((a, b))
    compare_with_oracle(engine, 0, SCORINGS[0][0], pairs)


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_multiband_wrap_vs_oracle(engine, algo, monkeypatch):
    """More bands than waves (m > 64*R*W): bands wrap round-robin over the waves of one
    workgroup (the single-workgroup few-pairs plan; SEQALIB_SPLIT=0 keeps it selected)."""
    monkeypatch.setenv("SEQALIB_SPLIT", "0")
    pairs = [(sa.synth_dna(31, 21000), sa.synth_dna(32, 97)), (sa.synth_dna(33, 9000), sa.synth_dna(34, 300)),
             (sa.synth_dna(35, 130), sa.synth_dna(36, 9000))]
    compare_with_oracle(engine, algo, SCORINGS[algo][1 % len(SCORINGS[algo])], pairs)
    assert engine.last_plan()[2] > 0


def split_pairs(seed):
    """Few pairs with 1..40 bands of 256 rows: ragged band counts inside one launch, thin and wide
    shapes, related pairs (long local paths crossing many bands), and empty sides."""
    rng = np.random.default_rng(seed)
    pairs = [(sa.synth_dna(seed, 10000), sa.synth_mutate(sa.synth_dna(seed, 10000), seed)[:9000]),
             (sa.synth_dna(seed + 1, 4096), sa.synth_dna(seed + 2, 4096)),
             (sa.synth_dna(seed + 3, 3000), sa.synth_dna(seed + 4, 70)),
             (sa.synth_dna(seed + 5, 300), sa.synth_dna(seed + 6, 5000)),
             (sa.synth_dna(seed + 7, 257), sa.synth_dna(seed + 8, 1)),
             (b"", sa.synth_dna(seed + 9, 40)), (sa.synth_dna(seed + 10, 600), b"")]
    for k in range(12):
        m, n = int(rng.integers(1, 2600)), int(rng.integers(1, 2600))
        a = sa.synth_dna(seed * 100 + 2 * k, m)
        b = sa.synth_mutate(a, k)[:n] if k % 2 else sa.synth_dna(seed * 100 + 2 * k + 1, n)
        pairs.append((a, b))
    return pairs


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_split_plan_vs_oracle(engine, algo, monkeypatch):
    """Few pairs take the multi-workgroup plan: one single-wave workgroup per (pair, band), band
    b+1 polling band b's last row through write-through {tag, value} granules (sa_fill_impl.h,
    SPLIT).  Every scoring of the algorithm (T16 + end-cell replay for DNA SW/NW with
    allow-mismatch, int32 otherwise), R = 2 (the default: padded records, sa_layout.h
    record_bpc), R = 1, 4 and 8 forced, and a custom match table, against the oracle; the result
    must not depend on the plan."""
    pairs = split_pairs(40 + algo)
    max_m = max(len(a) for a, _ in pairs)
    # sa_api.hip make_plan: the shortest bands (R = 2, then 4) while every band has a SIMD
    R0 = next((r for r in (2, 4) if len(pairs) * -(-max_m // (64 * r)) <= 1024), 8)
    for args in SCORINGS[algo]:
        compare_with_oracle(engine, algo, args, pairs)
        assert engine.last_plan()[1:] == (R0, 0), args
        assert all((r.flags & sa.SA_FLAG_TIMEOUT) == 0 for r in engine.align(algo, sc_obj(args), pairs[:2]))
    for r in (1, 2, 4, 8):
        monkeypatch.setenv("SEQALIB_PLAN", f"{r},0")
        for args in SCORINGS[algo][:2]:
            compare_with_oracle(engine, algo, args, pairs)
            assert engine.last_plan()[1:] == (r, 0), (r, args)
    monkeypatch.delenv("SEQALIB_PLAN")
    compare_with_oracle(engine, algo, SCORINGS[algo][0], pairs, "purine")
    assert engine.last_plan()[1:] == (R0, 0)
    # one long pair (configs 2 and 4): R = 2
    compare_with_oracle(engine, algo, SCORINGS[algo][0], pairs[1:2])
    assert engine.last_plan()[1:] == (2, 0)


T16_KERNELS = (sa.SA_KERNEL_T16, sa.SA_KERNEL_T16_ENDCELL)


def dna_pairs(seed, count, maxlen):
    rng = np.random.default_rng(seed)
    pairs = []
    for k in range(count):
        m, n = int(rng.integers(0, maxlen)), int(rng.integers(0, maxlen))
        a = sa.synth_dna(seed * 1000 + 2 * k, m)
        b = sa.synth_mutate(a, k)[:n] if k % 2 else sa.synth_dna(seed * 1000 + 2 * k + 1, n)
        pairs.append((a, b))
    return pairs


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_t16_and_int32_kernels_both_exact(engine, algo, monkeypatch):
    """DNA SW/NW/LocalGotoh/GlobalGotoh with allow-mismatch run on the tagged 16-bit kernels (the
    affine one for Gotoh); SEQALIB_T16=0 forces the int32 kernel.  Both must equal the oracle."""
    pairs = dna_pairs(7 + algo, 40, 900)
    full = 5 if algo >= 2 else 4   # argument count of the overload with AllowMismatch
    allow_scorings = [a for a in SCORINGS[algo] if len(a) == full - 1 or (len(a) == full and a[-1])]
    assert allow_scorings
    for args in allow_scorings:
        compare_with_oracle(engine, algo, args, pairs)
        assert engine.last_plan()[0] in T16_KERNELS, args
    monkeypatch.setenv("SEQALIB_T16", "0")
    for args in allow_scorings:
        compare_with_oracle(engine, algo, args, pairs)
        assert engine.last_plan()[0] == sa.SA_KERNEL_INT32, args


@pytest.mark.parametrize("algo", [0, 1])
def test_t16_eligibility(engine, algo):
    """Kernel choice follows the preconditions: <= 4 symbols, int16 headroom, allow-mismatch."""
    dna = dna_pairs(21 + algo, 6, 400)
    # fewer than four symbols (codes padded with absent bytes)
    two = [(bytes(b"AC"[x & 1] for x in a), bytes(b"CA"[x % 3 == 0] for x in b)) for a, b in dna]
    compare_with_oracle(engine, algo, (-1, 2, -1), two)
    assert engine.last_plan()[0] in T16_KERNELS
    # a fifth symbol -> int32 kernel
    five = dna[:-1] + [(dna[-1][0] + b"N", dna[-1][1])]
    compare_with_oracle(engine, algo, (-1, 2, -1), five)
    assert engine.last_plan()[0] == sa.SA_KERNEL_INT32
    # scores past the int16 headroom of 4*H: SW runs T16 and re-runs the pair on int32 (per-pair
    # retry); NW centres its score range with a constant offset, and only a range wider than
    # 2^14 goes to the int32 kernel
    big = [(sa.synth_dna(77, 3000), sa.synth_dna(77, 3000))]
    compare_with_oracle(engine, algo, (-1, 3, -1), big)
    assert engine.last_plan()[0] in T16_KERNELS
    compare_with_oracle(engine, algo, (-1, 2, -1), big)
    assert engine.last_plan()[0] in T16_KERNELS
    if algo == 1:
        compare_with_oracle(engine, algo, (-1, 5, -1), big)
        assert engine.last_plan()[0] == sa.SA_KERNEL_INT32
    # !allowMismatch runs T16 with a mismatch score below 2 * gap, which never wins a max (as the
    # reference's INT_MIN diagonal): t16_mode, sa_api.hip
    compare_with_oracle(engine, algo, (-2, 1, -1, False), dna)
    assert engine.last_plan()[0] in T16_KERNELS
    compare_with_oracle(engine, algo, (-1, 2), dna)   # the 2-argument ScoringSystem: !allow too
    assert engine.last_plan()[0] in T16_KERNELS
    # ... unless that score does not fit the int8 profile (gap -20: mismatch' = -41)
    compare_with_oracle(engine, algo, (-20, 1, -1, False), dna)
    assert engine.last_plan()[0] == sa.SA_KERNEL_INT32
    if algo == 0:
        # SW with gap 0: the T16 cell folds the zero clamp into a saturating up term, which needs
        # gap < 0 (sa_fill_impl.h), so the int32 kernel takes it
        compare_with_oracle(engine, algo, (0, 1, -1), dna)
        assert engine.last_plan()[0] == sa.SA_KERNEL_INT32


def test_t16_range_extension_large_probes(engine):
    """The reference's own 8192 x 8192 SW probe and its 4096 x 4096 NW probe at NW's default
    scoring (-1, 2, -1) run on the T16 kernel (SW: max score proven small at run time; NW: the
    constant offset) and equal the reference's golden vectors."""
    big = {e["id"]: e for e in load_golden("large.jsonl")}
    for pid in ("probe8192/sw/-1_1_-1/equal", "probe4096/nw/-1_2_-1/equal"):
        assert check_golden(engine, [big[pid]]) == 1
        assert engine.last_plan()[0] in T16_KERNELS, pid


def test_t16_sw_retry_mixed_batch(engine):
    """A T16 SW batch in which a few pairs score above the int16 headroom (identical 9,000-long
    sequences: score 9,000): exactly those pairs are re-run on the int32 kernel, on the batch
    plan (>= 1024 pairs) and on the few-pairs plan, and every pair equals the oracle."""
    rng = np.random.default_rng(17)
    pairs = [(sa.synth_dna(60_000 + k, int(rng.integers(50, 400))), sa.synth_dna(70_000 + k, int(rng.integers(50, 400))))
             for k in range(1100)]
    hot = sa.synth_dna(80_000, 9000)
    pairs[3] = (hot, hot)
    pairs[700] = (hot[:8500], sa.synth_mutate(hot, 3)[:8600])
    compare_with_oracle(engine, 0, (-1, 1, -1), pairs)
    assert engine.last_plan()[0] in T16_KERNELS
    compare_with_oracle(engine, 0, (-1, 1, -1), [pairs[3], pairs[5], pairs[700]])
    assert engine.last_plan()[0] in T16_KERNELS


def test_t16_affine_eligibility_and_retry(engine):
    """T16 affine kernel choice and headroom: LocalGotoh runs T16 at any size and re-runs on int32
    exactly the pairs whose maximum passes 4095 - match (8*M in int16), on the batch plan and the
    few-pairs plan; GlobalGotoh runs T16 while its affine path bounds fit (2048^2) and int32
    beyond (the reference's 4096^2 GlobalGotoh probe); !allowMismatch on T16 too (config 4's
    scoring, the reference's 8192^2 probe); five symbols -> int32."""
    lg = (-3, -1, 1, -1, True)
    rng = np.random.default_rng(29)
    pairs = [(sa.synth_dna(90_000 + k, int(rng.integers(50, 300))), sa.synth_dna(91_000 + k, int(rng.integers(50, 300))))
             for k in range(1100)]
    hot = sa.synth_dna(92_000, 5000)
    pairs[5] = (hot, hot)                                        # score 5000 > 4094: retried
    pairs[900] = (hot[:4600], sa.synth_mutate(hot, 5)[:4700])
    compare_with_oracle(engine, 2, lg, pairs)
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16_ENDCELL
    compare_with_oracle(engine, 2, lg, [pairs[5], pairs[6], pairs[900]])
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16_ENDCELL
    gg = (-3, -1, 1, -1, True)
    two = [(sa.synth_dna(93_000, 2048), sa.synth_dna(93_001, 2048)),
           (sa.synth_dna(93_002, 2000), sa.synth_mutate(sa.synth_dna(93_002, 2000), 4)[:2048])]
    compare_with_oracle(engine, 3, gg, two)
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16
    big = {e["id"]: e for e in load_golden("large.jsonl")}
    assert check_golden(engine, [big["probe4096/gg/-3_-1_1_-1_1/equal"]]) == 1
    assert engine.last_plan()[0] == sa.SA_KERNEL_INT32
    for pid in ("probe8192/lg/-3_-1_1_-1_1/equal", "mut4096/lg/-3_-1_1_-1_1/equal"):
        assert check_golden(engine, [big[pid]]) == 1
        assert engine.last_plan()[0] == sa.SA_KERNEL_T16_ENDCELL, pid
    dna = dna_pairs(31, 6, 400)
    compare_with_oracle(engine, 2, (-3, -1, 1, -1, False), dna)
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16_ENDCELL
    compare_with_oracle(engine, 3, (-3, -1, 1, -1, False), dna)
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16
    compare_with_oracle(engine, 2, (-3, -1, 1, -1, False), pairs)   # batch plan, retried pairs
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16_ENDCELL
    assert check_golden(engine, [big["probe8192/lg/-3_-1_1_-1_0/equal"]]) == 1   # config 4
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16_ENDCELL
    compare_with_oracle(engine, 2, (-9, -1, 1, -1, False), dna)   # 2 * GOE - 1 = -21: no int8 room
    assert engine.last_plan()[0] == sa.SA_KERNEL_INT32
    five = dna[:-1] + [(dna[-1][0] + b"N", dna[-1][1])]
    compare_with_oracle(engine, 3, gg, five)
    assert engine.last_plan()[0] == sa.SA_KERNEL_INT32


def test_t16_global_gotoh_screened_4096(engine, monkeypatch):
    """GlobalGotoh past the a-priori 16-bit width (4096^2 at (-3, -1, 1, -1): values in
    [-4104, 4096]) still runs the T16 affine kernel: the window sits at the low end (every pair's
    borders reach it) and the fill screens each pair by its symbol composition (every prefix
    alignment scores <= MA * sum_c min(count1(c), count2(c))).  Pairs above the cap -- identical or
    near-identical sequences -- are re-run exactly on the int32 kernel; the rest stay T16.  Batch
    plan (>= 1024 pairs) and the widened few-pairs plan (SEQALIB_SPLIT=0; SPLIT plans never take
    the screened kernel)."""
    gg = (-3, -1, 1, -1, True)
    hot = sa.synth_dna(95_000, 4096)
    big = [(sa.synth_dna(95_001, 4096), sa.synth_dna(95_002, 4096)),      # random: screened in
           (hot, hot),                                                   # score 4096: int32
           (hot, sa.synth_mutate(hot, 2)[:4096]),                         # near-identical: int32
           (sa.synth_dna(95_003, 4000), sa.synth_dna(95_004, 4096))]
    rng = np.random.default_rng(41)
    pairs = [(sa.synth_dna(96_000 + k, int(rng.integers(20, 200))), sa.synth_dna(97_000 + k, int(rng.integers(20, 200))))
             for k in range(1100)]
    pairs[10], pairs[500], pairs[501], pairs[1099] = big
    compare_with_oracle(engine, 3, gg, pairs)
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16
    monkeypatch.setenv("SEQALIB_SPLIT", "0")
    compare_with_oracle(engine, 3, gg, big)
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16
    # !allowMismatch: no mismatched diagonal, so the a-priori low end is the all-gap path
    # (2 GO + 8192 GE = -8198 at (4096, 4096)), wider than any 16-bit window: int32
    compare_with_oracle(engine, 3, (-3, -1, 1, -1, False), big)
    assert engine.last_plan()[0] == sa.SA_KERNEL_INT32
    monkeypatch.delenv("SEQALIB_SPLIT")
    compare_with_oracle(engine, 3, gg, big)   # few long pairs: SPLIT plan, int32
    assert engine.last_plan()[0] == sa.SA_KERNEL_INT32


def test_t16_global_gotoh_screened_lut(engine):
    """The screened T16 GlobalGotoh fill under a match table where DIFFERENT symbols match
    (ADVICE r03): all-'A' against all-'a' with a case-insensitive table scores ~4096 although the
    two sequences share no symbol, so the composition screen must count matches through the table
    (sum over a of min(count of a, count of the Seq2 symbols matching a)) and send the pair to the
    int32 re-run; purine/pyrimidine classes on DNA likewise.  Every pair against the oracle.
    (The T16 kernel codes at most four distinct bytes per batch: Seq1 over {A, C}, Seq2 over
    {a, c}.)"""
    gg = (-3, -1, 1, -1, True)
    ac = lambda seed, n: sa.synth_dna(seed, n).translate(bytes.maketrans(b"GT", b"AC"))
    big = [(b"A" * 4096, b"a" * 4096),
           (ac(95_101, 4096), ac(95_102, 4096).lower()),
           (b"AC" * 2048, b"ac" * 2048)]
    rng = np.random.default_rng(43)
    pairs = [(ac(96_500 + k, int(rng.integers(20, 120))), ac(97_500 + k, int(rng.integers(20, 120))).lower())
             for k in range(1100)]
    pairs[7], pairs[600], pairs[1099] = big
    compare_with_oracle(engine, 3, gg, pairs, match="caseless")
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16
    pur = [(sa.synth_dna(95_200 + k, 4096), sa.synth_dna(95_300 + k, 4096)) for k in range(2)]
    pur.append((b"AG" * 2048, b"GA" * 2048))
    pairs = [(sa.synth_dna(98_000 + k, 60), sa.synth_dna(99_000 + k, 60)) for k in range(1100)]
    pairs[3], pairs[700], pairs[1098] = pur
    compare_with_oracle(engine, 3, gg, pairs, match="purine")
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16


def test_endcell_replay_vs_oracle(engine, monkeypatch):
    """>= 1024 DNA SW pairs take the T16 plan with per-chunk maxima and the end-cell replay
    (sa_endcell.hip): one pair per wave at R = 32 (max_m 4200 -> 3 bands).  Cases: all-zero matrices (end cell = last cell; a
    2500 x 2000 one takes the dense launch), periodic sequences (many
    tied maxima across rows and chunks), identical sequences, multi-band pairs."""
    rng = np.random.default_rng(5)
    pairs = []
    for k in range(1030):
        kind = k % 6
        if kind == 0:
            a, b = b"A" * (1 + k % 70), b"C" * (1 + k % 50)
        elif kind == 1:
            a, b = b"AC" * (5 + k % 40), b"CA" * (3 + k % 45)
        elif kind == 2:
            a = sa.synth_dna(k, 1 + k % 97)
            b = a
        else:
            a = sa.synth_dna(50_000 + k, int(rng.integers(1, 300)))
            b = sa.synth_mutate(a, k)[: int(rng.integers(1, 300))]
        pairs.append((a, b))
    pairs[7] = (sa.synth_dna(1, 4200), sa.synth_dna(2, 3100))
    pairs[11] = (sa.synth_dna(3, 2100), sa.synth_mutate(sa.synth_dna(3, 2100), 9))
    pairs[13] = (b"ACGT" * 1050, b"ACGT" * 700)
    # all-zero and 2 bands: every lane block is a candidate (> kSoCand), the dense end-cell launch
    pairs[17] = (b"A" * 2500, b"C" * 2000)
    for args in [(-1, 1, -1), (-3, 2, -2), (-1, 2, -1)]:
        compare_with_oracle(engine, 0, args, pairs)
        assert engine.last_plan()[:2] == (sa.SA_KERNEL_T16_ENDCELL, 32), args
    # LocalGotoh: the affine end-cell replay (M, Iy and the last row's Ix per lane; the band's top
    # M and Ix rows), R = 16 (max_m 4200 -> 5 bands); the SPLIT plan's R = 2, 4, 8 replays below
    for args in [(-3, -1, 1, -1, True), (-2, -1, 2, -1, True), (-1, -1, 3, -2, True)]:
        compare_with_oracle(engine, 2, args, pairs)
        assert engine.last_plan()[:2] == (sa.SA_KERNEL_T16_ENDCELL, 16), args
    few = [pairs[7], pairs[11], pairs[13], pairs[1], pairs[2], pairs[0]]
    compare_with_oracle(engine, 2, (-3, -1, 1, -1, True), few)
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16_ENDCELL


@pytest.mark.parametrize("match", ["purine", "nwild", "caseless"])
def test_custom_match_fn_vs_oracle(engine, match):
    pairs = []
    for k in range(12):
        a = sa.synth_dna(40_000 + k, 300 + 17 * k)
        b = bytearray(sa.synth_mutate(a, k))
        for p in range(k % 5, len(b), 9):
            b[p] = ord("N") if match == "nwild" else (ord(chr(b[p]).lower()) if match == "caseless" else b[p])
        pairs.append((a, bytes(b)))
    for algo in range(4):
        compare_with_oracle(engine, algo, SCORINGS[algo][0], pairs, match)


def test_local_gotoh_size_hack(engine):
    """SALocalGotoh.h:484-488: these sizes are re-aligned with NW (parity unpinned: the
    reference reads an uninitialised Gap there; we use the ScoringSystem's gap = 0)."""
    pairs = [(sa.synth_dna(1, 60), sa.synth_dna(2, 57)), (sa.synth_dna(3, 314), sa.synth_dna(4, 288)),
             (sa.synth_dna(5, 61), sa.synth_dna(6, 58)), (sa.synth_dna(7, 61), sa.synth_dna(8, 59))]
    res = engine.align(2, sa.ScoringSystem(-3, -1, 1, -1, True), pairs)
    assert [bool(r.flags & sa.SA_FLAG_SIZE_HACK) for r in res] == [True, True, True, False]
    for (a, b), r in zip(pairs, res):
        o = oracle_align(2, (-3, -1, 1, -1, True), a, b)
        assert rows_of(2, a, b, r) == o["rows"]


def rescore(algo, args, a, b, r):
    """Score of the emitted local alignment under the scoring (independent of the DP)."""
    s = sa.ScoringSystem(*args)
    tot = 0
    prev = None
    for op in reversed(r.ops):
        c = chr(op)
        if c in "MS":
            tot += s.match if c == "M" else s.mismatch
        elif algo in (0, 1):
            tot += s.gap
        else:
            tot += s.gap_extend + (s.gap_open if prev != c else 0)
        prev = c if c in "UL" else None
    return tot


@pytest.mark.parametrize("pairs_n,length", [(1024, 4096)])
def test_full_size_properties(engine, pairs_n, length):
    """North-star shape (4096 x 4096 SW), 1024 pairs in one launch: every local alignment
    re-scores to the reported maximum, ends where the scores says, and a sample is bit-exact
    against the oracle."""
    s1, o1, s2, o2 = sa.synth_dna_batch(9_000_000_000, pairs_n, length, length, threads=16)
    args = (-1, 1, -1)
    res, ops = engine.align_packed(0, sa.ScoringSystem(*args), s1, o1, s2, o2)
    assert (res["flags"] == 0).all()
    assert (res["score"] > 0).all()
    for p in range(pairs_n):
        off = int(o1[p] + o2[p]) + p
        r = sa.PairResult(int(res["score"][p]), int(res["end_i"][p]), int(res["end_j"][p]),
                          int(res["start_i"][p]), int(res["start_j"][p]), 0,
                          ops[off:off + int(res["nops"][p])].tobytes())
        assert rescore(0, args, None, None, r) == r.score
        # the path consumes exactly (end - start) symbols of each sequence
        di = sum(1 for c in r.ops if chr(c) in "MSUX")
        dj = sum(1 for c in r.ops if chr(c) in "MSLX")
        assert (r.end_i - r.start_i, r.end_j - r.start_j) == (di, dj)
    for p in (0, 1, pairs_n // 2, pairs_n - 1):
        a = s1[o1[p]:o1[p + 1]].tobytes()
        b = s2[o2[p]:o2[p + 1]].tobytes()
        o = oracle_align(0, args, a, b)
        off = int(o1[p] + o2[p]) + p
        assert (int(res["score"][p]), int(res["end_i"][p]), int(res["end_j"][p])) == \
               (o["score"], o["end_i"], o["end_j"])
        assert ops[off:off + int(res["nops"][p])].tobytes() == o["ops"]


def test_affine_rescore_property(engine):
    pairs = [(sa.synth_dna(500 + k, 2000), sa.synth_mutate(sa.synth_dna(500 + k, 2000), k)) for k in range(64)]
    for algo, args in ((2, (-3, -1, 1, -1, True)), (3, (-3, -1, 1, -1, True))):
        res = engine.align(algo, sa.ScoringSystem(*args), pairs)
        for (a, b), r in zip(pairs, res):
            if algo == 2 and b"u" not in r.ops and b"l" not in r.ops:
                assert rescore(algo, args, a, b, r) == r.score


def test_device_api_and_timings(engine):
    """sa_align_batch_device on torch-owned HBM buffers, on torch's current stream."""
    torch = pytest.importorskip("torch")
    s1, o1, s2, o2 = sa.synth_dna_batch(123, 64, 512, 512)
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    d1, do1, d2, do2 = t(s1), t(o1), t(s2), t(o2)
    d_res = torch.zeros(64 * 32, dtype=torch.uint8, device=dev)
    d_ops = torch.zeros(len(s1) + len(s2) + 64, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    engine.align_device(0, sa.ScoringSystem(-1, 1, -1), d1.data_ptr(), do1.data_ptr(), d2.data_ptr(),
                        do2.data_ptr(), 64, 512, 512, d_res.data_ptr(), d_ops.data_ptr(), stream)
    torch.cuda.synchronize()
    res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE)
    ref, _ = engine.align_packed(0, sa.ScoringSystem(-1, 1, -1), s1, o1, s2, o2)
    assert (res["score"] == ref["score"]).all() and (res["end_i"] == ref["end_i"]).all()
    fill_ms, tb_ms, n = engine.last_timings()
    assert n >= 1 and fill_ms > 0


@pytest.mark.parametrize("algo", ["hb", "mm"])
def test_dc_device_api_bounds(engine, algo):
    """sa_align_batch_device for the linear-space aligners: no host wait inside the call (grid
    bounds from max_m / max_n); two back-to-back calls on one stream equal the host API; a pair
    longer than max_m is flagged SA_FLAG_BAD_SHAPE and the others are unaffected."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    A = sa.SA_HIRSCHBERG if algo == "hb" else sa.SA_MYERS_MILLER
    sc = sa.ScoringSystem(*((-1, 2, -1) if algo == "hb" else (-3, -1, 1, -1, True)))
    stream = torch.cuda.current_stream().cuda_stream
    outs = []
    for seed, lens in ((5, (300, 40, 0, 257)), (6, (120, 512, 33, 7))):
        pairs = [(sa.synth_dna(seed * 100 + k, m), sa.synth_dna(seed * 100 + 50 + k, (m * 7) % 300 + 1))
                 for k, m in enumerate(lens)]
        s1 = np.frombuffer(b"".join(a for a, _ in pairs), dtype=np.uint8)
        s2 = np.frombuffer(b"".join(b for _, b in pairs), dtype=np.uint8)
        o1 = np.cumsum([0] + [len(a) for a, _ in pairs]).astype(np.uint64)
        o2 = np.cumsum([0] + [len(b) for _, b in pairs]).astype(np.uint64)
        d = [t(s1.copy()), t(o1), t(s2.copy()), t(o2)]
        d_res = torch.zeros(len(pairs) * 32, dtype=torch.uint8, device=dev)
        d_ops = torch.zeros(len(s1) + len(s2) + len(pairs), dtype=torch.uint8, device=dev)
        max_m = 300   # the second batch's 512-row pair passes it
        engine.align_device(A, sc, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), len(pairs),
                            max_m, 300, d_res.data_ptr(), d_ops.data_ptr(), stream)
        outs.append((pairs, o1, o2, d, d_res, d_ops))
    torch.cuda.synchronize()
    for pairs, o1, o2, d, d_res, d_ops in outs:
        res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=sa.RESULT_DTYPE)
        ops = d_ops.cpu().numpy()
        ref = engine.align(A, sc, pairs)
        for p, ((a, b), r) in enumerate(zip(pairs, ref)):
            if len(a) > 300:
                assert res["flags"][p] & sa.SA_FLAG_BAD_SHAPE
                continue
            off = int(o1[p] + o2[p]) + p
            got = (int(res["score"][p]), int(res["end_i"][p]), int(res["end_j"][p]),
                   ops[off:off + int(res["nops"][p])].tobytes())
            assert got == (r.score, r.end_i, r.end_j, r.ops), (algo, p)


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_pipelined_device_api_matches_serial(engine, algo):
    """sa_set_pipeline: consecutive device calls overlap (traceback of call k with the fill of
    call k+1, two workspace slots); every call's results equal the host API's once sa_wait
    returns.  Different batches per call, so a slot mix-up cannot go unnoticed."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
    args = SCORINGS[algo][0]
    sc = sc_obj(args)
    stream = torch.cuda.current_stream().cuda_stream
    calls = []
    for k in range(5):
        L = (256, 700, 300, 1024, 128)[k]
        s1, o1, s2, o2 = sa.synth_dna_batch(900 + 17 * k, 48 + 16 * k, L, L - 5 * k)
        d = [t(x) for x in (s1, o1, s2, o2)]
        n = len(o1) - 1
        res = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
        ops = torch.zeros(len(s1) + len(s2) + n, dtype=torch.uint8, device=dev)
        calls.append(((s1, o1, s2, o2), d, n, L, res, ops))
    engine.set_pipeline(True)
    try:
        for (h, d, n, L, res, ops) in calls:
            engine.align_device(algo, sc, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), n, L, L,
                                res.data_ptr(), ops.data_ptr(), stream)
        engine.wait()
    finally:
        engine.set_pipeline(False)
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


def test_multi_gpu_threads_match_single(engine):
    """align_multi_gpu (one host thread + context per device; here two contexts on GPU 0) returns
    exactly what one sa_align_batch returns."""
    from seqalib_amd.multi import align_multi_gpu
    pairs = [(sa.synth_dna(700 + k, 200 + 31 * k), sa.synth_dna(900 + k, 150 + 17 * k)) for k in range(40)]
    s1, o1, s2, o2 = sa.pack_pairs(pairs)
    ref, ref_ops = engine.align_packed(0, sa.ScoringSystem(-1, 1, -1), s1, o1, s2, o2)
    res, ops = align_multi_gpu(0, sa.ScoringSystem(-1, 1, -1), s1, o1, s2, o2, devices=[0, 0])
    assert (res == ref).all()
    for p in range(len(pairs)):
        off = int(o1[p] + o2[p]) + p
        n = int(ref["nops"][p])
        assert ops[off:off + n].tobytes() == ref_ops[off:off + n].tobytes()


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
@pytest.mark.parametrize("tb", ["wave", "lane", "seg"])
def test_traceback_flavours_vs_oracle(engine, algo, tb, monkeypatch):
    """The traceback kernels on both plans: one wave per pair (sa_traceback_wave.hip, default
    below 1024 pairs), one lane per pair (sa_traceback.hip, default for batches) and the
    band-parallel walk of SPLIT fills (sa_traceback_seg.hip, "seg": every pair), forced with
    SEQALIB_TB.  Long related pairs cross many decode windows (128 rows x 16 diagonals) and drift
    across diagonals through gaps; the many-pairs batch takes the one-wave-per-pair fill."""
    monkeypatch.setenv("SEQALIB_TB", tb)
    pairs = split_pairs(60 + algo)
    for args in SCORINGS[algo][:2]:
        compare_with_oracle(engine, algo, args, pairs)
    many = []
    for k in range(1030):
        a = sa.synth_dna(90_000 + 2 * k, 100 + k % 300)
        b = sa.synth_mutate(a, k)[: 90 + k % 250] if k % 2 else sa.synth_dna(90_001 + 2 * k, 80 + k % 200)
        many.append((a, b))
    compare_with_oracle(engine, algo, SCORINGS[algo][0], many, "purine" if algo == 3 else None)


@pytest.mark.parametrize("algo", [0, 1, 2, 3])
def test_segmented_traceback_vs_oracle(engine, algo, monkeypatch):
    """Band-parallel traceback of SPLIT fills (sa_traceback_seg.hip): per band, walkers from every
    cell of its last row (score from the fill's hand-off granules) record where they leave the
    band; the path is then chained from the end cell and each band's segment re-walked at its op
    offset.  Forced for every pair (SEQALIB_TB=seg) on every SPLIT R, T16 and int32 kernels,
    related pairs (long paths over many bands, gaps across band edges) and a custom match table;
    and the default (long walks only) on one long related pair per algorithm."""
    rng = np.random.default_rng(300 + algo)
    pairs = []
    for k in range(6):
        m = int(rng.integers(300, 2300))
        a = sa.synth_dna(40_000 + 2 * k, m)
        b = sa.synth_mutate(a, 7 + k) if k % 3 else sa.synth_dna(40_001 + 2 * k, int(rng.integers(200, 2400)))
        pairs.append((a, b))
    pairs.append((sa.synth_dna(41_000, 700), sa.synth_dna(41_001, 1)))
    pairs.append((sa.synth_dna(41_002, 1), sa.synth_dna(41_003, 900)))
    monkeypatch.setenv("SEQALIB_TB", "seg")
    for r in (1, 2, 4, 8):
        monkeypatch.setenv("SEQALIB_PLAN", f"{r},0")
        for args in SCORINGS[algo]:
            compare_with_oracle(engine, algo, args, pairs)
            assert engine.last_plan()[1:] == (r, 0), (r, args)
    monkeypatch.setenv("SEQALIB_PLAN", "2,0")
    compare_with_oracle(engine, algo, SCORINGS[algo][0], pairs, "purine")
    monkeypatch.delenv("SEQALIB_PLAN")
    monkeypatch.delenv("SEQALIB_TB")
    a = sa.synth_dna(42_000 + algo, 3000)
    long_pairs = [(a, sa.synth_mutate(a, 99)), (sa.synth_dna(42_100, 2900), sa.synth_dna(42_101, 3100))]
    for args in SCORINGS[algo][:2]:
        compare_with_oracle(engine, algo, args, long_pairs)


@pytest.mark.parametrize("algo", [0, 2])
def test_keyed_end_cell_vs_oracle(engine, algo, monkeypatch):
    """SEQALIB_CMAX=0: the local modes' T16 fills keep per-cell (score, column) keys instead of the
    chunk maxima + end-cell replay; same results as the oracle on a many-pairs batch."""
    pairs = dna_pairs(60 + algo, 1100, 300)
    monkeypatch.setenv("SEQALIB_CMAX", "0")
    compare_with_oracle(engine, algo, SCORINGS[algo][0], pairs[:200] + pairs[-30:])
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16
    big = [(sa.synth_dna(61_000 + k, 700), sa.synth_mutate(sa.synth_dna(61_000 + k, 700), k)) for k in range(1100)]
    res = engine.align(algo, sc_obj(SCORINGS[algo][0]), big)
    assert engine.last_plan()[0] == sa.SA_KERNEL_T16
    for k in (0, 1, 517, 1099):
        o = oracle_align(algo, SCORINGS[algo][0], *big[k])
        assert (res[k].score, res[k].end_i, res[k].end_j, res[k].ops) == (o["score"], o["end_i"], o["end_j"], o["ops"])


def test_kernel_timing_switch(engine, monkeypatch):
    """SEQALIB_KERNEL_TIMING: sa_last_kernel_timings reports the fill kernels alone (<= the fill
    stream span) for a call made with it, and fails for a call made without it."""
    pairs = dna_pairs(70, 1100, 400)
    monkeypatch.setenv("SEQALIB_KERNEL_TIMING", "1")
    engine.align(0, sc_obj((-1, 1, -1)), pairs)
    fk, fs = engine.last_kernel_timings()
    assert 0 < fk <= fs * 1.001 + 1e-3
    assert fs <= engine.last_timings()[0] * 1.001 + 1e-3
    monkeypatch.delenv("SEQALIB_KERNEL_TIMING")
    engine.align(0, sc_obj((-1, 1, -1)), pairs)
    with pytest.raises(sa.SeqalibError):
        engine.last_kernel_timings()
