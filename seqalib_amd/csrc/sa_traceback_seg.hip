// sa_traceback_seg.hip — buildResult of the four reference aligners for FEW LONG pairs of a SPLIT
// fill (BASELINE configs 2 and 4), as a band-parallel walk instead of one serial walk.
//
// A traceback is a chain of dependent moves: ~4.7k for one 4096^2 local DNA pair, which the
// one-wave walker (sa_traceback_wave.hip) takes at ~0.2 us each.  But the walk is a pure
// function of (cell, state, carried score), and the SPLIT fill leaves every band's last row of
// scores in its hand-off granules (H, and Ix for Gotoh: sa_fill_impl.h).  So the walk can be cut
// at the band boundaries (rows b * 64R) and every segment computed independently:
//   1. EXIT MAP (seg_exit_kernel): for every band b below the end cell's band and every column c
//      and state st (M / Ix) of b's last row, a walker starts at that cell with the score the
//      fill left there and walks up to the first cell of band b - 1 (or to the walk's end).  It
//      records where it left (column, state), how many ops it emitted and, if it stopped, where.
//      One thread per walker, the band's records and symbols staged in LDS; the end cell's own
//      segment is one more walker.  ~B * n walkers, all in parallel.
//   2. EMIT (seg_emit_kernel): per band, one thread follows the exit maps from the end cell down
//      to its band (the op offset is the sum of the segment lengths above it) and, if the path
//      crosses the band, re-walks its segment writing the ops at that offset; the band where the
//      walk stops records (start_i, start_j, nops, flags) for the pair.
//   3. the wave walker kernel applies that record to sa_result (and walks the pairs not taken).
// Every segment is the reference's loop restated exactly as in sa_traceback_wave.hip:
//   SW  SASmithWaterman.h:232-334   NW  SANeedlemanWunsch.h:167-230
//   LG  SALocalGotoh.h:285-470      GG  SAGlobalGotoh.h:245-421
// A correct walk carries the exact score of its current cell (every move is an equality), so the
// segment that starts from the granule's score is the same walk.  Walkers off the path compute
// garbage that nobody reads; every move lowers i or j, so each stops.
// Crossing states: a row is crossed by a diagonal move (lands in M), or by an Ix move (extend:
// lands in Ix, open: in M); Iy moves stay on their row, except GlobalGotoh's edge rule at j == 0,
// where every state moves up alike (looked up as M).
#include <limits.h>

#include "sa_internal.h"

namespace sa {

constexpr int kSegTW = 256;                  // bottom-row columns per exit-map workgroup
constexpr uint32_t kSegStageBytes = 48 * 1024;  // LDS budget for a band's records
constexpr int kSegS2 = 1024;                 // Seq2 window bytes
// exit record / result flag bits (exit state at bits 2-3); kSegErr: a guard caught an inconsistent
// walk (never expected: the wave kernel then reports the pair with start (-1, -1))
constexpr uint32_t kSegStop = 1u, kSegDiv = 2u, kSegErr = 16u;

typedef uint8_t __attribute__((address_space(3))) sg_u8;

// Per-walker view of one band of one pair: records and symbols staged in LDS where they fall in
// the window, global memory otherwise.
struct SegBand {
    const uint8_t* dir;      // pair slot
    const uint8_t* s1;
    const uint8_t* s2;
    uint64_t stage_base;     // slot offset of the first staged record byte
    uint32_t stage_bytes;
    uint32_t pk_lo;          // first staged packet group of the band
    int s1_lo, s1_cnt;       // staged Seq1 [s1_lo, s1_lo + s1_cnt)
    int s2_lo, s2_cnt;       // staged Seq2 [s2_lo, s2_lo + s2_cnt)
    int m, n;
    uint32_t cap;            // EMIT: op bytes the walk may write
    const sg_u8* l_rec;
    const sg_u8* l_s1;
    const sg_u8* l_s2;
    const uint32_t* l_lut;   // LDS copy of the match bits (LUT)
};

// Stage the records of band b for steps [s_hi - (budget), s_hi], Seq1 rows of the band and the
// Seq2 window ending at column jmax (1-based), cooperatively by the workgroup.
template <int ALG, int R, bool LUT>
__device__ SegBand seg_stage(const TbParams& P, const Geom& g, const uint8_t* dir, const uint8_t* s1,
                             const uint8_t* s2, int m, int n, int b, int jmax, uint8_t* lds) {
    SegBand S;
    const int bps = g.bps, spp = g.spp, pps = g.pps;
    const uint32_t pk_bytes = (uint32_t)pps * kWave * 16;   // one packet group (spp steps)
    const uint32_t max_pk = kSegStageBytes / pk_bytes;
    const uint32_t total_pk = g.steps_pad / spp;
    const uint32_t pk_hi = min(total_pk, (uint32_t)(jmax + kWave - 1) / spp + 1);   // exclusive
    const uint32_t pk_lo = pk_hi > max_pk ? pk_hi - max_pk : 0u;
    (void)bps;
    S.dir = dir; S.s1 = s1; S.s2 = s2;
    S.m = m; S.n = n;
    S.cap = 0;
    S.stage_base = (uint64_t)b * g.band_stride + (uint64_t)pk_lo * pk_bytes;
    S.pk_lo = pk_lo;
    S.stage_bytes = (pk_hi - pk_lo) * pk_bytes;
    const int BR = kWave * R;
    S.s1_lo = b * BR;
    S.s1_cnt = max(0, min(BR, m - S.s1_lo));
    const int s2_hi = min(jmax, n);                 // Seq2 indices [.., s2_hi)
    S.s2_lo = max(0, s2_hi - kSegS2);
    S.s2_cnt = max(0, s2_hi - S.s2_lo);
    uint8_t* l_rec = lds;
    uint8_t* l_s1 = lds + kSegStageBytes;
    uint8_t* l_s2 = l_s1 + kWave * 8;
    uint32_t* l_lut = reinterpret_cast<uint32_t*>(l_s2 + kSegS2);
    const int nt = blockDim.x, t = threadIdx.x;
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const u4* src = reinterpret_cast<const u4*>(dir + S.stage_base);
    u4* dst = reinterpret_cast<u4*>(l_rec);
    for (uint32_t q = t; q < S.stage_bytes / 16; q += nt) dst[q] = src[q];
    for (int q = t; q < S.s1_cnt; q += nt) l_s1[q] = s1[S.s1_lo + q];
    for (int q = t; q < S.s2_cnt; q += nt) l_s2[q] = s2[S.s2_lo + q];
    if constexpr (LUT) {
        for (int q = t; q < 2048; q += nt) l_lut[q] = P.lutbits[q];
    }
    S.l_rec = (const sg_u8*)l_rec;
    S.l_s1 = (const sg_u8*)l_s1;
    S.l_s2 = (const sg_u8*)l_s2;
    S.l_lut = l_lut;
    return S;
}

// Off-window reads, out of line so that the walk loop keeps its few registers and branches.
__device__ __attribute__((noinline)) uint32_t seg_slow_rec(const Geom& g, const uint8_t* dir, int ci, int cj) {
    int sh;
    return dir[cell_byte(g, (uint32_t)ci, (uint32_t)cj, &sh)];
}
__device__ __attribute__((noinline)) uint32_t seg_slow_byte(const uint8_t* p) { return *p; }

// One segment of the walk: from (i, j) in state st with score V, until the walk stops or reaches
// row itop (> 0: the last row of band b - 1).  EMIT writes the op bytes at ops[k...].
// Returns true if the walk stopped (fin) inside the band.
template <int ALG, int R, bool LUT, bool TAG, bool EMIT>
__device__ bool seg_walk(const TbParams& P, const Geom& g, const SegBand& S, int itop, int& i, int& j, int& st,
                         int& V, uint32_t& k, uint32_t& fl, uint8_t* ops) {
    constexpr int BPC = bits_per_cell(ALG);
    constexpr uint32_t FMASK = (1u << BPC) - 1u;
    const bool vrec = P.vrec != 0, allow = P.allow != 0;
    const int G = P.gap, MA = P.match, MI = P.mismatch, GE = P.gap_extend;
    const int GOE = P.gap_open + P.gap_extend;
    const uint32_t obase = allow ? 'S' : 'X';
    auto emit = [&](uint32_t op) {
        if constexpr (EMIT) {
            if (k < S.cap) ops[k] = (uint8_t)op;
            else fl |= kSegErr;
        }
        ++k;
    };
    // flags of cell (i, j) in the int32 layout (fD/fU, or fD/fX/fXe/fYe) and its match bit.  The
    // record geometry is compile-time (R, TAG), so the staged offset is a few 32-bit shifts and
    // adds (sa_layout.h cell_byte restated); cells outside the staged window read HBM.
    constexpr int RBPC = record_bpc(ALG, R, TAG);
    constexpr int BPS = R * RBPC / 8, SPP = 16 / BPS;
    static_assert(BPS >= 1 && BPS <= 16 && 16 % BPS == 0, "SPLIT records: one packet per step group");
    constexpr int RPW = (R * RBPC < 32 ? R * RBPC : 32) / RBPC;   // rows per record word
    const uint32_t ib0 = (uint32_t)(itop);   // first row of the band, 0-based = b * BR
    auto cell = [&](int ci, int cj, uint32_t& mt) -> uint32_t {
        const uint32_t ii = (uint32_t)ci - 1u - ib0;
        const uint32_t t = ii / R, r = ii % R;
        const uint32_t sst = (uint32_t)cj - 1u + t;
        const uint32_t word = r / RPW, rr = r % RPW;
        const uint32_t lowbit = TAG ? RBPC * rr : (uint32_t)((R * RBPC < 32 ? R * RBPC : 32) - RBPC * (rr + 1));
        const uint32_t bir = word * 4 + lowbit / 8;
        const uint32_t rel = (sst / SPP - S.pk_lo) * 1024u + t * 16u + (sst % SPP) * BPS + bir;
        // The three LDS reads (record byte, Seq1 and Seq2 symbols) are issued together and
        // unconditionally (clamped indices); HBM is read only off the staged window (rare).
        // Seq1: the band's rows are all staged; Seq2: a window.
        const uint32_t x2 = (uint32_t)(cj - 1 - S.s2_lo);
        const uint32_t a = S.l_s1[ii];
        uint32_t bb = S.l_s2[min(x2, (uint32_t)S.s2_cnt - 1u)];
        uint32_t raw = S.l_rec[min(rel, S.stage_bytes - 1u)];
        if (rel >= S.stage_bytes) raw = seg_slow_rec(g, S.dir, ci, cj);
        if (!vrec && x2 >= (uint32_t)S.s2_cnt) bb = seg_slow_byte(S.s2 + (cj - 1));
        raw >>= (lowbit % 8);
        uint32_t f = raw & FMASK;
        if (BPC == 2 && TAG) f = (f == 3u) ? 2u : (uint32_t)(f == 2u);
        if (BPC == 4 && TAG) f = t16a_flags(raw & 0xffu);
        uint32_t me;
        if constexpr (LUT) me = (S.l_lut[(a << 3) | (bb >> 5)] >> (bb & 31)) & 1u;
        else me = (uint32_t)(a == bb);
        mt = vrec ? (BPC == 2 ? ((f >> 1) & f & 1u) : ((f >> 3) & (f >> 2) & 1u)) : me;
        return f;
    };
    // Branch-light move selection: every iteration computes (op, di, dj, dv, next state) and
    // applies them once; the loop leaves only at its top (band exit) or through `stop`.
    bool stop = false;
    for (;;) {
        if (i == itop && itop > 0) break;   // entered band b - 1
        if ((uint32_t)i > (uint32_t)S.m || (uint32_t)j > (uint32_t)S.n) { fl |= kSegErr; stop = true; break; }
        const bool inner = i > 0 && j > 0;
        uint32_t op = 0, f = 0, v = 0;
        int di = 0, dj = 0, dv = 0, nst = st;
        bool fin = false;
        if constexpr (ALG == SA_SW || ALG == SA_NW) {
            if (ALG == SA_SW ? (!inner || V == 0) : !(i > 0 || j > 0)) {
                fin = true;
            } else {
                f = 1u;   // NW edges: j == 0 -> up, i == 0 -> left
                if (inner) f = cell(i, j, v);
                else if (i == 0) f = 0u;
                const bool dg = (f & 2u) != 0, up = !dg && (f & 1u);
                op = dg ? (v ? 'M' : obase) : (up ? 'U' : 'L');
                dv = dg ? (v ? MA : MI) : G;
                di = (dg || up) ? 1 : 0;
                dj = up ? 0 : 1;
            }
        } else if constexpr (ALG == SA_LOCAL_GOTOH) {
            if (!inner) {
                fin = true;
            } else {
                f = cell(i, j, v);
                if (st == 0) {
                    if (V <= 0) fin = true;                       // M == max(D, 0) <= 0
                    else if (f & 8u) { op = v ? 'M' : obase; dv = v ? MA : MI; di = 1; dj = 1; }
                    else nst = (f & 4u) ? 1 : 2;                  // M == Ix, else M == Iy (same value)
                } else {
                    const bool ext = (st == 1 ? (f & 2u) : (f & 1u)) != 0;
                    if (ext) { dv = GE; }
                    else if (V > 0) { dv = GOE; nst = 0; }
                    else if (V == 0) { fin = true; }
                    else { fl |= kSegDiv; fin = true; }
                    if (ext || V >= 0) {
                        op = st == 1 ? (ext || V > 0 ? 'U' : 'u') : (ext || V > 0 ? 'L' : 'l');
                        if (ext || V > 0) { di = st == 1 ? 1 : 0; dj = st == 1 ? 0 : 1; }
                    }
                }
            }
        } else {  // SA_GLOBAL_GOTOH
            if (!(i > 0 || j > 0)) {
                fin = true;
            } else if (j == 0) {
                op = 'U'; di = 1;                              // edge rules hold in any state
            } else if (i == 0) {
                op = 'L'; dj = 1;
            } else {
                f = cell(i, j, v);
                if (st == 0) {
                    if (f & 8u) { op = v ? 'M' : obase; di = 1; dj = 1; }
                    else nst = (f & 4u) ? 1 : 2;
                } else if (st == 1) {
                    op = 'U'; di = 1;
                    if (!(f & 2u)) nst = 0;   // gap open: Ix == M[i-1][j] + GO + GE
                } else {
                    op = 'L'; dj = 1;
                    if (!(f & 1u)) nst = 0;
                }
            }
        }
        if (op) emit(op);
        if (fin) { stop = true; break; }
        i -= di;
        j -= dj;
        V -= dv;
        st = nst;
    }
    return stop;
}

// hand-off granule of band b (its last row), column j (1-based) -> the walk's score there, read
// as the fill's poller reads it (sc1).  The fill wrote every granule of columns 1..n with tag 1,
// so a zero tag means the scratch was overwritten: kSegErr (the pair is then walked serially and
// flagged SA_FLAG_RECOVERED).  (This guard found the pipeline slots' scratch overlap fixed in
// run_device, sa_api.hip: ~1 in 10 two-process runs of tests/test_gpu_multiproc.py.)
__device__ __forceinline__ int seg_hand(const TbParams& P, uint32_t slot, int b, int j, bool ix, uint32_t& fl) {
    if (j < 1) return 0;
    const uint64_t g = ((uint64_t)slot * P.split_bands + b) * P.max_n + (uint64_t)(j - 1) + (ix ? P.hand_x_off : 0);
    typedef const unsigned long long __attribute__((address_space(1))) cgu64;
    const unsigned long long x = __hip_atomic_load((cgu64*)(P.hand + g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((x >> 32) == 0) fl |= kSegErr;
    const int32_t v = (int32_t)(uint32_t)x;
    return P.hand_shift ? ((int)(int16_t)(v & 0xffff) >> P.hand_shift) : v;
}

template <int ALG, int R, bool LUT, bool TAG>
__global__ __launch_bounds__(512) void seg_exit_kernel(TbParams P) {
    constexpr int NST = is_affine(ALG) ? 2 : 1;
    __shared__ __attribute__((aligned(16))) uint8_t s_lds[kSegStageBytes + kWave * 8 + kSegS2 + (LUT ? 8192 : 0)];
    const uint32_t slot = blockIdx.z;
    const int b = blockIdx.y;
    const uint32_t tile = blockIdx.x;
    if (slot >= P.count) return;
    const uint32_t pidx = P.pair_base + slot;
    const sa_result res = P.res[pidx];
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    int b_e = 0;
    if (!seg_take<ALG, R>(P, res, m, n, &b_e)) return;
    if (b > b_e) return;
    const uint32_t ntile = (uint32_t)(n + 1 + kSegTW - 1) / kSegTW;
    const bool endw = (tile == ntile);   // the end cell's own segment
    if (endw != (b == b_e)) return;
    if (tile > ntile) return;
    const Geom g = make_geom(ALG, R, P.max_m, P.max_n, TAG ? 1 : 0);
    const int BR = kWave * R;
    const uint8_t* dir = P.dirs + (uint64_t)slot * P.dir_slot;
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    constexpr bool SCORED = (ALG == SA_SW || ALG == SA_LOCAL_GOTOH);
    const int c0 = (int)tile * kSegTW;
    const int jmax = endw ? (SCORED ? res.end_j : n) : min(n, c0 + kSegTW - 1);
    // This thread's walker and its record, fixed before the staging loops (the record address is
    // kept as one 64-bit pointer computed up front).
    const int t = threadIdx.x;
    const uint64_t rs = (uint64_t)NST * ((uint64_t)P.max_n + 1) + 1;   // records per band
    int4* const band_rec = P.seg_rec + ((uint64_t)slot * P.split_bands + (uint64_t)b) * rs;
    int i = 0, j = 0, st = 0, V = 0;
    uint32_t fl = 0;
    int4* out = nullptr;
    if (endw) {
        if (t == 0) {
            if (SCORED) { i = res.end_i; j = res.end_j; V = res.score; }
            else { i = m; j = n; }
            out = band_rec + (rs - 1);
        }
    } else {
        const int c = c0 + t % kSegTW;
        const int s0 = t / kSegTW;
        if (s0 < NST && c <= n) {
            st = s0;
            i = (b + 1) * BR;   // the band's last row (< m: b < b_e)
            j = c;
            if (SCORED) V = seg_hand(P, slot, b, c, st == 1, fl);
            out = band_rec + ((uint64_t)s0 * ((uint64_t)P.max_n + 1) + (uint64_t)c);
        }
    }
    const SegBand S = seg_stage<ALG, R, LUT>(P, g, dir, s1, s2, m, n, b, jmax, s_lds);
    __syncthreads();
    if (out == nullptr) return;
    uint32_t k = 0;
    const bool stop = seg_walk<ALG, R, LUT, TAG, false>(P, g, S, b * BR, i, j, st, V, k, fl, nullptr);
    int4 r;
    r.x = i; r.y = j; r.z = (int)k;
    r.w = (int)((stop ? kSegStop : 0u) | fl | ((uint32_t)st << 2));
    *out = r;
}

template <int ALG, int R, bool LUT, bool TAG>
__global__ __launch_bounds__(256) void seg_emit_kernel(TbParams P) {
    constexpr int NST = is_affine(ALG) ? 2 : 1;
    __shared__ __attribute__((aligned(16))) uint8_t s_lds[kSegStageBytes + kWave * 8 + kSegS2 + (LUT ? 8192 : 0)];
    __shared__ int s_entry[4];   // {j, st, offset, on path}
    const uint32_t slot = blockIdx.z;
    const int b = blockIdx.y;
    if (slot >= P.count) return;
    const uint32_t pidx = P.pair_base + slot;
    const sa_result res = P.res[pidx];
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    int b_e = 0;
    if (!seg_take<ALG, R>(P, res, m, n, &b_e)) return;
    if (b > b_e) return;
    const uint64_t rs = (uint64_t)NST * (P.max_n + 1) + 1;
    const int4* rec = P.seg_rec + (uint64_t)slot * P.split_bands * rs;
    constexpr bool SCORED = (ALG == SA_SW || ALG == SA_LOCAL_GOTOH);
    if (threadIdx.x == 0) {
        // follow the exit maps from the end cell's band down to this band
        int cb = b_e, cj = 0, cst = 0;
        uint64_t idx = rs - 1;
        uint32_t off = 0;
        bool on = true;
        while (cb > b) {
            const int4 r = rec[(uint64_t)cb * rs + idx];
            if (r.w & (kSegStop | kSegErr)) { on = false; break; }   // (kSegErr: no band records the end)
            off += (uint32_t)r.z;
            cj = r.y;
            cst = (r.w >> 2) & 3;
            if (cj == 0 || cst == 2) cst = 0;   // GlobalGotoh edge column: every state moves up alike
            if (cj < 0 || cj > n || cst >= NST || r.z < 0 || off > (uint32_t)(m + n + 1)) { on = false; break; }
            idx = (uint64_t)cst * (P.max_n + 1) + (uint64_t)cj;
            --cb;
        }
        s_entry[0] = cj; s_entry[1] = cst; s_entry[2] = (int)off; s_entry[3] = on ? 1 : 0;
    }
    __syncthreads();
    if (!s_entry[3]) return;
    const Geom g = make_geom(ALG, R, P.max_m, P.max_n, TAG ? 1 : 0);
    const int BR = kWave * R;
    const uint8_t* dir = P.dirs + (uint64_t)slot * P.dir_slot;
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    int i, j, st = s_entry[1], V = 0;
    uint32_t fl = 0;
    if (b == b_e) {
        st = 0;
        if (SCORED) { i = res.end_i; j = res.end_j; V = res.score; }
        else { i = m; j = n; }
    } else {
        i = (b + 1) * BR;
        j = s_entry[0];
        if (SCORED) V = seg_hand(P, slot, b, j, st == 1, fl);
    }
    const SegBand S = seg_stage<ALG, R, LUT>(P, g, dir, s1, s2, m, n, b, max(j, 1), s_lds);
    __syncthreads();
    if (threadIdx.x != 0) return;
    const uint32_t off = (uint32_t)s_entry[2];
    uint8_t* ops = P.ops + o1 + o2 + pidx + off;
    uint32_t k = 0;
    SegBand Sc = S;
    Sc.cap = (uint32_t)(m + n + 1) - min(off, (uint32_t)(m + n + 1));
    const bool stop = seg_walk<ALG, R, LUT, TAG, true>(P, g, Sc, b * BR, i, j, st, V, k, fl, ops);
    if (stop) {
        // the walk ends in this band: the pair's traceback result (applied by the wave kernel)
        int4 f;
        f.x = i; f.y = j; f.z = (int)(off + k); f.w = (int)fl;
        P.seg_fin[slot] = f;
    }
}

hipError_t launch_traceback_seg(int algo, int R, bool lut, const TbParams& p, hipStream_t stream, bool inject) {
    const int nst = is_affine(algo) ? 2 : 1;
    const uint32_t ntile = (p.max_n + 1 + kSegTW - 1) / kSegTW;
    const dim3 gx(ntile + 1, p.split_bands, p.count), bx(kSegTW * nst);
    const dim3 ge(1, p.split_bands, p.count), be(256);
    const uint64_t rs = (uint64_t)nst * ((uint64_t)p.max_n + 1) + 1;   // exit records per band
    const bool tag = p.tagged != 0;
#define SA_SEG(AA, RR, LL, TT)                                                              \
    if (algo == AA && R == RR && lut == LL && tag == TT) {                                  \
        hipLaunchKernelGGL((seg_exit_kernel<AA, RR, LL, TT>), gx, bx, 0, stream, p);        \
        hipError_t e = hipGetLastError();                                                   \
        if (e != hipSuccess) return e;                                                      \
        if (inject) {                                                                       \
            e = hipMemsetAsync(p.seg_rec, 0x40, (uint64_t)p.count * p.split_bands * rs * 16, stream); \
            if (e != hipSuccess) return e;                                                  \
        }                                                                                   \
        hipLaunchKernelGGL((seg_emit_kernel<AA, RR, LL, TT>), ge, be, 0, stream, p);        \
        return hipGetLastError();                                                           \
    }
#define SA_SEG_R(AA, LL, TT) SA_SEG(AA, 1, LL, TT) SA_SEG(AA, 2, LL, TT) SA_SEG(AA, 4, LL, TT) SA_SEG(AA, 8, LL, TT)
#define SA_SEG_A(AA) SA_SEG_R(AA, false, false) SA_SEG_R(AA, true, false) SA_SEG_R(AA, false, true) SA_SEG_R(AA, true, true)
    SA_SEG_A(SA_SW)
    SA_SEG_A(SA_NW)
    SA_SEG_A(SA_LOCAL_GOTOH)
    SA_SEG_A(SA_GLOBAL_GOTOH)
#undef SA_SEG_A
#undef SA_SEG_R
#undef SA_SEG
    return hipErrorInvalidValue;
}

}  // namespace sa
