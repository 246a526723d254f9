// sa_traceback.hip — buildResult of the four reference aligners, one lane per pair, reading the
// per-cell flags written by the fill kernel (sa_fill_impl.h) instead of a score matrix.
//
// Every move of the reference's traceback is an exact score equality, so the walk carries the
// score of its current cell: it starts from the end score the fill reported and steps back by
// the term that produced it (diag: the substitution score, up/left: the gap, Ix/Iy extend: GE,
// gap open: GO + GE).  With that value the zero tests and max(…, 0) clamps of the local modes
// are evaluated exactly as the reference does, and the stored flags only have to say which
// equality held at each cell.  Walks restated:
//   SW  SASmithWaterman.h:232-334   start at (MaxRow, MaxCol); stop when H == 0 or on an edge
//   NW  SANeedlemanWunsch.h:167-230 start at (m, n); diag > up > left; edges forced
//   LG  SALocalGotoh.h:285-470      3-state machine; stops on M == 0 / gap-open <= 0 / edge
//   GG  SAGlobalGotoh.h:245-421     3-state machine; j == 0 -> up, i == 0 -> left
// Ops are written in traceback order (include/seqalib_hip.h); forceGlobal is host work.
//
// Memory: a walk is a chain of dependent reads, one cell per move, and a 4k x 4k local path is
// ~5k moves long, so per-move HBM latency would dominate.  Each lane therefore keeps private LDS
// windows that one batch of independent loads refills:
//   flags: ~32 rows x 32 steps: lanes {t, t-1, ..} x step groups {G, G-1, ..} of its band
//          (16-byte packets, sa_layout.h) -- a walk only moves to smaller s = j-1+t and t;
//   Seq1 / Seq2: the 32 bytes below the current row / column.
// and refills are batched across the wave (see the round loop at the end of the kernel).
#include <limits.h>

#include "sa_internal.h"

namespace sa {

template <bool LUT>
__device__ __forceinline__ bool tb_match(const uint32_t* lut, uint8_t a, uint8_t b) {
    if constexpr (LUT) return (lut[(a << 3) | (b >> 5)] >> (b & 31)) & 1;
    else return a == b;
}

// Flag window ~32 rows x 32 steps whatever the geometry: max(1, 32/R) lanes x 32/SPP groups.
constexpr int kTbSeqWin = 32;                 // bytes per sequence window
constexpr int kTbMaxFlagBytes = 512;          // 128 * bits per cell
constexpr int kTbLaneWords = (kTbMaxFlagBytes + 2 * kTbSeqWin) / 4 + 1;   // odd: conflict-free LDS
static_assert(kTbLaneWords % 2 == 1, "per-lane LDS stride must be odd in words");

template <int ALG, int R, bool LUT>
__global__ __launch_bounds__(64) void traceback_kernel(TbParams P) {
    constexpr int BPC = bits_per_cell(ALG), BPS = R * BPC / 8, SPP = 16 / BPS;
    static_assert(BPS <= 16 && (SPP & (SPP - 1)) == 0, "one packet per step record");
    constexpr int kTbLanes = R >= 32 ? 1 : 32 / R;
    constexpr int kTbGroups = 32 / SPP;
    constexpr int kTbFlagBytes = kTbLanes * kTbGroups * 16;
    static_assert(kTbFlagBytes <= kTbMaxFlagBytes, "flag window");
    __shared__ uint32_t s_win[64 * kTbLaneWords];
    uint8_t* const win = reinterpret_cast<uint8_t*>(s_win + threadIdx.x * kTbLaneWords);
    uint8_t* const win1 = win + kTbFlagBytes;
    uint8_t* const win2 = win1 + kTbSeqWin;
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= P.count) return;
    const uint32_t pidx = P.pair_base + slot;
    sa_result res = P.res[pidx];
    if (res.flags & SA_FLAG_BAD_SHAPE) return;
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    const bool tagged = P.tagged != 0;
    const Geom g = make_geom(ALG, R, P.max_m, P.max_n, tagged);
    const uint8_t* dir = P.dirs + (uint64_t)slot * P.dir_slot;
    uint8_t* ops = P.ops + o1 + o2 + pidx;
    const bool allow = P.allow != 0;
    const int G = P.gap, MA = P.match, MI = P.mismatch, GE = P.gap_extend;
    const int GOE = P.gap_open + P.gap_extend;
    uint32_t k = 0;
    uint32_t flags = res.flags;

    // ---------------------------------------------------------------- windows
    const uint32_t band_rows = (uint32_t)kWave * R;
    int wb = -1, wt = 0, wg = 0;             // flag window: band, top lane, top step group
    int w1 = -kTbSeqWin, w2 = -kTbSeqWin;    // sequence windows cover [w, w + kTbSeqWin)
    int cb = 0, ct = 0, cgrp = 0, csub = 0, cr = 0;   // cell (i, j) decomposed by ready()
    auto locate = [&](int i, int j) {
        const uint32_t ii = (uint32_t)i - 1;
        cb = (int)(ii / band_rows);
        const uint32_t rem = ii - (uint32_t)cb * band_rows;
        ct = (int)(rem / R);
        cr = (int)(rem - (uint32_t)ct * R);
        const int s = j - 1 + ct;
        cgrp = s / SPP;               // s >= 0 whenever i, j > 0
        csub = s % SPP;
    };
    // true when everything a move at (i, j) may read is in the windows
    auto ready = [&](int i, int j) -> bool {
        if (!(i > 0 && j > 0)) return true;
        locate(i, j);
        return cb == wb && (unsigned)(wt - ct) < (unsigned)kTbLanes && (unsigned)(wg - cgrp) < (unsigned)kTbGroups &&
               (unsigned)(i - 1 - w1) < (unsigned)kTbSeqWin && (unsigned)(j - 1 - w2) < (unsigned)kTbSeqWin;
    };
    // one batch of independent loads re-anchors all three windows at (i, j)
    auto refill = [&](int i, int j) {
        if (!(i > 0 && j > 0)) return;       // edge moves read nothing (and (i-1) would wrap)
        locate(i, j);
        wb = cb; wt = ct; wg = cgrp;
        w1 = (i - kTbSeqWin) < 0 ? 0 : i - kTbSeqWin;
        w2 = (j - kTbSeqWin) < 0 ? 0 : j - kTbSeqWin;
        const uint8_t* base = dir + (uint64_t)cb * g.band_stride;
        // every load of the refill is issued before the first LDS store: one memory latency
        uint4 v[kTbLanes][kTbGroups];
#pragma unroll
        for (int dl = 0; dl < kTbLanes; ++dl)
#pragma unroll
            for (int dg = 0; dg < kTbGroups; ++dg) {
                const int lane = ct - dl, gg = cgrp - dg;
                v[dl][dg] = (lane >= 0 && gg >= 0)
                                ? *reinterpret_cast<const uint4*>(base + ((uint64_t)gg * kWave + lane) * 16)
                                : make_uint4(0, 0, 0, 0);
            }
        uint8_t b1[kTbSeqWin], b2[kTbSeqWin];
#pragma unroll
        for (int q = 0; q < kTbSeqWin; ++q) {
            b1[q] = (w1 + q < m) ? s1[w1 + q] : 0;
            b2[q] = (w2 + q < n) ? s2[w2 + q] : 0;
        }
#pragma unroll
        for (int dl = 0; dl < kTbLanes; ++dl)
#pragma unroll
            for (int dg = 0; dg < kTbGroups; ++dg) {
                uint32_t* w = reinterpret_cast<uint32_t*>(win + (dl * kTbGroups + dg) * 16);
                w[0] = v[dl][dg].x; w[1] = v[dl][dg].y; w[2] = v[dl][dg].z; w[3] = v[dl][dg].w;
            }
#pragma unroll
        for (int q = 0; q < kTbSeqWin; ++q) { win1[q] = b1[q]; win2[q] = b2[q]; }
    };
    // flags of the cell located by the last ready() (which returned true)
    auto cell = [&]() -> uint32_t {
        int word, lowbit;
        cell_word_bit(R, BPC, cr, &word, &lowbit, tagged);
        const int byte = ((wt - ct) * kTbGroups + (wg - cgrp)) * 16 + csub * BPS + word * 4 + lowbit / 8;
        return (uint32_t)(win[byte] >> (lowbit % 8));
    };
    // linear modes: flags fD (bit 1) / fU (bit 0); a T16 max tag (3 diag, 2 up, 1 left, 0 clamp)
    // says the same thing: diag wins iff H == D, else up iff H == U.
    auto lin = [&]() -> uint32_t {
        const uint32_t f = cell() & 3u;
        return tagged ? (f == 3u ? 2u : (f == 2u ? 1u : 0u)) : f;
    };
    // diagonal move: emits the op and returns the substitution term that was added
    auto diag = [&](int i, int j) -> int {
        const bool v = tb_match<LUT>(P.lutbits, win1[i - 1 - w1], win2[j - 1 - w2]);
        ops[k++] = v ? 'M' : (allow ? 'S' : 'X');
        return v ? MA : MI;
    };

    // ---------------------------------------------------------------- walk state
    int i, j, st = 0;
    int V = 0;          // SW: H; LG: M, Ix or Iy of the current cell, by state
    bool fin = false;
    if constexpr (ALG == SA_SW || ALG == SA_LOCAL_GOTOH) {
        i = res.end_i; j = res.end_j; V = res.score;
        if (ALG == SA_SW && (m == 0 || n == 0)) { i = 0; j = 0; }
    } else {
        i = m; j = n;
    }
    // One iteration of the reference's traceback loop (sets fin when it would leave the loop).
    auto move = [&]() {
        if constexpr (ALG == SA_SW) {
            if (!(i > 0 && j > 0) || V == 0) { fin = true; return; }   // H == 0: end of local path
            const uint32_t f = lin();
            if (f & 2u) { V -= diag(i, j); --i; --j; }
            else if (f & 1u) { ops[k++] = 'U'; V -= G; --i; }
            else { ops[k++] = 'L'; V -= G; --j; }
        } else if constexpr (ALG == SA_NW) {
            if (!(i > 0 || j > 0)) { fin = true; return; }
            if (i > 0 && j > 0) {
                const uint32_t f = lin();
                if (f & 2u) { diag(i, j); --i; --j; }
                else if (f & 1u) { ops[k++] = 'U'; --i; }
                else { ops[k++] = 'L'; --j; }
            } else if (i > 0) {
                ops[k++] = 'U'; --i;   // H[i][0] == H[i-1][0] + Gap always holds
            } else {
                ops[k++] = 'L'; --j;
            }
        } else if constexpr (ALG == SA_LOCAL_GOTOH) {
            // flags: bit3 = fD (M == diag), bit2 = fX (M == Ix), bit1 = Ix extends, bit0 = Iy extends
            if (!(i > 0 && j > 0)) { fin = true; return; }
            const uint32_t f = cell();
            if (st == 0) {
                if (V <= 0) { fin = true; return; }    // M == max(D, 0) <= 0
                if (f & 8u) { V -= diag(i, j); --i; --j; }
                else st = (f & 4u) ? 1 : 2;              // M == Ix, else M == Iy (same value)
            } else if (st == 1) {
                if (f & 2u) { ops[k++] = 'U'; V -= GE; --i; }
                else if (V > 0) { ops[k++] = 'U'; V -= GOE; --i; st = 0; }
                else if (V == 0) { ops[k++] = 'u'; fin = true; }
                else { flags |= SA_FLAG_DIVERGED; fin = true; }
            } else {
                if (f & 1u) { ops[k++] = 'L'; V -= GE; --j; }
                else if (V > 0) { ops[k++] = 'L'; V -= GOE; --j; st = 0; }
                else if (V == 0) { ops[k++] = 'l'; fin = true; }
                else { flags |= SA_FLAG_DIVERGED; fin = true; }
            }
        } else {  // SA_GLOBAL_GOTOH
            if (!(i > 0 || j > 0)) { fin = true; return; }
            if (j == 0) { ops[k++] = 'U'; --i; return; }   // edge rules hold in any state
            if (i == 0) { ops[k++] = 'L'; --j; return; }
            const uint32_t f = cell();
            if (st == 0) {
                if (f & 8u) { diag(i, j); --i; --j; }
                else st = (f & 4u) ? 1 : 2;
            } else if (st == 1) {
                ops[k++] = 'U'; --i;
                if (!(f & 2u)) st = 0;   // gap open: Ix == M[i-1][j] + GO + GE
            } else {
                ops[k++] = 'L'; --j;
                if (!(f & 1u)) st = 0;
            }
        }
    };

    // The 64 lanes of the wave walk 64 different pairs.  A lane whose next move would leave its
    // windows parks; once every unfinished lane is parked they all refill together, so the wave
    // pays one memory latency per round of ~kTbGroups*spp moves instead of one per move.
    bool parked = true;
    for (;;) {
        if (__builtin_amdgcn_ballot_w64(!fin && !parked) == 0) {
            if (__builtin_amdgcn_ballot_w64(!fin) == 0) break;
            if (!fin) { refill(i, j); parked = false; }
        }
        if (!fin && !parked) {
            if (ready(i, j)) move();
            else parked = true;
        }
    }
    res.start_i = i;
    res.start_j = j;
    res.nops = k;
    res.flags = flags;
    P.res[pidx] = res;
}

hipError_t launch_traceback(int algo, int R, bool lut, const TbParams& p, hipStream_t stream) {
    const dim3 block(64);
    const dim3 grid((p.count + 63) / 64);
#define SA_TB(AA, RR, LL)                                                                  \
    if (algo == AA && R == RR && lut == LL) {                                              \
        hipLaunchKernelGGL((traceback_kernel<AA, RR, LL>), grid, block, 0, stream, p);     \
        return hipGetLastError();                                                          \
    }
#define SA_TB_A(AA) SA_TB(AA, 4, false) SA_TB(AA, 8, false) SA_TB(AA, 16, false) \
                    SA_TB(AA, 4, true) SA_TB(AA, 8, true) SA_TB(AA, 16, true)
    SA_TB_A(SA_SW)
    SA_TB_A(SA_NW)
    SA_TB(SA_SW, 32, false) SA_TB(SA_SW, 32, true) SA_TB(SA_NW, 32, false) SA_TB(SA_NW, 32, true)
    SA_TB(SA_SW, 64, false) SA_TB(SA_SW, 64, true) SA_TB(SA_NW, 64, false) SA_TB(SA_NW, 64, true)
    SA_TB_A(SA_LOCAL_GOTOH)
    SA_TB_A(SA_GLOBAL_GOTOH)
#undef SA_TB_A
#undef SA_TB
    return hipErrorInvalidValue;
}

hipError_t launch_fill(int algo, const FillVariant& v, const FillParams& p, uint32_t grid,
                       hipStream_t stream) {
    switch (algo) {
        case SA_SW: return launch_fill_sw(v, p, grid, stream);
        case SA_NW: return launch_fill_nw(v, p, grid, stream);
        case SA_LOCAL_GOTOH: return launch_fill_lg(v, p, grid, stream);
        case SA_GLOBAL_GOTOH: return launch_fill_gg(v, p, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace sa
