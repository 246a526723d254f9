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

// Flag window ~32 rows x 32 steps whatever the geometry: max(1, 32/R) lanes x 32/SPP groups
// (<= 32 packets).  The windows live in LDS item-major ([item][lane]) because the refill is LDS DMA
// (global_load_lds: lane i's bytes land at base + i * size), which needs no staging registers:
//   flag packet q (16 B):           q * 1024 + lane * 16
//   sequence dword d (4 B, s1/s2):  kTbSeqOff{1,2} + d * 256 + lane * 4
// A sequence window is the 9 aligned dwords covering the 32 bytes below the current position;
// only dwords overlapping the pair's sequence are loaded (an aligned dword never crosses a page,
// so none of them can fault).
constexpr int kTbChunks = 32;
constexpr int kTbSeqWin = 32;
constexpr int kTbSeqItems = kTbSeqWin / 4 + 1;
constexpr int kTbSeqOff1 = kTbChunks * 1024;
constexpr int kTbSeqOff2 = kTbSeqOff1 + kTbSeqItems * 256;
// Ops are staged in LDS (64 per lane per round) and written to HBM once per round: a global
// store per move would put its latency on every iteration, because on gfx9 vmcnt counts stores
// too and the window reads must wait for vmcnt (the refill DMA).
constexpr int kTbOpsBuf = 64;
constexpr int kTbOpsOff = kTbSeqOff2 + kTbSeqItems * 256;
constexpr int kTbLdsBytes = kTbOpsOff + kTbOpsBuf * 64;

typedef const void __attribute__((address_space(1)))* tb_gptr;
typedef void __attribute__((address_space(3)))* tb_lptr;
// LDS / global byte pointers with explicit address spaces: a plain volatile pointer would be
// generic, i.e. flat loads and stores (vector-memory latency and vmcnt waits).
typedef volatile uint8_t __attribute__((address_space(3))) tb_lds_u8;
typedef uint8_t __attribute__((address_space(1))) tb_glb_u8;

#ifdef SA_TB_STATS
// Debug build only (-DSA_TB_STATS): [rounds, loop iterations, moves, wave cycles, refill cycles]
__device__ unsigned long long g_tb_stats[8];
#endif

// TAG: tagged affine records (T16 Gotoh fills, one byte per cell; sa_layout.h t16a_flags).
template <int ALG, int R, bool LUT, bool TAG = false>
__global__ __launch_bounds__(64) void traceback_kernel(TbParams P) {   // tb_mine: sa_internal.h
    constexpr int BPC = record_bpc(ALG, R, TAG), BPS = R * BPC / 8, SPP = 16 / BPS;
    static_assert(BPS >= 1 && BPS <= 16 && (SPP & (SPP - 1)) == 0, "one packet per step record");
    constexpr int kTbGroups = 32 / SPP;
    constexpr int kTbLanes = R >= 32 ? 1 : (32 / R < kTbChunks / kTbGroups ? 32 / R : kTbChunks / kTbGroups);
    static_assert(kTbLanes * kTbGroups <= kTbChunks, "flag window <= 32 packets");
    __shared__ __attribute__((aligned(16))) uint8_t s_tb[kTbLdsBytes];
    const int lane = threadIdx.x;
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= P.count) return;
    const uint32_t pidx = P.pair_base + slot;
    sa_result res = P.res[pidx];
    if (res.flags & SA_FLAG_BAD_SHAPE) return;
    if (!tb_mine(P, res.flags)) {
        tb_release(P, &P.res[pidx], res.flags);
        return;
    }
    res.flags &= tb_clear_mask(P);
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    const int tagged = P.tagged;   // record layout (sa_layout.h Geom::tagged)
    // Locals only below: lambdas capturing P or a Geom by reference keep them on the stack.
    const uint64_t band_stride = make_geom(ALG, R, P.max_m, P.max_n, tagged).band_stride;
    const uint32_t* const lutbits = P.lutbits;
    const uint8_t* dir = P.dirs + (uint64_t)slot * P.dir_slot;
    tb_glb_u8* ops = (tb_glb_u8*)(P.ops + o1 + o2 + pidx);
    const bool allow = P.allow != 0;
    const int G = P.gap, MA = P.match, MI = P.mismatch, GE = P.gap_extend;
    const int GOE = P.gap_open + P.gap_extend;
    uint32_t k = 0;        // ops emitted
    uint32_t k0 = 0;       // ops already written to HBM (the rest sit in the LDS buffer)
    uint32_t flags = res.flags;
    tb_lds_u8* const vtb = (tb_lds_u8*)s_tb;
    auto emit = [&](uint8_t op) __attribute__((always_inline)) {
        const uint32_t q = k - k0;
        vtb[kTbOpsOff + (q >> 2) * 256 + lane * 4 + (q & 3)] = op;
        ++k;
    };
    auto flush = [&]() __attribute__((always_inline)) {
        for (uint32_t q = 0; q < k - k0; ++q) ops[k0 + q] = vtb[kTbOpsOff + (q >> 2) * 256 + lane * 4 + (q & 3)];
        k0 = k;
    };

    // ---------------------------------------------------------------- windows
    const uint32_t band_rows = (uint32_t)kWave * R;
    int wb = -1, wt = 0, wg = 0;             // flag window: band, top lane, top step group
    int w1 = -kTbSeqWin, w2 = -kTbSeqWin;    // sequence windows cover indices [w, w + 32)
    uintptr_t a1 = 0, a2 = 0;                // ... from the aligned addresses a1 / a2
    int cb = 0, ct = 0, cgrp = 0, csub = 0, cr = 0;   // cell (i, j) decomposed by ready()
    auto locate = [&](int i, int j) __attribute__((always_inline)) {
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
    auto ready = [&](int i, int j) __attribute__((always_inline)) -> bool {
        if (k - k0 >= (uint32_t)kTbOpsBuf) return false;   // op buffer full: flush at the next round
        if (!(i > 0 && j > 0)) return true;
        locate(i, j);
        return cb == wb && (unsigned)(wt - ct) < (unsigned)kTbLanes && (unsigned)(wg - cgrp) < (unsigned)kTbGroups &&
               (unsigned)(i - 1 - w1) < (unsigned)kTbSeqWin && (unsigned)(j - 1 - w2) < (unsigned)kTbSeqWin;
    };
    // one batch of LDS-DMA loads (one memory latency) re-anchors all three windows at (i, j)
    auto refill = [&](int i, int j) __attribute__((always_inline)) {
        if (!(i > 0 && j > 0)) return;       // edge moves read nothing (and (i-1) would wrap)
        locate(i, j);
        wb = cb; wt = ct; wg = cgrp;
        const uint8_t* base = dir + (uint64_t)cb * band_stride;
#pragma unroll
        for (int dl = 0; dl < kTbLanes; ++dl)
#pragma unroll
            for (int dg = 0; dg < kTbGroups; ++dg) {
                const int l = ct - dl, gg = cgrp - dg;
                if (l >= 0 && gg >= 0)
                    __builtin_amdgcn_global_load_lds((tb_gptr)(base + ((uint64_t)gg * kWave + l) * 16),
                                                     (tb_lptr)(s_tb + (dl * kTbGroups + dg) * 1024), 16, 0, 0);
            }
        // sequence windows: the 9 aligned dwords covering indices [x - 31, x]
        w1 = i - kTbSeqWin;
        w2 = j - kTbSeqWin;
        a1 = (reinterpret_cast<uintptr_t>(s1) + w1) & ~(uintptr_t)3;
        a2 = (reinterpret_cast<uintptr_t>(s2) + w2) & ~(uintptr_t)3;
        const uintptr_t lo1 = reinterpret_cast<uintptr_t>(s1), hi1 = lo1 + (uintptr_t)m;
        const uintptr_t lo2 = reinterpret_cast<uintptr_t>(s2), hi2 = lo2 + (uintptr_t)n;
#pragma unroll
        for (int d = 0; d < kTbSeqItems; ++d) {
            const uintptr_t d1 = a1 + 4 * d, d2 = a2 + 4 * d;
            if (d1 + 4 > lo1 && d1 < hi1)
                __builtin_amdgcn_global_load_lds((tb_gptr)d1, (tb_lptr)(s_tb + kTbSeqOff1 + d * 256), 4, 0, 0);
            if (d2 + 4 > lo2 && d2 < hi2)
                __builtin_amdgcn_global_load_lds((tb_gptr)d2, (tb_lptr)(s_tb + kTbSeqOff2 + d * 256), 4, 0, 0);
        }
        // The DMA writes lane i's bytes at base + i * size, which alias analysis does not see, so
        // neither does the wait-count pass: wait for the DMA here, and keep every window read
        // after this point (compiler barrier).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    auto seqbyte = [&](int off, uintptr_t a, const uint8_t* sq, int x) __attribute__((always_inline)) -> uint8_t {
        const int o = (int)(reinterpret_cast<uintptr_t>(sq) + x - a);
        return vtb[off + (o >> 2) * 256 + lane * 4 + (o & 3)];
    };
    // flags of the cell located by the last ready() (which returned true)
    auto cell = [&]() __attribute__((always_inline)) -> uint32_t {
        int word, lowbit;
        cell_word_bit(R, BPC, cr, &word, &lowbit, tagged);
        const int q = (wt - ct) * kTbGroups + (wg - cgrp);
        const int byte = csub * BPS + word * 4 + lowbit / 8;
        return (uint32_t)(vtb[q * 1024 + lane * 16 + byte] >> (lowbit % 8));
    };
    // linear modes: flags fD (bit 1) / fU (bit 0); a T16 max tag (3 diag, 2 up, 1 left, 0 clamp)
    // says the same thing: diag wins iff H == D, else up iff H == U.
    auto lin = [&]() __attribute__((always_inline)) -> uint32_t {
        const uint32_t f = cell() & 3u;
        return tagged ? (f == 3u ? 2u : (f == 2u ? 1u : 0u)) : f;
    };
    // diagonal move: emits the op and returns the substitution term that was added (vrec: the
    // match bit is the record's fX position under fD, see sa_fill_impl.h kMatchBits)
    const bool vrec = P.vrec != 0;
    auto diag = [&](int i, int j, uint32_t f) __attribute__((always_inline)) -> int {
        const bool v = vrec ? ((f >> 2) & 1u) != 0
                            : tb_match<LUT>(lutbits, seqbyte(kTbSeqOff1, a1, s1, i - 1), seqbyte(kTbSeqOff2, a2, s2, j - 1));
        emit(v ? 'M' : (allow ? 'S' : 'X'));
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
    // The 64 lanes of the wave walk 64 different pairs.  A lane whose next move would leave its
    // windows parks; once every unfinished lane is parked they all refill together, so the wave
    // pays one memory latency per round of ~kTbGroups*spp moves instead of one per move.
    bool parked = true;
#ifdef SA_TB_STATS
    unsigned long long st_rounds = 0, st_iters = 0, st_rcyc = 0;
    const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();
#endif
    for (;;) {
#ifdef SA_TB_STATS
        ++st_iters;
#endif
        if (__builtin_amdgcn_ballot_w64(!fin && !parked) == 0) {
            if (__builtin_amdgcn_ballot_w64(!fin) == 0) break;
#ifdef SA_TB_STATS
            ++st_rounds;
            const unsigned long long r0 = __builtin_amdgcn_s_memtime();
#endif
            if (!fin) { flush(); refill(i, j); parked = false; }
#ifdef SA_TB_STATS
            __builtin_amdgcn_s_waitcnt(0);   // vmcnt(0) lgkmcnt(0): time the refill itself
            st_rcyc += __builtin_amdgcn_s_memtime() - r0;
#endif
        }
        if (!fin && !parked) {
            if (!ready(i, j)) {
                parked = true;
            } else {
                // one iteration of the reference's traceback loop (fin: it would leave the loop)
                do {
                    if constexpr (ALG == SA_SW || ALG == SA_NW) {
                        // Branch-free: the flag and both symbols are read together (one LDS latency), the
                        // move is selected arithmetically.  SW stops when H == 0 (diag test max(D,0) == 0).
                        const bool inner = i > 0 && j > 0;
                        if (ALG == SA_SW ? (!inner || V == 0) : !(i > 0 || j > 0)) { fin = true; break; }
                        uint32_t f = 1u;   // NW edges: j == 0 -> up (H[i][0] == H[i-1][0] + Gap), i == 0 -> left
                        bool v = false;
                        if (inner) {
                            f = lin();
                            v = vrec ? (f & 1u) != 0
                                     : tb_match<LUT>(lutbits, seqbyte(kTbSeqOff1, a1, s1, i - 1), seqbyte(kTbSeqOff2, a2, s2, j - 1));
                        } else if (i == 0) {
                            f = 0u;
                        }
                        const bool dg = (f & 2u) != 0, up = !dg && (f & 1u);
                        emit(dg ? (v ? 'M' : (allow ? 'S' : 'X')) : (up ? 'U' : 'L'));
                        if constexpr (ALG == SA_SW) V -= dg ? (v ? MA : MI) : G;
                        i -= (dg || up) ? 1 : 0;
                        j -= up ? 0 : 1;
                    } else if constexpr (ALG == SA_LOCAL_GOTOH) {
                        // flags: bit3 = fD (M == diag), bit2 = fX (M == Ix), bit1 = Ix extends, bit0 = Iy extends
                        if (!(i > 0 && j > 0)) { fin = true; break; }
                        const uint32_t f = TAG ? t16a_flags(cell()) : cell();
                        if (st == 0) {
                            if (V <= 0) { fin = true; break; }    // M == max(D, 0) <= 0
                            if (f & 8u) { V -= diag(i, j, f); --i; --j; }
                            else st = (f & 4u) ? 1 : 2;              // M == Ix, else M == Iy (same value)
                        } else if (st == 1) {
                            if (f & 2u) { emit('U'); V -= GE; --i; }
                            else if (V > 0) { emit('U'); V -= GOE; --i; st = 0; }
                            else if (V == 0) { emit('u'); fin = true; }
                            else { flags |= SA_FLAG_DIVERGED; fin = true; }
                        } else {
                            if (f & 1u) { emit('L'); V -= GE; --j; }
                            else if (V > 0) { emit('L'); V -= GOE; --j; st = 0; }
                            else if (V == 0) { emit('l'); fin = true; }
                            else { flags |= SA_FLAG_DIVERGED; fin = true; }
                        }
                    } else {  // SA_GLOBAL_GOTOH
                        if (!(i > 0 || j > 0)) { fin = true; break; }
                        if (j == 0) { emit('U'); --i; break; }   // edge rules hold in any state
                        if (i == 0) { emit('L'); --j; break; }
                        const uint32_t f = TAG ? t16a_flags(cell()) : cell();
                        if (st == 0) {
                            if (f & 8u) { diag(i, j, f); --i; --j; }
                            else st = (f & 4u) ? 1 : 2;
                        } else if (st == 1) {
                            emit('U'); --i;
                            if (!(f & 2u)) st = 0;   // gap open: Ix == M[i-1][j] + GO + GE
                        } else {
                            emit('L'); --j;
                            if (!(f & 1u)) st = 0;
                        }
                    }
                } while (false);
            }
        }
    }
    flush();
#ifdef SA_TB_STATS
    if (lane == __builtin_amdgcn_readfirstlane(lane)) {
        atomicAdd(&g_tb_stats[0], st_rounds);
        atomicAdd(&g_tb_stats[1], st_iters);
        atomicAdd(&g_tb_stats[3], __builtin_amdgcn_s_memtime() - st_t0);
        atomicAdd(&g_tb_stats[4], st_rcyc);
        atomicAdd(&g_tb_stats[5], 1ull);
    }
    atomicAdd(&g_tb_stats[2], (unsigned long long)k);
#endif
    res.start_i = i;
    res.start_j = j;
    res.nops = k;
    res.flags = flags;
    P.res[pidx] = res;
}

#ifdef SA_TB_STATS
extern "C" int sa_debug_tb_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tb_stats), sizeof(g_tb_stats)) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tb_stats), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif

hipError_t launch_traceback(int algo, int R, bool lut, const TbParams& p, hipStream_t stream) {
    const dim3 block(64);
    const dim3 grid((p.count + 63) / 64);
    const bool tag = p.tagged != 0 && is_affine(algo);
#define SA_TB(AA, RR, LL)                                                                  \
    if (algo == AA && R == RR && lut == LL && !tag) {                                      \
        hipLaunchKernelGGL((traceback_kernel<AA, RR, LL>), grid, block, 0, stream, p);     \
        return hipGetLastError();                                                          \
    }
#define SA_TBT(AA, RR, LL)                                                                 \
    if (algo == AA && R == RR && lut == LL && tag) {                                       \
        hipLaunchKernelGGL((traceback_kernel<AA, RR, LL, true>), grid, block, 0, stream, p); \
        return hipGetLastError();                                                          \
    }
#define SA_TBT_A(AA) SA_TBT(AA, 1, false) SA_TBT(AA, 2, false) SA_TBT(AA, 4, false) SA_TBT(AA, 8, false) \
                     SA_TBT(AA, 16, false) SA_TBT(AA, 1, true) SA_TBT(AA, 2, true) SA_TBT(AA, 4, true)    \
                     SA_TBT(AA, 8, true) SA_TBT(AA, 16, true)
    SA_TBT_A(SA_LOCAL_GOTOH)
    SA_TBT_A(SA_GLOBAL_GOTOH)
#undef SA_TBT_A
#undef SA_TBT
#define SA_TB_A(AA) SA_TB(AA, 4, false) SA_TB(AA, 8, false) SA_TB(AA, 16, false) \
                    SA_TB(AA, 4, true) SA_TB(AA, 8, true) SA_TB(AA, 16, true)   \
                    SA_TB(AA, 1, false) SA_TB(AA, 2, false) SA_TB(AA, 1, true) SA_TB(AA, 2, true)
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
