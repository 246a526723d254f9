// sa_fill_impl.h — the DP fill kernel (computeScoreMatrix of the four reference aligners),
// instantiated per algorithm by sa_fill_{sw,nw,lg,gg}.hip.
//
// Reference recurrences restated (all int32, wrapping):
//   SW  SASmithWaterman.h:89-117   H = max(Hd + s, Hu + Gap, Hl + Gap, 0), max cell = last
//                                  row-major (Score >= MaxScore, :110)
//   NW  SANeedlemanWunsch.h:69-86  H = max(max(Hd + s, Hu + Gap), Hl + Gap); H[i][0] = i*Gap
//   LG  SALocalGotoh.h:102-139     Ix = max(Mu + GO + GE, Ixu + GE); Iy = max(Ml + GO + GE,
//                                  Iyl + GE); M = max(Md + s, Ix, Iy, 0); Ix/Iy borders -10000
//   GG  SAGlobalGotoh.h:98-126     same without the 0 and with M[i][0] = GO + i*GE
//   !AllowMismatch: the diagonal term is (match ? Hd + Match : INT_MIN)  (e.g. :128-131).
//
// Mapping to CDNA4 (geometry: sa_layout.h):
//   * one workgroup = one pair; W waves = W concurrently running bands (software pipeline,
//     one __syncthreads per 32-step chunk);
//   * one lane = R rows held in VGPRs; per step it computes R cells of one column;
//   * the row above arrives from lane t-1 by DPP wave_shr:1 (no LDS round trip); lane 0 takes
//     it from the row buffer (previous band) or the top border, loaded once per chunk into a
//     VGPR and broadcast per step with v_readlane; the column symbol rides the same DPP shift;
//   * chunks where all 64 lanes are inside the matrix (all but the first two and the last
//     two of a band) run a branch-free body;
//   * each traceback flag costs one v_cmp (into an SGPR pair) + one v_addc_co_u32 that shifts
//     it into the lane's record; records leave as 16-byte-per-lane nontemporal stores
//     (1 KiB per wave instruction, fully coalesced);
//   * the running maximum of a row is one v_lshl_or (key = H << 16 | column) + one v_max_u32
//     (KEYED; the host checks scores and columns fit 16 bits), else a compare + 2 selects.
//
// T16 (tagged 16-bit profile kernel; SW and NW with allow-mismatch, batch alphabet <= 4 symbols,
// host-proven |4H| < 2^15).  gfx950 issues 16-bit VOP2 add/max and 32-bit bitwise ops at about
// twice the rate of 32-bit max/compare/carry ops (profiles/microbench_valu_issue_r01.txt), so:
//   * scores are kept as 4*H; every candidate carries its move tag in the two low bits
//     (diag 4D+3, up 4U+2, left 4L+1, clamp 0), so ONE v_max_i16 chain yields both the cell
//     value and the winning move with the reference's tie order (diag, then up, then left:
//     SASmithWaterman.h:274-312, SANeedlemanWunsch.h:181-214);
//   * the substitution term comes from a per-row byte profile with one v_bfe_i32 (offset =
//     8 * symbol code of the column) instead of a compare + select;
//   * the tag is pushed into the record with one v_alignbit_b32 (rec = rec >> 2 | T << 30) and
//     stripped from the value with one v_and_b32.
// Cell = bfe + 3 add_u16 + 2-3 max_i16 + and + alignbit (+ lshl_or + max_u32 for the key).
//
// T16 affine (LocalGotoh / GlobalGotoh with allow-mismatch, same alphabet and profile rules).
// Scores are kept as 8*V: bits 1-2 of a candidate carry its class in M's max (3 = diag, 2 = Ix,
// 1 = Iy, 0 = the zero clamp) and bit 0 says, inside Ix's / Iy's own max, extend (1) over open
// (0) -- the reference's tie orders (SALocalGotoh.h:304-468, SAGlobalGotoh.h:245-421).  Per cell:
//   Ix = max(Mu + 8GOE + 4, Xu + 8GE + 1)   LocalGotoh takes the open term as max(., 0) with one
//        saturating v_sub_u16, which also supplies M's zero clamp (max(Ix, 0) is exact wherever the
//        traceback reads Ix, and max(D, max(Ix, 0), Iy) == max(D, Ix, Iy, 0), class bits included);
//   Iy = max(Ml + 8GOE + 2, Yl + 8GE + 1);  M = max(D, Ix, Iy) with D = Md + (8s + 6) (profile);
//   one v_alignbit each pushes Ix's and Iy's extend bit and M's class into the record (one byte per
//   cell, sa_layout.h), one v_and each strips them (Ix/Iy keep their class bits).
// 16 VALU per cell (+2 for the LocalGotoh (M, column) key) against the int32 kernel's 21.
//
// CMAX (T16 SW and LocalGotoh, one-wave plans): instead of a (score, column) key per cell, each row keeps its
// maximum over the current 32-step chunk with one more v_max_i16 (fast class); at the chunk end
// the row's (max, chunk) pair joins its key and the lane stores a snapshot of its state (R
// 16-bit values + the diagonal input), and each band's top row is kept.  The fill then reports
// (score, row, chunk) and sa_endcell.hip replays that one chunk to find the exact column.
#pragma once
#include <limits.h>

#include <type_traits>

#include "sa_internal.h"

namespace sa {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kDppWaveShr1 = 0x138;  // DPP wave_shr:1 (GFX9-family wave-wide shift)

__device__ __forceinline__ int shr1(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, kDppWaveShr1, 0xf, 0xf, false);
}
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
// v_writelane_b32 through the LLVM intrinsic (the compiler routes the lane select via m0).
extern "C" __device__ int sa_writelane(int value, int lane, int old) __asm("llvm.amdgcn.writelane");

// rec = 2*rec + c, one v_cmp into an SGPR pair + one v_addc_co_u32.
__device__ __forceinline__ uint32_t push_bit(uint32_t rec, bool c) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(c);
    uint32_t out;
    unsigned long long co;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(out), "=s"(co) : "v"(rec), "s"(m));
    return out;
}
__device__ __forceinline__ uint32_t push_eq(uint32_t rec, int a, int b) { return push_bit(rec, a == b); }

// 8 * code of symbol b in the T16 alphabet (bytes of sym_pack are distinct; code 0 = byte 0).
__device__ __forceinline__ uint32_t t16_code8(uint32_t sp, uint32_t b) {
    return (b == ((sp >> 8) & 255u) ? 8u : 0u) | (b == ((sp >> 16) & 255u) ? 16u : 0u) |
           (b == (sp >> 24) ? 24u : 0u);
}

// SO profile word: the tagged profile bytes 4s + 3 (8s + 6 affine; decide_t16) back to s, byte by
// byte.
template <bool AFF = false>
__device__ __forceinline__ uint32_t so_profile(uint32_t w) {
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        o |= ((uint32_t)(AFF ? (((int)(int8_t)(w >> (8 * k)) - 6) >> 3) : (((int)(int8_t)(w >> (8 * k)) - 3) >> 2)) & 255u)
             << (8 * k);
    return o;
}

template <bool LUT>
__device__ __forceinline__ bool match_bit(const uint32_t* s_lut, int a, int b) {
    if constexpr (LUT) {
        return (s_lut[(a << 3) | (b >> 5)] >> (b & 31)) & 1;
    } else {
        return a == b;
    }
}

// Max workgroup size: 16 waves, except R = 32 (T16 only) and the T16 affine kernel at R = 16,
// which need > 128 VGPRs per lane.
template <int R, bool WIDE = false>
constexpr int fill_max_threads() { return (R >= 32 || (WIDE && R >= 16)) ? 256 : 1024; }

// Bounded wait of a SPLIT band for its producer: FillParams::wait_ticks (kSplitWaitTicksDefault,
// 0.2 s; SEQALIB_SPLIT_WAIT_TICKS overrides it for tests).  After one expiry the workgroup stops
// waiting altogether: the pair is flagged SA_FLAG_TIMEOUT and re-run by the call's
// single-workgroup fallback launch (run_device, sa_api.hip).

// SPLIT hand-off.  A SPLIT workgroup is three waves: the COMPUTE wave runs the band; the POLLER
// loads the producer band's last row -- write-through {tag, value} granules -- and copies it into
// an LDS ring (kRing columns), publishing how many columns are ready; the PUBLISHER reads this
// band's last row, which the compute wave parks per step in a second LDS ring, and stores it as
// granules for the next band.  The compute wave only touches LDS: every kHandGran steps it
// compares the poller's count (re-read only when short) and posts its own step count.  Polls or
// publishes in the compute wave cost +26..33 % per step (round 3, tools/split_stats.py): a vector
// load's s_waitcnt vmcnt also waits for every record store in flight (gfx9's vmcnt counts stores),
// and a publish is an LDS read + wait + store.  With the 32-column chunks of round 2 a band ran
// ~161 steps behind its producer (63 inherent, ~64 chunk quantisation, the rest latency).
// Steps per hand-off granule: 16 for the linear-gap cell, 8 for the affine one (configs 2 / 4 on
// one MI355X, tools/ab_split.py: SW 4096^2 fill 0.54 ms at 8, 0.49 at 16, 0.52 at 32, 0.63 at 4;
// LocalGotoh 8192^2 1.61 ms at 8, 1.64 at 16, 1.73 at 32).  SA_HAND_GRAN overrides both (A/B).

template <bool AFF>
constexpr int hand_gran() {
#ifdef SA_HAND_GRAN
    return SA_HAND_GRAN;
#else
    return AFF ? 8 : 16;
#endif
}
enum : int { kStepAny = 0, kStepSteady = 1, kStepStart = 2 };   // fill_kernel's step modes
static_assert(kChunk % hand_gran<false>() == 0 && kChunk % hand_gran<true>() == 0, "granules tile a chunk");

#ifdef SA_TB_STATS
// Debug build only (-DSA_TB_STATS, tools/split_stats.py): per SPLIT ticket {slot * bands + band,
// start, end, ticks spent polling for the producer} in s_memrealtime ticks (100 MHz, chip-wide).
// One copy per fill translation unit (no relocatable device code), read with
// sa_debug_split_stats_<algo> (SA_SPLIT_STATS_ACCESSOR in sa_fill_{sw,nw,lg,gg}.hip).
static __device__ unsigned long long g_split_stats[4096][4];
// hand-off events of the granule at columns kEvCol..kEvCol+7 (mid-band, steady state), same
// index: [0] the compute wave posts step kEvCol+71 (the granule parked), [1] the publisher sees
// that post, [2] the publisher has issued the granule's stores, [3] the poller publishes the
// granule to its compute wave, [6] the compute wave asks for the group at kEvCol, [4] it has its
// inputs.  Kept in registers, written when the wave leaves.
static __device__ unsigned long long g_split_ev[4096][12];
constexpr int kEvCol = 2048;
#define SA_SPLIT_STATS_ACCESSOR(NAME)                                                               \
    extern "C" int NAME(unsigned long long* out, int reset) {                                       \
        if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_split_stats), sizeof(g_split_stats)) != hipSuccess) \
            return 1;                                                                               \
        if (hipMemcpyFromSymbol(out + 4096 * 4, HIP_SYMBOL(g_split_ev), sizeof(g_split_ev)) != hipSuccess) \
            return 1;                                                                               \
        if (reset) {                                                                                \
            static unsigned long long z[4096][12];                                                   \
            if (hipMemcpyToSymbol(HIP_SYMBOL(g_split_stats), z, sizeof(g_split_stats)) != hipSuccess) return 1; \
            if (hipMemcpyToSymbol(HIP_SYMBOL(g_split_ev), z, sizeof(g_split_ev)) != hipSuccess) return 1; \
        }                                                                                           \
        return 0;                                                                                   \
    }
// many-pairs plans: per workgroup (slot) {start, end} in s_memrealtime ticks and {HW_ID, XCC_ID}
// (tools/fill_timeline.py: the fill's schedule -- generations, per-SIMD residency, the tail)
static __device__ unsigned long long g_fill_stats[32768][3];
#define SA_FILL_STATS_ACCESSOR(NAME)                                                               \
    extern "C" int NAME(unsigned long long* out, int reset) {                                       \
        if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fill_stats), sizeof(g_fill_stats)) != hipSuccess) \
            return 1;                                                                               \
        if (reset) {                                                                                \
            static unsigned long long z[32768][3];                                                  \
            if (hipMemcpyToSymbol(HIP_SYMBOL(g_fill_stats), z, sizeof(g_fill_stats)) != hipSuccess) return 1; \
        }                                                                                           \
        return 0;                                                                                   \
    }
#define SA_EV(k, cond) do { if (ev[k] == 0 && (cond)) ev[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define SA_EV_FLUSH() do { const uint64_t id_ = (uint64_t)slot * P.split_bands + band0;            \
    if (id_ < 4096 && lane == 0) for (int k_ = 0; k_ < 12; ++k_) if (ev[k_]) g_split_ev[id_][k_] = ev[k_]; } while (0)
#else
#define SA_SPLIT_STATS_ACCESSOR(NAME)
#define SA_FILL_STATS_ACCESSOR(NAME)
#define SA_EV(k, cond) do {} while (0)
#define SA_EV_FLUSH() do {} while (0)
#endif

// Band units (BU): the pair's final unit folds the per-unit words {tag << 32 | lost << 31 | maximum}
// of units [0, nparts) (segments past last_seg store none).  Each wait is bounded by wait_polls; an
// expired one counts as lost.  Returns this lane's maximum of the maxima it read (the caller reduces
// over the wave); lost (every lane) is set when any unit, or a wait here, lost its producer.
__device__ __forceinline__ uint32_t bu_fold_parts(const unsigned long long __attribute__((address_space(1)))* part,
                                                  uint32_t nparts, uint32_t last_seg, uint32_t segs, uint32_t tag,
                                                  uint32_t wait_polls, int lane, uint32_t& lost) {
    uint32_t mx = 0, ls = lost;
    for (uint32_t b = (uint32_t)lane; b < nparts; b += kWave) {
        if (b % segs > last_seg) continue;
        unsigned long long x = __hip_atomic_load(part + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t it = 0; (uint32_t)(x >> 32) != tag; ++it) {
            if (it >= wait_polls) { x = 1ull << 31; break; }
            __builtin_amdgcn_s_sleep(2);
            x = __hip_atomic_load(part + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        ls |= (uint32_t)(x >> 31) & 1u;
        mx = max(mx, (uint32_t)x & 0x7fffffffu);
    }
    lost = __builtin_amdgcn_ballot_w64(ls != 0) != 0 ? 1u : 0u;
    return mx;
}

// MM: how a cell learns whether its two symbols match -- kMatchEq (byte equality), kMatchLut (the
// 256 x 256 table of the user's match fn, LDS) or kMatchBits (a per-pair m x n match bitmap, the
// generic-Ty path: any symbol type and count, the reference's cacheAllMatches packed to bits).
// SO (score-only, T16 SW CMAX many-pairs plans): the cell carries no move tags and the fill writes
// no per-cell records -- only each lane's last row per step (the "edge" stream, 16 bits per
// lane-step).  With the per-chunk snapshots every (lane, chunk) block of R x 32 cells can be
// recomputed exactly from its left column (snapshot), its top row (edge stream of the lane above,
// or the band's top row) and its corner, which sa_traceback_so.hip does along the path.
template <int ALG, int R, int MM, bool ALLOW, bool KEYED, bool T16, bool CMAX, bool SPLIT, bool SO = false>
// (Asking the headline kernel for 4 waves per SIMD -- 128 VGPRs, 8 spills outside the step loops
// -- measured 29.6 ms per fill against 29.4 at its natural 3 waves: not taken.)
__device__ __forceinline__ void fill_body(const FillParams& P) {
    constexpr bool LUT = MM == kMatchLut;
    constexpr bool BITS = MM == kMatchBits;
    constexpr bool AFF = ALG >= SA_LOCAL_GOTOH;
    constexpr int kHandGran = hand_gran<AFF>();   // SPLIT hand-off granule (steps)
    constexpr bool LOCAL = (ALG == SA_SW || ALG == SA_LOCAL_GOTOH);
    constexpr int FBITS = AFF ? 4 : 2;            // flag bits per cell
    constexpr int BPC = record_bpc(ALG, R, T16);  // record bits per cell (padding above the flags)
    // bits per record (SO: the lane's last row, 16 bits; affine: its M and Ix - (GO + GE), 32 bits)
    constexpr int RB = SO ? (AFF ? 32 : 16) : R * BPC;
    constexpr int BPS = RB / 8;                // bytes per record
    constexpr int RW = (RB + 31) / 32;         // words per record
    constexpr int RPW = (RB < 32 ? RB : 32) / BPC;  // rows per record word
    constexpr int SPP = BPS >= 16 ? 1 : 16 / BPS;
    constexpr int PPS = BPS > 16 ? BPS / 16 : 1;
    constexpr int BAND = kWave * R;
    static_assert(kChunk % SPP == 0, "chunk must hold whole packets");
    static_assert(BPS >= 1, "record must be at least a byte");
    static_assert(!T16 || (ALLOW && MM == kMatchEq && (RB <= 32 || RB % 32 == 0)),
                  "T16: allow-mismatch, profile");
    static_assert(!T16 || !LOCAL || KEYED, "T16 local mode tracks its maximum with keys");
    constexpr int SC = SO ? 1 : T16 ? (AFF ? 8 : 4) : 1;   // score scale of the register values
    // SO: T16, many pairs; SW / LocalGotoh with the chunk-max end cell, or NW / GlobalGotoh (which
    // end at (m, n))
    static_assert(!SO || (T16 && !SPLIT && (LOCAL ? CMAX : !CMAX)), "SO: T16 chunk-max local or global, many pairs");
    // per-chunk snapshots of every lane's state (the end-cell replay and the SO traceback read them)
    constexpr bool SNAP = CMAX || SO;
    // BAND UNITS (SO): every (pair, band) is a work unit of its own -- one single-wave workgroup per
    // unit, units handed out by a ticket counter band-major (all bands 0, then all bands 1, ...), so
    // a unit's producer band started earlier and, at the batch sizes that fill the chip, has long
    // finished.  The launch tail is then the duration of one band, not of a whole pair (a 4096-row
    // pair is two R = 32 bands: 10,000 x 4096^2 fill 16.55 -> 15.23 ms measured as 20,000 x
    // 2048 x 4096, tools/fill_sweep.py).  The band's last row goes to the next band as 32-bit
    // {epoch, value} granules in the row buffer (written and read as agent-scope atomics, i.e.
    // coherent across the XCDs' L2s); a consumer re-reads a chunk's granules until they carry this
    // launch's epoch (rare: see above).  The bands' score maxima meet in epoch-tagged partials
    // that the last band folds into the pair's result.
    constexpr bool BU = SO && !AFF;
    // SOMAX (SO SW): the chunk maxima track only sampled cells (see the SW SO cell), the pair reports
    // their maximum smax and endcell_so_kernel finds S; SO LocalGotoh keeps the exact chunk maxima
    // of CMAX
    constexpr bool SOMAX = SO && ALG == SA_SW;
    constexpr int CSH = SO ? 0 : (AFF ? 3 : 2);   // CMAX: chunk maxima are H << CSH
    static_assert(!CMAX || (T16 && LOCAL && R % 2 == 0), "CMAX: T16 Smith-Waterman / LocalGotoh");

    // Dynamic LDS (sizes from lds_layout(), host and device agree):
    //   [match bits: 2048 words, LUT only][hand-off rings: W x kRing x (1|2) ints][Seq2 bytes, staged]
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    __shared__ int s_red[16 * 3];
    __shared__ int s_score;   // H[m][n] for the global modes, stored by the owning lane
    // SPLIT: [0] columns the poller has copied into the ring, [1] columns the compute wave has
    // consumed, [2] the poller's bounded wait expired; s_ticket: the band's ticket
    //   [3] steps the compute wave has run (its parked last-row values), [4] steps the publisher
    //   has stored
    __shared__ int s_sync[8];
    __shared__ uint32_t s_ticket;
    __shared__ int s_pring[SPLIT ? 2 * kRing : 1];   // SPLIT: the parked last row (H, then Ix), by step
    __shared__ uint32_t s_comp[(T16 && ALG == SA_GLOBAL_GOTOH) ? 8 : 1];   // symbol counts (GG screen)

    // the batch selected the other kernel variant: leave -- except an int32 launch re-running the
    // pairs a T16 fill flagged kFlagRetry (checked below, once the pair is known)
    bool redo = false;
    if (sa_skip(P.sel, P.sel_want)) {
        if (!P.redo) return;
        redo = true;
    }
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
    const int W = P.waves;
    const uint32_t symp = T16 ? P.prof[4] : 0u;   // T16: the symbols of codes 0..3
    // SPLIT (few pairs): one single-wave workgroup per (pair, band).  Bands are handed out by a
    // ticket counter in the order workgroups actually start, so band b's producer (ticket - 1)
    // is always already running or done: no wait can deadlock whatever the residency.
    uint32_t slot, band0 = 0, seg = 0;
    if constexpr (BU) {
        // tickets band-major, then segment-major: (band, segment, pair)
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(P.ticket, 1u);
        t = __builtin_amdgcn_readlane(t, 0);
        const uint32_t row = P.count * P.part_segs;
        band0 = t / row;
        const uint32_t rem = t - band0 * row;
        seg = rem / P.count;
        slot = rem - seg * P.count;
    } else if constexpr (SPLIT) {
        if (threadIdx.x == 0) {
            s_ticket = atomicAdd(P.ticket, 1u);
            s_sync[0] = 0; s_sync[1] = 0; s_sync[2] = 0; s_sync[3] = 0; s_sync[4] = 0;
        }
        __syncthreads();   // (the compute wave and the poller)
        const uint32_t t = __builtin_amdgcn_readfirstlane(s_ticket);
        slot = t / P.split_bands;
        band0 = t - slot * P.split_bands;
    } else {
        slot = blockIdx.x;
        if (slot >= P.count) return;   // (uniform) a grid larger than the launch's pairs
    }
    const uint32_t pidx = P.pair_base + slot;
    if (redo && !(P.res[pidx].flags & kFlagRetry)) return;   // uniform over the workgroup
    if (P.rerun && !(P.res[pidx].flags & SA_FLAG_TIMEOUT)) return;
#ifdef SA_TB_STATS
    const unsigned long long st_t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long st_wait = 0;
    // s_getreg HW_REG_HW_ID (4) and HW_REG_XCC_ID (20), all 32 bits
    const uint32_t st_hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t st_xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
#endif
    const uint64_t o1 = P.off1[pidx];
    const uint64_t o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);

    if ((uint32_t)m > P.max_m || (uint32_t)n > P.max_n) {  // whole block leaves together
        if (!SPLIT && threadIdx.x == 0 && band0 == 0) {   // SPLIT: split_reduce_kernel reports it
            sa_result r = {};
            r.flags = SA_FLAG_BAD_SHAPE;
            P.res[pidx] = r;
        }
        return;
    }
    // Screened T16 GlobalGotoh (t16_mode_affine, retry_above != INT_MAX): the 16-bit window holds
    // every value of a pair whose alignments of prefixes score at most retry_above.  Each such
    // score is <= MA * (its matches) <= MA * min(L, m, n), L a bound on the matches from the
    // symbol counts (below; sum over the <= 4 symbols of min(count in Seq1, count in Seq2) for
    // equality).  A pair above the cap leaves its fill to the int32
    // variant (kFlagRetry, re-run exactly by the redo launch).
    if constexpr (T16 && ALG == SA_GLOBAL_GOTOH && !SPLIT) {
        if (P.retry_above != INT_MAX) {
            if (threadIdx.x < 8) s_comp[threadIdx.x] = 0;
            __syncthreads();
            uint32_t ca[4] = {0, 0, 0, 0}, cb[4] = {0, 0, 0, 0};
            const uint8_t* q1 = P.seq1 + o1;
            const uint8_t* q2 = P.seq2 + o2;
            for (int k = threadIdx.x; k < m; k += blockDim.x) {
                const uint32_t c = t16_code8(symp, q1[k]) >> 3;
#pragma unroll
                for (int e = 0; e < 4; ++e) ca[e] += c == (uint32_t)e ? 1u : 0u;
            }
            for (int k = threadIdx.x; k < n; k += blockDim.x) {
                const uint32_t c = t16_code8(symp, q2[k]) >> 3;
#pragma unroll
                for (int e = 0; e < 4; ++e) cb[e] += c == (uint32_t)e ? 1u : 0u;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (ca[e]) atomicAdd(&s_comp[e], ca[e]);
                if (cb[e]) atomicAdd(&s_comp[4 + e], cb[e]);
            }
            __syncthreads();
            // L bounds the matches of any alignment of prefixes: a Seq1 symbol a is matched at most
            // min(count of a, count of the Seq2 symbols that match a) times -- and symmetrically.
            // With equality this is sum_a min(ca[a], cb[a]); with the caller's match table
            // (lutbits: the T16 profile follows it, decide_t16) different symbols may match.
            uint32_t mt = 0;
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint32_t xa = (symp >> (8 * a)) & 255u, xb = (symp >> (8 * b)) & 255u;
                    const bool v = P.lutbits ? ((P.lutbits[(xa << 3) | (xb >> 5)] >> (xb & 31u)) & 1u) != 0 : xa == xb;
                    mt |= (v ? 1u : 0u) << (4 * a + b);
                }
            int64_t L1 = 0, L2 = 0;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                int64_t r1 = 0, r2 = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    if ((mt >> (4 * a + b)) & 1u) r1 += s_comp[4 + b];   // Seq2 symbols matching a
                    if ((mt >> (4 * b + a)) & 1u) r2 += s_comp[b];       // Seq1 symbols matching a
                }
                L1 += min<int64_t>(s_comp[a], r1);
                L2 += min<int64_t>(s_comp[4 + a], r2);
            }
            const int64_t L = min(L1, L2);
            const int64_t hi = (int64_t)max(P.match, 0) * min<int64_t>(L, min(m, n));
            if (hi > (int64_t)P.retry_above) {   // uniform over the workgroup
                if (threadIdx.x == 0) {
                    sa_result r = {};
                    r.flags = kFlagRetry;
                    P.res[pidx] = r;
                }
                return;
            }
        }
    }
    const LdsLayout lay = lds_layout(LUT, AFF, W, P.stage_seq2 ? P.max_n : 0);
    uint32_t* const s_lut = smem;
    int32_t* const s_ring = reinterpret_cast<int32_t*>(smem + lay.ring_off / 4);
    uint8_t* const s_seq2 = reinterpret_cast<uint8_t*>(smem) + lay.seq_off;
    // LDS-fed steps: a chunk's lane-0 inputs and column symbols are read per step as LDS
    // broadcasts straight into the DPP shift's old operand, and the band's last row is parked per
    // step by an LDS write of lane 63 (lanes 0..62 write a discard slot, so the address is a
    // per-lane constant and the step offset an immediate): no v_readlane / v_writelane / v_mov.
    int32_t* const s_step = reinterpret_cast<int32_t*>(smem + lay.step_off / 4) + w * kStepBufWords;
    int32_t* const s_park = s_step + (lane == 63 ? 96 : 160);
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    if constexpr (LUT) {
        for (int k = threadIdx.x; k < 2048; k += blockDim.x) s_lut[k] = P.lutbits[k];
    }
    if (P.stage_seq2) {
        // (BU: the columns of this unit's chunks and the 64 before them)
        int k0 = 0, k1 = n;
        if constexpr (BU) {
            const uint32_t nc = chunks_per_band((uint32_t)n);
            const uint32_t sp = max(1u, min(P.part_segs, nc / 2)), cp = (nc + sp - 1) / sp;
            k0 = max(0, (int)(seg * cp * kChunk) - kWave);
            k1 = min(n, (int)((seg + 1) * cp * kChunk));
        }
        for (int k = k0 + (int)threadIdx.x; k < k1; k += blockDim.x)
            s_seq2[k] = T16 ? (uint8_t)t16_code8(symp, s2[k]) : s2[k];
    }
    if constexpr (SPLIT) {   // tag 0 = no column yet (LDS holds a previous workgroup's data)
        for (int k = threadIdx.x; k < (AFF ? 2 : 1) * kRing; k += blockDim.x) s_ring[k] = 0;
    }
    __syncthreads();
    const int G = P.gap, MA = P.match, MI = P.mismatch;
    const int GO = P.gap_open, GE = P.gap_extend;
    const int GOE = GO + GE;
    // T16 tagged gaps.  Local modes take the up term as max(4U + 2, 0) = hu - CU with unsigned
    // saturation (v_sub_u16 clamp; hu >= 0, CU = -(4G + 2) > 0 since t16_ok demands G < 0),
    // which also applies the zero clamp of the cell: max(D, max(U, 0), L) == max(D, U, L, 0).
    const uint32_t CU = SO ? ((uint32_t)(-G) & 0xffffu)
                       : LOCAL ? ((uint32_t)(-(4 * G + 2)) & 0xffffu) : (uint32_t)(4 * G + 2);
    const uint32_t CL = SO ? ((uint32_t)G & 0xffffu) : (uint32_t)(4 * G + 1);   // (SO NW: the shared gap term)
    // T16 affine: class / extend tagged gap terms (u16 arithmetic, sa_fill_impl.h header).  The
    // LocalGotoh Ix open term is max(Mu + 8GOE + 4, 0) = Mu - CXO with unsigned saturation (Mu >= 0,
    // CXO = -(8GOE + 4) > 0 since t16_mode demands GOE < 0).
    const uint32_t CXO = (uint32_t)(LOCAL ? -(8 * GOE + 4) : 8 * GOE + 4) & 0xffffu;
    const uint32_t CXE = (uint32_t)(8 * GE + 1) & 0xffffu;
    const uint32_t CYO = (uint32_t)(8 * GOE + 2) & 0xffffu;
    // SO affine: CGE = GE; CGOE = -(GO + GE) (LocalGotoh, by saturation) or GO + GE (GlobalGotoh)
    const uint32_t CGE = (uint32_t)GE & 0xffffu;
    const uint32_t CGOE = (uint32_t)(LOCAL ? -GOE : GOE) & 0xffffu;
    // Ix / Iy borders (the reference's -10000): T16 affine uses a value below every candidate
    const int XB = (T16 && AFF) ? P.t16_sent : -10000;

    const int B = (m > 0 && n > 0) ? (m + BAND - 1) / BAND : 0;
    if (SPLIT && (int)band0 >= B) return;   // uniform: this pair has fewer bands
    if (BU && (int)band0 >= (B > 0 ? B : 1)) return;   // (an empty pair: unit 0 reports it)
    const uint32_t nch = chunks_per_band((uint32_t)n);
    const uint32_t period = sched_period(nch, W);
    // BU column segments: this unit runs chunks [c0, c1) of its band (a segment past the pair's
    // chunks is empty and leaves at once); every boundary c0 >= 2 lies where all 64 lanes have
    // reached their first column, so the unit starts from the state the previous segment handed on
    const uint32_t SEGS = BU ? P.part_segs : 1u;
    const uint32_t segs_p = max(1u, min(SEGS, nch / 2));   // this pair's (at least 2 chunks each)
    const uint32_t cps = (nch + segs_p - 1) / segs_p;
    const uint32_t c0 = BU ? seg * cps : 0u;
    const uint32_t c1 = BU ? min(nch, c0 + cps) : nch;
    const uint32_t last_seg = BU && nch > 0 ? (nch - 1) / cps : 0u;
    if (BU && seg > (B > 0 ? last_seg : 0u)) return;   // (uniform) an empty segment (an empty pair: unit 0 reports)
    const uint32_t total = SPLIT ? nch : BU ? (B > 0 ? c1 : 0u) : total_phases((uint32_t)B, (uint32_t)n, W);
    const uint32_t epoch16 = P.epoch << 16;   // BU: this launch's hand-off tag (P.epoch in [1, 65535])
    // SPLIT hand-off: band b's last row as 8-byte {tag = 1, value} granules written
    // write-through (sc1) per column, polled by band b+1 with sc1 loads; the data is its own flag
    // (cdna_hip_programming.md Guideline 16, R2).  The host zeroes them before every launch.
    typedef unsigned long long __attribute__((address_space(1))) gu64;
    gu64* const hand_pair = SPLIT ? (gu64*)(P.hand + (uint64_t)slot * P.split_bands * P.max_n) : nullptr;
    uint32_t tmo = 0;   // SPLIT: a bounded wait expired
    uint32_t seg_lost = 0;   // BU: a wait for a producer's hand-off expired (the pair is re-run in int32)
#ifdef SA_TB_STATS
    unsigned long long ev[12] = {};
#endif
    // SPLIT poller (wave 1, see kHandGran): copies the producer band's granules into the LDS ring
    // s_ring (the hand-off ring of the multi-wave plans, unused here) and publishes the count of
    // ready columns, never more than kRing columns beyond what the compute wave has consumed.
    // Its loads wait only for themselves; on a bounded-wait expiry it flags the band and releases
    // the compute wave (the pair is flagged SA_FLAG_TIMEOUT and re-run by the call's fallback).
    if constexpr (SPLIT) {
        if (w == 1) {
            if (band0 == 0) return;   // band 0 has no producer
            gu64* const src = hand_pair + (uint64_t)(band0 - 1) * P.max_n;
            int pub = 0;
            uint64_t t0 = 0;
            // two window loads in flight (A and B alternate): a granule is seen about half a load
            // round trip after it lands.  The loads are write-through-coherent (sc1) vector loads
            // in inline asm with explicit vmcnt waits tied to their results: compiled from C++, the
            // loop-header wait the compiler inserts drains both (vmcnt(0)).
            auto issue = [&](int b, unsigned long long& x, unsigned long long& y) {
                const int cl = min(b + lane, n - 1);
                gu64* const pa = src + cl;
                asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=&v"(x) : "v"(pa) : "memory");
                y = 1ull << 32;
                if constexpr (AFF) {
                    gu64* const px = pa + P.hand_x_off;
                    asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=&v"(y) : "v"(px) : "memory");
                }
            };
            // the older window's loads are done once only the newer window's remain in flight
            auto settle = [&](unsigned long long& x, unsigned long long& y) {
                if constexpr (AFF) asm volatile("s_waitcnt vmcnt(2)" : "+v"(x), "+v"(y) :: "memory");
                else asm volatile("s_waitcnt vmcnt(1)" : "+v"(x) :: "memory");
            };
            // columns b + lane of one window: extend the ready run from pub; false once the
            // bounded wait expired (the band is flagged and the compute wave released)
            auto take = [&](int b, unsigned long long x, unsigned long long y) -> bool {
                const int cons = __hip_atomic_load(&s_sync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const int lim = min(n, cons + kRing);
                const int c = b + lane;
                const bool ok = c < lim && (x >> 32) != 0 && (y >> 32) != 0;
                const uint64_t bad = __builtin_amdgcn_ballot_w64(c >= pub && !ok);
                const int npub = max(pub, b + (bad ? (int)__builtin_ctzll(bad) : kWave));
                if (npub > pub) {
                    if (c >= pub && c < npub) {
                        // T16: the 16-bit value tagged with its granule number + 1 in the upper
                        // half, so the compute wave's read of a granule is its own readiness check
                        const uint32_t tg = T16 ? ((uint32_t)c / kHandGran + 1u) << 16 : 0u;
                        const uint32_t vm = T16 ? 0xffffu : 0xffffffffu;
                        s_ring[c & (kRing - 1)] = (int)(((uint32_t)x & vm) | tg);
                        if constexpr (AFF) s_ring[kRing + (c & (kRing - 1))] = (int)(((uint32_t)y & vm) | tg);
                    }
                    pub = npub;
                    __hip_atomic_store(&s_sync[0], pub, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    SA_EV(3, pub >= kEvCol + 8);
                    t0 = 0;
                } else if (lim <= pub) {
                    __builtin_amdgcn_s_sleep(1);   // ring full: the compute wave is behind
                } else {
                    const uint64_t now = __builtin_amdgcn_s_memrealtime();
                    if (t0 == 0) {
                        t0 = now;
                    } else if (now - t0 > P.wait_ticks) {
                        __hip_atomic_store(&s_sync[2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(&s_sync[0], n, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        return false;
                    }
                }
                return true;
            };
            unsigned long long xa, ya, xb, yb;
            int ba = pub, bb;
            issue(ba, xa, ya);
            while (true) {
                bb = pub;
                issue(bb, xb, yb);
                settle(xa, ya);
                if (!take(ba, xa, ya) || pub >= n) break;
                ba = pub;
                issue(ba, xa, ya);
                settle(xb, yb);
                if (!take(bb, xb, yb) || pub >= n) break;
            }
            // the window load still in flight: its registers stay live up to here, so no exit
            // code (the compiler sinks the timeout stores to the exit) can take them before the
            // load lands
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(xa), "+v"(ya), "+v"(xb), "+v"(yb) :: "memory");
            SA_EV_FLUSH();
            return;
        }
        if (w == 2) {
            // PUBLISHER: step s of the band parked lane 63's value, the last row at column s - 63,
            // in ring slot s % kRing; store the columns of every step the compute wave has posted
            if ((int)band0 + 1 >= B) return;   // the last band has no consumer
            gu64* const dst = hand_pair + (uint64_t)band0 * P.max_n;
            const int total_steps = n + kWave - 1;
            int done = 0;
            while (done < total_steps) {
                const int avail = min(total_steps, __hip_atomic_load(&s_sync[3], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                if (avail <= done) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                SA_EV(1, avail >= kEvCol + 72);
                for (int s0 = done; s0 < avail; s0 += kWave) {
                    const int st = s0 + lane;
                    const int col = st - (kWave - 1);
                    if (st < avail && col >= 0) {
                        __hip_atomic_store(dst + col, (1ull << 32) | (uint32_t)s_pring[st & (kRing - 1)],
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if constexpr (AFF)
                            __hip_atomic_store(dst + P.hand_x_off + col,
                                               (1ull << 32) | (uint32_t)s_pring[kRing + (st & (kRing - 1))],
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                done = avail;
                SA_EV(2, avail >= kEvCol + 72);
                __hip_atomic_store(&s_sync[4], done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            SA_EV_FLUSH();
            return;
        }
    }

    uint8_t* const dslot = P.dirs + (uint64_t)slot * P.dir_slot;
    int32_t* const rb_h = P.rowbuf + (uint64_t)slot * P.rowbuf_slot;
    // affine: [M rows][Ix rows], the halves of the slot
    int32_t* const rb_x = rb_h + P.rowbuf_slot / 2;
    // CMAX (the end-cell replay) and BU (the units of a pair run concurrently) keep every band's
    // top row (row buffer = bands x max_n per component); otherwise one row is reused
    const uint64_t rbs = (CMAX || BU) ? P.max_n : 0;
    typedef uint32_t __attribute__((address_space(1))) gu32;
    gu32* const rb_g = (gu32*)rb_h;   // BU: the granules

    // Per-lane state for the current band.
    int a[R];      // Seq1 symbols of my rows
    uint32_t mwin[BITS ? R : 1];   // BITS: match bits of my rows at this chunk's 32 columns
    int Hp[R];     // H (or M) of my rows at the previous column
    int Yp[R];     // Iy of my rows at the previous column (affine)
    int bh[R];     // best per row: key (KEYED) or score
    int bj[R];     // its column (0-based), !KEYED
    uint32_t cml = 0;  // CMAX: the lane's maximum over the current chunk (4H >= 0)
    // CMAX: the lane's best chunk of the band so far as one key H << 12 | chunk + 1 (H < 2^13 by
    // t16_ok, chunks < 4096 since n < 65535): highest score, then last chunk
    uint32_t lkey = 0;
    uint32_t smax = 0;   // SO: the lane's largest tracked cell (the wave's: a lower bound of S)
    int hl = 0, xl = 0, sym = 0, prev_up = 0;
    int row0 = 0;
    // Running best of this lane over its bands: (score, i, j), 1-based cell.
    int best_h = INT_MIN, best_i = 0, best_j = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) { a[r] = 0; Hp[r] = 0; Yp[r] = 0; bh[r] = 0; bj[r] = 0; }

    // One step: lane computes column j = s - lane for its R rows.  STEADY: every lane is in
    // range, no exec-mask branch.  Returns the packed record words in rec.
    uint32_t kprev[R];   // T16 steady chunks: the previous step's keys, merged pairwise by v_max3
    // where step q of the current chunk reads lane 0's row-above inputs: the step buffer, or for a
    // SPLIT band > 0 the poller's ring at the chunk's first column
    const int32_t* in_h = s_step;
    const int32_t* in_x = s_step + 32;
    // where step q parks lane 63's last-row values (the other lanes write a discard slot)
    int32_t* park_h = s_park;
    int32_t* park_x = s_park + 32;
    // vh / vx / vs: lane 0's row-above inputs (H, Ix) and the column symbol of this step
    // Step modes (kStepAny: any lane may be outside the matrix, per-lane branch; kStepSteady: every
    // lane inside; kStepStart, T16 local CMAX only: the band's first chunks, where lanes left of
    // their first column run the cell on garbage and are reset to the matrix border at it -- no
    // per-lane branch, so a lone SPLIT wave's first granule is not slowed by the band's start)
    auto step = [&](auto mode, int q, int s, int vh, int vx, int vs, uint32_t (&rec)[RW], auto phase) {
        constexpr int MODE = (int)decltype(mode)::value;
        constexpr bool STEADY = MODE == kStepSteady;
        constexpr bool START = MODE == kStepStart;
        // T16 records narrower than a word: pushed straight into the packet word (acc_rec); SO
        // pushes every step of every mode (a lane-step outside the matrix leaves a stale value in
        // the edge stream, which the traceback never reads)
        constexpr bool ACC = T16 && RB < 32 && (MODE != kStepAny || SO);
        constexpr int PH = decltype(phase)::value;   // the step's index in its chunk, mod 4
        constexpr bool ODD = (PH & 1) != 0;
        const int up_h = shr1(vh, hl);
        int up_x = 0;
        if constexpr (AFF) up_x = shr1(vx, xl);
        sym = shr1(vs, sym);
        const int j = s - lane;
        // T16: the v_alignbit pushes shift every bit a word held out of it, and a lane-step outside
        // the matrix only fills its own (never read) record bytes -- except a narrow record of
        // kStepAny, ORed into its packet word unshifted when the lane-step is outside: zeroed
        if constexpr (!T16 || (RB < 32 && !ACC) || (RB > 32 && RB % 32 != 0)) {
#pragma unroll
            for (int e = 0; e < RW; ++e) rec[e] = 0;
        }
        if (STEADY || START || (unsigned)j < (unsigned)n) {
            const int jkey = j + 1;      // 1-based column, < 2^16 when KEYED
            if constexpr (START) {
                // this lane's first column: the left border (H = 0, Iy = border) and the
                // diagonal of its first row (H[i-1][0] = 0); the chunk maximum restarts
                const bool f = j == 0;
                prev_up = f ? 0 : prev_up;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    Hp[r] = f ? 0 : Hp[r];
                    if constexpr (AFF) Yp[r] = f ? XB : Yp[r];
                }
                cml = f ? 0u : cml;
            }
            int hd = prev_up;            // H[i-1][j-1] of my first row
            int hu = up_h;               // H[i-1][j]
            int xu = up_x;               // Ix[i-1][j]
            uint32_t dcur = 0;           // T16: tagged diagonal candidate of the current row
            if constexpr (T16) {
                asm("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0"
                    : "=&v"(dcur) : "v"(a[0]), "v"(sym), "v"(hd));
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                uint32_t& rw = rec[r / RPW];
                int Hc;
                if constexpr (SO && AFF) {
                    // Score-only affine cell (SALocalGotoh.h:108-130, SAGlobalGotoh.h:98-126), no tags.
                    // Registers hold A = Ix - (GO + GE) (down the rows: xu) and B = Iy - (GO + GE) (Yp):
                    //   A = max(Mu, Au + GE), B = max(Ml, Bl + GE), M = max(D, max(A, B) + GO + GE)
                    // (LocalGotoh: max(., 0) of the second term by unsigned saturation: A, B >= M >= 0),
                    // D = Md + s from the profile: 8 fast 16-bit ops + v_bfe_i32, against 16 for the
                    // tagged cell.
#define SA_SOA_HEAD                                                                                \
    "v_add_u16 %[xa], %[cge], %[xu]\n\t"                                                            \
    "v_add_u16 %[yb], %[cge], %[yp]\n\t"                                                            \
    "v_max_i16 %[xa], %[hu], %[xa]\n\t"                                                             \
    "v_max_i16 %[yp], %[hp], %[yb]\n\t"
#define SA_SOA_NEXT "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\tv_add_u16 %[dn], %[hp], %[dn]\n\t"
#define SA_SOA_TAIL_L "v_max_i16 %[t], %[xa], %[yp]\n\tv_sub_u16_e64 %[t], %[t], %[cgoe] clamp\n\tv_max_i16 %[hp], %[dr], %[t]"
#define SA_SOA_TAIL_G "v_max_i16 %[t], %[xa], %[yp]\n\tv_add_u16 %[t], %[cgoe], %[t]\n\tv_max_i16 %[hp], %[dr], %[t]"
#define SA_SOA_OUT [xa] "=&v"(xa), [yb] "=&v"(yb), [t] "=&v"(tt), [hp] "+v"(Hp[r]), [yp] "+v"(Yp[r])
#define SA_SOA_IN [dr] "v"(dcur), [hu] "v"(hu), [xu] "v"(xu), [cge] "s"(CGE), [cgoe] "s"(CGOE)
                    uint32_t xa, yb, tt;
                    if (r + 1 < R) {
                        uint32_t dn;
                        const uint32_t tabn = (uint32_t)a[r + 1 < R ? r + 1 : r];
                        if constexpr (LOCAL)
                            asm(SA_SOA_HEAD SA_SOA_NEXT SA_SOA_TAIL_L : SA_SOA_OUT, [dn] "=&v"(dn)
                                : SA_SOA_IN, [tabn] "v"(tabn), [sym] "v"(sym));
                        else
                            asm(SA_SOA_HEAD SA_SOA_NEXT SA_SOA_TAIL_G : SA_SOA_OUT, [dn] "=&v"(dn)
                                : SA_SOA_IN, [tabn] "v"(tabn), [sym] "v"(sym));
                        dcur = dn;
                    } else {
                        if constexpr (LOCAL) asm(SA_SOA_HEAD SA_SOA_TAIL_L : SA_SOA_OUT : SA_SOA_IN);
                        else asm(SA_SOA_HEAD SA_SOA_TAIL_G : SA_SOA_OUT : SA_SOA_IN);
                    }
#undef SA_SOA_HEAD
#undef SA_SOA_NEXT
#undef SA_SOA_TAIL_L
#undef SA_SOA_TAIL_G
#undef SA_SOA_OUT
#undef SA_SOA_IN
                    (void)yb;
                    if constexpr (CMAX) {   // the lane's chunk maximum of M (>= 0), one v_max3_u32 per two rows
                        if (r & 1)
                            asm("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r >= 1 ? r - 1 : 0]), "v"(Hp[r]));
                    }
                    xu = (int)xa;
                    Hc = Hp[r];
                } else if constexpr (T16 && AFF) {
                    // One asm block per cell (see the header): Ix and Iy terms, M's max, the three
                    // record pushes and strips, the next row's diagonal candidate from Hp[r] before
                    // Hp[r] is updated, and (LocalGotoh) the (M, column) key: Hp = 8M, so
                    // Hp << 13 == M << 16.
                    uint32_t t0, t1, xr, yr, xs;
                    const uint32_t jk = (uint32_t)jkey;
#define SA_T16A_HEAD_L "v_sub_u16_e64 %[t0], %[hu], %[cxo] clamp\n\t"
#define SA_T16A_HEAD_G "v_add_u16 %[t0], %[cxo], %[hu]\n\t"
#define SA_T16A_GAPS                                                                          \
    "v_add_u16 %[t1], %[cyo], %[hp]\n\t"                                                       \
    "v_add_u16 %[xr], %[cxe], %[xu]\n\t"                                                       \
    "v_add_u16 %[yr], %[cxe], %[yp]\n\t"                                                       \
    "v_max_i16 %[xr], %[t0], %[xr]\n\t"                                                        \
    "v_max_i16 %[yr], %[t1], %[yr]\n\t"
#define SA_T16A_MN                                                                            \
    "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\t"                                                  \
    "v_max_i16 %[t0], %[dr], %[xr]\n\t"                                                        \
    "v_add_u16 %[dn], %[hp], %[dn]\n\t"                                                        \
    "v_max_i16 %[t0], %[yr], %[t0]\n\t"
#define SA_T16A_M "v_max_i16 %[t0], %[dr], %[xr]\n\tv_max_i16 %[t0], %[yr], %[t0]\n\t"
#define SA_T16A_TAIL                                                                          \
    "v_alignbit_b32 %[rec], %[xr], %[rec], 1\n\t"                                              \
    "v_and_b32 %[xs], -2, %[xr]\n\t"                                                           \
    "v_alignbit_b32 %[rec], %[yr], %[rec], 1\n\t"                                              \
    "v_and_b32 %[yp], -2, %[yr]\n\t"                                                           \
    "v_alignbit_b32 %[rec], %[t0], %[rec], 6\n\t"                                              \
    "v_and_b32 %[hp], -8, %[t0]\n\t"
#define SA_T16A_KEY "v_lshl_or_b32 %[t1], %[hp], 13, %[jk]\n\tv_max_u32 %[bh], %[bh], %[t1]\n\t"
#define SA_T16A_OUT [t0] "=&v"(t0), [t1] "=&v"(t1), [xr] "=&v"(xr), [yr] "=&v"(yr), [xs] "=&v"(xs), \
                    [hp] "+v"(Hp[r]), [yp] "+v"(Yp[r]), [rec] "+v"(rw)
#define SA_T16A_IN [dr] "v"(dcur), [hu] "v"(hu), [xu] "v"(xu), [cxo] "s"(CXO), [cxe] "s"(CXE), [cyo] "s"(CYO)
                    if (r + 1 < R) {
                        uint32_t dn;
                        const uint32_t tabn = (uint32_t)a[r + 1 < R ? r + 1 : r];
                        if constexpr (LOCAL && CMAX)
                            asm(SA_T16A_HEAD_L SA_T16A_GAPS SA_T16A_MN SA_T16A_TAIL
                                : SA_T16A_OUT, [dn] "=&v"(dn)
                                : SA_T16A_IN, [tabn] "v"(tabn), [sym] "v"(sym));
                        else if constexpr (LOCAL)
                            asm(SA_T16A_HEAD_L SA_T16A_GAPS SA_T16A_MN SA_T16A_TAIL SA_T16A_KEY
                                : SA_T16A_OUT, [dn] "=&v"(dn), [bh] "+v"(bh[r])
                                : SA_T16A_IN, [tabn] "v"(tabn), [sym] "v"(sym), [jk] "v"(jk));
                        else
                            asm(SA_T16A_HEAD_G SA_T16A_GAPS SA_T16A_MN SA_T16A_TAIL
                                : SA_T16A_OUT, [dn] "=&v"(dn)
                                : SA_T16A_IN, [tabn] "v"(tabn), [sym] "v"(sym));
                        dcur = dn;
                    } else {
                        if constexpr (LOCAL && CMAX)
                            asm(SA_T16A_HEAD_L SA_T16A_GAPS SA_T16A_M SA_T16A_TAIL : SA_T16A_OUT : SA_T16A_IN);
                        else if constexpr (LOCAL)
                            asm(SA_T16A_HEAD_L SA_T16A_GAPS SA_T16A_M SA_T16A_TAIL SA_T16A_KEY
                                : SA_T16A_OUT, [bh] "+v"(bh[r])
                                : SA_T16A_IN, [jk] "v"(jk));
                        else
                            asm(SA_T16A_HEAD_G SA_T16A_GAPS SA_T16A_M SA_T16A_TAIL : SA_T16A_OUT : SA_T16A_IN);
                    }
#undef SA_T16A_HEAD_L
#undef SA_T16A_HEAD_G
#undef SA_T16A_GAPS
#undef SA_T16A_MN
#undef SA_T16A_M
#undef SA_T16A_TAIL
#undef SA_T16A_KEY
#undef SA_T16A_OUT
#undef SA_T16A_IN
                    if constexpr (CMAX) {   // the lane's chunk maximum (8M >= 0), as for SW below
                        if (r & 1)
                            asm("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r >= 1 ? r - 1 : 0]), "v"(Hp[r]));
                    }
                    xu = (int)xs;
                    Hc = Hp[r];
                } else if constexpr (SO && ALG == SA_NW) {
                    // Score-only NW cell (Hp = H - delta, no tags, no clamp): both gap candidates
                    // share G, so max(U + G, L + G) = max(U, L) + G; the cell is max(D, that), the
                    // next row's diagonal Hp_old + s from the profile (SANeedlemanWunsch.h:69-86)
                    uint32_t t1;
                    if (r + 1 < R) {
                        uint32_t dn;
                        const uint32_t tabn = (uint32_t)a[r + 1 < R ? r + 1 : r];
                        asm("v_max_i16 %[t1], %[hu], %[hp]\n\t"
                            "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\t"
                            "v_add_u16 %[dn], %[hp], %[dn]\n\t"
                            "v_add_u16 %[t1], %[cg], %[t1]\n\t"
                            "v_max_i16 %[hp], %[dr], %[t1]"
                            : [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                            : [dr] "v"(dcur), [hu] "v"(hu), [cg] "s"(CL), [tabn] "v"(tabn), [sym] "v"(sym));
                        dcur = dn;
                    } else {
                        asm("v_max_i16 %[t1], %[hu], %[hp]\n\t"
                            "v_add_u16 %[t1], %[cg], %[t1]\n\t"
                            "v_max_i16 %[hp], %[dr], %[t1]"
                            : [t1] "=&v"(t1), [hp] "+v"(Hp[r])
                            : [dr] "v"(dcur), [hu] "v"(hu), [cg] "s"(CL));
                    }
                    Hc = Hp[r];
                } else if constexpr (SO) {
                    // Score-only cell (Hp = H, no tags).  Both gap candidates share G: max(U + G,
                    // L + G, 0) = max(U, L) - (-G) with unsigned saturation (U, L = H >= 0, so the zero
                    // clamp is free), and the cell is max(D, sat(max(U, L) - CU)): 4 fast-class 16-bit
                    // ops + v_bfe_i32 for the next row's diagonal Hp_old + s from the profile.  No
                    // single fast-class op does the 4-symbol lookup (round 5, tools/microbench_ops3.hip:
                    // v_perm / dot4 / sdwa forms issue at the v_bfe rate or slower).
                    uint32_t t1;
                    if (r + 1 < R) {
                        uint32_t dn;
                        const uint32_t tabn = (uint32_t)a[r + 1 < R ? r + 1 : r];
                        asm("v_max_i16 %[t1], %[hu], %[hp]\n\t"
                            "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\t"
                            "v_add_u16 %[dn], %[hp], %[dn]\n\t"
                            "v_sub_u16_e64 %[t1], %[t1], %[cu] clamp\n\t"
                            "v_max_i16 %[hp], %[dr], %[t1]"
                            : [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                            : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [tabn] "v"(tabn), [sym] "v"(sym));
                        dcur = dn;
                    } else {
                        asm("v_max_i16 %[t1], %[hu], %[hp]\n\t"
                            "v_sub_u16_e64 %[t1], %[t1], %[cu] clamp\n\t"
                            "v_max_i16 %[hp], %[dr], %[t1]"
                            : [t1] "=&v"(t1), [hp] "+v"(Hp[r])
                            : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU));
                    }
                    (void)CL;
                    // The lane's chunk maximum (H >= 0, one v_max3_u32 per two tracked cells).  Steady
                    // chunks track only the rows 3 mod 4 at the steps 3 mod 4: every cell (i, j) of
                    // the chunk has the tracked cell (i | 3, j | 3) of the same lane and chunk, and a
                    // cell is at most its right / lower neighbour - G (their left / up candidates), so
                    // H(i, j) <= tracked - kSoSlack G (kSoSlack = 6): the lane's true maximum is at most
                    // cml - 6G and the end-cell replay (endcell_so_kernel) recomputes every lane block
                    // that could hold S.  Ramp chunks (columns past the matrix edge) track every cell.
                    if constexpr (STEADY) {
                        if constexpr (R >= 8) {
                            if (PH == 3 && (r & 7) == 7)
                                asm("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r >= 4 ? r - 4 : 0]), "v"(Hp[r]));
                        } else if (PH == 3 && (r & 3) == 3) {
                            asm("v_max_u32 %0, %0, %1" : "+v"(cml) : "v"(Hp[r]));
                        }
                    } else if (r & 1) {
                        asm("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r >= 1 ? r - 1 : 0]), "v"(Hp[r]));
                    }
                    Hc = Hp[r];
                } else if constexpr (T16) {
                    // One asm block per cell (plain VALU->VALU dependences need no wait
                    // states; the compiler pads s_nop between separate asm statements).  The
                    // block also forms the NEXT row's diagonal candidate from Hp[r] before
                    // updating Hp[r] in place, so no register copies are needed.  Its
                    // substitution term is v_bfe_i32 of the row's 4-byte profile at 8 x the
                    // column's symbol code (an SDWA byte select from a per-step LDS column profile
                    // is one instruction fewer but measured slower: tools/microbench_cellmix.hip).
                    uint32_t t0, t1;
                    // R >= 32: the row-max key update (lshl_or + max_u32, in place) joins the
                    // block -- separate statements would cost s_nops and register renaming.
                    constexpr bool KIN = LOCAL && R >= 32 && !CMAX;
                    const uint32_t jk = (uint32_t)jkey;
#define SA_T16_LEFT "v_add_u16 %[t0], %[cl], %[hp]\n\t"
#define SA_T16_UPC "v_sub_u16_e64 %[t1], %[hu], %[cu] clamp\n\t"
#define SA_T16_UP "v_add_u16 %[t1], %[cu], %[hu]\n\t"
#define SA_T16_MAX                                                                           \
    "v_max_i16 %[t0], %[dr], %[t0]\n\t"                                                      \
    "v_max_i16 %[t0], %[t1], %[t0]\n\t"
#define SA_T16_NEXT                                                                          \
    "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\t"                                                \
    "v_add_u16 %[dn], %[hp], %[dn]\n\t"
#define SA_T16_TAIL                                                                          \
    "v_and_b32 %[hp], -4, %[t0]\n\t"                                                         \
    "v_alignbit_b32 %[rec], %[t0], %[rec], %[bpc]\n\t"
#define SA_T16_KEY                                                                           \
    "v_lshl_or_b32 %[t1], %[hp], 14, %[jk]\n\t"                                              \
    "v_max_u32 %[bh], %[bh], %[t1]\n\t"
#define SA_T16_OUT [t0] "=&v"(t0), [t1] "=&v"(t1), [hp] "+v"(Hp[r]), [rec] "+v"(rw)
#define SA_T16_IN [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL), [bpc] "i"(BPC)
#define SA_T16_PW [tabn] "v"(tabn), [sym] "v"(sym)
                    if (r + 1 < R) {
                        uint32_t dn;
                        const uint32_t tabn = (uint32_t)a[r + 1 < R ? r + 1 : r];
                        if constexpr (KIN)
                            asm(SA_T16_LEFT SA_T16_NEXT SA_T16_UPC SA_T16_MAX SA_T16_TAIL SA_T16_KEY
                                : SA_T16_OUT, [dn] "=&v"(dn), [bh] "+v"(bh[r])
                                : SA_T16_IN, SA_T16_PW, [jk] "v"(jk));
                        else if constexpr (LOCAL)
                            asm(SA_T16_LEFT SA_T16_NEXT SA_T16_UPC SA_T16_MAX SA_T16_TAIL
                                : SA_T16_OUT, [dn] "=&v"(dn)
                                : SA_T16_IN, SA_T16_PW);
                        else
                            asm(SA_T16_LEFT SA_T16_NEXT SA_T16_UP SA_T16_MAX SA_T16_TAIL
                                : SA_T16_OUT, [dn] "=&v"(dn)
                                : SA_T16_IN, SA_T16_PW);
                        dcur = dn;
                    } else {
                        if constexpr (KIN)
                            asm(SA_T16_LEFT SA_T16_UPC SA_T16_MAX SA_T16_TAIL SA_T16_KEY
                                : SA_T16_OUT, [bh] "+v"(bh[r]) : SA_T16_IN, [jk] "v"(jk));
                        else if constexpr (LOCAL)
                            asm(SA_T16_LEFT SA_T16_UPC SA_T16_MAX SA_T16_TAIL : SA_T16_OUT : SA_T16_IN);
                        else
                            asm(SA_T16_LEFT SA_T16_UP SA_T16_MAX SA_T16_TAIL : SA_T16_OUT : SA_T16_IN);
                    }
                    if constexpr (CMAX) {
                        // the lane's chunk maximum: one v_max3_u32 per two rows instead of a
                        // v_max_i16 per cell (tools/microbench_cellmix.hip V8 vs V2)
                        if (r & 1)
                            asm("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r >= 1 ? r - 1 : 0]), "v"(Hp[r]));
                    }
#undef SA_T16_UPC
#undef SA_T16_LEFT
#undef SA_T16_UP
#undef SA_T16_MAX
#undef SA_T16_TAIL
#undef SA_T16_NEXT
#undef SA_T16_KEY
#undef SA_T16_OUT
#undef SA_T16_IN
#undef SA_T16_PW
                    Hc = Hp[r];
                } else {
                bool v;
                if constexpr (BITS) v = (mwin[r] >> q) & 1u;
                else v = match_bit<LUT>(s_lut, a[r], sym);
                int D;
                if constexpr (ALLOW) D = hd + (v ? MA : MI);
                else D = v ? hd + MA : INT_MIN;
                if constexpr (BPC > FBITS) rw <<= BPC - FBITS;   // record padding (R <= 2)
                if constexpr (!AFF) {
                    const int U = hu + G;
                    const int L = Hp[r] + G;
                    int H = imax(imax(D, U), L);
                    if constexpr (LOCAL) H = imax(H, 0);
                    rw = push_eq(rw, H, D);   // fD
                    // BITS: the second bit is the match bit when fD is set (the traceback's diag
                    // move then needs no symbols), fU otherwise
                    if constexpr (BITS) rw = push_bit(rw, H == D ? v : H == U);
                    else rw = push_eq(rw, H, U);   // fU
                    Hc = H;
                } else {
                    const int XE = xu + GE;
                    const int X = imax(hu + GOE, XE);
                    const int YE = Yp[r] + GE;
                    const int Y = imax(Hp[r] + GOE, YE);
                    int M = imax(imax(D, X), Y);
                    if constexpr (LOCAL) M = imax(M, 0);
                    rw = push_eq(rw, M, D);   // fD
                    if constexpr (BITS) rw = push_bit(rw, M == D ? v : M == X);   // fX, or v under fD
                    else rw = push_eq(rw, M, X);   // fX
                    rw = push_eq(rw, X, XE);  // fXe: Ix extends
                    rw = push_eq(rw, Y, YE);  // fYe: Iy extends
                    Yp[r] = Y;
                    xu = X;
                    Hc = M;
                }
                }
                if constexpr (LOCAL) {
                    if constexpr (CMAX || (T16 && (R >= 32 || AFF))) {
                        // chunk max / key already updated by the cell's asm block
                    } else if constexpr (T16 && STEADY) {
                        // Hc = 4H with clear tag bits, so Hc << 14 == H << 16.  Two steps' keys
                        // per v_max3, in place (lets the compiler keep bh[] in fixed registers).
                        const uint32_t k = ((uint32_t)Hc << 14) | (uint32_t)jkey;
                        if constexpr (!ODD) kprev[r] = k;
                        else asm("v_max3_u32 %0, %0, %1, %2" : "+v"(bh[r]) : "v"(kprev[r]), "v"(k));
                    } else if constexpr (KEYED) {
                        bh[r] = (int)max((uint32_t)bh[r], ((uint32_t)Hc << (T16 ? 14 : 16)) | (uint32_t)jkey);
                    } else {
                        if (Hc >= bh[r]) { bh[r] = Hc; bj[r] = j; }
                    }
                }
                if constexpr (!T16) {
                    hd = Hp[r];
                    Hp[r] = Hc;
                }
                hu = Hc;
            }
            prev_up = up_h;
            hl = Hp[R - 1];
            if constexpr (AFF) xl = xu;
            if constexpr (T16 && RB < 32 && !ACC) rec[0] >>= (32 - RB);   // alignbit filled from the top
        }
        // SO: the step's record is the lane's last row, pushed into the packet word from the top
        // (two steps per word)
        if constexpr (SO && AFF) rec[0] = __builtin_amdgcn_perm((uint32_t)xl, (uint32_t)hl, 0x05040100u);   // M | A << 16
        else if constexpr (SO) rec[0] = __builtin_amdgcn_alignbit((uint32_t)hl, rec[0], 16u);
    };

    // SPLIT compute wave, before the group of SG steps at step q of the chunk at kC: back-pressure
    // from the publisher (the park ring slots of the next kHandGran steps held steps kRing earlier),
    // then, band > 0, the group's lane-0 inputs.  T16 ring entries carry their granule number, so
    // a whole group inside the matrix is read and checked in one LDS round trip (re-read while
    // stale); otherwise the poller's column count is awaited first.
    int have = 0, pubd = 0;
    auto split_inputs = [&](int band, int kC, int q, auto sg, int* gh, int* gx, int* gs) {
        constexpr int G_ = decltype(sg)::value;
        if constexpr (SPLIT) {
            if (q % kHandGran == 0 && band + 1 < B && pubd < kC + q + kHandGran - kRing) {
                do {
                    pubd = __hip_atomic_load(&s_sync[4], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (pubd >= kC + q + kHandGran - kRing) break;
                    __builtin_amdgcn_s_sleep(1);
                } while (true);
            }
            const bool tagged = T16 && band > 0 && kC + q + G_ <= n;
            if (band > 0 && !tagged) {
                const int need = min(n, kC + q + G_);
                if (have < need) {
                    have = __hip_atomic_load(&s_sync[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (have < need) {
#ifdef SA_TB_STATS
                        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#endif
                        do {
                            __builtin_amdgcn_s_sleep(1);
                            have = __hip_atomic_load(&s_sync[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        } while (have < need);
#ifdef SA_TB_STATS
                        st_wait += __builtin_amdgcn_s_memrealtime() - t0;
#endif
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < G_; ++k) {
                gh[k] = in_h[q + k];
                gs[k] = s_step[64 + q + k];
                if constexpr (AFF) gx[k] = in_x[q + k];
            }
            if constexpr (T16) {
                if (tagged) {
                    const uint32_t want = ((uint32_t)(kC + q) / kHandGran + 1u) << 16;
                    auto fresh = [&]() {
                        uint32_t mn = (uint32_t)gh[0];
#pragma unroll
                        for (int k = 1; k < G_; ++k) mn = min(mn, (uint32_t)gh[k]);
                        if constexpr (AFF) {
#pragma unroll
                            for (int k = 0; k < G_; ++k) mn = min(mn, (uint32_t)gx[k]);
                        }
                        return mn >= want;
                    };
                    if (!fresh()) {
#ifdef SA_TB_STATS
                        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#endif
                        do {
                            // the poller's bounded wait expired: go on (the pair is re-run)
                            if (__hip_atomic_load(&s_sync[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                            __builtin_amdgcn_s_sleep(1);
#pragma unroll
                            for (int k = 0; k < G_; ++k) {
                                gh[k] = __hip_atomic_load(&in_h[q + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                if constexpr (AFF) gx[k] = __hip_atomic_load(&in_x[q + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            }
                        } while (!fresh());
#ifdef SA_TB_STATS
                        st_wait += __builtin_amdgcn_s_memrealtime() - t0;
#endif
                    }
                }
            }
        }
    };
    // One chunk of kChunk steps of one band.
    auto run_chunk = [&](auto steady, int band, int kC, int bch, int bcx, int symc, int& acc_h,
                         int& acc_x) {
        uint8_t* const dband = dslot + (uint64_t)band * P.band_stride;
#pragma unroll 1
        for (int q0 = 0; q0 < kChunk; q0 += SPP) {
            uint32_t pk[4 * PPS];
#pragma unroll
            for (int e = 0; e < 4 * PPS; ++e) pk[e] = 0;
            static_assert(SPP % 2 == 0 || !T16 || R >= 32 || AFF, "steps pair up for the key max3");
            // SPLIT (a lone wave, whose LDS read latency no other wave hides): a group of SG steps'
            // inputs is read into registers at once (broadcast reads), not one read per step
            constexpr int SG = SPP >= kHandGran ? kHandGran : SPP;
            int gh[SPLIT ? SG : 1], gx[SPLIT ? SG : 1], gs[SPLIT ? SG : 1];
#pragma unroll
            for (int g = 0; g < SPP; ++g) {
                const int q = q0 + g;
                int vh, vx = 0, vs;
                if constexpr (SPLIT) {
                    if (g % SG == 0) {
                        SA_EV(6, kC + q >= kEvCol);
                        split_inputs(band, kC, q, std::integral_constant<int, SG>{}, gh, gx, gs);
                        SA_EV(4, kC + q >= kEvCol);
                    }
                    vh = gh[g % SG];
                    vs = gs[g % SG];
                    if constexpr (AFF) vx = gx[g % SG];
                } else {
                    vh = in_h[q];
                    vs = s_step[64 + q];
                    if constexpr (AFF) vx = in_x[q];
                }
                constexpr bool ACC = T16 && RB < 32 && ((int)decltype(steady)::value != kStepAny || SO);
                if constexpr (ACC) {
                    // every lane pushes every step: the packet word fills from the top, step by
                    // step, into the same byte layout as the shifted-and-ORed records below
                    uint32_t(&acc_rec)[1] = *reinterpret_cast<uint32_t(*)[1]>(&pk[(g * BPS) / 4]);
                    switch (g & 3) {   // (g is unrolled: one case remains)
                        case 0: step(steady, q, kC + q, vh, vx, vs, acc_rec, std::integral_constant<int, 0>{}); break;
                        case 1: step(steady, q, kC + q, vh, vx, vs, acc_rec, std::integral_constant<int, 1>{}); break;
                        case 2: step(steady, q, kC + q, vh, vx, vs, acc_rec, std::integral_constant<int, 2>{}); break;
                        default: step(steady, q, kC + q, vh, vx, vs, acc_rec, std::integral_constant<int, 3>{}); break;
                    }
                } else {
                    uint32_t rec[RW];
                    switch (g & 3) {
                        case 0: step(steady, q, kC + q, vh, vx, vs, rec, std::integral_constant<int, 0>{}); break;
                        case 1: step(steady, q, kC + q, vh, vx, vs, rec, std::integral_constant<int, 1>{}); break;
                        case 2: step(steady, q, kC + q, vh, vx, vs, rec, std::integral_constant<int, 2>{}); break;
                        default: step(steady, q, kC + q, vh, vx, vs, rec, std::integral_constant<int, 3>{}); break;
                    }
                    if constexpr (BPS >= 4) {
#pragma unroll
                        for (int e = 0; e < RW; ++e) pk[g * RW + e] = rec[e];
                    } else {
                        pk[(g * BPS) / 4] |= rec[0] << (((g * BPS) % 4) * 8);
                    }
                }
                // lane 63 holds the band's last row at column kC + q - 63: park it in LDS (SPLIT: in
                // the park ring, posting the step count every kHandGran steps for the publisher)
                park_h[q] = hl;
                if constexpr (AFF) park_x[q] = xl;
                if constexpr (SPLIT) {
                    // (every lane stores the same count: no exec-mask switch)
                    if ((q + 1) % kHandGran == 0 && band + 1 < B) {
                        __hip_atomic_store(&s_sync[3], kC + q + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        SA_EV(0, kC + q + 1 >= kEvCol + 72);
                    }
                }
            }
            const uint64_t pkt0 = (uint64_t)((kC + q0) / SPP) * PPS;
#pragma unroll
            for (int pp = 0; pp < PPS; ++pp) {
                u32x4* dst = reinterpret_cast<u32x4*>(dband + ((pkt0 + pp) * kWave + lane) * 16);
                const u32x4 v4 = {pk[pp * 4 + 0], pk[pp * 4 + 1], pk[pp * 4 + 2], pk[pp * 4 + 3]};
                __builtin_nontemporal_store(v4, dst);
            }
        }
        // lane q < kChunk: the band's last row at column kC + q - 63
        acc_h = s_step[96 + (lane & 31)];
        if constexpr (AFF) acc_x = s_step[128 + (lane & 31)];
    };

    // Band -> band hand-off.  The last row of band b (H and, affine, Ix) goes to band b+1 through
    // an LDS ring of kRing columns owned by wave (b+1) % W — unless b+1 wraps round to wave 0
    // (more bands than waves), which uses the per-pair global row buffer.  Everything a steady
    // chunk reads is in LDS, so the only memory traffic of the chunk loop is the fire-and-forget
    // flag stores (no s_waitcnt vmcnt behind them).
    auto ring = [&](int wave, int comp) -> int32_t* {
        return s_ring + (wave * (AFF ? 2 : 1) + comp) * kRing;
    };
    // Lane q < kChunk of the returned registers holds column c0 + q: the row-above value for
    // lane 0 (top border, or the previous band's last row) and Seq2[c].
    auto load_chunk = [&](int band, int c0, int& vh, int& vx, int& vs) {
        const int c = c0 + lane;
        vh = 0; vx = XB; vs = 0;
        if (lane < kChunk && c < n) {
            if (P.stage_seq2) vs = (int)s_seq2[c];
            else vs = T16 ? (int)t16_code8(symp, s2[c]) : (int)s2[c];
            if (band == 0) {
                const int J = c + 1;
                if constexpr (ALG == SA_NW) vh = SC * (J * G - P.t16_delta);
                else if constexpr (ALG == SA_GLOBAL_GOTOH) vh = SC * (GO + J * GE - P.t16_delta);
            } else if constexpr (SPLIT) {
                // polled per granule group inside the chunk (split_sub)
            } else if constexpr (BU) {
                vh = (int)__hip_atomic_load(rb_g + (uint64_t)(band - 1) * rbs + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (band % W != 0) {
                vh = ring(band % W, 0)[c % kRing];
                if constexpr (AFF) vx = ring(band % W, 1)[c % kRing];
            } else {
                vh = rb_h[(uint64_t)(band - 1) * rbs + c];
                if constexpr (AFF) vx = rb_x[(uint64_t)(band - 1) * rbs + c];
            }
        }
        // SPLIT, band > 0: the lane-0 inputs are polled per granule group inside the chunk
        // (split_sub); the values written to s_step here are placeholders
        if constexpr (BU) {
            if (band > 0) {   // (uniform) the producer band's granules of this chunk, this launch's
                // (bounded, as the segment wait: after a lost producer the unit runs on without
                // waiting and the pair is flagged for the int32 re-run)
                const bool want = lane < kChunk && c < n;
                for (uint32_t it = 0; !seg_lost && __builtin_amdgcn_ballot_w64(want && ((uint32_t)vh & 0xffff0000u) != epoch16) != 0; ++it) {
                    if (it >= P.wait_polls) { seg_lost = 1; break; }
                    __builtin_amdgcn_s_sleep(2);
                    if (want)
                        vh = (int)__hip_atomic_load(rb_g + (uint64_t)(band - 1) * rbs + c, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
                }
                vh &= 0xffff;
            }
        }
    };

    for (uint32_t ph = BU ? c0 : 0u; ph < total; ++ph) {
        const int rel = (int)ph - w * kLagPhases;
        if (SPLIT || BU || rel >= 0) {
            const uint32_t k = (SPLIT || BU) ? 0u : (uint32_t)rel / period;
            const uint32_t chunk = (SPLIT || BU) ? ph : (uint32_t)rel - k * period;
            const int band = (SPLIT || BU) ? (int)band0 : w + (int)k * W;
            if (chunk < nch && band < B) {
                // ---------------------------------------------------------------- band start
                if (chunk == (BU ? c0 : 0u)) {
                    row0 = band * BAND + lane * R;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int row = row0 + r;
                        // CMAX: rows past m get substitution -128 (with gap < 0 their values stay
                        // below the matrix maximum, so they never win the lane's chunk maximum)
                        if constexpr (SO) a[r] = row < m ? (int)so_profile<AFF>(P.prof[t16_code8(symp, s1[row]) >> 3]) : (CMAX ? (int)0x80808080u : 0);
                        else if constexpr (T16) a[r] = row < m ? (int)P.prof[t16_code8(symp, s1[row]) >> 3] : (CMAX ? (int)0x80808080u : 0);
                        else a[r] = row < m ? (int)s1[row] : 0;
                        const int i = row + 1;
                        if constexpr (ALG == SA_NW) Hp[r] = SC * (i * G - P.t16_delta);
                        else if constexpr (ALG == SA_GLOBAL_GOTOH) Hp[r] = SC * (GO + i * GE - P.t16_delta);
                        else Hp[r] = 0;
                        Yp[r] = XB;
                        bh[r] = KEYED ? 0 : INT_MIN;
                        bj[r] = 0;
                    }
                    lkey = 0;
                    cml = 0;
                    have = 0;
                    // retire the row loads above here, once per band: left pending, they make the
                    // compiler wait vmcnt(0) at every chunk's loop entry, which also drains the
                    // record stores in flight (gfx9's vmcnt counts stores) -- a stall per chunk
                    // that a lone wave (SPLIT) cannot hide
                    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
                    if constexpr (ALG == SA_NW) prev_up = SC * (row0 * G - P.t16_delta);
                    else if constexpr (ALG == SA_GLOBAL_GOTOH) prev_up = SC * ((row0 == 0 ? 0 : GO + row0 * GE) - P.t16_delta);
                    else prev_up = 0;
                    if constexpr (BU) {
                        if (c0 > 0) {
                            // a later segment: this lane's R values and diagonal input at column
                            // 32 c0 - 1 - lane from the previous segment's unit (epoch-tagged, polled
                            // as the band granules are), its last-row value for the lane below and
                            // the column symbol the DPP shift hands it at the first step
                            const uint32_t* hs = P.seg_hand + (uint64_t)slot * P.seg_slot +
                                                 ((uint64_t)band * SEGS + seg - 1) * (R + 1) * kWave + lane;
                            uint32_t hv[R + 1];
                            auto rd = [&]() __attribute__((always_inline)) {
#pragma unroll
                                for (int r = 0; r <= R; ++r)
                                    hv[r] = __hip_atomic_load(hs + r * kWave, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            };
                            auto stale = [&]() __attribute__((always_inline)) -> bool {
                                bool st = false;
#pragma unroll
                                for (int r = 0; r <= R; ++r) st |= (hv[r] & 0xffff0000u) != epoch16;
                                return st;
                            };
                            rd();
                            // (bounded: a producer that never comes leaves the unit after
                            // wait_polls polls with the pair flagged for the int32 re-run)
                            for (uint32_t it = 0; !seg_lost && __builtin_amdgcn_ballot_w64(stale()) != 0; ++it) {
                                if (it >= P.wait_polls) { seg_lost = 1; break; }
                                __builtin_amdgcn_s_sleep(2);
                                rd();
                            }
#pragma unroll
                            for (int r = 0; r < R; ++r) Hp[r] = (int)(hv[r] & 0xffffu);
                            prev_up = (int)(hv[R] & 0xffffu);
                            hl = Hp[R - 1];
                            const int cs = (int)(c0 * kChunk) - 1 - lane;
                            sym = cs >= 0 && cs < n ? (P.stage_seq2 ? (int)s_seq2[cs] : (int)t16_code8(symp, s2[cs])) : 0;
                        }
                    }
                }
                // ---------------------------------------------------------------- one chunk
                const int kC = (int)chunk * kChunk;
                int bch, bcx, symc;
                load_chunk(band, kC, bch, bcx, symc);
                if (SPLIT && band > 0) {
                    // the poller may now refill the ring slots of the columns before kC
                    __hip_atomic_store(&s_sync[1], kC, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    in_h = s_ring + (kC & (kRing - 1));
                    in_x = s_ring + kRing + (kC & (kRing - 1));
                }
                if constexpr (SPLIT) {
                    park_h = lane == 63 ? s_pring + (kC & (kRing - 1)) : s_step + 160;
                    park_x = lane == 63 ? s_pring + kRing + (kC & (kRing - 1)) : s_step + 192;
                }
                if (lane < kChunk) {   // the chunk's per-step broadcast inputs (LDS-fed steps)
                    s_step[lane] = bch;
                    if constexpr (AFF) s_step[32 + lane] = bcx;
                    s_step[64 + lane] = symc;
                }
                if constexpr (BITS) {
                    // my rows' match bits at columns [kC - lane, kC - lane + 32): bit q = step q
                    const int c0 = kC - lane;
                    const uint32_t wn = ((uint32_t)n + 31u) >> 5;
                    const uint32_t* mrow = P.mbits + P.mbits_off[pidx];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int row = row0 + r;
                        uint32_t w = 0;
                        if (row < m && c0 < n && c0 > -32) {
                            const uint32_t* rp = mrow + (uint64_t)row * wn;
                            if (c0 >= 0) {
                                const uint32_t k = (uint32_t)c0 >> 5;
                                const uint32_t lo = rp[k], hi = k + 1 < wn ? rp[k + 1] : 0u;
                                w = __builtin_amdgcn_alignbit(hi, lo, (uint32_t)c0 & 31u);
                            } else {
                                w = rp[0] << (uint32_t)(-c0);
                            }
                        }
                        mwin[r] = w;
                    }
                }
                int acc_h = 0, acc_x = 0;
                const bool steady = kC >= kWave - 1 && kC + kChunk <= n;
                if constexpr (SPLIT) {
                    SA_EV(7, true);   // [7] chunk 0, [5] chunk 2 (the first steady one)
                    SA_EV(5, kC >= 64);
                    SA_EV(8, kC >= 64 + 32 * 8);   // chunk 10
                }
                if (steady) {
                    run_chunk(std::integral_constant<int, kStepSteady>{}, band, kC, bch, bcx, symc, acc_h, acc_x);
                } else if (T16 && LOCAL && CMAX && SPLIT && n >= kWave && kC < kWave - 1) {
                    // a band's first chunks (n >= 64: every lane reaches its first column inside
                    // them, so none starts from start-mode garbage in a kStepAny chunk).  SPLIT
                    // only: a third chunk body costs the many-pairs R = 32 kernel 31 VGPRs (138 ->
                    // 169, i.e. 3 -> 2 waves per SIMD and a 6 % slower headline fill), and its
                    // ramp chunks are hidden by the other waves anyway
                    if constexpr (T16 && LOCAL && CMAX && SPLIT)
                        run_chunk(std::integral_constant<int, kStepStart>{}, band, kC, bch, bcx, symc, acc_h, acc_x);
                } else {
                    run_chunk(std::integral_constant<int, kStepAny>{}, band, kC, bch, bcx, symc, acc_h, acc_x);
                }
                // hand the band's last row (columns kC-63 .. kC-32) to the next band
                if (band + 1 < B) {
                    const int cc = kC + lane - (kWave - 1);
                    if (lane < kChunk && cc >= 0 && cc < n) {
                        const int nw = (band + 1) % W;
                        if constexpr (SPLIT) {
                            // stored by the publisher wave from the park ring
                        } else if constexpr (BU) {
                            __hip_atomic_store(rb_g + (uint64_t)band * rbs + cc, epoch16 | ((uint32_t)acc_h & 0xffffu),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        } else if (nw != 0) {
                            ring(nw, 0)[cc % kRing] = acc_h;
                            if constexpr (AFF) ring(nw, 1)[cc % kRing] = acc_x;
                        } else {
                            rb_h[(uint64_t)band * rbs + cc] = acc_h;
                            if constexpr (AFF) rb_x[(uint64_t)band * rbs + cc] = acc_x;
                        }
                    }
                }
                // ------------------------------------------------ CMAX: chunk maxima, snapshot
                if constexpr (SNAP) {
                    const uint64_t e = (uint64_t)band * P.snap_nch + chunk;
                    if constexpr (!CMAX) {
                        // (SO NW: snapshots only)
                    } else if constexpr (SOMAX) {
                        // per (band, chunk, lane): the lane's maximum of its tracked cells -- the
                        // end-cell replay then recomputes only the lane blocks that may hold S
                        if (kC + kChunk - 1 < lane) cml = 0;   // (a lane that has not reached its first column)
                        P.snap_m[(uint64_t)slot * P.snap_p_slot + e * kWave + lane] = (int32_t)cml;
                        smax = max(smax, cml);   // (per lane; reduced over the wave at the end)
                        // the wave's maximum of the chunk (DPP row prefix maxima, then the row
                        // broadcasts: lane 63 holds it), for the end-cell replay's first-level scan
                        uint32_t wm = cml;
                        wm = max(wm, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0x111, 0xf, 0xf, false));
                        wm = max(wm, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0x112, 0xf, 0xf, false));
                        wm = max(wm, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0x114, 0xf, 0xf, false));
                        wm = max(wm, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0x118, 0xf, 0xf, false));
                        wm = max(wm, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0x142, 0xa, 0xf, false));
                        wm = max(wm, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0x143, 0xc, 0xf, false));
                        if (lane == kWave - 1) P.snap_c[(uint64_t)slot * P.part_bands * P.snap_nch + e] = (int32_t)wm;
                    } else {
                        // (start mode: a lane that has not reached its first column holds garbage)
                        if (kC + kChunk - 1 < lane) cml = 0;
                        P.snap_m[(uint64_t)slot * P.snap_p_slot + e * kWave + lane] = (int32_t)cml;
                        lkey = max(lkey, (cml >> CSH) << 12 | (chunk + 1));
                    }
                    cml = 0;
                    if (chunk + 1 < nch) {   // state entering chunk + 1, for the end-cell replay
                        // R 16-bit values (affine: then the R Iy values and the last row's Ix)
                        constexpr int SW = AFF ? R + 1 : R / 2;
                        // word-major ([chunk][word][lane]): every store is one coalesced 256 B row
                        uint32_t* sh = P.snap_h + (uint64_t)slot * P.snap_h_slot + e * SW * kWave + lane;
#pragma unroll
                        for (int q = 0; q < R / 2; ++q)
                            sh[q * kWave] = ((uint32_t)Hp[2 * q] & 0xffffu) | ((uint32_t)Hp[2 * q + 1] << 16);
                        if constexpr (AFF) {
#pragma unroll
                            for (int q = 0; q < R / 2; ++q)
                                sh[(R / 2 + q) * kWave] = ((uint32_t)Yp[2 * q] & 0xffffu) | ((uint32_t)Yp[2 * q + 1] << 16);
                            sh[R * kWave] = (uint32_t)xl;
                        }
                        P.snap_p[(uint64_t)slot * P.snap_p_slot + e * kWave + lane] = prev_up;
                    }
                }
                if constexpr (BU) {
                    if (chunk + 1 == c1 && c1 < nch) {   // hand this lane's state on to the next segment
                        uint32_t* hs = P.seg_hand + (uint64_t)slot * P.seg_slot +
                                       ((uint64_t)band * SEGS + seg) * (R + 1) * kWave + lane;
#pragma unroll
                        for (int r = 0; r < R; ++r)
                            __hip_atomic_store(hs + r * kWave, epoch16 | ((uint32_t)Hp[r] & 0xffffu), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(hs + R * kWave, epoch16 | ((uint32_t)prev_up & 0xffffu), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                // ---------------------------------------------------------------- band end
                if (chunk == nch - 1) {
                    if constexpr (CMAX) {
                        // (score, lane, chunk): best_i names the lane by its last row; the end-cell
                        // replay (sa_endcell.hip) finds the row and the column
                        const int h = (int)(lkey >> 12);
                        if (lkey != 0 && h >= best_h) {
                            best_h = h;
                            best_i = row0 + R;
                            best_j = (int)(lkey & 4095u);
                        }
                    } else if constexpr (LOCAL) {
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            int h, jj;
                            if constexpr (KEYED || CMAX) { h = (int)((uint32_t)bh[r] >> 16); jj = bh[r] & 0xffff; }
                            else { h = bh[r]; jj = bj[r] + 1; }
                            if (row0 + r < m && h >= best_h) {
                                best_h = h;
                                best_i = row0 + r + 1;
                                best_j = jj;
                            }
                        }
                    } else {
                        const int last = m - 1;
                        if (band == last / BAND && lane == (last % BAND) / R) {
                            const int rr = last % R;
                            int v = 0;
#pragma unroll
                            for (int r = 0; r < R; ++r) v = (r == rr) ? Hp[r] : v;
                            s_score = T16 ? ((int)(int16_t)(v & 0xffff)) / SC + P.t16_delta : v;
                        }
                    }
                }
            }
        }
        if constexpr (!SPLIT) __syncthreads();   // (SPLIT: one compute wave; the poller takes no barriers)
    }

    // ------------------------------------------------------------------------ results
    if constexpr (SPLIT) {
        // per-band partial {score, i, j, timeout}; split_reduce_kernel folds them per pair
        if constexpr (LOCAL) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                const int oh = __shfl_xor(best_h, off);
                const int oi = __shfl_xor(best_i, off);
                const int oj = __shfl_xor(best_j, off);
                const bool take = oh > best_h || (oh == best_h && (oi > best_i || (oi == best_i && oj > best_j)));
                if (take) { best_h = oh; best_i = oi; best_j = oj; }
            }
        } else {
            best_h = ((m - 1) / BAND == (int)band0) ? s_score : 0;   // ordered by the loop's barrier
        }
        tmo = (uint32_t)__hip_atomic_load(&s_sync[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (threadIdx.x == 0) {
            int32_t* q = P.part + ((uint64_t)slot * P.split_bands + band0) * 4;
            q[0] = best_h; q[1] = best_i; q[2] = best_j; q[3] = (int32_t)tmo;
#ifdef SA_TB_STATS
            const uint64_t id = (uint64_t)slot * P.split_bands + band0;
            if (id < 4096) {
                g_split_stats[id][0] = id + 1;
                g_split_stats[id][1] = st_t0;
                g_split_stats[id][2] = __builtin_amdgcn_s_memrealtime();
                g_split_stats[id][3] = st_wait;
            }
            SA_EV_FLUSH();
#endif
        }
    } else if constexpr (LOCAL) {
        if constexpr (BU) {
            // this band's maximum of its tracked cells; the pair's last band folds the partials
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) smax = max(smax, (uint32_t)__shfl_xor((int)smax, off));
            typedef unsigned long long __attribute__((address_space(1))) gu64p;
            gu64p* const part = (gu64p*)(P.band_part + (uint64_t)slot * P.part_bands * SEGS);
            // the pair's final unit (last band, last segment) folds the other units' partials
            const uint32_t me = band0 * SEGS + seg, nparts = B > 0 ? (uint32_t)(B - 1) * SEGS + last_seg : 0u;
            if (me != nparts) {
                if (lane == 0)
                    __hip_atomic_store(part + me, (unsigned long long)epoch16 << 32 | smax | seg_lost << 31, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
#ifdef SA_TB_STATS
                const uint64_t sid = ((uint64_t)band0 * SEGS + seg) * P.count + slot;
                if (threadIdx.x == 0 && sid < 32768) {
                    g_fill_stats[sid][0] = st_t0;
                    g_fill_stats[sid][1] = __builtin_amdgcn_s_memrealtime();
                    g_fill_stats[sid][2] = (unsigned long long)st_hwid | ((unsigned long long)st_xcc << 32);
                }
#endif
                return;
            }
            // (the last band: every earlier band finished its last chunk before this one's last
            // chunk could read it, so its partial is at most a few instructions away)
            smax = max(smax, bu_fold_parts(part, nparts, last_seg, SEGS, epoch16, P.wait_polls, lane, seg_lost));
        }
#ifdef SA_TB_STATS
        const uint64_t sid = BU ? ((uint64_t)band0 * SEGS + seg) * P.count + slot : slot;   // (BU: one entry per unit)
        if (threadIdx.x == 0 && sid < 32768) {
            g_fill_stats[sid][0] = st_t0;
            g_fill_stats[sid][1] = __builtin_amdgcn_s_memrealtime();
            g_fill_stats[sid][2] = (unsigned long long)st_hwid | ((unsigned long long)st_xcc << 32);
        }
#endif
        if constexpr (SOMAX) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) smax = max(smax, (uint32_t)__shfl_xor((int)smax, off));
        }
        // lexicographic max over (score, i, j): the reference's last row-major maximum
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const int oh = __shfl_xor(best_h, off);
            const int oi = __shfl_xor(best_i, off);
            const int oj = __shfl_xor(best_j, off);
            const bool take = oh > best_h || (oh == best_h && (oi > best_i || (oi == best_i && oj > best_j)));
            if (take) { best_h = oh; best_i = oi; best_j = oj; }
        }
        if (lane == 0) { s_red[w * 3 + 0] = best_h; s_red[w * 3 + 1] = best_i; s_red[w * 3 + 2] = best_j; }
        __syncthreads();
        if (threadIdx.x == 0) {
            int h = INT_MIN, bi = 0, bjj = 0;
            for (int v = 0; v < W; ++v) {
                const int oh = s_red[v * 3], oi = s_red[v * 3 + 1], oj = s_red[v * 3 + 2];
                if (oh > h || (oh == h && (oi > bi || (oi == bi && oj > bjj)))) { h = oh; bi = oi; bjj = oj; }
            }
            sa_result r = {};
            if (B == 0) {
                // empty input: SW keeps MaxScore = INT_MIN, (MaxRow, MaxCol) = (0, 0);
                // LocalGotoh reads M[0][0] = 0 there
                r.score = (ALG == SA_SW) ? INT_MIN : 0;
            } else if constexpr (SOMAX) {
                // S >= smax and S <= smax - kSoSlack G: endcell_so_kernel finds S and the last
                // row-major cell
                h = (int)smax - kSoSlack * G;   // (the retry test below: the largest S this pair may have)
                r.score = (int)smax; r.end_i = 0; r.end_j = 0;
                r.reserved = 1;
            } else if constexpr (CMAX) {
                r.score = h; r.end_i = bi; r.end_j = 0;
                r.reserved = (uint32_t)bjj;   // chunk + 1: sa_endcell.hip resolves the column
            } else {
                r.score = h; r.end_i = bi; r.end_j = bjj;
            }
            if (T16 && B != 0 && h > P.retry_above) r.flags |= kFlagRetry;
            if (BU && seg_lost) r.flags |= kFlagRetry;
            if (redo) r.flags |= kFlagRedo;
            if (P.rerun) r.flags |= kFlagRerun;
            P.res[pidx] = r;
        }
    } else {
        if constexpr (BU) {
            // every unit's lost flag meets in the per-unit words (no maxima: NW reports H[m][n]), so
            // a lost hand-off anywhere in the pair reaches the unit holding (m, n), which flags the
            // pair for the int32 re-run
            typedef unsigned long long __attribute__((address_space(1))) gu64p;
            gu64p* const part = (gu64p*)(P.band_part + (uint64_t)slot * P.part_bands * SEGS);
            const uint32_t me = band0 * SEGS + seg, nparts = B > 0 ? (uint32_t)(B - 1) * SEGS + last_seg : 0u;
            if (me != nparts) {   // (uniform; B > 0 here: an empty pair has one unit, me == 0 == nparts)
                if (lane == 0)
                    __hip_atomic_store(part + me, (unsigned long long)epoch16 << 32 | seg_lost << 31, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
            (void)bu_fold_parts(part, nparts, last_seg, SEGS, epoch16, P.wait_polls, lane, seg_lost);
        }
        if (threadIdx.x == 0) {   // the phase loop's last barrier orders the owner's s_score store
            sa_result r = {};
            r.end_i = m;
            r.end_j = n;
            if (B == 0) {
                const int k = m > n ? m : n;
                if constexpr (ALG == SA_NW) r.score = k * G;
                else r.score = k == 0 ? 0 : GO + k * GE;
            } else {
                r.score = s_score;
            }
            if (BU && seg_lost) r.flags |= kFlagRetry;
            if (redo) r.flags |= kFlagRedo;
            if (P.rerun) r.flags |= kFlagRerun;
            P.res[pidx] = r;
        }
    }
}

template <int ALG, int R, int MM, bool ALLOW, bool KEYED, bool T16, bool CMAX, bool SPLIT, bool SO = false>
__global__ __launch_bounds__((fill_max_threads<R, (T16 && ALG >= SA_LOCAL_GOTOH)>())) void fill_kernel(FillParams P) {
    fill_body<ALG, R, MM, ALLOW, KEYED, T16, CMAX, SPLIT, SO>(P);
}
// The score-only kernel (one wave per workgroup): 4 waves per SIMD.  Its cell needs no record
// registers, and the fourth wave hides the cell's dependent 16-bit chain (tools/microbench_so.hip:
// 8,054 vs 7,520 GCUPS-equivalent at 4 vs 3 waves per SIMD).
template <int ALG, int R>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void fill_so_kernel(FillParams P) {
    constexpr bool LOCAL = ALG == SA_SW || ALG == SA_LOCAL_GOTOH;
    fill_body<ALG, R, kMatchEq, true, LOCAL, true, LOCAL, false, true>(P);
}

template <int ALG>
hipError_t launch_fill_alg(const FillVariant& v, const FillParams& p, uint32_t grid, hipStream_t stream) {
    constexpr bool LOCAL = (ALG == SA_SW || ALG == SA_LOCAL_GOTOH);
    const int R = v.R;
    if (v.so && (!v.t16 || v.split || v.cmax != LOCAL)) return hipErrorInvalidValue;
    const bool lut = (v.t16 || v.bits) ? false : v.lut, allow = v.allow;
    const bool keyed = LOCAL && v.keyed;
    // SPLIT: the compute wave + its poller and publisher waves (see kHandGran); LDS for one
    // compute wave
    const dim3 block(kWave * (v.split ? 3 : p.waves));
    const size_t lds = lds_layout(lut, is_affine(ALG), p.waves, p.stage_seq2 ? p.max_n : 0).total;
    if (lds > kMaxLds) return hipErrorInvalidConfiguration;
    const bool split = v.split;
    if (split && (p.waves != 1 || (R != 1 && R != 2 && R != 4 && R != 8))) return hipErrorInvalidConfiguration;
    if constexpr (ALG == SA_SW || ALG == SA_NW) {
        if (v.t16) {
            if (!allow || (LOCAL && !keyed)) return hipErrorInvalidValue;
            if ((int)block.x > (R >= 32 ? fill_max_threads<32>() : fill_max_threads<16>()))
                return hipErrorInvalidConfiguration;
#define SA_LAUNCH16S(RR, SP)                                                                         \
    if (R == RR && split == SP) {                                                                    \
        if constexpr ((ALG == SA_SW || ALG == SA_NW) && !SP && RR <= 32) {                            \
            if (v.so) {                                                                              \
                hipLaunchKernelGGL((fill_so_kernel<ALG, RR>), dim3(grid), block, lds, stream, p);       \
                return hipGetLastError();                                                            \
            }                                                                                        \
        }                                                                                            \
        if (v.so) return hipErrorInvalidValue;                                                       \
        if constexpr (ALG == SA_SW) {                                                                \
            if (v.cmax) {                                                                            \
                hipLaunchKernelGGL((fill_kernel<ALG, RR, kMatchEq, true, LOCAL, true, true, SP>), dim3(grid), \
                                   block, lds, stream, p);                                           \
                return hipGetLastError();                                                            \
            }                                                                                        \
        }                                                                                            \
        hipLaunchKernelGGL((fill_kernel<ALG, RR, kMatchEq, true, LOCAL, true, false, SP>), dim3(grid), block, \
                           lds, stream, p);                                                          \
        return hipGetLastError();                                                                    \
    }
            SA_LAUNCH16S(4, false)
            SA_LAUNCH16S(8, false)
            SA_LAUNCH16S(16, false)
            SA_LAUNCH16S(32, false)
            SA_LAUNCH16S(64, false)
            SA_LAUNCH16S(2, true)
            SA_LAUNCH16S(4, true)
            SA_LAUNCH16S(8, true)
#undef SA_LAUNCH16S
            if (R == 1 && split && !v.cmax && !v.so) {   // R = 1: the per-cell key (CMAX pairs rows)
                hipLaunchKernelGGL((fill_kernel<ALG, 1, kMatchEq, true, LOCAL, true, false, true>), dim3(grid), block,
                                   lds, stream, p);
                return hipGetLastError();
            }
            return hipErrorInvalidValue;
        }
    }
    if constexpr (ALG == SA_LOCAL_GOTOH || ALG == SA_GLOBAL_GOTOH) {
        if (v.t16) {   // T16 affine: one-wave plans (R <= 16) and SPLIT bands (R <= 8)
            if (!allow || (v.cmax && !LOCAL) || (LOCAL && !keyed)) return hipErrorInvalidValue;
            if ((int)block.x > (R >= 16 ? fill_max_threads<16, true>() : fill_max_threads<8>()))
                return hipErrorInvalidConfiguration;
#define SA_LAUNCH16A(RR, SP)                                                                           \
    if (R == RR && split == SP) {                                                                      \
        if constexpr (!SP && RR >= 4) {                                                                \
            if (v.so) {                                                                                \
                hipLaunchKernelGGL((fill_so_kernel<ALG, RR>), dim3(grid), block, lds, stream, p);         \
                return hipGetLastError();                                                              \
            }                                                                                          \
        }                                                                                              \
        if (v.so) return hipErrorInvalidValue;                                                         \
        if constexpr (LOCAL && RR % 2 == 0) {                                                          \
            if (v.cmax) {                                                                              \
                hipLaunchKernelGGL((fill_kernel<ALG, RR, kMatchEq, true, true, true, true, SP>), dim3(grid), block, \
                                   lds, stream, p);                                                    \
                return hipGetLastError();                                                              \
            }                                                                                          \
        }                                                                                              \
        if (v.cmax) return hipErrorInvalidValue;                                                       \
        hipLaunchKernelGGL((fill_kernel<ALG, RR, kMatchEq, true, LOCAL, true, false, SP>), dim3(grid), block, \
                           lds, stream, p);                                                            \
        return hipGetLastError();                                                                      \
    }
            SA_LAUNCH16A(4, false)
            SA_LAUNCH16A(8, false)
            SA_LAUNCH16A(16, false)
            SA_LAUNCH16A(1, true)
            SA_LAUNCH16A(2, true)
            SA_LAUNCH16A(4, true)
            SA_LAUNCH16A(8, true)
#undef SA_LAUNCH16A
            return hipErrorInvalidValue;
        }
    }
    if (v.t16 || v.cmax || v.so) return hipErrorInvalidValue;
    const int mm = v.bits ? kMatchBits : lut ? kMatchLut : kMatchEq;
#define SA_LAUNCH(RR, MMV, AA, KK)                                                             \
    if (R == RR && mm == MMV && allow == AA && keyed == KK) {                                  \
        if (split) {                                                                           \
            if constexpr (RR <= 8) {                                                           \
                hipLaunchKernelGGL((fill_kernel<ALG, RR, MMV, AA, KK, false, false, true>), dim3(grid), block, lds, \
                                   stream, p);                                                 \
                return hipGetLastError();                                                      \
            }                                                                                  \
            return hipErrorInvalidConfiguration;                                               \
        }                                                                                      \
        hipLaunchKernelGGL((fill_kernel<ALG, RR, MMV, AA, KK, false, false, false>), dim3(grid), block, lds, stream, p); \
        return hipGetLastError();                                                              \
    }
#define SA_LAUNCH_K(RR, MMV, AA) \
    SA_LAUNCH(RR, MMV, AA, false) \
    if constexpr (LOCAL) { SA_LAUNCH(RR, MMV, AA, true) }
#define SA_LAUNCH_R(RR)                  \
    SA_LAUNCH_K(RR, kMatchEq, true)      \
    SA_LAUNCH_K(RR, kMatchEq, false)     \
    SA_LAUNCH_K(RR, kMatchLut, true)     \
    SA_LAUNCH_K(RR, kMatchLut, false)    \
    SA_LAUNCH_K(RR, kMatchBits, true)    \
    SA_LAUNCH_K(RR, kMatchBits, false)
    SA_LAUNCH_R(4)
    SA_LAUNCH_R(8)
    SA_LAUNCH_R(16)
#undef SA_LAUNCH_R
    // R = 1, 2: the few-pairs (SPLIT) plans only
#define SA_LAUNCH_S(RR, MMV, AA, KK)                                                            \
    if (split && R == RR && mm == MMV && allow == AA && keyed == KK) {                          \
        hipLaunchKernelGGL((fill_kernel<ALG, RR, MMV, AA, KK, false, false, true>), dim3(grid), block, lds, stream, p); \
        return hipGetLastError();                                                               \
    }
#define SA_LAUNCH_SK(RR, MMV, AA) \
    SA_LAUNCH_S(RR, MMV, AA, false) \
    if constexpr (LOCAL) { SA_LAUNCH_S(RR, MMV, AA, true) }
#define SA_LAUNCH_SR(RR)                 \
    SA_LAUNCH_SK(RR, kMatchEq, true)     \
    SA_LAUNCH_SK(RR, kMatchEq, false)    \
    SA_LAUNCH_SK(RR, kMatchLut, true)    \
    SA_LAUNCH_SK(RR, kMatchLut, false)   \
    SA_LAUNCH_SK(RR, kMatchBits, true)   \
    SA_LAUNCH_SK(RR, kMatchBits, false)
    SA_LAUNCH_SR(1)
    SA_LAUNCH_SR(2)
#undef SA_LAUNCH_SR
#undef SA_LAUNCH_SK
#undef SA_LAUNCH_S
#undef SA_LAUNCH_K
#undef SA_LAUNCH
    return hipErrorInvalidValue;
}

}  // namespace sa
