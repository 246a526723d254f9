// sa_hirschberg.hip — HirschbergSA::getAlignment (SAHirschberg.h:102-184) on the GPU, batched over
// pairs: linear-space global alignment whose result is exactly the reference's (its own split
// tie rule and NW base case), not merely an optimal alignment.
//
// The recursion is run breadth-first over all pairs at once:
//   * device levels: every subproblem with more than kHbLeafRows rows of Seq1 and >= 2 columns
//     is split.  Its two NWScore sweeps (:131 forward over the top half, :136 over the reversed
//     bottom half and reversed Seq2) become two rows of one batched launch of hb_sweep_kernel
//     (score-only NW, one wave per sweep, anti-diagonal wavefront as in the fill kernel, the
//     last DP row written out); hb_split_kernel then takes, per subproblem, the LAST i in
//     [0, |Seq2|) maximising Fwd[i] + Rev[|Seq2|-i] (:138-149; i never reaches |Seq2|) and
//     writes the two children (:151-161) as the next level's subproblems.
//   * leaves: everything smaller (and every base case) is finished by hb_leaf_kernel, one
//     thread per subproblem running the same recursion iteratively (explicit stack, left child
//     first), including the NW base case of :119-126 with the reference's NW traceback rules.
//   * assembly: a pair's leaves cover disjoint, increasing ranges of Seq1, so its alignment is
//     the concatenation of its leaves' forward op lists in Seq1 order; dc_assemble_kernel
//     (sa_dc.hip) reverses it into the engine's traceback-order op stream (include/seqalib_hip.h).
// The level loop never returns to the host: subproblems are classified on the device and every
// buffer is addressed by the subproblem's key a0 + b0 (sa_dc.hip); the host only launches, with
// grid sizes from upper bounds (the largest subproblem halves per level).
// Score reported: NW H[m][n] (the reference exposes none): max over i in [0, n] of the level-0
// split sums, or the leaf's own full NWScore.
#include <hip/hip_runtime.h>
#include <limits.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "sa_dc.h"
#include "sa_internal.h"

namespace sa {

constexpr int kHbLeafRows = 12;   // subproblems with <= this many Seq1 rows are leaves (tuned, tools/ab_dc.sh)

struct HbSweep {       // NWScore over A (alen) x B (blen) -> rows[out .. out+blen]
    uint64_t a, b;     // index of A[0] / B[0] in seq1 / seq2 (rev: of the LAST element read first)
    int32_t alen, blen;
    int32_t rev;       // 1: A and B are both read backwards
    int32_t pad;
    uint64_t out;      // int32 index into the row buffer
};

// Sweep rows of a split subproblem live at 2 * key (forward) and 2 * key + n + 1 (reverse):
// 2 (n + 1) <= 2 (m + n) ints, inside its key span.
__device__ __forceinline__ HbSweep hb_sweep_of(const DcSub& s, int rev) {
    const int mid = s.m / 2;
    const uint64_t key = s.a0 + s.b0;
    if (!rev) return HbSweep{s.a0, s.b0, mid, s.n, 0, 0, 2 * key};
    return HbSweep{s.a0 + (uint64_t)s.m - 1, s.b0 + (uint64_t)s.n - 1, s.m - mid, s.n, 1, 0, 2 * key + s.n + 1};
}

struct HbScore {
    int32_t gap, match, mismatch, allow;
};

// NW cell as NWScore computes it (:40-44 / :56-59).
__device__ __forceinline__ int32_t hb_cell(int32_t hd, int32_t hu, int32_t hl, bool v, const HbScore& s) {
    const int32_t sub = s.allow ? hd + (v ? s.match : s.mismatch) : (v ? hd + s.match : INT_MIN);
    return max(max(sub, hu + s.gap), hl + s.gap);
}

// The same cell with AllowMismatch fixed at compile time (branch-free), v = match(a, b).
template <bool ALLOW>
__device__ __forceinline__ int32_t hb_cell_v(int32_t hd, int32_t hu, int32_t hl, bool v, const HbScore& s) {
    int32_t sub;
    if constexpr (ALLOW) sub = hd + (v ? s.match : s.mismatch);
    else sub = v ? hd + s.match : INT_MIN;
    return max(max(sub, hu + s.gap), hl + s.gap);
}

// ------------------------------------------------------------------ batched NWScore sweeps
// 16-bit band of a whole-wave NWScore sweep (Dc16, sa_dc.h): registers hold H - delta in their low
// 16 bits; per cell max(Hd + s, max(Hu, Hl) + Gap) = v_max_i16, v_add_u16, v_bfe_i32 (the row's
// byte profile at 8 x the column's symbol code), v_add_u16, v_max_i16 -- one 32-bit op, four
// 16-bit ops, against seven 32-bit ops of the int32 cell.  Same wavefront and hand-off as below.
template <int R>
__device__ __forceinline__ void hb_band16(const HbSweep& d, const uint8_t* s1, const uint8_t* s2, const uint32_t* aux,
                                          int32_t delta, int32_t G, int band, int lastb, int tl, int rl, int32_t* out,
                                          int32_t& hl, int32_t* s_park) {
    const int lane = threadIdx.x;
    const int m = d.alen, n = d.blen;
    constexpr int BAND = 64 * R;
    const uint32_t symp = aux[kAuxProf + 4];
    const uint32_t g16 = (uint32_t)G & 0xffffu;
    const int row0 = band * BAND + lane * R;
    uint32_t a[R];
    int32_t Hp[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        a[r] = row < m ? aux[kAuxProf + (dc_code8(symp, d.rev ? s1[d.a - row] : s1[d.a + row]) >> 3)] : 0u;
        Hp[r] = (row + 1) * G - delta;                      // H[i][0] = i * Gap (:37)
    }
    int32_t prev_up = row0 * G - delta;                      // H[row0][0]
    auto load_chunk = [&](int c0, int32_t& vu, uint32_t& vs) {
        const int j = c0 + lane;
        vu = 0;
        vs = 0;
        if (j < n) {
            vu = (band == 0 ? (j + 1) * G : out[j + 1]) - delta;
            vs = dc_code8(symp, d.rev ? s2[d.b - j] : s2[d.b + j]);
        }
    };
    int32_t vup, nvup;
    uint32_t vsym, nvsym, sym = 0;
    // the R cells of one step, updated in place: row r's block also forms row r+1's diagonal + s
    // from the OLD Hp[r] before overwriting it, so the step needs no register copies
    auto cells = [&](int32_t up_h) __attribute__((always_inline)) {
        uint32_t dcur;
        asm("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(dcur) : "v"(a[0]), "v"(sym), "v"(prev_up));
        int32_t hu = up_h;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t t0, dn = 0;
            if (r + 1 < R) {
                asm("v_max_i16 %[t0], %[hu], %[hp]\n\t"   // max(up, left) + gap
                    "v_add_u16 %[t0], %[g], %[t0]\n\t"
                    "v_bfe_i32 %[dn], %[an], %[sym], 8\n\t"   // next row: s + diagonal (old H)
                    "v_add_u16 %[dn], %[hp], %[dn]\n\t"
                    "v_max_i16 %[hp], %[dr], %[t0]"
                    : [t0] "=&v"(t0), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                    : [hu] "v"(hu), [g] "s"(g16), [an] "v"(a[r + 1 < R ? r + 1 : r]), [sym] "v"(sym), [dr] "v"(dcur));
            } else {
                asm("v_max_i16 %[t0], %[hu], %[hp]\n\t"
                    "v_add_u16 %[t0], %[g], %[t0]\n\t"
                    "v_max_i16 %[hp], %[dr], %[t0]"
                    : [t0] "=&v"(t0), [hp] "+v"(Hp[r])
                    : [hu] "v"(hu), [g] "s"(g16), [dr] "v"(dcur));
            }
            dcur = dn;
            hu = Hp[r];
        }
    };
    // the lane and register holding the row this band hands on: its last row (lane 63, Hp[R-1]),
    // or in the last band row m of the sweep (lane tl, Hp[rl])
    const int src_lane = band < lastb ? 63 : tl;
    const int src_r = band < lastb ? R - 1 : rl;
    // Steady chunk (c0 >= 63, c0 + 64 <= n: every lane inside the matrix for all 64 steps): no
    // per-lane branch, and the handed-on row is parked per step by an LDS write of every lane
    // (src_lane into its slot, the others into a discard slot) and stored once per chunk,
    // coalesced -- instead of an exec-masked global store per step.  SRC: src_r at compile time.
    auto steady_park = [&](int c0, auto SRC) {
        constexpr int SR = decltype(SRC)::value;
        int32_t* const park = s_park + (lane == src_lane ? 0 : 64);
#pragma unroll 1
        for (int q = 0; q < 64; ++q) {
            const int32_t up_h = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vup, q), hl, 0x138, 0xf, 0xf, false);
            sym = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vsym, q), sym, 0x138, 0xf, 0xf, false);
            cells(up_h);
            prev_up = up_h;
            hl = Hp[R - 1];
            park[q] = Hp[SR];
        }
        __syncthreads();   // (one wave: orders the parked writes before the reads)
        out[c0 - src_lane + 1 + lane] = dc_unpack16(s_park[lane], delta);
        __syncthreads();
    };
    load_chunk(0, vup, vsym);
    for (int c0 = 0; c0 < n + 63; c0 += 64) {
        load_chunk(c0 + 64, nvup, nvsym);
        if (s_park && c0 >= 63 && c0 + 64 <= n) {
            dc_row_dispatch<R>(src_r, [&](auto SRC) { steady_park(c0, SRC); });   // (uniform)
            vup = nvup;
            vsym = nvsym;
            continue;
        }
        const int steps = min(64, n + 63 - c0);
        // steady chunk without parking (SEQALIB_DC16_PARK=0): every lane is inside the matrix for
        // all 64 steps, so the per-lane range branch is skipped (the hand-off store keeps its lane test)
        const bool steady = c0 >= 63 && c0 + 64 <= n;
        for (int q = 0; q < steps; ++q) {
            const int s = c0 + q;
            const int32_t up_h = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vup, q), hl, 0x138, 0xf, 0xf, false);
            sym = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vsym, q), sym, 0x138, 0xf, 0xf, false);
            const int j0 = s - lane;
            if (steady || (j0 >= 0 && j0 < n)) {
                cells(up_h);
                prev_up = up_h;
                hl = Hp[R - 1];
                if (band < lastb) {
                    if (lane == 63) out[j0 + 1] = dc_unpack16(hl, delta);   // this band's last row, in place
                } else if (lane == tl) {
                    int32_t v = Hp[0];
#pragma unroll
                    for (int r = 1; r < R; ++r)
                        if (r == rl) v = Hp[r];
                    out[j0 + 1] = dc_unpack16(v, delta);                   // row m of the sweep
                }
            }
        }
        vup = nvup;
        vsym = nvsym;
    }
}

// MM: kMatchEq / kMatchLut (byte symbols) or kMatchBits (pair-local indices + the pair's match
// bitmap, the generic-Ty path; DcSrc in sa_dc.h).  d16.aux: the 16-bit path may run (the device's
// alphabet decision picks it, uniformly for the grid).
template <int R, int MM, bool ALLOW>
__global__ __launch_bounds__(64) void hb_sweep_kernel(const uint8_t* s1, const uint8_t* s2, const DcSub* split,
                                                      const DcLevel* lvl, int32_t* rows, const uint32_t* lutbits,
                                                      DcBits bits, HbScore sc, Dc16 d16) {
    constexpr bool LUT = MM == kMatchLut;
    if (MM != kMatchBits && d16.seg16 && d16.aux && d16.aux[kAuxSel] == 1) return;   // (hb_sweep_seg16_kernel)
    __shared__ uint32_t s_lut[LUT ? 2048 : 1];
    __shared__ int32_t s_park[128];   // Dc16 steady chunks: the handed-on row, parked per step
    const int lane = threadIdx.x;
    if (blockIdx.x / 2 >= lvl->nsplit) return;   // grid sized from an upper bound
    if constexpr (LUT) {
        for (int k = lane; k < 2048; k += 64) s_lut[k] = lutbits[k];
        __syncthreads();
    }
    // One sweep per block, or a grid-stride loop when the grid was capped (launched beside the
    // 16-bit seg16 kernel, this kernel usually returns at once and a full grid would cost more
    // than the skip itself).
    auto one = [&](uint32_t bid) {
        const DcSub sub = split[bid / 2];
        const HbSweep d = hb_sweep_of(sub, bid & 1);
        const DcSrc<MM> src = bits.src<MM>(s1, s2, s_lut, sub.pair, true);
        int32_t* out = rows + d.out;
        const int m = d.alen, n = d.blen, G = sc.gap;
        if constexpr (MM != kMatchBits) {
            if (d16.aux && d16.aux[kAuxSel] == 1) {
                constexpr int BAND = 64 * R;
                const int bands = (m + BAND - 1) / BAND;
                const int tl = ((m - 1) % BAND) / R, rl = (m - 1) % R;
                int32_t hl = 0;
                for (int band = 0; band < bands; ++band) {
                    hb_band16<R>(d, s1, s2, d16.aux, d16.delta, G, band, bands - 1, tl, rl, out, hl, d16.park ? s_park : nullptr);
                    __threadfence_block();
                    __syncthreads();
                }
                if (lane == 0) out[0] = m * G;
                return;
            }
        }
        auto symA = [&](int k) -> uint32_t { return src.a(d.rev ? d.a - k : d.a + k); };
        auto symB = [&](int k) -> uint32_t { return src.b(d.rev ? d.b - k : d.b + k); };
        constexpr int BAND = 64 * R;
        const int bands = (m + BAND - 1) / BAND;
        const int lastb = bands - 1;
        const int tl = ((m - 1) % BAND) / R, rl = (m - 1) % R;   // owner of row m-1 in the last band
        int hl = 0;
        for (int band = 0; band < bands; ++band) {
            const int row0 = band * BAND + lane * R;
            uint32_t a[R];
            int32_t Hp[R];
    #pragma unroll
            for (int r = 0; r < R; ++r) {
                a[r] = row0 + r < m ? symA(row0 + r) : 0u;
                Hp[r] = (row0 + r + 1) * G;                      // H[i][0] = i * Gap (:37)
            }
            int32_t prev_up = row0 * G;                          // H[row0][0]
            // Per 64-step chunk, lane k holds column c0+k's row-above value (for lane 0) and Seq2
            // symbol, loaded one chunk ahead; both reach their lane by DPP wave_shr:1 like the fill.
            auto load_chunk = [&](int c0, int32_t& vu, uint32_t& vs) {
                const int j = c0 + lane;
                vu = 0;
                vs = 0;
                if (j < n) {
                    vu = band == 0 ? (j + 1) * G : out[j + 1];
                    vs = symB(j);
                }
            };
            int32_t vup, nvup;
            uint32_t vsym, nvsym, sym = 0;
            load_chunk(0, vup, vsym);
            for (int c0 = 0; c0 < n + 63; c0 += 64) {
                load_chunk(c0 + 64, nvup, nvsym);
                const int steps = min(64, n + 63 - c0);
                const bool steady = c0 >= 63 && c0 + 64 <= n;   // every lane inside (as the 16-bit sweep)
                for (int q = 0; q < steps; ++q) {
                    const int s = c0 + q;
                    const int32_t up_h = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vup, q), hl, 0x138, 0xf,
                                                                     0xf, false);
                    sym = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vsym, q), sym, 0x138, 0xf, 0xf, false);
                    const int j0 = s - lane;
                    if (steady || (j0 >= 0 && j0 < n)) {
                        int32_t hd = prev_up, hu = up_h;
    #pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const int32_t h = hb_cell_v<ALLOW>(hd, hu, Hp[r], src.match(a[r], sym), sc);
                            hd = Hp[r];
                            Hp[r] = h;
                            hu = h;
                        }
                        prev_up = up_h;
                        hl = Hp[R - 1];
                        if (band < lastb) {
                            if (lane == 63) out[j0 + 1] = hl;    // this band's last row, in place
                        } else if (lane == tl) {
                            out[j0 + 1] = Hp[rl];                // row m of the sweep (uniform index)
                        }
                    }
                }
                vup = nvup;
                vsym = nvsym;
            }
            __threadfence_block();
            __syncthreads();
        }
        if (lane == 0) out[0] = m * G;
    };
    for (uint32_t bid = blockIdx.x; bid / 2 < lvl->nsplit; bid += gridDim.x) {
        one(bid);
        __syncthreads();
    }
}

// Deep levels of the 16-bit sweeps (Dc16): TWO sweeps per wave, 32 lanes x R rows each (a sweep
// of at most 32 R rows, one band), instead of one 64-lane sweep per wave with R / 2 rows per lane:
// the ramp is 31 steps instead of 63 and the per-step hand-off (two readlanes, two DPP moves) is
// paid for twice the cells.  Lanes 0 and 32 take their segment's top row value and column symbol
// (readlane of their own half of the chunk registers) where the other lanes take lane - 1's by
// wave_shr:1.  The cells are hb_band16's (in place, 16-bit, value - delta).  Runs only when the
// device's alphabet decision picked the 16-bit path; hb_sweep_kernel<R / 2> (launched beside it,
// Dc16::seg16) returns at once then, and runs the int32 sweeps otherwise.
template <int R>
__global__ __launch_bounds__(64) void hb_sweep_seg16_kernel(const uint8_t* s1, const uint8_t* s2, const DcSub* split,
                                                            const DcLevel* lvl, int32_t* rows, HbScore sc, Dc16 d16) {
    if (!(d16.aux && d16.aux[kAuxSel] == 1)) return;   // the int32 sweeps run (hb_sweep_kernel)
    const int lane = threadIdx.x;
    const uint32_t nsw = 2 * lvl->nsplit;
    if (blockIdx.x * 2 >= nsw) return;   // grid sized from an upper bound (uniform exit)
    const int seg = lane >> 5, ls = lane & 31;
    const uint32_t swi = blockIdx.x * 2 + seg;
    const bool active = swi < nsw;
    HbSweep d{};
    if (active) d = hb_sweep_of(split[swi / 2], swi & 1);
    const uint32_t* aux = d16.aux;
    const int32_t delta = d16.delta;
    const int m = d.alen, n = d.blen, G = sc.gap;
    const uint32_t symp = aux[kAuxProf + 4];
    const uint32_t g16 = (uint32_t)G & 0xffffu;
    const int row0 = ls * R;
    uint32_t a[R];
    int32_t Hp[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        a[r] = active && row < m ? aux[kAuxProf + (dc_code8(symp, d.rev ? s1[d.a - row] : s1[d.a + row]) >> 3)] : 0u;
        Hp[r] = (row + 1) * G - delta;                      // H[i][0] = i * Gap (:37)
    }
    int32_t prev_up = row0 * G - delta;                      // H[row0][0]
    const int tl = active ? (m - 1) / R : -1, rl = active ? (m - 1) % R : 0;   // owner of row m
    int32_t* const out = rows + d.out;
    uint32_t sym = 0;
    auto cells = [&](int32_t up_h) __attribute__((always_inline)) {   // as hb_band16's
        uint32_t dcur;
        asm("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(dcur) : "v"(a[0]), "v"(sym), "v"(prev_up));
        int32_t hu = up_h;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t t0, dn = 0;
            if (r + 1 < R) {
                asm("v_max_i16 %[t0], %[hu], %[hp]\n\t"
                    "v_add_u16 %[t0], %[g], %[t0]\n\t"
                    "v_bfe_i32 %[dn], %[an], %[sym], 8\n\t"
                    "v_add_u16 %[dn], %[hp], %[dn]\n\t"
                    "v_max_i16 %[hp], %[dr], %[t0]"
                    : [t0] "=&v"(t0), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                    : [hu] "v"(hu), [g] "s"(g16), [an] "v"(a[r + 1 < R ? r + 1 : r]), [sym] "v"(sym), [dr] "v"(dcur));
            } else {
                asm("v_max_i16 %[t0], %[hu], %[hp]\n\t"
                    "v_add_u16 %[t0], %[g], %[t0]\n\t"
                    "v_max_i16 %[hp], %[dr], %[t0]"
                    : [t0] "=&v"(t0), [hp] "+v"(Hp[r])
                    : [hu] "v"(hu), [g] "s"(g16), [dr] "v"(dcur));
            }
            dcur = dn;
            hu = Hp[r];
        }
    };
    // per 32-step chunk, lane k of a segment holds its column c0 + k's top value and symbol
    auto load_chunk = [&](int c0, int32_t& vu, uint32_t& vs) {
        const int j = c0 + ls;
        vu = 0;
        vs = 0;
        if (active && j < n) {
            vu = (j + 1) * G - delta;                       // top row H[0][j+1] (:35)
            vs = dc_code8(symp, d.rev ? s2[d.b - j] : s2[d.b + j]);
        }
    };
    int steps = active ? n + 31 : 0;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) steps = max(steps, __shfl_xor(steps, off));
    int32_t vup, nvup, hl = Hp[R - 1];
    uint32_t vsym, nvsym;
    load_chunk(0, vup, vsym);
    for (int c0 = 0; c0 < steps; c0 += 32) {
        load_chunk(c0 + 32, nvup, nvsym);
        const int qn = min(32, steps - c0);
        for (int q = 0; q < qn; ++q) {
            int32_t up_h = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vup, q), hl, 0x138, 0xf, 0xf, false);
            sym = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vsym, q), sym, 0x138, 0xf, 0xf, false);
            const int32_t up_b = __builtin_amdgcn_readlane(vup, 32 + q);
            const uint32_t sym_b = __builtin_amdgcn_readlane(vsym, 32 + q);
            if (lane == 32) {   // the second segment's first lane: its own top row and symbol
                up_h = up_b;
                sym = sym_b;
            }
            const int j0 = c0 + q - ls;
            if (active && j0 >= 0 && j0 < n) {
                cells(up_h);
                prev_up = up_h;
                hl = Hp[R - 1];
                if (ls == tl) {
                    int32_t v = Hp[0];
#pragma unroll
                    for (int r = 1; r < R; ++r)
                        if (r == rl) v = Hp[r];
                    out[j0 + 1] = dc_unpack16(v, delta);   // row m of the sweep
                }
            }
        }
        vup = nvup;
        vsym = nvsym;
    }
    if (active && ls == 0) out[0] = m * G;
}

// Packed sweeps for the deep levels (every sweep of the level has alen <= G = 8, 16 or 32 rows): 64 / G sweeps
// per wave, G lanes each, one row per lane, so a sweep takes n + G - 1 steps on G lanes instead
// of n + 63 steps on a whole wave.  The row-above value and column symbol still arrive by DPP
// wave_shr:1; a segment's first lane takes the top border (H[0][j] = j * gap) and its column
// symbol (one ds_bpermute from the segment's chunk of Seq2, loaded a chunk ahead) instead.
template <int G, int MM, bool ALLOW>
__global__ __launch_bounds__(64) void hb_sweep_seg_kernel(const uint8_t* s1, const uint8_t* s2, const DcSub* split,
                                                          const DcLevel* lvl, int32_t* rows, const uint32_t* lutbits,
                                                          DcBits bits, HbScore sc) {
    constexpr int P = 64 / G;
    constexpr bool LUT = MM == kMatchLut;
    __shared__ uint32_t s_lut[LUT ? 2048 : 1];
    const int lane = threadIdx.x;
    const uint32_t nsw = 2 * lvl->nsplit;
    if (blockIdx.x * P >= nsw) return;   // grid sized from an upper bound (uniform exit)
    if constexpr (LUT) {
        for (int k = lane; k < 2048; k += 64) s_lut[k] = lutbits[k];
        __syncthreads();
    }
    const int seg = lane / G, ls = lane % G;
    const uint32_t swi = blockIdx.x * P + seg;
    const bool active = swi < nsw;
    HbSweep d{};
    uint32_t pair = 0;
    if (active) {
        const DcSub sub = split[swi / 2];
        d = hb_sweep_of(sub, swi & 1);
        pair = sub.pair;
    }
    const DcSrc<MM> src = bits.src<MM>(s1, s2, s_lut, pair, active);
    const int m = d.alen, n = d.blen, Gp = sc.gap;
    int32_t* out = rows + d.out;
    int steps = n + G - 1;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) steps = max(steps, __shfl_xor(steps, off));
    auto symB = [&](int k) -> uint32_t { return src.b(d.rev ? d.b - k : d.b + k); };
    const uint32_t a = ls < m ? src.a(d.rev ? d.a - ls : d.a + ls) : 0u;
    int32_t Hp = (ls + 1) * Gp;          // H[ls + 1][0]
    int32_t prev_up = ls * Gp;           // H[ls][0]: the diagonal of column 1
    int32_t hl = Hp;
    uint32_t sym = 0;
    const bool last_row = ls == m - 1;
    uint32_t vs = ls < n ? symB(ls) : 0u, nvs;
    for (int c0 = 0; c0 < steps; c0 += G) {
        nvs = c0 + G + ls < n ? symB(c0 + G + ls) : 0u;
        const int qn = min(G, steps - c0);
        for (int q = 0; q < qn; ++q) {
            const int s = c0 + q;
            const uint32_t b0 = __shfl(vs, seg * G + q);
            const int32_t up_d = __builtin_amdgcn_update_dpp(0, hl, 0x138, 0xf, 0xf, false);
            const uint32_t sy_d = __builtin_amdgcn_update_dpp(0u, sym, 0x138, 0xf, 0xf, false);
            const int32_t up_h = ls == 0 ? (s + 1) * Gp : up_d;
            sym = ls == 0 ? b0 : sy_d;
            const int j0 = s - ls;
            if (j0 >= 0 && j0 < n && ls < m) {
                const int32_t h = hb_cell_v<ALLOW>(prev_up, up_h, Hp, src.match(a, sym), sc);
                Hp = h;
                prev_up = up_h;
                hl = h;
                if (last_row) out[j0 + 1] = h;   // row m of the sweep
            }
        }
        vs = nvs;
    }
    if (active && ls == 0) out[0] = m * Gp;
}

// ---------------------------------------------------------------------------- split
template <int GS>
__global__ __launch_bounds__(64) void hb_split_kernel(const DcSub* split, const DcLevel* lvl, const int32_t* rows,
                                                      DcSub* next, sa_result* res) {
    // GS lanes per split, 64 / GS splits per wave (deep levels: short rows, many splits)
    const int lane = threadIdx.x, sl = lane % GS;
    const uint32_t k = blockIdx.x * (64 / GS) + lane / GS;
    const uint32_t ns = lvl->nsplit;
    if (blockIdx.x * (64 / GS) >= ns) return;   // (uniform)
    const bool act = k < ns;
    DcSub d{};
    if (act) d = split[k];
    const int32_t* F = rows + 2 * (d.a0 + d.b0);
    const int n = act ? d.n : 0;
    const int32_t* B = F + n + 1;
    int32_t best = INT_MIN;
    int idx = 0;
    for (int i = sl; i < n; i += GS) {
        const int32_t s = F[i] + B[n - i];
        if (s >= best) { best = s; idx = i; }
    }
    // lexicographic (sum, i) maximum = the reference's last maximum (S >= MaxScore, :144)
#pragma unroll
    for (int off = GS / 2; off >= 1; off >>= 1) {
        const int32_t ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(idx, off);
        if (ob > best || (ob == best && oi > idx)) { best = ob; idx = oi; }
    }
    if (act && sl == 0) {
        if (d.top) res[d.pair].score = max(best, F[n] + B[0]);   // NW H[m][n] over i in [0, n]
        const int mid = d.m / 2;
        next[2 * k] = DcSub{d.a0, d.b0, mid, idx, 0, 0, d.pair, 0};
        next[2 * k + 1] = DcSub{d.a0 + (uint64_t)mid, d.b0 + (uint64_t)idx, d.m - mid, n - idx, 0, 0, d.pair, 0};
    }
}

// ---------------------------------------------------------------------------- leaves
// The leaf solvers take the symbols as a sequence view (Seq: GSeq / LSeq bytes, ISeq pair-local
// indices) and the match as a functor (Match: DcLutMatch, DcBitsMatch).
// NWScore's last row (:31-66) into F[0..blen], one row updated in place (the cell above is read
// before it is overwritten; its old value is the next column's diagonal).
template <typename Row, typename Seq, typename Match>
__device__ void hb_nwscore(Seq A, int alen, int arev, Seq B, int blen, int brev,
                           const Match& mt, const HbScore& sc, Row F) {
    F[0] = 0;
    for (int j = 1; j <= blen; ++j) F[j] = F[j - 1] + sc.gap;
    for (int i = 1; i <= alen; ++i) {
        const uint32_t ai = arev ? A[alen - i] : A[i - 1];
        int32_t diag = F[0];
        int32_t left = diag + sc.gap;
        F[0] = left;
        for (int j = 1; j <= blen; ++j) {
            const uint32_t bj = brev ? B[blen - j] : B[j - 1];
            const int32_t up = F[j];
            left = hb_cell(diag, up, left, mt(ai, bj), sc);
            F[j] = left;
            diag = up;
        }
    }
}

// NeedlemanWunschSA::getAlignment on a 1 x k or k x 1 view (:119-126): full matrix + the
// reference NW traceback (SANeedlemanWunsch.h:167-230); writes forward-order ops at out.
template <typename Row, typename Seq, typename Match>
__device__ int hb_nw_small(Seq A, int m, Seq B, int n, const Match& mt, const HbScore& sc, Row H, uint8_t* out) {
    const int w = n + 1;
    for (int i = 0; i <= m; ++i) H[i * w] = i * sc.gap;
    for (int j = 0; j <= n; ++j) H[j] = j * sc.gap;
    for (int i = 1; i <= m; ++i)
        for (int j = 1; j <= n; ++j)
            H[i * w + j] = hb_cell(H[(i - 1) * w + j - 1], H[(i - 1) * w + j], H[i * w + j - 1], mt(A[i - 1], B[j - 1]), sc);
    int k = 0, i = m, j = n;
    while (i > 0 || j > 0) {
        if (i > 0 && j > 0) {
            const bool v = mt(A[i - 1], B[j - 1]);
            const int32_t hd = H[(i - 1) * w + j - 1];
            const int32_t dt = sc.allow ? hd + (v ? sc.match : sc.mismatch) : (v ? hd + sc.match : INT_MIN);
            if (H[i * w + j] == dt) {
                out[k++] = (v || sc.allow) ? (v ? 'M' : 'S') : 'X';
                --i; --j;
                continue;
            }
        }
        if (i > 0 && H[i * w + j] == H[(i - 1) * w + j] + sc.gap) { out[k++] = 'U'; --i; }
        else { out[k++] = 'L'; --j; }
    }
    for (int p = 0, q = k - 1; p < q; ++p, --q) { const uint8_t t = out[p]; out[p] = out[q]; out[q] = t; }
    return k;
}

// One leaf: the whole HirschbergRec below it (explicit stack, left child first), forward ops.
template <typename Row, typename Seq, typename Match>
__device__ int hb_leaf_solve(Seq S1, Seq S2, int alen, int blen, bool top, Row F, Row Cc, Row Hs, uint8_t* out,
                             int32_t* score, const Match& mt, const HbScore& sc) {
    if (top) {
        int32_t s;
        if (alen == 0) s = blen * sc.gap;
        else if (blen == 0) s = alen * sc.gap;
        else { hb_nwscore(S1, alen, 0, S2, blen, 0, mt, sc, F); s = F[blen]; }
        *score = s;
    }
    int k = 0;
    int stk[40][4];   // pending right children; depth <= 2 + log2(alen)
    int sp = 0;
    stk[sp][0] = 0; stk[sp][1] = alen; stk[sp][2] = 0; stk[sp][3] = blen; ++sp;
    while (sp > 0) {
        --sp;
        const int x0 = stk[sp][0], xl = stk[sp][1], y0 = stk[sp][2], yl = stk[sp][3];
        if (xl == 0) {
            for (int q = 0; q < yl; ++q) out[k++] = 'L';
        } else if (yl == 0) {
            for (int q = 0; q < xl; ++q) out[k++] = 'U';
        } else if (xl == 1 || yl == 1) {
            k += hb_nw_small(S1.shifted(x0), xl, S2.shifted(y0), yl, mt, sc, Hs, out + k);
        } else {
            const int mid = xl / 2;
            const Seq A0 = S1.shifted(x0), B0 = S2.shifted(y0), A1 = S1.shifted(x0 + mid);
            hb_nwscore(A0, mid, 0, B0, yl, 0, mt, sc, F);
            for (int q = 0; q <= yl; ++q) Cc[q] = F[q];
            hb_nwscore(A1, xl - mid, 1, B0, yl, 1, mt, sc, F);
            int mid2 = 0;
            int32_t best = INT_MIN;
            for (int i = 0; i < yl; ++i) {
                const int32_t s = Cc[i] + F[yl - i];
                if (s >= best) { best = s; mid2 = i; }
            }
            // right child below, left child on top: left is finished first (:155, :161)
            stk[sp][0] = x0 + mid; stk[sp][1] = xl - mid; stk[sp][2] = y0 + mid2; stk[sp][3] = yl - mid2; ++sp;
            stk[sp][0] = x0; stk[sp][1] = mid; stk[sp][2] = y0; stk[sp][3] = mid2; ++sp;
        }
    }
    return k;
}

// Leaves with |Seq1|, |Seq2| <= kHbLdsCols run with LDS rows + symbols: 2 rows + 2 symbol
// strings per thread, 15.8 KiB per 64-thread block at 24 (at 64 with a third row it was 58 KiB:
// 2 blocks per CU).  Leaves have <= kHbLeafRows rows; wider ones take the global-scratch path.
// Measured (tools/ab_dc.sh, 10,000 x 1024^2; profiles/ab_dc_r02*.txt): 64 cols / 48-row leaves
// 21.3 ms, 48 / 48 17.1, 32 / 24 12.6, then with packed sweeps 32 / 12 9.2, 24 / 12 9.0 ms.
#ifndef SA_HB_LDS_COLS
#define SA_HB_LDS_COLS 24
#endif
constexpr int kHbLdsCols = SA_HB_LDS_COLS;

// A leaf's global scratch lives at 6 * key (F, -, Cc: 3 (blen + 1); base-case matrix:
// 2 (max(alen, blen) + 1); together <= 6 (alen + blen) whenever alen, blen >= 1, the only
// leaves that use scratch), its forward ops at stage[key], its op count at mark[key].
// BITS: the generic-Ty path (symbols = pair-local indices, match = the pair's bitmap).
template <bool BITS>
__global__ __launch_bounds__(64) void hb_leaf_kernel(const uint8_t* s1, const uint8_t* s2, const DcSub* leaves,
                                                     const uint32_t* nleaves, int32_t* scratch, uint8_t* stage,
                                                     int32_t* mark, sa_result* res, const uint32_t* lut,
                                                     DcBits bits, HbScore sc) {
    __shared__ int32_t s_rows[2 * (kHbLdsCols + 1) * 64];
    __shared__ uint8_t s_seq[BITS ? 1 : 2 * kHbLdsCols * 64];
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= *nleaves) return;
    const int t = threadIdx.x;
    const DcSub L = leaves[id];
    const uint64_t key = L.a0 + L.b0;
    int32_t* Fg = scratch + 6 * key;
    int32_t* Hs = Fg + 3 * (L.n + 1);
    uint8_t* out = stage + key;
    int32_t* score = &res[L.pair].score;   // written only for a top leaf
    const bool in_lds = L.m <= kHbLdsCols && L.n <= kHbLdsCols;
    dc_lds_i32* r0 = (dc_lds_i32*)s_rows + t;
    const LRow F{r0}, Cc{r0 + (kHbLdsCols + 1) * 64};
    int k;
    if constexpr (BITS) {
        uint64_t b1, b2;
        const DcBitsMatch mt = bits.of(L.pair, &b1, &b2);
        const ISeq S1{(uint32_t)(L.a0 - b1)}, S2{(uint32_t)(L.b0 - b2)};
        if (in_lds) k = hb_leaf_solve(S1, S2, L.m, L.n, L.top != 0, F, Cc, F, out, score, mt, sc);
        else k = hb_leaf_solve(S1, S2, L.m, L.n, L.top != 0, GRow{Fg}, GRow{Fg + 2 * (L.n + 1)}, GRow{Hs}, out, score, mt, sc);
    } else {
        const uint8_t* g1 = s1 + L.a0;
        const uint8_t* g2 = s2 + L.b0;
        const DcLutMatch mt{lut};
        if (in_lds) {
            dc_lds_u8* q1 = (dc_lds_u8*)s_seq + t;
            dc_lds_u8* q2 = q1 + kHbLdsCols * 64;
            for (int c = 0; c < L.m; ++c) q1[c * 64] = g1[c];
            for (int c = 0; c < L.n; ++c) q2[c * 64] = g2[c];
            // a base case's (<= 2 x (kHbLdsCols + 1)) matrix reuses F and Cc, both dead by then
            k = hb_leaf_solve(LSeq{q1}, LSeq{q2}, L.m, L.n, L.top != 0, F, Cc, F, out, score, mt, sc);
        } else {
            k = hb_leaf_solve(GSeq{g1}, GSeq{g2}, L.m, L.n, L.top != 0, GRow{Fg}, GRow{Fg + 2 * (L.n + 1)}, GRow{Hs},
                              out, score, mt, sc);
        }
    }
    if (k) mark[key] = k;
}

// ---------------------------------------------------------------------------- host driver
namespace {

struct HbLaunch {
    const uint8_t* d1;
    const uint8_t* d2;
    const DcSub* split;
    const DcLevel* lvl;
    int32_t* rows;
    const uint32_t* lut;
    DcBits bits;
    HbScore sc;
    Dc16 d16;
};

template <int MM, bool ALLOW>
void launch_sweeps_t(int R, int G, uint32_t count, const HbLaunch& a_in, hipStream_t st) {
    const dim3 block(64);
    HbLaunch a = a_in;
    // 16-bit sweeps of <= 128 rows (whole-wave R = 1, 2): two per wave (hb_sweep_seg16_kernel, 2R rows per lane), the
    // whole-wave kernel beside it for the int32 case
    if (MM != kMatchBits && a.d16.aux && G == 0 && R <= 2) {
        const dim3 grid2((count + 1) / 2);
        if (R == 1) hipLaunchKernelGGL(hb_sweep_seg16_kernel<2>, grid2, block, 0, st, a.d1, a.d2, a.split, a.lvl, a.rows, a.sc, a.d16);
        else hipLaunchKernelGGL(hb_sweep_seg16_kernel<4>, grid2, block, 0, st, a.d1, a.d2, a.split, a.lvl, a.rows, a.sc, a.d16);
        a.d16.seg16 = 1;
    }
#define SA_HB_SEG(GG)                                                                                           \
    hipLaunchKernelGGL((hb_sweep_seg_kernel<GG, MM, ALLOW>), dim3((count + 64 / GG - 1) / (64 / GG)), block, 0, st, \
                       a.d1, a.d2, a.split, a.lvl, a.rows, a.lut, a.bits, a.sc)
#define SA_HB_SW(RR) \
    hipLaunchKernelGGL((hb_sweep_kernel<RR, MM, ALLOW>), dim3(a.d16.seg16 ? std::min(count, kDcSkipGrid) : count), block, 0, st, a.d1, a.d2, a.split, a.lvl, a.rows, a.lut, a.bits, a.sc, a.d16)
    if (G == 8) SA_HB_SEG(8);
    else if (G == 16) SA_HB_SEG(16);
    else if (G == 32) SA_HB_SEG(32);
    else if (R == 1) SA_HB_SW(1);
    else if (R == 2) SA_HB_SW(2);
    else if (R == 4) SA_HB_SW(4);
    else if (R == 8) SA_HB_SW(8);
    else if (R == 16) SA_HB_SW(16);
    else SA_HB_SW(32);
#undef SA_HB_SEG
#undef SA_HB_SW
}

// G = 8 / 16 / 32: packed sweeps (maxa <= G); G = 0: R rows per lane, one sweep per wave.
hipError_t launch_sweeps(int R, int G, uint32_t count, const HbLaunch& a, hipStream_t st) {
    const int mm = a.bits.mbits ? kMatchBits : a.lut ? kMatchLut : kMatchEq;
    if (mm == kMatchBits) a.sc.allow ? launch_sweeps_t<kMatchBits, true>(R, G, count, a, st)
                                     : launch_sweeps_t<kMatchBits, false>(R, G, count, a, st);
    else if (mm == kMatchLut) a.sc.allow ? launch_sweeps_t<kMatchLut, true>(R, G, count, a, st)
                                         : launch_sweeps_t<kMatchLut, false>(R, G, count, a, st);
    else a.sc.allow ? launch_sweeps_t<kMatchEq, true>(R, G, count, a, st) : launch_sweeps_t<kMatchEq, false>(R, G, count, a, st);
    return hipGetLastError();
}

}  // namespace

// Host driver: inputs, results and the traceback-order op streams (pair p's at
// o1[p] + o2[p] + p) all on the device; enqueued on st without waiting for it (grid
// bounds from b).
int hirschberg_run(DcWork& w, hipEvent_t prev, const sa_scoring* scoring, const DcInputs& in, const DcBounds& b,
                   hipStream_t st, sa_result* d_res, uint8_t* d_ops, std::string* err) {
    int leaf_rows = kHbLeafRows;   // tuning override: SEQALIB_HB_LEAF
    if (const char* lr = getenv("SEQALIB_HB_LEAF")) leaf_rows = std::max(2, atoi(lr));
    const char* segenv = getenv("SEQALIB_DC_SEG");   // 0: whole-wave sweeps only (A/B, tests)
    const bool seg_sweeps = !segenv || atoi(segenv) != 0;
    constexpr int rmax = 32;                         // the sweep's largest R
    const uint32_t npairs = in.npairs;
    HbScore sc;
    sc.gap = scoring->gap;
    sc.match = scoring->match;
    sc.allow = scoring->allow_mismatch != 0;
    sc.mismatch = sc.allow ? scoring->mismatch : INT_MIN;
    const bool bits = in.bits.mbits != nullptr;
    SA_DC_HIP(w.prepare(b, npairs, leaf_rows, 2, 2, 6, st, prev));
    // 16-bit whole-wave sweeps when the shapes and scoring admit them (sa_dc.h Dc16); the device
    // takes them when the batch alphabet has <= 4 symbols
    Dc16 d16 = bits ? Dc16{} : dc16_plan(false, scoring, b.max_m, b.max_n);
    if (d16.aux) {
        SA_DC_HIP(w.aux.alloc(kAuxWords));
        SA_DC_HIP(launch_alphabet_scan(in.d1, in.o1, in.d2, in.o2, npairs, w.aux.p, st));
        SA_DC_HIP(launch_decide_t16(in.lutbits, sc.match, d16.mismatch, 2, w.aux.p, st));
        d16.aux = w.aux.p;
    }
    SA_DC_HIP(hipMemsetAsync(d_res, 0, sizeof(sa_result) * npairs, st));
    SA_DC_HIP(dc_launch_init(in.o1, in.o2, npairs, 0, b, w.cur.p, d_res, st));
    uint32_t cap = npairs;     // upper bound on this level's subproblems
    int maxm = (int)b.max_m;        // upper bound on their Seq1 length
    for (int l = 0;; ++l) {
        SA_DC_HIP(dc_launch_classify(w.cur.p, cap, npairs, l ? w.lvl.p + l - 1 : nullptr, 2, leaf_rows, 2,
                                     w.lvl.p + l, w.split.p, w.leaves.p, w.nleaf(), st));
        if (maxm <= leaf_rows) break;
        const uint32_t splits = std::min<uint64_t>(cap, w.max_splits);
        const int maxa = (maxm + 1) / 2;
        int R = 1;
        while (R < rmax && 64 * R < maxa) R *= 2;   // bands of 64 R rows
        const int G = !seg_sweeps ? 0 : maxa <= 8 ? 8 : maxa <= 16 ? 16 : maxa <= 32 ? 32 : 0;
        const HbLaunch a{in.d1, in.d2, w.split.p, w.lvl.p + l, w.rows.p, in.lutbits, in.bits, sc, d16};
        SA_DC_HIP(launch_sweeps(R, G, 2 * splits, a, st));
        // lanes per split: the level's rows bound the split's columns only loosely (n ~ m for
        // similar pairs), any n is exact, a wider one just loops
        const int gs = dc_split_lanes(maxm);
        if (gs == 64)
            hipLaunchKernelGGL(hb_split_kernel<64>, dim3(splits), dim3(64), 0, st, w.split.p, w.lvl.p + l, w.rows.p,
                               w.next.p, d_res);
        else if (gs == 16)
            hipLaunchKernelGGL(hb_split_kernel<16>, dim3((splits + 3) / 4), dim3(64), 0, st, w.split.p, w.lvl.p + l,
                               w.rows.p, w.next.p, d_res);
        else
            hipLaunchKernelGGL(hb_split_kernel<8>, dim3((splits + 7) / 8), dim3(64), 0, st, w.split.p, w.lvl.p + l,
                               w.rows.p, w.next.p, d_res);
        SA_DC_HIP(hipGetLastError());
        w.cur.swap(w.next);
        cap = 2 * splits;
        maxm = maxa;
    }
    if (bits)
        hipLaunchKernelGGL(hb_leaf_kernel<true>, dim3((w.leaf_cap + 63) / 64), dim3(64), 0, st, in.d1, in.d2, w.leaves.p,
                           w.nleaf(), w.scratch.p, w.stage.p, w.mark.p, d_res, in.lutbits, in.bits, sc);
    else
        hipLaunchKernelGGL(hb_leaf_kernel<false>, dim3((w.leaf_cap + 63) / 64), dim3(64), 0, st, in.d1, in.d2, w.leaves.p,
                           w.nleaf(), w.scratch.p, w.stage.p, w.mark.p, d_res, in.lutbits, in.bits, sc);
    SA_DC_HIP(hipGetLastError());
    SA_DC_HIP(dc_launch_assemble(in.o1, in.o2, npairs, w.mark.p, w.stage.p, d_res, d_ops, st));
    return 0;
}

}  // namespace sa
