// sa_myersmiller.hip — MyersMillerSA::getAlignment (SAMyersMiller.h:43-420) on the GPU, batched
// over pairs: linear-space affine-gap global alignment whose result is exactly the reference's
// (its midpoint tie rules, boundary gap opens tb/te and base cases), not merely an optimal one.
//
// Breadth-first over all pairs at once, like sa_hirschberg.hip:
//   * device levels: every subproblem with more than kMmLeafRows rows of Seq1 and >= 1 column is
//     split.  Its forward sweep (CC/DD over the top half, :172-238) and reverse sweep (RR/SS over
//     the bottom half read backwards, :247-313) become two rows of one batched launch of
//     mm_sweep_kernel (score-only affine DP, one wave per sweep, anti-diagonal wavefront; each
//     sweep writes its last C and D rows); mm_split_kernel then takes, per subproblem, the FIRST
//     j in [0, N] maximising max(CC[j] + RR[j], DD[j] + SS[j] - g) and the midpoint type
//     (type 2 iff the gap term is not strictly smaller, :320-340) and writes the children with
//     their tb/te (:358-395) as the next level's subproblems (three slots per split; a type-1
//     midpoint leaves the third empty).  A type-2 midpoint's two deletions (:390-392) become a leaf
//     of 2 rows and 0 columns, which emits exactly those.
//   * leaves: mm_leaf_kernel, one thread per subproblem, runs the same recursion iteratively
//     (explicit stack, left child first) including the base cases N == 0, M == 0 and M == 1
//     (:57-160, with its "failsafe" pair of gap entries).
//   * assembly: dc_assemble_kernel (sa_dc.hip).  The level loop stays on the device (sa_dc.hip:
//     key-addressed buffers, device-side classification).
// Score reported (the reference exposes none): the top call's optimum — its midpoint maximum,
// the M == 1 maximum, or the boundary value of an empty side (oracle: align_myers_miller).
//
// The reverse sweep is computed as a forward sweep over the reversed sequences with t0 = te, so
// RR[j] = Crev[N - j] and SS[j] = Drev[N - j] (including SS[N] = RR[N], :313).
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "sa_dc.h"
#include "sa_internal.h"

namespace sa {

constexpr int kMmLeafRows = 12;   // subproblems with <= this many Seq1 rows are leaves (tuned, tools/ab_dc.sh)

struct MmSweep {       // affine sweep over A (alen) x B (blen) -> C row at out, D row at out + blen + 1
    uint64_t a, b;     // index of A[0] / B[0] in seq1 / seq2 (rev: of the LAST element, read first)
    int32_t alen, blen;
    int32_t rev;       // 1: A and B are both read backwards
    int32_t t0;        // gap open charged on column 0 (tb forwards, te backwards)
    uint64_t out;      // int32 index into the row buffer
};

struct MmScore {
    int32_t g, h, match, mismatch, allow;   // mismatch = INT_MIN when !allow (:15)
};

// Sweep rows of a split subproblem live at 4 * key: forward C, D, reverse C, D, n + 1 ints
// each (4 (n + 1) <= 4 (m + n), inside its key span).
__device__ __forceinline__ MmSweep mm_sweep_of(const DcSub& s, int rev) {
    const int mid = s.m / 2;
    const uint64_t base = 4 * (s.a0 + s.b0);
    if (!rev) return MmSweep{s.a0, s.b0, mid, s.n, 0, s.tb, base};
    return MmSweep{s.a0 + (uint64_t)s.m - 1, s.b0 + (uint64_t)s.n - 1, s.m - mid, s.n, 1, s.te,
                   base + 2ull * ((uint64_t)s.n + 1)};
}

// diagonal candidate of c = max({DD, e, s + Similarity}) (:218-232); INT_MIN drops out of the max
__device__ __forceinline__ int32_t mm_diag(int32_t s, bool v, const MmScore& sc) {
    return (sc.allow || v) ? s + (v ? sc.match : sc.mismatch) : INT_MIN;
}

// ------------------------------------------------------------------ batched affine sweeps
// Lane t owns R consecutive rows of a 64R-row band and computes column s - t at step s.  Per
// row it keeps C and e (the horizontal-gap state) of the previous column; (C, D) of the row
// above come from the lane above via DPP wave_shr:1 (lane 0: the previous band's last row,
// written in place to the output rows, or the top boundary).  The match source (MM: DcSrc in
// sa_dc.h) and ALLOW are compile-time so the cell is branch-free; LAST (the band holding row m)
// also captures D of row m.
template <bool ALLOW>
__device__ __forceinline__ int32_t mm_diag_v(int32_t cd, bool v, const MmScore& sc) {
    if constexpr (ALLOW) return cd + (v ? sc.match : sc.mismatch);
    else return v ? cd + sc.match : INT_MIN;
}

template <int R, int MM, bool ALLOW, bool LAST>
__device__ __forceinline__ void mm_band(const MmSweep& d, const DcSrc<MM>& src, const MmScore& sc, int band,
                                        int32_t* outC, int32_t* outD, int tl, int rl, int32_t& cl, int32_t& dl) {
    const int lane = threadIdx.x;
    const int m = d.alen, n = d.blen, g = sc.g, h = sc.h;
    constexpr int BAND = 64 * R;
    const int row0 = band * BAND + lane * R;
    uint32_t a[R];
    int32_t Cp[R], Ep[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        a[r] = row0 + r < m ? src.a(d.rev ? d.a - (row0 + r) : d.a + (row0 + r)) : 0u;
        Cp[r] = d.t0 + h * (row0 + r + 1);                   // C[i][0] = t0 + i h (:192-197)
        Ep[r] = Cp[r] + g;                                   // e = t + g (:198)
    }
    int32_t prev_up = row0 == 0 ? 0 : d.t0 + h * row0;       // C[row0][0]; C[0][0] = 0 (:172)
    // Per 64-step chunk, lane k holds column c0+k's row-above (C, D) (for lane 0) and Seq2
    // symbol, loaded one chunk ahead; they reach their lane by DPP like the fill kernel.
    auto load_chunk = [&](int c0, int32_t& vc, int32_t& vd, uint32_t& vs) {
        const int j = c0 + lane;
        vc = 0;
        vd = 0;
        vs = 0;
        if (j < n) {
            if (band == 0) {
                vc = g + h * (j + 1);                        // CC[j] = g + j h, DD[j] = CC[j] + g (:183-188)
                vd = vc + g;
            } else {
                vc = outC[j + 1];
                vd = outD[j + 1];
            }
            vs = src.b(d.rev ? d.b - j : d.b + j);
        }
    };
    int32_t vc, vd, nvc, nvd;
    uint32_t vs, nvs, sym = 0;
    load_chunk(0, vc, vd, vs);
    for (int c0 = 0; c0 < n + 63; c0 += 64) {
        load_chunk(c0 + 64, nvc, nvd, nvs);
        const int steps = min(64, n + 63 - c0);
        const bool steady = c0 >= 63 && c0 + 64 <= n;   // every lane inside (as the 16-bit sweep)
        for (int q = 0; q < steps; ++q) {
            const int s = c0 + q;
            const int32_t up_c = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vc, q), cl, 0x138, 0xf, 0xf, false);
            const int32_t up_d = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vd, q), dl, 0x138, 0xf, 0xf, false);
            sym = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vs, q), sym, 0x138, 0xf, 0xf, false);
            const int j0 = s - lane;
            if (steady || (j0 >= 0 && j0 < n)) {
                int32_t cd = prev_up, cu = up_c, du = up_d, dsel = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int32_t e = max(Ep[r], Cp[r] + g) + h;   // :202
                    const int32_t dd = max(du, cu + g) + h;        // :203
                    const int32_t c = max(max(dd, e), mm_diag_v<ALLOW>(cd, src.match(a[r], sym), sc));
                    cd = Cp[r];
                    Cp[r] = c;
                    Ep[r] = e;
                    cu = c;
                    du = dd;
                    if constexpr (LAST) {
                        if (r == rl) dsel = dd;
                    }
                }
                prev_up = up_c;
                cl = Cp[R - 1];
                dl = du;
                if constexpr (!LAST) {
                    if (lane == 63) {                         // this band's last row, in place
                        outC[j0 + 1] = cl;
                        outD[j0 + 1] = dl;
                    }
                } else if (lane == tl) {
                    int32_t csel = Cp[0];
#pragma unroll
                    for (int r = 1; r < R; ++r)
                        if (r == rl) csel = Cp[r];
                    outC[j0 + 1] = csel;                      // row m of the sweep
                    outD[j0 + 1] = dsel;
                }
            }
        }
        vc = nvc;
        vd = nvd;
        vs = nvs;
    }
}

// 16-bit band of a whole-wave affine sweep (Dc16, sa_dc.h): C, e and D kept as value - delta in the
// low 16 bits.  Per cell (per row): e = max(Ep, Cp + g) + h and D = max(Du, Cu + g) + h (three
// 16-bit ops each), the diagonal Cd + s (v_bfe_i32 of the row's byte profile + v_add_u16), and
// C = max(max(D, e), diag) (two v_max_i16): ten instructions, one of them 32-bit.
template <int R, bool LAST>
__device__ __forceinline__ void mm_band16(const MmSweep& d, const uint8_t* s1, const uint8_t* s2, const uint32_t* aux,
                                          int32_t delta, const MmScore& sc, int band, int32_t* outC, int32_t* outD,
                                          int tl, int rl, int32_t& cl, int32_t& dl, int32_t* s_park) {
    const int lane = threadIdx.x;
    const int m = d.alen, n = d.blen, g = sc.g, h = sc.h;
    constexpr int BAND = 64 * R;
    const uint32_t symp = aux[kAuxProf + 4];
    const uint32_t g16 = (uint32_t)g & 0xffffu, h16 = (uint32_t)h & 0xffffu;
    const int row0 = band * BAND + lane * R;
    uint32_t a[R];
    int32_t Cp[R], Ep[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        a[r] = row < m ? aux[kAuxProf + (dc_code8(symp, d.rev ? s1[d.a - row] : s1[d.a + row]) >> 3)] : 0u;
        Cp[r] = d.t0 + h * (row + 1) - delta;                // C[i][0] = t0 + i h (:192-197)
        Ep[r] = Cp[r] + g;                                   // e = t + g (:198)
    }
    int32_t prev_up = (row0 == 0 ? 0 : d.t0 + h * row0) - delta;   // C[row0][0]; C[0][0] = 0 (:172)
    auto load_chunk = [&](int c0, int32_t& vc, int32_t& vd, uint32_t& vs) {
        const int j = c0 + lane;
        vc = 0;
        vd = 0;
        vs = 0;
        if (j < n) {
            if (band == 0) {
                vc = g + h * (j + 1);                        // CC[j] = g + j h, DD[j] = CC[j] + g (:183-188)
                vd = vc + g;
            } else {
                vc = outC[j + 1];
                vd = outD[j + 1];
            }
            vc -= delta;
            vd -= delta;
            vs = dc_code8(symp, d.rev ? s2[d.b - j] : s2[d.b + j]);
        }
    };
    int32_t vc, vd, nvc, nvd;
    uint32_t vs, nvs, sym = 0;
    // the R cells of one step, updated in place (Cp, Ep): row r's block also forms row r+1's
    // diagonal + s from the OLD Cp[r] before overwriting it, so the step needs no register copies;
    // on_d(r, D) sees every row's new D; returns the last row's D
    auto cells = [&](int32_t up_c, int32_t up_d, auto&& on_d) __attribute__((always_inline)) -> int32_t {
        uint32_t tcur;
        asm("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(tcur) : "v"(a[0]), "v"(sym), "v"(prev_up));
        int32_t cu = up_c, du = up_d;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t tmp, dd, tn = 0;
            if (r + 1 < R) {
                asm("v_add_u16 %[tmp], %[g], %[cp]\n\t"   // e = max(Ep, Cp + g) + h      (:202)
                    "v_max_i16 %[ep], %[ep], %[tmp]\n\t"
                    "v_add_u16 %[ep], %[h], %[ep]\n\t"
                    "v_add_u16 %[dd], %[g], %[cu]\n\t"    // D = max(Du, Cu + g) + h      (:203)
                    "v_max_i16 %[dd], %[du], %[dd]\n\t"
                    "v_add_u16 %[dd], %[h], %[dd]\n\t"
                    "v_bfe_i32 %[tn], %[an], %[sym], 8\n\t"   // next row: Cd + s(a, b) (old Cp)
                    "v_add_u16 %[tn], %[cp], %[tn]\n\t"
                    "v_max_i16 %[tmp], %[dd], %[ep]\n\t"  // C = max(max(D, e), diag)
                    "v_max_i16 %[cp], %[tc], %[tmp]"
                    : [tmp] "=&v"(tmp), [dd] "=&v"(dd), [tn] "=&v"(tn), [cp] "+v"(Cp[r]), [ep] "+v"(Ep[r])
                    : [g] "s"(g16), [h] "s"(h16), [cu] "v"(cu), [du] "v"(du), [an] "v"(a[r + 1 < R ? r + 1 : r]),
                      [sym] "v"(sym), [tc] "v"(tcur));
            } else {
                asm("v_add_u16 %[tmp], %[g], %[cp]\n\t"
                    "v_max_i16 %[ep], %[ep], %[tmp]\n\t"
                    "v_add_u16 %[ep], %[h], %[ep]\n\t"
                    "v_add_u16 %[dd], %[g], %[cu]\n\t"
                    "v_max_i16 %[dd], %[du], %[dd]\n\t"
                    "v_add_u16 %[dd], %[h], %[dd]\n\t"
                    "v_max_i16 %[tmp], %[dd], %[ep]\n\t"
                    "v_max_i16 %[cp], %[tc], %[tmp]"
                    : [tmp] "=&v"(tmp), [dd] "=&v"(dd), [cp] "+v"(Cp[r]), [ep] "+v"(Ep[r])
                    : [g] "s"(g16), [h] "s"(h16), [cu] "v"(cu), [du] "v"(du), [tc] "v"(tcur));
            }
            tcur = tn;
            cu = Cp[r];
            du = (int32_t)dd;
            on_d(r, (int32_t)dd);
        }
        return du;
    };
    // Steady chunk (c0 >= 63, c0 + 64 <= n; as hb_band16): no per-lane branch; the handed-on row
    // (C and D of lane 63's last row, or of row m at lane tl / register rl in the last band) is
    // parked per step in LDS by every lane (others into a discard slot) and stored per chunk.
    const int src_lane = LAST ? tl : 63;
    auto steady_park = [&](int c0, auto SRC) {
        constexpr int SR = decltype(SRC)::value;
        int32_t* const park = s_park + (lane == src_lane ? 0 : 64);
#pragma unroll 1
        for (int q = 0; q < 64; ++q) {
            const int32_t up_c = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vc, q), cl, 0x138, 0xf, 0xf, false);
            const int32_t up_d = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vd, q), dl, 0x138, 0xf, 0xf, false);
            sym = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vs, q), sym, 0x138, 0xf, 0xf, false);
            int32_t dsel = 0;
            dl = cells(up_c, up_d, [&](int r, int32_t dd) __attribute__((always_inline)) { if (r == SR) dsel = dd; });
            prev_up = up_c;
            cl = Cp[R - 1];
            park[q] = Cp[SR];
            park[128 + q] = dsel;
        }
        __syncthreads();   // (one wave: orders the parked writes before the reads)
        outC[c0 - src_lane + 1 + lane] = dc_unpack16(s_park[lane], delta);
        outD[c0 - src_lane + 1 + lane] = dc_unpack16(s_park[128 + lane], delta);
        __syncthreads();
    };
    load_chunk(0, vc, vd, vs);
    for (int c0 = 0; c0 < n + 63; c0 += 64) {
        load_chunk(c0 + 64, nvc, nvd, nvs);
        if (s_park && c0 >= 63 && c0 + 64 <= n) {
            const int src_r = LAST ? rl : R - 1;
            dc_row_dispatch<R>(src_r, [&](auto SRC) { steady_park(c0, SRC); });   // (uniform)
            vc = nvc;
            vd = nvd;
            vs = nvs;
            continue;
        }
        const int steps = min(64, n + 63 - c0);
        // steady chunk without parking (SEQALIB_DC16_PARK=0): every lane is inside the matrix for
        // all 64 steps, so the per-lane range branch is skipped (the hand-off store keeps its lane test)
        const bool steady = c0 >= 63 && c0 + 64 <= n;
        for (int q = 0; q < steps; ++q) {
            const int s = c0 + q;
            const int32_t up_c = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vc, q), cl, 0x138, 0xf, 0xf, false);
            const int32_t up_d = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vd, q), dl, 0x138, 0xf, 0xf, false);
            sym = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vs, q), sym, 0x138, 0xf, 0xf, false);
            const int j0 = s - lane;
            if (steady || (j0 >= 0 && j0 < n)) {
                int32_t dsel = 0;
                dl = cells(up_c, up_d, [&](int r, int32_t dd) __attribute__((always_inline)) {
                    if constexpr (LAST) {
                        if (r == rl) dsel = dd;
                    }
                });
                prev_up = up_c;
                cl = Cp[R - 1];
                if constexpr (!LAST) {
                    if (lane == 63) {                         // this band's last row, in place
                        outC[j0 + 1] = dc_unpack16(cl, delta);
                        outD[j0 + 1] = dc_unpack16(dl, delta);
                    }
                } else if (lane == tl) {
                    int32_t csel = Cp[0];
#pragma unroll
                    for (int r = 1; r < R; ++r)
                        if (r == rl) csel = Cp[r];
                    outC[j0 + 1] = dc_unpack16(csel, delta);  // row m of the sweep
                    outD[j0 + 1] = dc_unpack16(dsel, delta);
                }
            }
        }
        vc = nvc;
        vd = nvd;
        vs = nvs;
    }
}

// Deep levels of the 16-bit sweeps (Dc16): TWO sweeps per wave, 32 lanes x R rows each (as
// hb_sweep_seg16_kernel): a sweep of at most 32 R rows is one band; lanes 0 and 32 take their own
// segment's top row (C, D) and column symbol.  Cells as mm_band16's.  Runs only when the device
// picked the 16-bit path; mm_sweep_kernel (launched beside it, Dc16::seg16) returns at once then.
template <int R>
__global__ __launch_bounds__(64) void mm_sweep_seg16_kernel(const uint8_t* s1, const uint8_t* s2, const DcSub* split,
                                                            const DcLevel* lvl, int32_t* rows, MmScore sc, Dc16 d16) {
    if (!(d16.aux && d16.aux[kAuxSel] == 1)) return;   // the int32 sweeps run (mm_sweep_kernel)
    const int lane = threadIdx.x;
    if (blockIdx.x * 2 >= 2 * lvl->nsplit) return;   // grid sized from an upper bound (uniform exit)
    const int seg = lane >> 5, ls = lane & 31;
    const uint32_t swi = blockIdx.x * 2 + seg;
    const bool active = swi < 2 * lvl->nsplit;
    MmSweep d{};
    if (active) d = mm_sweep_of(split[swi / 2], swi & 1);
    const uint32_t* aux = d16.aux;
    const int32_t delta = d16.delta;
    const int m = d.alen, n = d.blen, g = sc.g, h = sc.h;
    const uint32_t symp = aux[kAuxProf + 4];
    const uint32_t g16 = (uint32_t)g & 0xffffu, h16 = (uint32_t)h & 0xffffu;
    const int row0 = ls * R;
    uint32_t a[R];
    int32_t Cp[R], Ep[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        a[r] = active && row < m ? aux[kAuxProf + (dc_code8(symp, d.rev ? s1[d.a - row] : s1[d.a + row]) >> 3)] : 0u;
        Cp[r] = d.t0 + h * (row + 1) - delta;                // C[i][0] = t0 + i h (:192-197)
        Ep[r] = Cp[r] + g;                                   // e = t + g (:198)
    }
    int32_t prev_up = (row0 == 0 ? 0 : d.t0 + h * row0) - delta;   // C[row0][0]; C[0][0] = 0 (:172)
    const int tl = active ? (m - 1) / R : -1, rl = active ? (m - 1) % R : 0;   // owner of row m
    int32_t* const outC = rows + d.out;
    int32_t* const outD = outC + n + 1;
    uint32_t sym = 0;
    auto cells = [&](int32_t up_c, int32_t up_d, int32_t& dsel) __attribute__((always_inline)) -> int32_t {
        uint32_t tcur;
        asm("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(tcur) : "v"(a[0]), "v"(sym), "v"(prev_up));
        int32_t cu = up_c, du = up_d;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t tmp, dd, tn = 0;
            if (r + 1 < R) {
                asm("v_add_u16 %[tmp], %[g], %[cp]\n\t"
                    "v_max_i16 %[ep], %[ep], %[tmp]\n\t"
                    "v_add_u16 %[ep], %[h], %[ep]\n\t"
                    "v_add_u16 %[dd], %[g], %[cu]\n\t"
                    "v_max_i16 %[dd], %[du], %[dd]\n\t"
                    "v_add_u16 %[dd], %[h], %[dd]\n\t"
                    "v_bfe_i32 %[tn], %[an], %[sym], 8\n\t"
                    "v_add_u16 %[tn], %[cp], %[tn]\n\t"
                    "v_max_i16 %[tmp], %[dd], %[ep]\n\t"
                    "v_max_i16 %[cp], %[tc], %[tmp]"
                    : [tmp] "=&v"(tmp), [dd] "=&v"(dd), [tn] "=&v"(tn), [cp] "+v"(Cp[r]), [ep] "+v"(Ep[r])
                    : [g] "s"(g16), [h] "s"(h16), [cu] "v"(cu), [du] "v"(du), [an] "v"(a[r + 1 < R ? r + 1 : r]),
                      [sym] "v"(sym), [tc] "v"(tcur));
            } else {
                asm("v_add_u16 %[tmp], %[g], %[cp]\n\t"
                    "v_max_i16 %[ep], %[ep], %[tmp]\n\t"
                    "v_add_u16 %[ep], %[h], %[ep]\n\t"
                    "v_add_u16 %[dd], %[g], %[cu]\n\t"
                    "v_max_i16 %[dd], %[du], %[dd]\n\t"
                    "v_add_u16 %[dd], %[h], %[dd]\n\t"
                    "v_max_i16 %[tmp], %[dd], %[ep]\n\t"
                    "v_max_i16 %[cp], %[tc], %[tmp]"
                    : [tmp] "=&v"(tmp), [dd] "=&v"(dd), [cp] "+v"(Cp[r]), [ep] "+v"(Ep[r])
                    : [g] "s"(g16), [h] "s"(h16), [cu] "v"(cu), [du] "v"(du), [tc] "v"(tcur));
            }
            tcur = tn;
            cu = Cp[r];
            du = (int32_t)dd;
            if (r == rl) dsel = (int32_t)dd;
        }
        return du;
    };
    auto load_chunk = [&](int c0, int32_t& vc, int32_t& vd, uint32_t& vs) {
        const int j = c0 + ls;
        vc = 0;
        vd = 0;
        vs = 0;
        if (active && j < n) {
            vc = g + h * (j + 1);                            // CC[j] = g + j h, DD[j] = CC[j] + g (:183-188)
            vd = vc + g;
            vc -= delta;
            vd -= delta;
            vs = dc_code8(symp, d.rev ? s2[d.b - j] : s2[d.b + j]);
        }
    };
    int steps = active ? n + 31 : 0;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) steps = max(steps, __shfl_xor(steps, off));
    int32_t vc, vd, nvc, nvd, cl = Cp[R - 1], dl = Ep[R - 1];
    uint32_t vs, nvs;
    load_chunk(0, vc, vd, vs);
    for (int c0 = 0; c0 < steps; c0 += 32) {
        load_chunk(c0 + 32, nvc, nvd, nvs);
        const int qn = min(32, steps - c0);
        for (int q = 0; q < qn; ++q) {
            int32_t up_c = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vc, q), cl, 0x138, 0xf, 0xf, false);
            int32_t up_d = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vd, q), dl, 0x138, 0xf, 0xf, false);
            sym = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vs, q), sym, 0x138, 0xf, 0xf, false);
            const int32_t up_cb = __builtin_amdgcn_readlane(vc, 32 + q), up_db = __builtin_amdgcn_readlane(vd, 32 + q);
            const uint32_t sym_b = __builtin_amdgcn_readlane(vs, 32 + q);
            if (lane == 32) {   // the second segment's first lane: its own top row and symbol
                up_c = up_cb;
                up_d = up_db;
                sym = sym_b;
            }
            const int j0 = c0 + q - ls;
            if (active && j0 >= 0 && j0 < n) {
                int32_t dsel = 0;
                dl = cells(up_c, up_d, dsel);
                prev_up = up_c;
                cl = Cp[R - 1];
                if (ls == tl) {
                    int32_t csel = Cp[0];
#pragma unroll
                    for (int r = 1; r < R; ++r)
                        if (r == rl) csel = Cp[r];
                    outC[j0 + 1] = dc_unpack16(csel, delta);   // row m of the sweep
                    outD[j0 + 1] = dc_unpack16(dsel, delta);
                }
            }
        }
        vc = nvc;
        vd = nvd;
        vs = nvs;
    }
    if (active && ls == 0) {
        outC[0] = d.t0 + sc.h * m;
        outD[0] = outC[0];                                    // DD[0] = CC[0] (:238)
    }
}

template <int R, int MM, bool ALLOW>
__global__ __launch_bounds__(64) void mm_sweep_kernel(const uint8_t* s1, const uint8_t* s2, const DcSub* split,
                                                      const DcLevel* lvl, int32_t* rows, const uint32_t* lutbits,
                                                      DcBits bits, MmScore sc, Dc16 d16) {
    constexpr bool LUT = MM == kMatchLut;
    if (MM != kMatchBits && d16.seg16 && d16.aux && d16.aux[kAuxSel] == 1) return;   // (mm_sweep_seg16_kernel)
    __shared__ uint32_t s_lut[LUT ? 2048 : 1];
    __shared__ int32_t s_park[256];   // Dc16 steady chunks: the handed-on C and D rows, per step
    const int lane = threadIdx.x;
    if (blockIdx.x / 2 >= lvl->nsplit) return;   // grid sized from an upper bound
    if constexpr (LUT) {
        for (int k = lane; k < 2048; k += 64) s_lut[k] = lutbits[k];
        __syncthreads();
    }
    // One sweep per block, or a grid-stride loop over a capped grid (kDcSkipGrid).
    auto one = [&](uint32_t bid) {
        const DcSub sub = split[bid / 2];
        const MmSweep d = mm_sweep_of(sub, bid & 1);
        const DcSrc<MM> src = bits.src<MM>(s1, s2, s_lut, sub.pair, true);
        const int m = d.alen, n = d.blen;
        int32_t* outC = rows + d.out;
        int32_t* outD = outC + n + 1;
        constexpr int BAND = 64 * R;
        const int bands = (m + BAND - 1) / BAND;
        const int tl = ((m - 1) % BAND) / R, rl = (m - 1) % R;   // owner of row m-1 in the last band
        int32_t cl = 0, dl = 0;                                   // this lane's last row: C, D
        bool b16 = false;
        if constexpr (MM != kMatchBits) b16 = d16.aux && d16.aux[kAuxSel] == 1;   // uniform over the grid
        for (int band = 0; band < bands; ++band) {
            if constexpr (MM != kMatchBits) {
                if (b16) {
                    if (band < bands - 1)
                        mm_band16<R, false>(d, s1, s2, d16.aux, d16.delta, sc, band, outC, outD, tl, rl, cl, dl, d16.park ? s_park : nullptr);
                    else
                        mm_band16<R, true>(d, s1, s2, d16.aux, d16.delta, sc, band, outC, outD, tl, rl, cl, dl, d16.park ? s_park : nullptr);
                    __threadfence_block();
                    __syncthreads();
                    continue;
                }
            }
            if (band < bands - 1)
                mm_band<R, MM, ALLOW, false>(d, src, sc, band, outC, outD, tl, rl, cl, dl);
            else
                mm_band<R, MM, ALLOW, true>(d, src, sc, band, outC, outD, tl, rl, cl, dl);
            __threadfence_block();
            __syncthreads();
        }
        if (lane == 0) {
            outC[0] = d.t0 + sc.h * m;
            outD[0] = outC[0];                                    // DD[0] = CC[0] (:238)
        }
    };
    for (uint32_t bid = blockIdx.x; bid / 2 < lvl->nsplit; bid += gridDim.x) {
        one(bid);
        __syncthreads();
    }
}

// Packed sweeps for the deep levels (every sweep has alen <= G rows): 64 / G sweeps per wave, G
// lanes each, one row per lane (as hb_sweep_seg_kernel).  A segment's first lane takes the top
// border (CC[j] = g + j h, DD[j] = CC[j] + g, :183-188) and its column symbol by ds_bpermute.
template <int G, int MM, bool ALLOW>
__global__ __launch_bounds__(64) void mm_sweep_seg_kernel(const uint8_t* s1, const uint8_t* s2, const DcSub* split,
                                                          const DcLevel* lvl, int32_t* rows, const uint32_t* lutbits,
                                                          DcBits bits, MmScore sc) {
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
    MmSweep d{};
    uint32_t pair = 0;
    if (active) {
        const DcSub sub = split[swi / 2];
        d = mm_sweep_of(sub, swi & 1);
        pair = sub.pair;
    }
    const DcSrc<MM> src = bits.src<MM>(s1, s2, s_lut, pair, active);
    const int m = d.alen, n = d.blen, g = sc.g, h = sc.h;
    int32_t* outC = rows + d.out;
    int32_t* outD = outC + n + 1;
    int steps = n + G - 1;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) steps = max(steps, __shfl_xor(steps, off));
    auto symB = [&](int k) -> uint32_t { return src.b(d.rev ? d.b - k : d.b + k); };
    const uint32_t a = ls < m ? src.a(d.rev ? d.a - ls : d.a + ls) : 0u;
    int32_t Cp = d.t0 + h * (ls + 1);                 // C[i][0] = t0 + i h (:192-197)
    int32_t Ep = Cp + g;                              // e = t + g (:198)
    int32_t prev_up = ls == 0 ? 0 : d.t0 + h * ls;    // C[ls][0]; C[0][0] = 0 (:172)
    int32_t cl = Cp, dl = 0;
    uint32_t sym = 0;
    const bool last_row = ls == m - 1;
    uint32_t vs = ls < n ? symB(ls) : 0u, nvs;
    for (int c0 = 0; c0 < steps; c0 += G) {
        nvs = c0 + G + ls < n ? symB(c0 + G + ls) : 0u;
        const int qn = min(G, steps - c0);
        for (int q = 0; q < qn; ++q) {
            const int s = c0 + q;
            const uint32_t b0 = __shfl(vs, seg * G + q);
            const int32_t c_d = __builtin_amdgcn_update_dpp(0, cl, 0x138, 0xf, 0xf, false);
            const int32_t d_d = __builtin_amdgcn_update_dpp(0, dl, 0x138, 0xf, 0xf, false);
            const uint32_t sy_d = __builtin_amdgcn_update_dpp(0u, sym, 0x138, 0xf, 0xf, false);
            const int32_t bc = g + h * (s + 1);
            const int32_t up_c = ls == 0 ? bc : c_d;
            const int32_t up_d = ls == 0 ? bc + g : d_d;
            sym = ls == 0 ? b0 : sy_d;
            const int j0 = s - ls;
            if (j0 >= 0 && j0 < n && ls < m) {
                const int32_t e = max(Ep, Cp + g) + h;                  // :202
                const int32_t dd = max(up_d, up_c + g) + h;             // :203
                const int32_t c = max(max(dd, e), mm_diag_v<ALLOW>(prev_up, src.match(a, sym), sc));
                Cp = c;
                Ep = e;
                prev_up = up_c;
                cl = c;
                dl = dd;
                if (last_row) {                                         // row m of the sweep
                    outC[j0 + 1] = c;
                    outD[j0 + 1] = dd;
                }
            }
        }
        vs = nvs;
    }
    if (active && ls == 0) {
        outC[0] = d.t0 + h * m;
        outD[0] = outC[0];                                              // DD[0] = CC[0] (:238)
    }
}

// ---------------------------------------------------------------------------- split
template <int GS>
__global__ __launch_bounds__(64) void mm_split_kernel(const DcSub* split, const DcLevel* lvl, const int32_t* rows,
                                                      DcSub* next, sa_result* res, int32_t g) {
    // GS lanes per split, 64 / GS splits per wave (dc_split_lanes)
    const int lane = threadIdx.x, sl = lane % GS;
    const uint32_t k = blockIdx.x * (64 / GS) + lane / GS;
    const uint32_t ns = lvl->nsplit;
    if (blockIdx.x * (64 / GS) >= ns) return;   // (uniform)
    const bool act = k < ns;
    DcSub d{};
    if (act) d = split[k];
    const int n = act ? d.n : -1;
    const int32_t* C = rows + 4 * (d.a0 + d.b0);
    const int32_t* D = C + n + 1;
    const int32_t* Cr = D + n + 1;
    const int32_t* Dr = Cr + n + 1;
    int32_t best = INT_MIN;
    int idx = 0, ty = 0;
    for (int j = sl; j <= n; j += GS) {
        const int32_t c1 = C[j] + Cr[n - j];
        const int32_t c2 = D[j] + Dr[n - j] - g;
        const int32_t t = max(c1, c2);
        if (t > best) { best = t; idx = j; ty = c1 > c2 ? 0 : 1; }
    }
    // lexicographic (max, -j): the reference keeps the FIRST maximum (temp > max, :326)
#pragma unroll
    for (int off = GS / 2; off >= 1; off >>= 1) {
        const int32_t ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(idx, off);
        const int ot = __shfl_xor(ty, off);
        if (ob > best || (ob == best && oi < idx)) { best = ob; idx = oi; ty = ot; }
    }
    if (act && sl == 0) {
        if (d.top) res[d.pair].score = best;
        const int mid = d.m / 2, j = idx;
        DcSub* c = next + 3 * k;
        if (!ty) {   // type 1 (:358-374)
            c[0] = DcSub{d.a0, d.b0, mid, j, d.tb, g, d.pair, 0};
            c[1] = DcSub{d.a0 + (uint64_t)mid, d.b0 + (uint64_t)j, d.m - mid, n - j, g, d.te, d.pair, 0};
            c[2] = DcSub{0, 0, -1, 0, 0, 0, d.pair, 0};
        } else {     // type 2 (:375-395): the two deletions of :390-392 as a 2-row, 0-column leaf
            c[0] = DcSub{d.a0, d.b0, mid - 1, j, d.tb, 0, d.pair, 0};
            c[1] = DcSub{d.a0 + (uint64_t)mid - 1, d.b0 + (uint64_t)j, 2, 0, 0, 0, d.pair, 0};
            c[2] = DcSub{d.a0 + (uint64_t)mid + 1, d.b0 + (uint64_t)j, d.m - mid - 1, n - j, 0, d.te, d.pair, 0};
        }
    }
}

// ---------------------------------------------------------------------------- leaves
// One sweep of buildResultRec (forward :172-238, or reversed = :247-313) into C, D [0..blen].
// (Seq / Match: as hb_leaf_solve, sa_hirschberg.hip.)
template <typename Row, typename Seq, typename Match>
__device__ void mm_sweep_thread(Seq A, int alen, int rev, Seq B, int blen, int32_t t0, const Match& mt,
                                const MmScore& sc, Row C, Row D) {
    const int32_t g = sc.g, h = sc.h;
    int32_t t = g;
    C[0] = 0;
    for (int j = 1; j <= blen; ++j) {
        t += h;
        C[j] = t;
        D[j] = t + g;
    }
    t = t0;
    for (int i = 1; i <= alen; ++i) {
        const uint32_t ai = rev ? A[alen - i] : A[i - 1];
        int32_t s = C[0];
        t += h;
        int32_t c = t;
        C[0] = c;
        int32_t e = t + g;
        for (int j = 1; j <= blen; ++j) {
            const uint32_t bj = rev ? B[blen - j] : B[j - 1];
            e = max(e, c + g) + h;
            const int32_t cj = C[j];
            const int32_t dj = max(D[j], cj + g) + h;
            D[j] = dj;
            c = max(max(dj, e), mm_diag(s, mt(ai, bj), sc));
            s = cj;
            C[j] = c;
        }
    }
    D[0] = C[0];
}

template <typename Row, typename Seq, typename Match>
__device__ int mm_leaf_solve(Seq S1, Seq S2, int alen, int blen, int32_t tb0, int32_t te0, bool top, Row C, Row D,
                             Row Cr, Row Dr, uint8_t* out, int32_t* score, const Match& mt, const MmScore& sc) {
    const int32_t g = sc.g, h = sc.h;
    int k = 0;
    int stk[48][6];   // pending subproblems (x0, xl, y0, yl, tb, te); <= 3 per level of a leaf
    int sp = 0;
    auto push = [&](int x0, int xl, int y0, int yl, int32_t tb, int32_t te) {
        stk[sp][0] = x0; stk[sp][1] = xl; stk[sp][2] = y0; stk[sp][3] = yl; stk[sp][4] = tb; stk[sp][5] = te;
        ++sp;
    };
    push(0, alen, 0, blen, tb0, te0);
    bool first = top;
    while (sp > 0) {
        --sp;
        const int x0 = stk[sp][0], M = stk[sp][1], y0 = stk[sp][2], N = stk[sp][3];
        const int32_t tb = stk[sp][4], te = stk[sp][5];
        int32_t sval = 0;
        if (N == 0) {                                               // :57-66
            for (int q = 0; q < M; ++q) out[k++] = 'U';
            sval = M > 0 ? tb + h * M : 0;
        } else if (M == 0) {                                        // :67-74
            for (int q = 0; q < N; ++q) out[k++] = 'L';
            sval = g + h * N;
        } else if (M == 1) {                                        // :75-160
            const uint32_t a = S1[x0];
            const int32_t base = max(tb, te) + h + (g + h * N);
            int32_t best = INT_MIN;
            int index = 0;
            for (int j = 1; j <= N; ++j) {
                const bool v = mt(a, S2[y0 + j - 1]);
                int32_t t = base;
                if (sc.allow || v) t = max(t, g + h * (j - 1) + (v ? sc.match : sc.mismatch) + g + h * (N - j));
                if (t > best) { best = t; index = j; }
            }
            for (int j = 1; j <= N; ++j) {
                if (j == index) {
                    const bool v = mt(a, S2[y0 + j - 1]);
                    if (!sc.allow && !v) { out[k++] = 'U'; out[k++] = 'L'; }   // :141-147
                    else out[k++] = v ? 'M' : 'S';
                } else {
                    out[k++] = 'L';
                }
            }
            sval = best;
        } else {
            const int mid = M / 2;
            mm_sweep_thread(S1.shifted(x0), mid, 0, S2.shifted(y0), N, tb, mt, sc, C, D);
            mm_sweep_thread(S1.shifted(x0 + mid), M - mid, 1, S2.shifted(y0), N, te, mt, sc, Cr, Dr);
            int index = 0, type2 = 0;
            int32_t best = INT_MIN;
            for (int j = 0; j <= N; ++j) {                          // :320-340
                const int32_t c1 = C[j] + Cr[N - j];
                const int32_t c2 = D[j] + Dr[N - j] - g;
                const int32_t t = max(c1, c2);
                if (t > best) { best = t; index = j; type2 = c1 > c2 ? 0 : 1; }
            }
            sval = best;
            // children pushed right first: the left one is finished first (:371-372, :388-394)
            if (!type2) {
                push(x0 + mid, M - mid, y0 + index, N - index, g, te);
                push(x0, mid, y0, index, tb, g);
            } else {
                push(x0 + mid + 1, M - mid - 1, y0 + index, N - index, 0, te);
                push(x0 + mid - 1, 2, y0 + index, 0, 0, 0);         // the two deletions :390-392
                push(x0, mid - 1, y0, index, tb, 0);
            }
        }
        if (first) {
            *score = sval;
            first = false;
        }
    }
    return k;
}

// Leaves with |Seq1|, |Seq2| <= kMmLdsCols run with LDS rows (C, D, Cr, Dr) + symbols: 19 KiB
// per 64-thread block at 16 (8 blocks per CU).  Measured with 12-row leaves (tools/ab_dc.sh,
// 10,000 x 1024^2): 32 cols 14.1 ms, 24 13.9, 16 13.6 ms; wider leaves use global scratch.
#ifndef SA_MM_LDS_COLS
#define SA_MM_LDS_COLS 16
#endif
constexpr int kMmLdsCols = SA_MM_LDS_COLS;

// Leaves beyond the LDS size keep their four rows at 6 * key (4 (blen + 1) <= 6 (alen + blen));
// forward ops at stage[key], op count at mark[key].  BITS: the generic-Ty path (symbols =
// pair-local indices, match = the pair's bitmap).
template <bool BITS>
__global__ __launch_bounds__(64) void mm_leaf_kernel(const uint8_t* s1, const uint8_t* s2, const DcSub* leaves,
                                                     const uint32_t* nleaves, int32_t* scratch, uint8_t* stage,
                                                     int32_t* mark, sa_result* res, const uint32_t* lut,
                                                     DcBits bits, MmScore sc) {
    __shared__ int32_t s_rows[4 * (kMmLdsCols + 1) * 64];
    __shared__ uint8_t s_seq[BITS ? 1 : 2 * kMmLdsCols * 64];
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= *nleaves) return;
    const int t = threadIdx.x;
    const DcSub L = leaves[id];
    const uint64_t key = L.a0 + L.b0;
    uint8_t* out = stage + key;
    int32_t* score = &res[L.pair].score;   // written only for a top leaf
    const bool in_lds = L.m <= kMmLdsCols && L.n <= kMmLdsCols;
    dc_lds_i32* r0 = (dc_lds_i32*)s_rows + t;
    constexpr int W = (kMmLdsCols + 1) * 64;
    int32_t* F = scratch + 6 * key;
    const int Wg = L.n + 1;
    int k;
    if constexpr (BITS) {
        uint64_t b1, b2;
        const DcBitsMatch mt = bits.of(L.pair, &b1, &b2);
        const ISeq S1{(uint32_t)(L.a0 - b1)}, S2{(uint32_t)(L.b0 - b2)};
        if (in_lds)
            k = mm_leaf_solve(S1, S2, L.m, L.n, L.tb, L.te, L.top != 0, LRow{r0}, LRow{r0 + W}, LRow{r0 + 2 * W},
                              LRow{r0 + 3 * W}, out, score, mt, sc);
        else
            k = mm_leaf_solve(S1, S2, L.m, L.n, L.tb, L.te, L.top != 0, GRow{F}, GRow{F + Wg}, GRow{F + 2 * Wg},
                              GRow{F + 3 * Wg}, out, score, mt, sc);
    } else {
        const uint8_t* g1 = s1 + L.a0;
        const uint8_t* g2 = s2 + L.b0;
        const DcLutMatch mt{lut};
        if (in_lds) {
            dc_lds_u8* q1 = (dc_lds_u8*)s_seq + t;
            dc_lds_u8* q2 = q1 + kMmLdsCols * 64;
            for (int c = 0; c < L.m; ++c) q1[c * 64] = g1[c];
            for (int c = 0; c < L.n; ++c) q2[c * 64] = g2[c];
            k = mm_leaf_solve(LSeq{q1}, LSeq{q2}, L.m, L.n, L.tb, L.te, L.top != 0, LRow{r0}, LRow{r0 + W},
                              LRow{r0 + 2 * W}, LRow{r0 + 3 * W}, out, score, mt, sc);
        } else {
            k = mm_leaf_solve(GSeq{g1}, GSeq{g2}, L.m, L.n, L.tb, L.te, L.top != 0, GRow{F}, GRow{F + Wg},
                              GRow{F + 2 * Wg}, GRow{F + 3 * Wg}, out, score, mt, sc);
        }
    }
    if (k) mark[key] = k;
}

// ---------------------------------------------------------------------------- host driver
namespace {

struct MmLaunch {
    const uint8_t* d1;
    const uint8_t* d2;
    const DcSub* split;
    const DcLevel* lvl;
    int32_t* rows;
    const uint32_t* lut;
    DcBits bits;
    MmScore sc;
    Dc16 d16;
};

template <int MM, bool ALLOW>
void launch_mm_sweeps_t(int R, int G, uint32_t count, const MmLaunch& a_in, hipStream_t st) {
    const dim3 block(64);
    MmLaunch a = a_in;
    // 16-bit sweeps of <= 128 rows (whole-wave R = 1, 2): two per wave (mm_sweep_seg16_kernel, 2R rows per lane), the
    // whole-wave kernel beside it for the int32 case
    if (MM != kMatchBits && a.d16.aux && G == 0 && R <= 2) {
        const dim3 grid2((count + 1) / 2);
        if (R == 1) hipLaunchKernelGGL(mm_sweep_seg16_kernel<2>, grid2, block, 0, st, a.d1, a.d2, a.split, a.lvl, a.rows, a.sc, a.d16);
        else hipLaunchKernelGGL(mm_sweep_seg16_kernel<4>, grid2, block, 0, st, a.d1, a.d2, a.split, a.lvl, a.rows, a.sc, a.d16);
        a.d16.seg16 = 1;
    }
#define SA_MM_SEG(GG)                                                                                           \
    hipLaunchKernelGGL((mm_sweep_seg_kernel<GG, MM, ALLOW>), dim3((count + 64 / GG - 1) / (64 / GG)), block, 0, st, \
                       a.d1, a.d2, a.split, a.lvl, a.rows, a.lut, a.bits, a.sc)
#define SA_MM_SW(RR) \
    hipLaunchKernelGGL((mm_sweep_kernel<RR, MM, ALLOW>), dim3(a.d16.seg16 ? std::min(count, kDcSkipGrid) : count), block, 0, st, a.d1, a.d2, a.split, a.lvl, a.rows, a.lut, a.bits, a.sc, a.d16)
    if (G == 8) SA_MM_SEG(8);
    else if (G == 16) SA_MM_SEG(16);
    else if (G == 32) SA_MM_SEG(32);
    else if (R == 1) SA_MM_SW(1);
    else if (R == 2) SA_MM_SW(2);
    else if (R == 4) SA_MM_SW(4);
    else if (R == 8) SA_MM_SW(8);
    else if (R == 16) SA_MM_SW(16);
    else SA_MM_SW(32);
#undef SA_MM_SEG
#undef SA_MM_SW
}

// G = 8 / 16 / 32: packed sweeps (maxa <= G); G = 0: R rows per lane, one sweep per wave.
hipError_t launch_mm_sweeps(int R, int G, uint32_t count, const MmLaunch& a, hipStream_t st) {
    const int mm = a.bits.mbits ? kMatchBits : a.lut ? kMatchLut : kMatchEq;
    if (mm == kMatchBits) a.sc.allow ? launch_mm_sweeps_t<kMatchBits, true>(R, G, count, a, st)
                                     : launch_mm_sweeps_t<kMatchBits, false>(R, G, count, a, st);
    else if (mm == kMatchLut) a.sc.allow ? launch_mm_sweeps_t<kMatchLut, true>(R, G, count, a, st)
                                         : launch_mm_sweeps_t<kMatchLut, false>(R, G, count, a, st);
    else a.sc.allow ? launch_mm_sweeps_t<kMatchEq, true>(R, G, count, a, st)
                    : launch_mm_sweeps_t<kMatchEq, false>(R, G, count, a, st);
    return hipGetLastError();
}

}  // namespace

// Host driver: same contract as hirschberg_run (device results and op streams, enqueued on st).
int myersmiller_run(DcWork& w, hipEvent_t prev, const sa_scoring* scoring, const DcInputs& in, const DcBounds& b,
                    hipStream_t st, sa_result* d_res, uint8_t* d_ops, std::string* err) {
    int leaf_rows = kMmLeafRows;   // tuning override: SEQALIB_MM_LEAF (the leaf stack bounds it)
    if (const char* lr = getenv("SEQALIB_MM_LEAF")) leaf_rows = std::min(4096, std::max(2, atoi(lr)));
    const char* segenv = getenv("SEQALIB_DC_SEG");   // 0: whole-wave sweeps only (A/B, tests)
    const bool seg_sweeps = !segenv || atoi(segenv) != 0;
    constexpr int rmax = 32;                         // the sweep's largest R
    const uint32_t npairs = in.npairs;
    MmScore sc;
    sc.g = scoring->gap_open;
    sc.h = scoring->gap_extend;
    sc.match = scoring->match;
    sc.allow = scoring->allow_mismatch != 0;
    sc.mismatch = sc.allow ? scoring->mismatch : INT_MIN;
    const bool bits = in.bits.mbits != nullptr;
    SA_DC_HIP(w.prepare(b, npairs, leaf_rows, 3, 4, 6, st, prev));
    // 16-bit whole-wave sweeps (sa_dc.h Dc16), as hirschberg_run
    Dc16 d16 = bits ? Dc16{} : dc16_plan(true, scoring, b.max_m, b.max_n);
    if (d16.aux) {
        SA_DC_HIP(w.aux.alloc(kAuxWords));
        SA_DC_HIP(launch_alphabet_scan(in.d1, in.o1, in.d2, in.o2, npairs, w.aux.p, st));
        SA_DC_HIP(launch_decide_t16(in.lutbits, sc.match, d16.mismatch, 2, w.aux.p, st));
        d16.aux = w.aux.p;
    }
    SA_DC_HIP(hipMemsetAsync(d_res, 0, sizeof(sa_result) * npairs, st));
    // getAlignment: buildResultRec(.., GapOpen, GapOpen) (:417)
    SA_DC_HIP(dc_launch_init(in.o1, in.o2, npairs, sc.g, b, w.cur.p, d_res, st));
    uint32_t cap = npairs;
    int maxm = (int)b.max_m;
    for (int l = 0;; ++l) {
        SA_DC_HIP(dc_launch_classify(w.cur.p, cap, npairs, l ? w.lvl.p + l - 1 : nullptr, 3, leaf_rows, 1,
                                     w.lvl.p + l, w.split.p, w.leaves.p, w.nleaf(), st));
        if (maxm <= leaf_rows) break;
        const uint32_t splits = std::min<uint64_t>(cap, w.max_splits);
        const int maxa = (maxm + 1) / 2;
        int R = 1;
        while (R < rmax && 64 * R < maxa) R *= 2;   // bands of 64 R rows
        const int G = !seg_sweeps ? 0 : maxa <= 8 ? 8 : maxa <= 16 ? 16 : maxa <= 32 ? 32 : 0;
        const MmLaunch a{in.d1, in.d2, w.split.p, w.lvl.p + l, w.rows.p, in.lutbits, in.bits, sc, d16};
        SA_DC_HIP(launch_mm_sweeps(R, G, 2 * splits, a, st));
        const int gs = dc_split_lanes(maxm);
        if (gs == 64)
            hipLaunchKernelGGL(mm_split_kernel<64>, dim3(splits), dim3(64), 0, st, w.split.p, w.lvl.p + l, w.rows.p,
                               w.next.p, d_res, sc.g);
        else if (gs == 16)
            hipLaunchKernelGGL(mm_split_kernel<16>, dim3((splits + 3) / 4), dim3(64), 0, st, w.split.p, w.lvl.p + l,
                               w.rows.p, w.next.p, d_res, sc.g);
        else
            hipLaunchKernelGGL(mm_split_kernel<8>, dim3((splits + 7) / 8), dim3(64), 0, st, w.split.p, w.lvl.p + l,
                               w.rows.p, w.next.p, d_res, sc.g);
        SA_DC_HIP(hipGetLastError());
        w.cur.swap(w.next);
        cap = 3 * splits;
        maxm = maxa;
    }
    if (bits)
        hipLaunchKernelGGL(mm_leaf_kernel<true>, dim3((w.leaf_cap + 63) / 64), dim3(64), 0, st, in.d1, in.d2, w.leaves.p,
                           w.nleaf(), w.scratch.p, w.stage.p, w.mark.p, d_res, in.lutbits, in.bits, sc);
    else
        hipLaunchKernelGGL(mm_leaf_kernel<false>, dim3((w.leaf_cap + 63) / 64), dim3(64), 0, st, in.d1, in.d2, w.leaves.p,
                           w.nleaf(), w.scratch.p, w.stage.p, w.mark.p, d_res, in.lutbits, in.bits, sc);
    SA_DC_HIP(hipGetLastError());
    SA_DC_HIP(dc_launch_assemble(in.o1, in.o2, npairs, w.mark.p, w.stage.p, d_res, d_ops, st));
    return 0;
}

}  // namespace sa
