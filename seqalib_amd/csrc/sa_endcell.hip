// sa_endcell.hip — exact end cell (MaxRow, MaxCol) after a CMAX fill (sa_fill_impl.h).
//
// The reference keeps the LAST row-major maximum of the score matrix (SASmithWaterman.h:110:
// Score >= MaxScore inside the i-then-j loops).  A CMAX fill reports, per pair, the maximum
// score S, the last lane (band b, lane t) holding it and the last 32-step chunk c in which lane t
// reached S; it also stores every lane's maximum of every chunk.  This kernel replays, in order,
// each chunk c' <= c of band b in which lane t's maximum equals S, from the snapshot the fill
// stored at the end of chunk c'-1 (every lane's R row values and its diagonal input; the band's
// top row comes from the per-band row buffer), and keeps the last row of lane t holding S and
// that row's last column.  An all-zero matrix (S = 0) ends at (m, n) without a replay.
// The replay repeats the fill's recurrence and its wavefront order exactly (lane t computes
// column s - t at step s; the row above comes from lane t-1's previous step), in int32 on the
// unscaled scores, so it yields the same cell values the fill produced.
//
// One wave per pair; 32 steps x R rows per lane per replayed chunk (usually one): ~0.05% of the
// fill's work at 4096 x 4096.
#include <limits.h>

#include "sa_endcell_so.h"
#include "sa_internal.h"

namespace sa {


// the band's top row: the fill's row buffer or, SPLIT, its write-through hand-off granules, read
// as the fill's poller reads them (sc1), like sa_traceback_seg.hip's seg_hand
__device__ __forceinline__ int32_t ec_top(const int32_t* p) {
    typedef const int32_t __attribute__((address_space(1))) cgi32;
    return __hip_atomic_load((cgi32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


template <int R>
__global__ __launch_bounds__(64) void endcell_kernel(EndcellParams P) {
    if (sa_skip(P.sel, P.sel_want)) return;
    const int lane = threadIdx.x;
    const uint32_t slot = blockIdx.x;
    if (slot >= P.count) return;
    const uint32_t symp = P.prof[4];
    const uint32_t pidx = P.pair_base + slot;
    sa_result res = P.res[pidx];
    if (res.reserved == 0 || (res.flags & (SA_FLAG_BAD_SHAPE | kFlagRetry))) return;   // uniform over the wave
    const int c = (int)res.reserved - 1;
    const int S = res.score;
    const int iend = res.end_i;
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    constexpr int BAND = kWave * R;
    const int b = (iend - 1) / BAND;
    const int tstar = ((iend - 1) % BAND) / R;
    const int row0 = b * BAND + lane * R;
    const int G = P.gap;
    const int hs = P.hshift;   // values stored as H << hs: 4H (tagged fill) or H (score-only fill)

    if (S == 0) {   // every cell is 0: the last cell is the reference's maximum (MaxScore from INT_MIN)
        if (lane == 0) {
            res.end_i = m;
            res.end_j = n;
            res.reserved = 0;
            P.res[pidx] = res;
        }
        return;
    }
    uint32_t tab[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        tab[r] = row < m ? P.prof[ec_code8(symp, s1[row]) >> 3] : 0u;
    }
    const uint32_t rs = P.rowbuf_stride;
    const int32_t* top = b > 0 ? P.rowbuf + (uint64_t)slot * P.rowbuf_slot + (uint64_t)(b - 1) * P.max_n * rs : nullptr;
    const int32_t* lmax = P.snap_m + (uint64_t)slot * P.snap_p_slot + (uint64_t)b * P.snap_nch * kWave + tstar;
    int rbest = -1, jbest = -1;
    __shared__ uint8_t s_sym[kWave + kChunk];   // the chunk's column codes, columns cc*32 - 63 ..
    __shared__ int s_top[kChunk];               // the band's top row at the chunk's columns
    // the chunks to replay, found 64 at a time (one load per lane, not a dependent load per chunk)
    for (int base = 0; base <= c; base += kWave) {
        const int ccl = base + lane;
        uint64_t hits = __builtin_amdgcn_ballot_w64(ccl <= c && lmax[(uint64_t)ccl * kWave] == (S << hs));
        while (hits) {
        const int cc = base + (int)__builtin_ctzll(hits);
        hits &= hits - 1;
        int Hp[R];
#pragma unroll
        for (int r = 0; r < R; ++r) Hp[r] = 0;
        int prev_up = 0;
        if (cc > 0) {
            const uint64_t e = (uint64_t)b * P.snap_nch + (cc - 1);
            const uint32_t* sh = P.snap_h + (uint64_t)slot * P.snap_h_slot + e * (R / 2) * kWave + lane;
#pragma unroll
            for (int q = 0; q < R / 2; ++q) {
                const uint32_t w = sh[q * kWave];
                Hp[2 * q] = (int)(w & 0xffffu) >> hs;        // stored as H << hs (non-negative)
                Hp[2 * q + 1] = (int)(w >> 16) >> hs;
            }
            prev_up = (int)(P.snap_p[(uint64_t)slot * P.snap_p_slot + e * kWave + lane] & 0xffff) >> hs;
        }
        __syncthreads();   // (a previous candidate's reads of the staging arrays)
        for (int k = lane; k < kWave + kChunk; k += kWave) {
            const int j = cc * kChunk - (kWave - 1) + k;
            s_sym[k] = (uint8_t)(j >= 0 && j < n ? ec_code8(symp, s2[j]) : 0u);
        }
        if (lane < kChunk) {
            const int j = cc * kChunk + lane;
            s_top[lane] = (top && j < n) ? (ec_top(top + (uint64_t)j * rs) >> hs) : 0;
        }
        __syncthreads();
        int hl = Hp[R - 1];
        for (int q = 0; q < kChunk; ++q) {
            const int s = cc * kChunk + q;
            const int j0 = s - lane;
            int up_h = __shfl_up(hl, 1);
            if (lane == 0) up_h = s_top[q];
            if (j0 >= 0 && j0 < n) {
                if (j0 == 0) {   // the lane's first column: the matrix border (the fill's snapshot
                    prev_up = 0; // of a lane that had not started holds its start-mode garbage)
#pragma unroll
                    for (int r = 0; r < R; ++r) Hp[r] = 0;
                }
                const uint32_t sym = s_sym[q - lane + (kWave - 1)];
                int hd = prev_up, hu = up_h;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    // profile byte = 4s+3 (signed); the builtin returns unsigned: shift as int
                    const int sub = ((int)__builtin_amdgcn_sbfe(tab[r], sym, 8) - 3) >> 2;
                    int H = hd + sub;
                    H = max(H, hu + G);
                    H = max(H, Hp[r] + G);
                    H = max(H, 0);
                    hd = Hp[r];
                    Hp[r] = H;
                    hu = H;
                    // last row of the lane holding S, then its last column (chunks ascend)
                    if (lane == tstar && row0 + r < m && H == S && (r > rbest || (r == rbest && j0 > jbest))) {
                        rbest = r;
                        jbest = j0;
                    }
                }
                prev_up = up_h;
                hl = Hp[R - 1];
            }
        }
        }
    }
    if (lane == tstar) {
        res.end_i = row0 + rbest + 1;   // 1-based; rbest >= 0 whenever the fill's report is consistent
        res.end_j = jbest + 1;
        res.reserved = 0;
        P.res[pidx] = res;
    }
}

// Score-only SW fill (sa_fill_impl.h SO): the fill tracked the rows 3 mod 4 at the steps 3 mod 4
// of its steady chunks (every cell of ramp chunks) and stored, per (band, chunk, lane), the lane's
// maximum of its tracked cells; every cell is at most a tracked cell of the same lane and chunk -
// kSoSlack G, so S lies in [smax, smax - kSoSlack G] and only the LANE BLOCKS (R rows x 32 columns)
// whose tracked maximum reaches smax + kSoSlack G can hold it.  This kernel lists those blocks and recomputes each one alone,
// as the score-only traceback recomputes a block on the path (sa_traceback_so.hip): its left
// column from the snapshot of the chunk before, its top row from the edge stream (the last row of
// the lane above, per step), one row per lane in a 32 + R - 1 step wavefront, 64 / R blocks per
// round.  Every lane keeps the lexicographically largest (H, i, j) of its cells -- the reference's
// last row-major maximum, SASmithWaterman.h:110 -- and the wave reduces them.  A pair with more
// than kSoCand candidate blocks (an all-zero or low-scoring matrix: smax = 0 lists every block)
// replays whole chunks instead (64 lanes, from the snapshots), as endcell_kernel does.
constexpr int kSoCand = 1024;
#ifdef SA_TB_STATS
// Debug build only (-DSA_TB_STATS, tools/so4_stats.py): [pairs, candidate lane blocks, dense
// fallbacks, wave cycles, cycles to the scan's first load (parameters, result, offsets), first-level
// scan cycles, second-level cycles, summed over waves; [7]: the wave lifetime's maximum]
__device__ unsigned long long g_ecso_stats[8];
extern "C" int sa_debug_ecso_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ecso_stats), sizeof(g_ecso_stats)) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_ecso_stats), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif

// DENSE = false: the candidate scan and the lane-block replay; a pair with more than kSoCand
// candidate blocks is left pending (reserved != 0) for the DENSE = true launch behind it, which
// replays whole chunks -- a kernel of its own so that its R-row register arrays do not set the
// common kernel's occupancy (121 -> fewer VGPRs, more resident waves).
template <int R, bool DENSE>
__global__ __launch_bounds__(64) void endcell_so_kernel(EndcellParams P) {
    if constexpr (DENSE) {   // (after the fill: its count is final) to the host's pinned word
        if (P.f16_count && blockIdx.x == 0 && threadIdx.x == 0)
            __hip_atomic_store(P.f16_host, (unsigned long long)P.f16_seq << 32 | *P.f16_count, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (sa_skip(P.sel, P.sel_want)) return;
    const int lane = threadIdx.x;
    const uint32_t slot = blockIdx.x;
    if (slot >= P.count) return;
    const uint32_t symp = P.prof[4];
    const uint32_t pidx = P.pair_base + slot;
    sa_result res = P.res[pidx];
    if (res.reserved == 0 || (res.flags & (SA_FLAG_BAD_SHAPE | kFlagRetry))) return;   // uniform over the wave
    if constexpr (!DENSE) {
        __shared__ uint32_t s_cand[kSoCand], s_hit[kSoCand];
        __shared__ __attribute__((aligned(16))) uint32_t s_pk[kWave / R][kEcPk<R>];
#ifdef SA_TB_STATS
        const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();
        int cnt = 0;
        unsigned long long ph[3] = {st_t0, st_t0, st_t0};
        const bool done = endcell_so_lanes<R, kSoCand>(P, slot, res.score, s_cand, s_hit, s_pk, &cnt, ph);
        if (lane == 0) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            atomicAdd(&g_ecso_stats[0], 1ull);
            atomicAdd(&g_ecso_stats[1], (unsigned long long)cnt);
            atomicAdd(&g_ecso_stats[2], done ? 0ull : 1ull);
            atomicAdd(&g_ecso_stats[3], t1 - st_t0);
            atomicAdd(&g_ecso_stats[4], ph[0] - st_t0);
            atomicAdd(&g_ecso_stats[5], ph[1] - ph[0]);
            atomicAdd(&g_ecso_stats[6], ph[2] - ph[1]);
            atomicMax(&g_ecso_stats[7], t1 - st_t0);
        }
#else
        (void)endcell_so_lanes<R, kSoCand>(P, slot, res.score, s_cand, s_hit, s_pk);
#endif
        (void)symp;
        return;
    }
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    constexpr int BAND = kWave * R;
    const int B = (m + BAND - 1) / BAND;
    const int nch = (int)chunks_per_band((uint32_t)n);
    const uint32_t snch = P.snap_nch;
    const int G = P.gap;
    const int thr = res.score + kSoSlack * G;   // lane blocks whose tracked maximum reaches this may hold S
    const int32_t* cm = P.snap_m + (uint64_t)slot * P.snap_p_slot;   // [band][chunk][lane]
    const uint32_t* sh_base = P.snap_h + (uint64_t)slot * P.snap_h_slot;
    const int32_t* sp_base = P.snap_p + (uint64_t)slot * P.snap_p_slot;
    int bv = -1, bi = -1, bj = -1;       // this lane's best (H, row, column), 0-based
    auto take = [&](int H, int row, int col) __attribute__((always_inline)) {
        if (H > bv || (H == bv && (row > bi || (row == bi && col > bj)))) { bv = H; bi = row; bj = col; }
    };
    {
        // ---- dense: whole chunks holding a candidate lane, all 64 lanes from the snapshots
        __shared__ uint8_t s_sym[kWave + kChunk];
        __shared__ int s_top[kChunk];
        for (int b = 0; b < B; ++b) {
            const int row0 = b * BAND + lane * R;
            uint32_t tab[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int row = row0 + r;
                tab[r] = row < m ? P.prof[ec_code8(symp, s1[row]) >> 3] : 0u;
            }
            const int32_t* top = b > 0 ? P.rowbuf + (uint64_t)slot * P.rowbuf_slot + (uint64_t)(b - 1) * P.max_n : nullptr;
            for (int cc = 0; cc < nch; ++cc) {
                if (__builtin_amdgcn_ballot_w64(cm[((uint64_t)b * snch + cc) * kWave + lane] >= thr) == 0) continue;
                int Hp[R];
#pragma unroll
                for (int r = 0; r < R; ++r) Hp[r] = 0;
                int prev_up = 0;
                if (cc > 0) {
                    const uint64_t e = (uint64_t)b * snch + (cc - 1);
                    const uint32_t* sh = sh_base + e * (R / 2) * kWave + lane;
#pragma unroll
                    for (int q = 0; q < R / 2; ++q) {
                        const uint32_t w = sh[q * kWave];
                        Hp[2 * q] = (int)(w & 0xffffu);
                        Hp[2 * q + 1] = (int)(w >> 16);
                    }
                    prev_up = (int)(sp_base[e * kWave + lane] & 0xffff);
                }
                __syncthreads();   // (a previous candidate's reads of the staging arrays)
                for (int k = lane; k < kWave + kChunk; k += kWave) {
                    const int j = cc * kChunk - (kWave - 1) + k;
                    s_sym[k] = (uint8_t)(j >= 0 && j < n ? ec_code8(symp, s2[j]) : 0u);
                }
                if (lane < kChunk) {
                    const int j = cc * kChunk + lane;
                    s_top[lane] = (top && j < n) ? (ec_top(top + j) & 0xffff) : 0;   // ({epoch, H} granules)
                }
                __syncthreads();
                int hl = Hp[R - 1];
                for (int q = 0; q < kChunk; ++q) {
                    const int s = cc * kChunk + q;
                    const int j0 = s - lane;
                    int up_h = __shfl_up(hl, 1);
                    if (lane == 0) up_h = s_top[q];
                    if (j0 >= 0 && j0 < n) {
                        if (j0 == 0) {   // the lane's first column: the matrix border
                            prev_up = 0;
#pragma unroll
                            for (int r = 0; r < R; ++r) Hp[r] = 0;
                        }
                        const uint32_t sym = s_sym[q - lane + (kWave - 1)];
                        int hd = prev_up, hu = up_h;
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            // profile byte = 4s+3 (signed); the builtin returns unsigned: shift as int
                            const int sub = ((int)__builtin_amdgcn_sbfe(tab[r], sym, 8) - 3) >> 2;
                            int H = hd + sub;
                            H = max(H, hu + G);
                            H = max(H, Hp[r] + G);
                            H = max(H, 0);
                            hd = Hp[r];
                            Hp[r] = H;
                            hu = H;
                            if (row0 + r < m) take(H, row0 + r, j0);
                        }
                        prev_up = up_h;
                        hl = Hp[R - 1];
                    }
                }
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const int ov = __shfl_xor(bv, off), oi = __shfl_xor(bi, off), oj = __shfl_xor(bj, off);
        if (ov > bv || (ov == bv && (oi > bi || (oi == bi && oj > bj)))) { bv = ov; bi = oi; bj = oj; }
    }
    if (lane == 0) {   // (the other fields stay as the fill wrote them)
        sa_result* const o = P.res + pidx;
        o->score = bv;
        o->end_i = bi + 1;
        o->end_j = bj + 1;
        o->reserved = 0;
    }
}


// LocalGotoh (T16 affine CMAX fill): the same replay on the three-state recurrence
// (SALocalGotoh.h:108-130).  The fill's snapshot of a lane holds its R values of M (8M), then its
// R values of Iy (8Iy + 2) and the Ix of its last row (8Ix + 4, or 0 where the fill's clamped Ix
// open term floored it); the band's top row holds M and Ix.  Replayed Ix values may differ from
// the reference's below 0 (the fill keeps max(Ix, 0) there), which leaves every M unchanged:
// M = max(D, Ix, Iy, 0) and max(max(Ix, 0) + GE, GE) keeps max(., 0) of the chain (GE < 0).
// SO (score-only LocalGotoh fill, hshift 0): the snapshots and top rows hold M, B = Iy - (GO + GE)
// and A = Ix - (GO + GE) unscaled and exact (sa_fill_impl.h, the SO affine cell); the chunk maxima M.
template <int R, bool SO>
__global__ __launch_bounds__(64) void endcell_lg_kernel(EndcellParams P) {
    if (sa_skip(P.sel, P.sel_want)) return;
    const int lane = threadIdx.x;
    const uint32_t slot = blockIdx.x;
    if (slot >= P.count) return;
    const uint32_t symp = P.prof[4];
    const uint32_t pidx = P.pair_base + slot;
    sa_result res = P.res[pidx];
    if (res.reserved == 0 || (res.flags & (SA_FLAG_BAD_SHAPE | kFlagRetry))) return;   // uniform over the wave
    const int c = (int)res.reserved - 1;
    const int S = res.score;
    const int iend = res.end_i;
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    constexpr int BAND = kWave * R;
    const int b = (iend - 1) / BAND;
    const int tstar = ((iend - 1) % BAND) / R;
    const int row0 = b * BAND + lane * R;
    const int GE = P.gap_extend, GOE = P.gap_open + P.gap_extend;
    constexpr int kNeg = INT_MIN / 4;   // the Ix / Iy borders: below every candidate

    if (S == 0) {   // every M is 0: the last cell is the reference's maximum (MaxScore from INT_MIN)
        if (lane == 0) {
            res.end_i = m;
            res.end_j = n;
            res.reserved = 0;
            P.res[pidx] = res;
        }
        return;
    }
    uint32_t tab[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        tab[r] = row < m ? P.prof[ec_code8(symp, s1[row]) >> 3] : 0u;
    }
    const uint32_t rs = P.rowbuf_stride;
    const int32_t* top = b > 0 ? P.rowbuf + (uint64_t)slot * P.rowbuf_slot + (uint64_t)(b - 1) * P.max_n * rs : nullptr;
    const int32_t* topx = top ? top + P.rowbuf_x_off : nullptr;
    const int32_t* lmax = P.snap_m + (uint64_t)slot * P.snap_p_slot + (uint64_t)b * P.snap_nch * kWave + tstar;
    int rbest = -1, jbest = -1;
    __shared__ uint8_t s_sym[kWave + kChunk];
    __shared__ int s_top[2 * kChunk];   // M, then Ix, of the band's top row at the chunk's columns
    for (int base = 0; base <= c; base += kWave) {   // candidate chunks, as endcell_kernel
        const int ccl = base + lane;
        uint64_t hits = __builtin_amdgcn_ballot_w64(ccl <= c && lmax[(uint64_t)ccl * kWave] == (SO ? S : 8 * S));
        while (hits) {
        const int cc = base + (int)__builtin_ctzll(hits);
        hits &= hits - 1;
        int Mp[R], Yp[R];
#pragma unroll
        for (int r = 0; r < R; ++r) { Mp[r] = 0; Yp[r] = kNeg; }
        int prev_up = 0, xl = kNeg;
        if (cc > 0) {
            const uint64_t e = (uint64_t)b * P.snap_nch + (cc - 1);
            const uint32_t* sh = P.snap_h + (uint64_t)slot * P.snap_h_slot + e * (R + 1) * kWave + lane;
            constexpr int SH = SO ? 0 : 3;   // SO: M, B, A unscaled; tagged: 8M, 8Iy + 2, 8Ix + 4
            const int off = SO ? GOE : 0;
#pragma unroll
            for (int q = 0; q < R / 2; ++q) {
                const uint32_t w = sh[q * kWave], y = sh[(R / 2 + q) * kWave];
                Mp[2 * q] = (int)(w & 0xffffu) >> SH;   // M >= 0
                Mp[2 * q + 1] = (int)(w >> 16) >> SH;
                Yp[2 * q] = ((int)(int16_t)(y & 0xffffu) >> SH) + off;   // Iy (the border: far below)
                Yp[2 * q + 1] = ((int)(int16_t)(y >> 16) >> SH) + off;
            }
            xl = ((int)(int16_t)(sh[R * kWave] & 0xffffu) >> SH) + off;
            prev_up = (int)(P.snap_p[(uint64_t)slot * P.snap_p_slot + e * kWave + lane] & 0xffff) >> SH;
        }
        __syncthreads();
        for (int k = lane; k < kWave + kChunk; k += kWave) {
            const int j = cc * kChunk - (kWave - 1) + k;
            s_sym[k] = (uint8_t)(j >= 0 && j < n ? ec_code8(symp, s2[j]) : 0u);
        }
        if (lane < kChunk) {
            const int j = cc * kChunk + lane;
            const bool t = top && j < n;
            s_top[lane] = t ? ((ec_top(top + (uint64_t)j * rs) & (SO ? 0xffff : -1)) >> (SO ? 0 : 3)) : 0;
            s_top[kChunk + lane] = t ? (((int)(int16_t)(ec_top(topx + (uint64_t)j * rs) & 0xffff) >> (SO ? 0 : 3)) + (SO ? GOE : 0)) : kNeg;
        }
        __syncthreads();
        int hl = Mp[R - 1];
        for (int q = 0; q < kChunk; ++q) {
            const int s = cc * kChunk + q;
            const int j0 = s - lane;
            int up_h = __shfl_up(hl, 1);
            int up_x = __shfl_up(xl, 1);
            if (lane == 0) {
                up_h = s_top[q];
                up_x = s_top[kChunk + q];
            }
            if (j0 >= 0 && j0 < n) {
                if (j0 == 0) {   // the lane's first column: the matrix border (as endcell_kernel)
                    prev_up = 0;
#pragma unroll
                    for (int r = 0; r < R; ++r) { Mp[r] = 0; Yp[r] = kNeg; }
                }
                const uint32_t sym = s_sym[q - lane + (kWave - 1)];
                int hd = prev_up, hu = up_h, xu = up_x;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    // profile byte = 8s+6 (signed); the builtin returns unsigned: shift as int
                    const int sub = ((int)__builtin_amdgcn_sbfe(tab[r], sym, 8) - 6) >> 3;
                    const int X = max(hu + GOE, xu + GE);
                    const int Y = max(Mp[r] + GOE, Yp[r] + GE);
                    const int M = max(max(hd + sub, X), max(Y, 0));
                    hd = Mp[r];
                    Mp[r] = M;
                    Yp[r] = Y;
                    hu = M;
                    xu = X;
                    // last row of the lane holding S, then its last column (chunks ascend)
                    if (lane == tstar && row0 + r < m && M == S && (r > rbest || (r == rbest && j0 > jbest))) {
                        rbest = r;
                        jbest = j0;
                    }
                }
                prev_up = up_h;
                hl = Mp[R - 1];
                xl = xu;
            }
        }
        }
    }
    if (lane == tstar) {
        res.end_i = row0 + rbest + 1;
        res.end_j = jbest + 1;
        res.reserved = 0;
        P.res[pidx] = res;
    }
}

// SPLIT fills (sa_fill_impl.h): fold each pair's per-band partials {score, i, j, timeout} into
// its result — local modes: the lexicographic max over (score, i, j), i.e. the reference's last
// row-major maximum; global modes: H[m][n] from the band holding row m.  One thread per pair.
template <int ALG>
__global__ void split_reduce_kernel(SplitReduceParams P) {
    bool redo = false;
    if (sa_skip(P.sel, P.sel_want)) {
        if (!P.redo) return;
        redo = true;
    }
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= P.count) return;
    const uint32_t pidx = P.pair_base + slot;
    if (redo && !(P.res[pidx].flags & kFlagRetry)) return;
    const int m = (int)(P.off1[pidx + 1] - P.off1[pidx]);
    const int n = (int)(P.off2[pidx + 1] - P.off2[pidx]);
    sa_result r = {};
    if ((uint32_t)m > P.max_m || (uint32_t)n > P.max_n) {
        r.flags = SA_FLAG_BAD_SHAPE;
        P.res[pidx] = r;
        return;
    }
    const int BR = (int)P.band_rows;
    const int B = (m > 0 && n > 0) ? (m + BR - 1) / BR : 0;
    const int32_t* q = P.part + (uint64_t)slot * P.split_bands * 4;
    uint32_t tmo = 0;
    for (int b = 0; b < B; ++b) tmo |= (uint32_t)q[4 * b + 3];
    if (tmo) r.flags |= SA_FLAG_TIMEOUT;
    constexpr bool LOCAL = (ALG == SA_SW || ALG == SA_LOCAL_GOTOH);
    if constexpr (LOCAL) {
        int h = INT_MIN, bi = 0, bj = 0;
        for (int b = 0; b < B; ++b) {
            const int oh = q[4 * b], oi = q[4 * b + 1], oj = q[4 * b + 2];
            if (oh > h || (oh == h && (oi > bi || (oi == bi && oj > bj)))) { h = oh; bi = oi; bj = oj; }
        }
        if (B == 0) {
            r.score = (ALG == SA_SW) ? INT_MIN : 0;   // as the single-workgroup fill reports it
        } else if (P.cmax) {
            r.score = h; r.end_i = bi; r.end_j = 0;
            r.reserved = (uint32_t)bj;   // chunk + 1: endcell_kernel resolves the column
        } else {
            r.score = h; r.end_i = bi; r.end_j = bj;
        }
        if (B != 0 && h > P.retry_above) r.flags |= kFlagRetry;
    } else {
        r.end_i = m;
        r.end_j = n;
        if (B == 0) {
            const int k = m > n ? m : n;
            if constexpr (ALG == SA_NW) r.score = k * P.gap;
            else r.score = k == 0 ? 0 : P.gap_open + k * P.gap_extend;
        } else {
            r.score = q[4 * (B - 1)];
        }
    }
    if (redo) r.flags |= kFlagRedo;
    P.res[pidx] = r;
}

hipError_t launch_split_reduce(int algo, const SplitReduceParams& p, hipStream_t stream) {
    const dim3 grid((p.count + 255) / 256), block(256);
    switch (algo) {
        case SA_SW: hipLaunchKernelGGL(split_reduce_kernel<SA_SW>, grid, block, 0, stream, p); break;
        case SA_NW: hipLaunchKernelGGL(split_reduce_kernel<SA_NW>, grid, block, 0, stream, p); break;
        case SA_LOCAL_GOTOH: hipLaunchKernelGGL(split_reduce_kernel<SA_LOCAL_GOTOH>, grid, block, 0, stream, p); break;
        case SA_GLOBAL_GOTOH: hipLaunchKernelGGL(split_reduce_kernel<SA_GLOBAL_GOTOH>, grid, block, 0, stream, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_endcell_so(int R, const EndcellParams& p, hipStream_t stream) {
    const dim3 grid(p.count), block(64);
    // the lane-block kernel, then the dense one for the pairs it left pending (most return at once)
#define SA_EC_SO(RR)                                                                       \
    hipLaunchKernelGGL((endcell_so_kernel<RR, false>), grid, block, 0, stream, p);          \
    if (hipPeekAtLastError() == hipSuccess)                                                 \
        hipLaunchKernelGGL((endcell_so_kernel<RR, true>), grid, block, 0, stream, p);
    switch (R) {
        case 4: SA_EC_SO(4) break;
        case 8: SA_EC_SO(8) break;
        case 16: SA_EC_SO(16) break;
        case 32: SA_EC_SO(32) break;
        default: return hipErrorInvalidValue;
    }
#undef SA_EC_SO
    return hipGetLastError();
}

hipError_t launch_endcell(int algo, int R, const EndcellParams& p, hipStream_t stream) {
    const dim3 grid(p.count), block(64);
    if (algo == SA_LOCAL_GOTOH) {
        const bool so = p.hshift == 0;   // the score-only fill's unscaled snapshots
        switch (R) {
            case 2: if (so) return hipErrorInvalidValue; hipLaunchKernelGGL((endcell_lg_kernel<2, false>), grid, block, 0, stream, p); break;
            case 4: if (so) hipLaunchKernelGGL((endcell_lg_kernel<4, true>), grid, block, 0, stream, p);
                    else hipLaunchKernelGGL((endcell_lg_kernel<4, false>), grid, block, 0, stream, p); break;
            case 8: if (so) hipLaunchKernelGGL((endcell_lg_kernel<8, true>), grid, block, 0, stream, p);
                    else hipLaunchKernelGGL((endcell_lg_kernel<8, false>), grid, block, 0, stream, p); break;
            case 16: if (so) hipLaunchKernelGGL((endcell_lg_kernel<16, true>), grid, block, 0, stream, p);
                     else hipLaunchKernelGGL((endcell_lg_kernel<16, false>), grid, block, 0, stream, p); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (algo != SA_SW) return hipErrorInvalidValue;
    switch (R) {
        case 2: hipLaunchKernelGGL(endcell_kernel<2>, grid, block, 0, stream, p); break;
        case 4: hipLaunchKernelGGL(endcell_kernel<4>, grid, block, 0, stream, p); break;
        case 8: hipLaunchKernelGGL(endcell_kernel<8>, grid, block, 0, stream, p); break;
        case 16: hipLaunchKernelGGL(endcell_kernel<16>, grid, block, 0, stream, p); break;
        case 32: hipLaunchKernelGGL(endcell_kernel<32>, grid, block, 0, stream, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sa
