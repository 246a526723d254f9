// sa_endcell_so.h — the lane-block end-cell replay of the score-only SW fill as a device function
// (endcell_so_kernel, sa_endcell.hip, runs it one wave per pair after the fill).  Round 6 also ran
// it inside the two-pairs-per-wave fill's final units (after an agent-scope release / acquire of
// the units' streams): the last units of a fill are final units, so the replay moved into the
// fill's critical path instead of off it -- fill kernel 16.3 -> 16.8 ms, step unchanged
// (profiles/so2_fused_ab_r06.txt); not kept.
#pragma once
#include <limits.h>

#include "sa_internal.h"

namespace sa {

__device__ __forceinline__ uint32_t ec_code8(uint32_t sp, uint32_t b) {
    return (b == ((sp >> 8) & 255u) ? 8u : 0u) | (b == ((sp >> 16) & 255u) ? 16u : 0u) |
           (b == (sp >> 24) ? 24u : 0u);
}
#ifndef SA_EC_SCAN
#define SA_EC_SCAN 16
#endif
constexpr int kEcScan = SA_EC_SCAN;
// words per block row of the replay's LDS staging (endcell_so_lanes): one per step, rounded to
// whole 16-byte groups, and the corner
template <int R>
constexpr int kEcPk = ((kChunk + R - 1 + 3) & ~3) + 4;

// The score-only fill tracked the rows 3 mod 4 at the steps 3 mod 4 and stored, per (band, chunk,
// lane), the lane's maximum of its tracked cells; every cell is at most a tracked cell of the same
// lane and chunk - kSoSlack G, so S lies in [score, score - kSoSlack G] (score = the fill's smax)
// and only the LANE BLOCKS (R rows x 32 columns) whose tracked maximum reaches score + kSoSlack G
// can hold it.  Lists those blocks (first level: the (band, chunk) wave maxima snap_c, kEcScan x 64
// per round of loads; second level: the 64 lane maxima of each hit) into s_cand (CAND entries;
// s_hit: CAND) and recomputes each block alone -- its left column from the snapshot of the chunk
// before, its top row from the edge stream, one row per lane in a 32 + R - 1 step wavefront,
// 64 / R blocks per round (s_pk: 64 / R x kEcPk<R> words, 16-byte aligned) -- keeping per lane the
// lexicographically largest (H, i, j): the reference's last row-major maximum,
// SASmithWaterman.h:110.  Writes (score, end_i, end_j, reserved = 0) of pair `slot` and returns
// true; with more than CAND candidate blocks it writes nothing and returns false (the pair stays
// pending for endcell_so_kernel<R, DENSE = true>).  *ncand (if given): the candidate count.  One wave.
template <int R, int CAND>
__device__ __forceinline__ bool endcell_so_lanes(const EndcellParams& P, uint32_t slot, int score, uint32_t* s_cand,
                                                 uint32_t* s_hit, uint32_t (*s_pk)[kEcPk<R>], int* ncand = nullptr,
                                                 unsigned long long* ph = nullptr) {
    const int lane = threadIdx.x;
    const uint32_t symp = P.prof[4];
    const uint32_t pidx = P.pair_base + slot;
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
    const int thr = score + kSoSlack * G;   // lane blocks whose tracked maximum reaches this may hold S
    const int32_t* cm = P.snap_m + (uint64_t)slot * P.snap_p_slot;   // [band][chunk][lane]
    const uint32_t* sh_base = P.snap_h + (uint64_t)slot * P.snap_h_slot;
    const int32_t* sp_base = P.snap_p + (uint64_t)slot * P.snap_p_slot;
    int bv = -1, bi = -1, bj = -1;       // this lane's best (H, row, column), 0-based
    auto take = [&](int H, int row, int col) __attribute__((always_inline)) {
        if (H > bv || (H == bv && (row > bi || (row == bi && col > bj)))) { bv = H; bi = row; bj = col; }
    };
    // ---- the candidate lane blocks, in [band][chunk][lane] order.  First level: the fill's
    // (band, chunk) maxima of the lane maxima (FillParams::snap_c), kEcScan x 64 entries per round of
    // loads issued together; second level: the 64 lane maxima of each (band, chunk) that reaches thr
    // s_cand: band << 22 | chunk << 6 | lane; s_hit: (band, chunk) entries whose maximum reaches thr
    const uint32_t total = (uint32_t)B * snch;
    const int32_t* const sc = P.snap_c + (uint64_t)slot * P.snap_c_slot;
    int nhit = 0;
    if (ph) ph[0] = __builtin_amdgcn_s_memtime();
    for (uint32_t e0 = 0; e0 < total; e0 += kWave * kEcScan) {
        int v[kEcScan];
#pragma unroll
        for (int k = 0; k < kEcScan; ++k) {
            const uint32_t e = e0 + (uint32_t)(k * kWave + lane);
            v[k] = e < total && (int)(e % snch) < nch ? sc[e] : INT_MIN;
        }
#pragma unroll
        for (int k = 0; k < kEcScan; ++k) {
            const bool hit = v[k] >= thr;
            const uint64_t hits = __builtin_amdgcn_ballot_w64(hit);
            if (hit) {
                const int pos = nhit + (int)__builtin_popcountll(hits & ((1ull << lane) - 1));
                if (pos < CAND) s_hit[pos] = e0 + (uint32_t)(k * kWave + lane);
            }
            nhit += (int)__builtin_popcountll(hits);
        }
    }
    const bool over = nhit > CAND;   // (uniform) more chunks than the list holds: the DENSE launch
    nhit = min(nhit, CAND);
    __syncthreads();
    if (ph) ph[1] = __builtin_amdgcn_s_memtime();
    int cnt = over ? CAND + 1 : 0;
    for (int h0 = 0; h0 < (over ? 0 : nhit); h0 += kEcScan) {
        int v[kEcScan];
        uint32_t ee[kEcScan];
#pragma unroll
        for (int k = 0; k < kEcScan; ++k) {   // (wave-uniform)
            ee[k] = h0 + k < nhit ? s_hit[h0 + k] : 0u;
            v[k] = h0 + k < nhit ? cm[(uint64_t)ee[k] * kWave + lane] : INT_MIN;
        }
#pragma unroll
        for (int k = 0; k < kEcScan; ++k) {
            const bool hit = v[k] >= thr;
            const uint64_t hits = __builtin_amdgcn_ballot_w64(hit);
            if (hit) {
                const int pos = cnt + (int)__builtin_popcountll(hits & ((1ull << lane) - 1));
                const uint32_t bb = ee[k] / snch, cc = ee[k] - bb * snch;
                if (pos < CAND) s_cand[pos] = bb << 22 | cc << 6 | (uint32_t)lane;
            }
            cnt += (int)__builtin_popcountll(hits);
        }
    }
    __syncthreads();
    if (ph) ph[2] = __builtin_amdgcn_s_memtime();
    if (ncand) *ncand = cnt;

    if (cnt > CAND) return false;   // (uniform) pending: the DENSE launch takes the pair
    {
        // ---- lane blocks: 64 / R per round, lane = block g's row r
        constexpr int NB = kWave / R;
        const int g = lane / R, r = lane % R;
        // s_pk[NB][kEcPk<R>]: per block, entry q = 0 .. 31 = column code | top H << 16 (the value row
        // 0 reads at step q), the corner (top H at q = -1) in the row's last word
        const uint8_t* const dir = P.dirs + (uint64_t)slot * P.dir_slot;
        const uint64_t bst = P.band_stride;
        // Round k+1's loads (left word, top values, Seq2 / Seq1 bytes) are issued before round k's
        // steps and consumed after them, so a round's dependent global reads do not stall it; the
        // profile words are registers (no load behind the Seq1 byte).
        constexpr int QN = (kChunk + R) / R;   // q = r - 1 + R k < kChunk: at most QN per lane
        const uint32_t pf0 = P.prof[0], pf1 = P.prof[1], pf2 = P.prof[2], pf3 = P.prof[3];
        struct Pre {
            uint32_t w, s1c;
            uint32_t top[QN], s2c[QN];
        };
        auto fetch = [&](int c0, Pre& x) __attribute__((always_inline)) {
            const int ci = c0 + g;
            const bool act = ci < cnt;
            const uint32_t cd = act ? s_cand[ci] : 0u;
            const int b = (int)(cd >> 22), c = (int)((cd >> 6) & 0xffffu), t = (int)(cd & 63u);
            const int i = b * BAND + t * R + r;
            const int j0 = kChunk * c - t;
            x.w = 0;
            if (act && j0 >= 1 && i < m) x.w = sh_base[(((uint64_t)b * snch + (c - 1)) * (R / 2) + (r >> 1)) * kWave + t];
            // the top row (row i0 - 1, the last row of lane t - 1, or of lane 63 of band b - 1) and the
            // column codes: lane tp computed column jj at step jj + tp of its band's edge stream
            const bool has_top = !(b == 0 && t == 0);
            const int bp = t > 0 ? b : b - 1, tp = t > 0 ? t - 1 : kWave - 1;
#pragma unroll
            for (int k = 0; k < QN; ++k) {
                const int q = r - 1 + R * k, jj = j0 + q;
                x.top[k] = 0;
                x.s2c[k] = 0;
                if (q < kChunk && act && jj >= 0 && jj < n) {
                    if (has_top) {
                        if (q < 0 && j0 >= 1) {
                            x.top[k] = (uint32_t)sp_base[((uint64_t)b * snch + (c - 1)) * kWave + t] & 0xffffu;
                        } else {
                            const int st = jj + tp;
                            x.top[k] = *reinterpret_cast<const uint16_t*>(dir + (uint64_t)bp * bst +
                                                                        ((uint64_t)(st >> 3) * kWave + tp) * 16 + (st & 7) * 2);
                        }
                    }
                    x.s2c[k] = s2[jj];
                }
            }
            x.s1c = act && i < m ? s1[i] : 0u;
        };
        // steps of a round, rounded up to whole ds_read_b128 groups: the extra steps only touch
        // columns q >= kChunk, which no lane takes and no lane below reads inside its block
        constexpr int kSteps = (kChunk + R - 1 + 3) & ~3;
        static_assert(kSteps <= kEcPk<R> - 1, "s_pk row holds every step's word and the corner");
        Pre cur, nxt;
        fetch(0, cur);
        for (int c0 = 0; c0 < cnt; c0 += NB) {
            const int ci = c0 + g;
            const bool act = ci < cnt;
            const uint32_t cd = act ? s_cand[ci] : 0u;
            const int b = (int)(cd >> 22), c = (int)((cd >> 6) & 0xffffu), t = (int)(cd & 63u);
            const int i = b * BAND + t * R + r;   // this lane's row (0-based)
            const int j0 = kChunk * c - t;        // the block's first column
            // H at column j0 - 1 (left of the block; 0 where j0 <= 0: the left border)
            int h = (int)((r & 1) ? (cur.w >> 16) : (cur.w & 0xffffu));
#pragma unroll
            for (int k = 0; k < QN; ++k) {
                const int q = r - 1 + R * k, jj = j0 + q;
                const uint32_t code = (act && jj >= 0 && jj < n) ? ec_code8(symp, cur.s2c[k]) : 0u;
                if (q < 0) s_pk[g][kEcPk<R> - 1] = cur.top[k] << 16;
                else if (q < kChunk) s_pk[g][q] = code | cur.top[k] << 16;
            }
            // this lane's substitution scores by column code (bytes 0, 8, 16, 24), the profile's
            // (s * 4 + 3) bytes decoded once per round
            const uint32_t c8 = ec_code8(symp, cur.s1c);
            const uint32_t tab = c8 == 0 ? pf0 : c8 == 8 ? pf1 : c8 == 16 ? pf2 : pf3;
            uint32_t sub4 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                sub4 |= ((uint32_t)(((int)__builtin_amdgcn_sbfe(tab, 8u * k, 8u) - 3) >> 2) & 0xffu) << (8 * k);
            // the cells this lane takes: steps u = q + r with 0 <= q < kChunk and 0 <= j = j0 + q < n;
            // h advances from the first step with q >= 0 and j >= 0 (cells left of column 0 keep 0)
            const int ustart = r + max(0, -j0);
            const int uend = min(r + kChunk, r - j0 + n);
            const uint32_t span = act && i < m && uend > ustart ? (uint32_t)(uend - ustart) : 0u;
            if (c0 + NB < cnt) fetch(c0 + NB, nxt);
            __syncthreads();
            const bool row0 = r == 0;
            uint32_t pk = 0;   // (column code | top H << 16) of this lane's current column
            int up_prev = (int)(s_pk[g][kEcPk<R> - 1] >> 16);   // row 0: the corner; other rows: set below
            int rbv = -1, ru = 0;   // this round's best H and its step (ties: the later column)
            for (int u0 = 0; u0 < kSteps; u0 += 4) {
                const uint4 w4 = *reinterpret_cast<const uint4*>(&s_pk[g][u0]);
                const uint32_t wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int u = u0 + k;
                    // row r at column q = u - r: up = row r - 1's H at q (its previous step), diagonal =
                    // row r - 1's H at q - 1 (the up of this lane's previous step)
                    const int up_d = __builtin_amdgcn_update_dpp(0, h, 0x138, 0xf, 0xf, true);   // wave_shr:1
                    const uint32_t pk_d = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pk, 0x138, 0xf, 0xf, true);
                    pk = row0 ? wv[k] : pk_d;
                    const int up = row0 ? (int)(wv[k] >> 16) : up_d;
                    const int diag = up_prev;
                    up_prev = up;
                    const int sub = (int)__builtin_amdgcn_sbfe(sub4, pk, 8);
                    const int H = max(max(diag + sub, max(up, h) + G), 0);
                    h = u >= ustart ? H : h;
                    const bool tk = (uint32_t)(u - ustart) < span && H >= rbv;
                    rbv = tk ? H : rbv;
                    ru = tk ? u : ru;
                }
            }
            if (rbv >= 0) take(rbv, i, j0 + ru - r);
            __syncthreads();   // (s_pk and s_cand reads of this round)
            cur = nxt;
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
    return true;
}


}  // namespace sa
