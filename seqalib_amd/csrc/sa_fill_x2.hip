// sa_fill_x2.hip — the T16 Smith-Waterman fill for TWO pairs per wave (packed 16-bit halves).
//
// Same recurrence, tags, chunk-max end cell and record format as the T16 CMAX kernel of
// sa_fill_impl.h (SASmithWaterman.h:89-117; H kept as 4H + tag, tags 3 diag / 2 up / 1 left /
// 0 zero clamp), but every register holds pair A (this workgroup's first pair) in its low 16
// bits and pair B in its high 16 bits, and the cell runs on VOP3P packed ops: per row and step
// ONE instruction sequence updates the cells of both pairs.
//
// Per row (2 cells):
//   v_pk_add_u16     left   = Hp + (4G + 1)
//   v_perm_b32       the next row's substitution bytes of both pairs (high byte of each half),
//                    from the two column profiles (DPP-shifted per step like the row-above value)
//                    and the row's selector (its symbol codes)
//   v_pk_ashrrev_i16 sign-extend them, v_pk_add_u16 next row's diagonal = Hp + s
//   v_pk_sub_u16     up     = max(Hu + 4G + 2, 0)   (clamp: the zero clamp of the cell)
//   2 v_pk_max_i16   the tagged max chain (value and winning move with the reference's ties)
//   v_and_b32        strip both tags;  v_and_b32 + v_lshl_add_u32  push both tags
//   v_pk_max_i16     the lane's chunk maximum (end cell)
// = 11 VALU per 2 cells (the one-pair kernel: 8.7 per cell).  tools/microbench_pk.hip measured
// the packed ops at ~4.3 cycles each against ~3.3 for the one-pair mix (net +16 % at equal
// occupancy), and the packed kernel needs about half the registers per cell (5 waves / SIMD).
//
// Records: the tag push (rec = 4 rec + tags) accumulates 8 rows per 16-bit half, first row
// highest; v_perm_b32 splits two packed words into one record word per pair, so a pair's record
// word holds rows 8g..8g+7 at bits 16(g%2) + 2(7 - r%8) (sa_layout.h, "tagged = 2").  Both
// pairs' records, row buffers, snapshots and results go to their own per-pair slots in exactly
// the layout sa_endcell.hip and the tracebacks read for the one-pair kernel.
//
// Ragged pairs: the wave runs the larger shape; rows past a pair's m select the byte 0xFF
// (substitution -1 in 4s+3 form) and columns past its n get an all-0xFF column profile, so with
// gap < 0 those cells stay strictly below the pair's maximum (the end cell is unchanged) and
// their records are never read.
#include <limits.h>

#include "sa_internal.h"

namespace sa {

namespace {

typedef unsigned int x2_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t x2_shr1(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x138, 0xf, 0xf, false);
}

__device__ __forceinline__ uint32_t x2_code(uint32_t sp, uint32_t b) {   // T16 code 0..3 of symbol b
    return (b == ((sp >> 8) & 255u) ? 1u : 0u) | (b == ((sp >> 16) & 255u) ? 2u : 0u) | (b == (sp >> 24) ? 3u : 0u);
}

}  // namespace

template <int R>
__global__ __launch_bounds__(64, R == 16 ? 5 : 3) void fill_x2_kernel(FillParams P) {
    static_assert(R == 16 || R == 32, "8-row packed record groups, whole record words");
    constexpr int NPW = R / 8;          // packed record words per step (8 rows each)
    constexpr int RW = R / 16;          // record words per pair per step (2 bits x R rows)
    constexpr int SPP = 4 / RW;         // steps per 16-byte packet
    constexpr int BAND = kWave * R;
    if (sa_skip(P.sel, P.sel_want)) return;   // the batch selected the int32 variant

    // LDS (~1 KiB, so 20 workgroups fit a CU): the transposed profile and the per-step buffers
    //   [0, 32) lane-0 row-above input, [32, 64) / [64, 96) column profiles of A / B,
    //   [96, 128) the band's last row parked by lane 63, [128, 160) lanes 0..62's discard slots
    __shared__ uint32_t s_tprof[4];
    __shared__ __attribute__((aligned(16))) int32_t s_step[160];
    const int lane = threadIdx.x;
    const uint32_t symp = P.prof[4];
    if (lane < 4) {   // tprof[b] byte a = prof[a] byte b: the column profile of column code b
        uint32_t w = 0;
        for (int a = 0; a < 4; ++a) w |= ((P.prof[a] >> (8 * lane)) & 255u) << (8 * a);
        s_tprof[lane] = w;
    }
    const uint32_t slot[2] = {2 * blockIdx.x, 2 * blockIdx.x + 1};
    int m[2], n[2];
    uint64_t o1[2], o2[2];
    bool ok[2];
    // has[1] is false for the odd last pair of a launch: that half computes on empty input and
    // never touches memory (its slot would be past the launch's workspace)
    const bool has[2] = {true, slot[1] < P.count};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t pidx = P.pair_base + (has[h] ? slot[h] : slot[0]);
        o1[h] = P.off1[pidx];
        o2[h] = P.off2[pidx];
        m[h] = has[h] ? (int)(P.off1[pidx + 1] - o1[h]) : 0;
        n[h] = has[h] ? (int)(P.off2[pidx + 1] - o2[h]) : 0;
        ok[h] = has[h] && (uint32_t)m[h] <= P.max_m && (uint32_t)n[h] <= P.max_n;
        if (!ok[h]) { m[h] = 0; n[h] = 0; }
    }
    const int MM = max(m[0], m[1]), NN = max(n[0], n[1]);
    const int B = (MM > 0 && NN > 0) ? (MM + BAND - 1) / BAND : 0;
    const uint8_t* s1[2] = {P.seq1 + o1[0], P.seq1 + o1[1]};
    const uint8_t* s2[2] = {P.seq2 + o2[0], P.seq2 + o2[1]};
    __syncthreads();
    // Seq2 symbols of a chunk are loaded one chunk ahead (lanes 0..31: column kC + lane)
    auto ld2 = [&](int c, int h) -> uint32_t { return c < n[h] ? (uint32_t)s2[h][c] : 0u; };

    const int G = P.gap;
    // tagged gap terms, both halves: up = max(4Hu + 4G + 2, 0) as a saturating subtract (t16_ok:
    // G < 0), left = 4Hl + 4G + 1
    const uint32_t cu = (uint32_t)(-(4 * G + 2)) & 0xffffu, cl = (uint32_t)(4 * G + 1) & 0xffffu;
    const uint32_t CU2 = cu | cu << 16, CL2 = cl | cl << 16;
    const uint32_t SM2 = 0xfffcfffcu, SH8 = 0x00080008u;
    const uint32_t nch = chunks_per_band((uint32_t)NN);
    int32_t* const s_park = s_step + (lane == 63 ? 96 : 128);   // lanes 0..62: discard slots
    const uint32_t sl1 = has[1] ? slot[1] : slot[0];   // an absent half reads pair A's buffers, writes nothing
    uint8_t* const dslot[2] = {P.dirs + (uint64_t)slot[0] * P.dir_slot, P.dirs + (uint64_t)sl1 * P.dir_slot};
    int32_t* const rb[2] = {P.rowbuf + (uint64_t)slot[0] * P.rowbuf_slot, P.rowbuf + (uint64_t)sl1 * P.rowbuf_slot};

    uint32_t rs[R];   // per row: perm selector [0x00, A's code, 0x00, 4 + B's code] (13: past m)
    uint32_t Hp[R];   // 4H of both pairs at the previous column
    uint32_t hl = 0, cA = 0, cB = 0, prev_up = 0, cml = 0;
    uint32_t lkey[2] = {0, 0};
    int best_h[2] = {INT_MIN, INT_MIN}, best_i[2] = {0, 0}, best_j[2] = {0, 0};
    int row0 = 0;

    for (int band = 0; band < B; ++band) {
        row0 = band * BAND + lane * R;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int row = row0 + r;
            const uint32_t ca = row < m[0] ? x2_code(symp, s1[0][row]) : 13u;
            const uint32_t cb = row < m[1] ? 4u + x2_code(symp, s1[1][row]) : 13u;
            rs[r] = 0x000c000cu | ca << 8 | cb << 24;   // bytes 0, 2: selector 12 = 0x00
            Hp[r] = 0;
        }
        lkey[0] = lkey[1] = 0;
        cml = 0;
        prev_up = 0;
        hl = 0;
        uint32_t nx[2] = {ld2(lane, 0), ld2(lane, 1)};
        for (uint32_t chunk = 0; chunk < nch; ++chunk) {
            const int kC = (int)chunk * kChunk;
            // this chunk's lane-0 inputs: the row above (band 0: the zero border; else both pairs'
            // previous-band rows) and both column profiles (past a pair's n: all 0xFF)
            if (lane < kChunk) {
                const int c = kC + lane;
                uint32_t up = 0;
                if (band > 0 && c < NN) {
                    const uint64_t e = (uint64_t)(band - 1) * P.max_n + c;
                    up = ((uint32_t)rb[0][e] & 0xffffu) | (uint32_t)rb[1][e] << 16;
                }
                s_step[lane] = (int32_t)up;
                s_step[32 + lane] = (int32_t)(c < n[0] ? s_tprof[x2_code(symp, nx[0])] : 0xffffffffu);
                s_step[64 + lane] = (int32_t)(c < n[1] ? s_tprof[x2_code(symp, nx[1])] : 0xffffffffu);
                nx[0] = ld2(c + kChunk, 0);   // next chunk's, in flight meanwhile
                nx[1] = ld2(c + kChunk, 1);
            }
            __syncthreads();
            const bool steady = kC >= kWave - 1 && kC + kChunk <= NN;
#pragma unroll 1
            for (int q0 = 0; q0 < kChunk; q0 += SPP) {
                uint32_t pk[2][4];
#pragma unroll
                for (int g = 0; g < SPP; ++g) {
                    const int q = q0 + g;
                    const uint32_t up_h = x2_shr1((uint32_t)s_step[q], hl);
                    cA = x2_shr1((uint32_t)s_step[32 + q], cA);
                    cB = x2_shr1((uint32_t)s_step[64 + q], cB);
                    const int j = kC + q - lane;
                    uint32_t pw[NPW];
                    if (steady || (unsigned)j < (unsigned)NN) {
                        uint32_t dcur;
                        asm("v_perm_b32 %0, %1, %2, %3\n\tv_pk_ashrrev_i16 %0, %4, %0\n\tv_pk_add_u16 %0, %5, %0"
                            : "=&v"(dcur) : "v"(cB), "v"(cA), "v"(rs[0]), "s"(SH8), "v"(prev_up));
                        uint32_t hu = up_h;
#pragma unroll
                        for (int e = 0; e < NPW; ++e) pw[e] = 0;   // 8 pushes per word: shifted once only
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            uint32_t& w = pw[r / 8];
                            uint32_t t0, t1;
#define X2_HEAD                                                                               \
    "v_pk_add_u16 %[t0], %[cl], %[hp]\n\t"
#define X2_NEXT                                                                               \
    "v_perm_b32 %[dn], %[cb], %[ca], %[rsn]\n\t"                                              \
    "v_pk_ashrrev_i16 %[dn], %[sh8], %[dn]\n\t"                                               \
    "v_pk_add_u16 %[dn], %[hp], %[dn]\n\t"
#define X2_TAIL                                                                               \
    "v_pk_sub_u16 %[t1], %[hu], %[cu] clamp\n\t"                                              \
    "v_pk_max_i16 %[t0], %[dr], %[t0]\n\t"                                                    \
    "v_pk_max_i16 %[t0], %[t1], %[t0]\n\t"                                                    \
    "v_and_b32 %[hp], %[sm], %[t0]\n\t"                                                       \
    "v_and_b32 %[t1], 0x30003, %[t0]\n\t"                                                     \
    "v_lshl_add_u32 %[w], %[w], 2, %[t1]\n\t"                                                 \
    "v_pk_max_i16 %[cm], %[cm], %[hp]\n\t"
#define X2_OUT [t0] "=&v"(t0), [t1] "=&v"(t1), [hp] "+v"(Hp[r]), [w] "+v"(w), [cm] "+v"(cml)
#define X2_IN [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU2), [cl] "s"(CL2), [sm] "s"(SM2)
                            if (r + 1 < R) {
                                uint32_t dn;
                                asm(X2_HEAD X2_NEXT X2_TAIL
                                    : X2_OUT, [dn] "=&v"(dn)
                                    : X2_IN, [ca] "v"(cA), [cb] "v"(cB), [rsn] "v"(rs[r + 1 < R ? r + 1 : r]), [sh8] "s"(SH8));
                                dcur = dn;
                            } else {
                                asm(X2_HEAD X2_TAIL : X2_OUT : X2_IN);
                            }
#undef X2_HEAD
#undef X2_NEXT
#undef X2_TAIL
#undef X2_OUT
#undef X2_IN
                            hu = Hp[r];
                        }
                        prev_up = up_h;
                        hl = Hp[R - 1];
                    } else {
#pragma unroll
                        for (int e = 0; e < NPW; ++e) pw[e] = 0;
                    }
                    // one record word per pair and 16 rows: [rows 16k..16k+7 | rows 16k+8..16k+15]
#pragma unroll
                    for (int e = 0; e < RW; ++e) {
                        pk[0][g * RW + e] = __builtin_amdgcn_perm(pw[2 * e + 1], pw[2 * e], 0x05040100u);
                        pk[1][g * RW + e] = __builtin_amdgcn_perm(pw[2 * e + 1], pw[2 * e], 0x07060302u);
                    }
                    s_park[q] = (int32_t)hl;   // lane 63: the band's last row at column kC + q - 63
                }
                const uint64_t off = (uint64_t)band * P.band_stride + ((uint64_t)((kC + q0) / SPP) * kWave + lane) * 16;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const x2_u32x4 v4 = {pk[h][0], pk[h][1], pk[h][2], pk[h][3]};
                    if (has[h]) __builtin_nontemporal_store(v4, reinterpret_cast<x2_u32x4*>(dslot[h] + off));
                }
            }
            // hand the band's last row (columns kC-63 .. kC-32) to the next band, per pair
            if (band + 1 < B && lane < kChunk) {
                const int cc = kC + lane - (kWave - 1);
                if (cc >= 0 && cc < NN) {
                    const uint32_t v = (uint32_t)s_step[96 + lane];
                    const uint64_t e = (uint64_t)band * P.max_n + cc;
                    rb[0][e] = (int32_t)(v & 0xffffu);
                    if (has[1]) rb[1][e] = (int32_t)(v >> 16);
                }
            }
            // chunk maxima and the snapshot entering chunk + 1, per pair (sa_endcell.hip layout)
            {
                const uint32_t ck = chunk + 1;
                const uint64_t e = (uint64_t)band * P.snap_nch + chunk;
                const uint32_t cmh[2] = {cml & 0xffffu, cml >> 16};
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (has[h]) P.snap_m[(uint64_t)slot[h] * P.snap_p_slot + e * kWave + lane] = (int32_t)cmh[h];
                    lkey[h] = max(lkey[h], (cmh[h] >> 2) << 12 | ck);
                }
                cml = 0;
                if (chunk + 1 < nch) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        if (!has[h]) continue;
                        uint32_t* sh = P.snap_h + (uint64_t)slot[h] * P.snap_h_slot + e * (R / 2) * kWave + lane;
                        const uint32_t sel = h ? 0x07060302u : 0x05040100u;
#pragma unroll
                        for (int q = 0; q < R / 2; ++q) sh[q * kWave] = __builtin_amdgcn_perm(Hp[2 * q + 1], Hp[2 * q], sel);
                        P.snap_p[(uint64_t)slot[h] * P.snap_p_slot + e * kWave + lane] = (int32_t)(h ? prev_up >> 16 : prev_up & 0xffffu);
                    }
                }
            }
            __syncthreads();
        }
        // band end: (score, lane, chunk) per pair; sa_endcell.hip finds the row and the column
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int hh = (int)(lkey[h] >> 12);
            if (lkey[h] != 0 && hh >= best_h[h]) {
                best_h[h] = hh;
                best_i[h] = row0 + R;
                best_j[h] = (int)(lkey[h] & 4095u);
            }
        }
    }

    // results: lexicographic max over (score, i, j) per pair, the reference's last row-major max
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        int bh = best_h[h], bi = best_i[h], bj = best_j[h];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const int oh = __shfl_xor(bh, off), oi = __shfl_xor(bi, off), oj = __shfl_xor(bj, off);
            if (oh > bh || (oh == bh && (oi > bi || (oi == bi && oj > bj)))) { bh = oh; bi = oi; bj = oj; }
        }
        if (lane == 0 && slot[h] < P.count) {
            sa_result r = {};
            if (!ok[h]) {
                r.flags = SA_FLAG_BAD_SHAPE;
            } else if (m[h] == 0 || n[h] == 0) {
                r.score = INT_MIN;   // empty input: SW keeps MaxScore = INT_MIN, (MaxRow, MaxCol) = (0, 0)
            } else {
                r.score = bh; r.end_i = bi; r.end_j = 0;
                r.reserved = (uint32_t)bj;   // chunk + 1: sa_endcell.hip resolves the column
                if (bh > P.retry_above) r.flags |= kFlagRetry;
            }
            P.res[P.pair_base + slot[h]] = r;
        }
    }
}

hipError_t launch_fill_sw_x2(int R, const FillParams& p, uint32_t pairs, hipStream_t stream) {
    const dim3 grid((pairs + 1) / 2), block(64);
    switch (R) {
        case 16: hipLaunchKernelGGL(fill_x2_kernel<16>, grid, block, 0, stream, p); break;
        case 32: hipLaunchKernelGGL(fill_x2_kernel<32>, grid, block, 0, stream, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sa
