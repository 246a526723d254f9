// sa_fill_so2.hip — the score-only Smith-Waterman fill with TWO pairs per wave (the headline path:
// T16 SW, many pairs, R = 32 band units), bit-for-bit the per-pair outputs of fill_so_kernel<SW, R>.
//
// Recurrence (SASmithWaterman.h:89-117): H = max(0, Hd + s, Hu + Gap, Hl + Gap).
//
// Why two pairs.  The shipped one-pair cell is 4 16-bit VOP2 ops + one v_bfe_i32 per cell, at its
// issue floor (profiles/fill_cell_ab_r05.txt).  Packed VOP3P ops and v_perm_b32 issue at the
// v_bfe rate, but each carries two cells when the two 16-bit halves of every register hold two
// independent pairs -- lane t runs rows [t R, t R + R) of pair A in the low halves and the same
// rows of pair B in the high halves, in the same band geometry, so every stream the traceback and
// the end-cell replay read (edge stream, snapshots, chunk maxima, band rows) keeps its layout per
// pair.  Per 2 cells, 6 ops (tools/microbench_pk6.hip: 14.15 vs 16.04 SIMD-cycles per 64 cells at
// 4 waves per SIMD, profiles/microbench_pk6_r06.txt):
//   p  = v_perm_b32(colB, colA, sel_r)   s(a_r, c) + 128 of both pairs: sel_r selects, per half, the
//                                        row symbol's byte of the column's table word (byte x =
//                                        s(x, c) + 128), and a zero high byte
//   dn = v_pk_add_u16(hp, p)             the next row's diagonal Hd + s, biased +128
//   t  = v_pk_max_i16(hu, hp)            max(Hu, Hl)
//   t  = v_pk_add_u16(t, Gap + 128)      max(Hu, Hl) + Gap, biased +128
//   h  = v_pk_max_i16(t, dr)             max(Hu + Gap, Hl + Gap, Hd + s) + 128  (>= 0: dr >= 0)
//   hp = v_pk_sub_u16(h, 128) clamp      ... and the zero clamp, by unsigned saturation
// Rows past a pair's m and columns past its n take the selector / table byte 0 (s = -128, as the
// one-pair kernel's rows past m): their cells are the recurrence's values for that substitution,
// never above their left or upper neighbour + Gap, so they never raise a chunk maximum above the
// matrix maximum and never feed a cell inside the matrix; the walks and the replay read no cell
// outside it.  The two pairs of a unit may differ in shape: the unit runs the larger band count and
// column count; a half whose pair has no band here is carried along and writes nothing.
//
// Work units, tickets, column segments, {tag, value} hand-off words, bounded waits and the per-unit
// maxima are those of the one-pair band units (sa_fill_impl.h BU), per pair.
//
// FK (round 6, SW): the cell in f16 arithmetic, 5 ops per 2 cells (tools/microbench_pk6.hip PK5F:
// 12.11 vs 14.15 SIMD-cycles per 64 cells, profiles/microbench_pk5f_r06.txt):
//   p  = v_perm_b32(colB, colA, sel_r)   s(a_r, c) as an f16 whose low byte is 0 (the table byte is
//                                        its high byte; sel_r selects it into the high byte of each
//                                        half and the constant 0 into the low byte)
//   dn = v_pk_add_f16(hp, p)             Hd + s
//   t  = v_pk_max_i16(hu, hp)            max(Hu, Hl) (H >= 0: f16 patterns order as integers)
//   t  = v_pk_add_f16(t, Gap)
//   hp = v_pk_maximum3_f16(t, dr, 0)     max(0, Hu + Gap, Hl + Gap, Hd + s)
// Exact while every value stays below 2048 (f16 integers); the host takes it when match and mismatch
// are such f16 values (sa_api.hip so2_f16_scoring) and flags for the int32 re-run every pair whose
// sampled maximum says a value may have reached 2048 (retry_above <= kSo2F16RetryAbove: the first
// such cell is computed >= 2048 and the sampled cell below it >= 2048 + kSoSlack Gap - kSoSlack).
// Every word other kernels read (edge stream, snapshots, chunk maxima, band rows) is converted to
// the integers of the 16-bit path on its way out (v_cvt_u16_f16, 2 ops per word), and band rows
// back to f16 on their way in; the segment hand-off words stay f16 (only this kernel reads them).
// Rows past a pair's m take s = 0 (the selector's constant byte), columns past its n s = -128:
// s <= 0 keeps those cells at most the matrix maximum, all the bounds above need.
//
// ALG = SA_NW (round 6): the same cell without the clamp (SANeedlemanWunsch.h:69-86; registers hold
// H - delta, the T16 window of t16_mode), the borders i Gap - delta / j Gap - delta in the left
// column, the corner and band 0's top row, no chunk maxima.  H[m][n] of each pair is taken at the
// one step where its lane computes column n - 1 of row m - 1 (columns past n run on, as in SW), and
// reaches the couple's final unit through the per-unit words.
#include "sa_fill_impl.h"

namespace sa {

namespace {

__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_pk_max_u16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ uint32_t lo16(uint32_t x) { return x & 0xffffu; }
// the lane index through an opaque move: per-lane addresses built from it inside the chunk loop are
// not hoisted out of it (as loop invariants they would each hold a 64-bit VGPR pair across the
// steps, and the 128-VGPR budget of 4 waves per SIMD spills them, with a scratch round trip --
// and an s_waitcnt vmcnt(0) that drains the edge-stream stores -- per reload)
__device__ __forceinline__ uint32_t lane_here() {
    uint32_t l;
    asm volatile("v_mov_b32 %0, %1" : "=v"(l) : "v"((uint32_t)threadIdx.x));
    return l;
}
__device__ __forceinline__ uint32_t hi16(uint32_t x) { return x >> 16; }
// the wave's maximum of each half, in lane 63 (DPP row prefix maxima, then the row broadcasts)
__device__ __forceinline__ uint32_t wave_pk_max(uint32_t v) {
    v = pk_max_u16(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = pk_max_u16(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = pk_max_u16(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = pk_max_u16(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = pk_max_u16(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = pk_max_u16(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}
__device__ __forceinline__ uint32_t pk_max_i16(uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_pk_max_i16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
// both halves: f16 integer -> u16 integer, and back
__device__ __forceinline__ uint32_t f16x2_to_u16x2(uint32_t x) {
    uint32_t d;
    asm("v_cvt_u16_f16_sdwa %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0\n\t"
        "v_cvt_u16_f16_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1"
        : "=&v"(d) : "v"(x));
    return d;
}
__device__ __forceinline__ uint32_t u16x2_to_f16x2(uint32_t x) {
    uint32_t d;
    asm("v_cvt_f16_u16_sdwa %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0\n\t"
        "v_cvt_f16_u16_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1"
        : "=&v"(d) : "v"(x));
    return d;
}
__device__ __forceinline__ uint32_t f16_bits(int s) {
    const _Float16 h = (_Float16)(float)s;
    return (uint32_t)__builtin_bit_cast(uint16_t, h);
}

}  // namespace

template <int ALG, int R, bool FK>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void fill_so2_kernel(FillParams P) {
    constexpr bool NWK = ALG == SA_NW;
    static_assert(!(FK && NWK), "the f16 cell is SW's");
    if (sa_skip(P.sel, P.sel_want)) return;   // (the score-only variant has no redo launch)
    static_assert(R >= 8 && R % 2 == 0, "the sampled chunk maximum needs 8 rows per lane");
    constexpr int BAND = kWave * R;
    constexpr int SPP = 8;   // steps per 16-byte edge-stream packet (16 bits per lane-step)
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    // step buffer: [0, 32) lane 0's row-above input (A | B << 16) of the chunk's steps, [32, 96)
    // the column table words (A, B interleaved), [96, 128) the last row parked by lane 63 per step,
    // [160, 192) the discard slots of lanes 0..62's parking writes
    uint32_t* const s_step = smem;
    const int lane = threadIdx.x;
    uint32_t* const s_park = s_step + (lane == 63 ? 96 : 160);
    const uint32_t SEGS = P.part_segs;
    const uint32_t ncp = (P.count + 1) / 2;   // couples of this launch (the last may hold one pair)
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(P.ticket, 1u);
    t = __builtin_amdgcn_readlane(t, 0);
    // tickets (band, segment, couple)-major: every producer of a unit holds a smaller ticket
    const uint32_t rowt = ncp * SEGS;
    const uint32_t band0 = t / rowt;
    const uint32_t rem = t - band0 * rowt;
    const uint32_t seg = rem / ncp;
    const uint32_t cp = rem - seg * ncp;
    const uint32_t sA = 2 * cp;
    const bool hasB = 2 * cp + 1 < P.count;
    const uint32_t sB = hasB ? 2 * cp + 1 : sA;
    const uint32_t pA = P.pair_base + sA, pB = P.pair_base + sB;
    const uint64_t o1A = P.off1[pA], o2A = P.off2[pA], o1B = P.off1[pB], o2B = P.off2[pB];
    const int mA = (int)(P.off1[pA + 1] - o1A), nA = (int)(P.off2[pA + 1] - o2A);
    const int mB = hasB ? (int)(P.off1[pB + 1] - o1B) : 0, nB = hasB ? (int)(P.off2[pB + 1] - o2B) : 0;
    const bool badA = (uint32_t)mA > P.max_m || (uint32_t)nA > P.max_n;
    const bool badB = hasB && ((uint32_t)mB > P.max_m || (uint32_t)nB > P.max_n);
    const int BA = (!badA && mA > 0 && nA > 0) ? (mA + BAND - 1) / BAND : 0;
    const int BB = (hasB && !badB && mB > 0 && nB > 0) ? (mB + BAND - 1) / BAND : 0;
    const int B2 = max(BA, BB);
    const int n2 = max(BA ? nA : 0, BB ? nB : 0);
    if ((int)band0 >= (B2 > 0 ? B2 : 1)) return;   // (uniform) a band neither pair has
    const uint32_t nch2 = chunks_per_band((uint32_t)n2);
    const uint32_t segs_p = max(1u, min(SEGS, nch2 / 2));
    const uint32_t cps = (nch2 + segs_p - 1) / segs_p;
    const uint32_t c0 = seg * cps, c1 = B2 > 0 ? min(nch2, c0 + cps) : 0u;
    const uint32_t last_seg = (nch2 - 1) / cps;
    if (seg > (B2 > 0 ? last_seg : 0u)) return;   // (uniform) an empty segment
    const uint32_t nchA = chunks_per_band((uint32_t)nA), nchB = chunks_per_band((uint32_t)nB);
    const bool liveA = (int)band0 < BA, liveB = (int)band0 < BB;
    const uint32_t epoch16 = P.epoch << 16;
    const uint32_t symp = P.prof[4];
    const int G = P.gap;
    const int D0 = P.t16_delta;
    // NW border H(i, 0) = H(0, i) = i Gap as H - delta in both halves (SW: 0)
    auto border2 = [&](int i) __attribute__((always_inline)) -> uint32_t {
        return NWK ? ((uint32_t)(i * G - D0) & 0xffffu) * 0x10001u : 0u;
    };
    uint32_t seg_lost = 0;

    // the column table words: byte x of cw[c] = s(x, c) + 128 (x: row symbol code, c: column code)
    uint32_t cw[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        uint32_t w = 0;
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            const int s = (int)(int8_t)(so_profile(P.prof[x]) >> (8 * c));
            if constexpr (FK) w |= (f16_bits(s) >> 8) << (8 * x);
            else w |= ((uint32_t)(s + 128) & 255u) << (8 * x);
        }
        cw[c] = w;
    }
    const uint8_t* const s1A = P.seq1 + o1A;
    const uint8_t* const s1B = P.seq1 + o1B;
    const uint8_t* const s2A = P.seq2 + o2A;
    const uint8_t* const s2B = P.seq2 + o2B;
    // Seq2 symbol codes of this unit's columns [k0, k0 + so2_stage) of both pairs, staged in LDS
    // (the 64 columns before its first chunk included), when the host gave the room
    const bool staged = P.so2_stage != 0;
    const int k0 = max(0, (int)(c0 * kChunk) - kWave);
    uint8_t* const s_cA = reinterpret_cast<uint8_t*>(smem + kStepBufWords);
    uint8_t* const s_cB = s_cA + P.so2_stage;
    if (staged) {
        const int k1 = min(n2, (int)(c1 * kChunk));
        for (int k = k0 + lane; k < k1; k += kWave) {
            s_cA[k - k0] = (uint8_t)(liveA && k < nA ? t16_code8(symp, s2A[(uint32_t)k]) >> 3 : 0u);
            s_cB[k - k0] = (uint8_t)(liveB && k < nB ? t16_code8(symp, s2B[(uint32_t)k]) >> 3 : 0u);
        }
        __syncthreads();
    }
    // the column table word of column c of each pair (substitution -128 outside it: 0, FK 0xd8 = -128.0)
    constexpr uint32_t kOut = FK ? 0xd8d8d8d8u : 0u;
    auto col_pair = [&](int c, uint32_t& wa, uint32_t& wb) {
        const bool ia = liveA && c >= 0 && c < nA, ib = liveB && c >= 0 && c < nB;
        uint32_t xa, xb;
        if (staged) {
            xa = ia ? (uint32_t)s_cA[c - k0] : 0u;
            xb = ib ? (uint32_t)s_cB[c - k0] : 0u;
        } else {
            xa = ia ? (t16_code8(symp, s2A[(uint32_t)c]) >> 3) : 0u;
            xb = ib ? (t16_code8(symp, s2B[(uint32_t)c]) >> 3) : 0u;
        }
        wa = ia ? (xa == 0 ? cw[0] : xa == 1 ? cw[1] : xa == 2 ? cw[2] : cw[3]) : kOut;
        wb = ib ? (xb == 0 ? cw[0] : xb == 1 ? cw[1] : xb == 2 ? cw[2] : cw[3]) : kOut;
    };
    // (FK: the packed f16 Gap)
    const uint32_t G128 = FK ? f16_bits(G) * 0x10001u : ((uint32_t)(G + 128) & 0xffffu) * 0x10001u;
    const uint32_t C128 = 0x00800080u;

    typedef uint32_t __attribute__((address_space(1))) gu32;
    gu32* const rbA = (gu32*)(P.rowbuf + (uint64_t)sA * P.rowbuf_slot);
    gu32* const rbB = (gu32*)(P.rowbuf + (uint64_t)sB * P.rowbuf_slot);
    const uint64_t rbs = P.max_n;

    // ------------------------------------------------------------------ band start
    // (per-lane addresses below are a wave-uniform base plus a 32-bit lane offset, so the stores
    // and loads take the SGPR-base form and no 64-bit address pair stays live across the chunks)
    const int row0 = (int)band0 * BAND + lane * R;
    uint32_t Hp[R], sel[R];
    uint32_t prev_up = border2(row0), colA = 0, colB = 0, cml = 0, smax = 0;   // (the lane's last row: Hp[R - 1])
#pragma unroll
    for (int r = 0; r < R; ++r) Hp[r] = border2(row0 + r + 1);
    // NW: H[m][n] of each pair is Hp[rr] of lane L after wavefront step n - 1 + L of the band holding
    // row m - 1 (-1: not this unit's band); cap*: the value, in lane L, took*: this unit's segment
    // holds that step
    // (capI = (m - 1) mod BAND = L R + rr: one scalar per pair besides the step)
    int capSA = -1, capSB = -1, capIA = 0, capIB = 0;
    uint32_t capA = 0, capB = 0;
    bool tookA = false, tookB = false;   // (uniform) this unit ran the step
    if constexpr (NWK) {
        if (liveA && mA > 0 && nA > 0 && (int)band0 == (mA - 1) / BAND) {
            capIA = (mA - 1) % BAND;
            capSA = nA - 1 + capIA / R;
        }
        if (liveB && mB > 0 && nB > 0 && (int)band0 == (mB - 1) / BAND) {
            capIB = (mB - 1) % BAND;
            capSB = nB - 1 + capIB / R;
        }
    }
    if (c0 > 0) {
        // a later segment: this lane's R values and diagonal input of each pair at column
        // 32 c0 - 1 - lane, handed on by the previous segment's unit (tagged, bounded wait).  Pair
        // A's words land in Hp, pair B's in sel (built after this).
        const uint64_t hoff = ((uint64_t)band0 * SEGS + seg - 1) * (R + 1) * kWave;
        const uint32_t* const hsA = P.seg_hand + (uint64_t)sA * P.seg_slot + hoff;
        const uint32_t* const hsB = P.seg_hand + (uint64_t)sB * P.seg_slot + hoff;
        uint32_t pa_ = 0, pb_ = 0;
        auto rd = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                Hp[r] = liveA ? __hip_atomic_load(hsA + (uint32_t)(r * kWave + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : epoch16;
                sel[r] = liveB ? __hip_atomic_load(hsB + (uint32_t)(r * kWave + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : epoch16;
            }
            pa_ = liveA ? __hip_atomic_load(hsA + (uint32_t)(R * kWave + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : epoch16;
            pb_ = liveB ? __hip_atomic_load(hsB + (uint32_t)(R * kWave + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : epoch16;
        };
        auto stale = [&]() __attribute__((always_inline)) -> bool {
            bool st = ((pa_ & 0xffff0000u) != epoch16) | ((pb_ & 0xffff0000u) != epoch16);
#pragma unroll
            for (int r = 0; r < R; ++r) st |= ((Hp[r] & 0xffff0000u) != epoch16) | ((sel[r] & 0xffff0000u) != epoch16);
            return st;
        };
        rd();
        for (uint32_t it = 0; !seg_lost && __builtin_amdgcn_ballot_w64(stale()) != 0; ++it) {
            if (it >= P.wait_polls) { seg_lost = 1; break; }
            __builtin_amdgcn_s_sleep(2);
            rd();
        }
#pragma unroll
        for (int r = 0; r < R; ++r) Hp[r] = lo16(Hp[r]) | sel[r] << 16;
        prev_up = lo16(pa_) | pb_ << 16;
        col_pair((int)(c0 * kChunk) - 1 - lane, colA, colB);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        const uint32_t ca = (liveA && row < mA) ? (t16_code8(symp, s1A[(uint32_t)row]) >> 3) : 12u;
        const uint32_t cb = (liveB && row < mB) ? (4u + (t16_code8(symp, s1B[(uint32_t)row]) >> 3)) : 12u;
        sel[r] = FK ? 0x0cu | ca << 8 | 0x0c0000u | cb << 24 : ca | 0x0c00u | cb << 16 | 0x0c000000u;
    }

    // One step of the chunk at kC: lane t computes column j = kC + q - t of its R rows of both
    // pairs (RAMP: a lane left of its first column keeps its border state).
    // (sq = s_step + q0, sc = s_step + 32 + 2 q0, g the step in its packet: one LDS address per
    // packet and array, immediate offsets)
    auto step = [&](auto ramp, auto gc, int kC, int q0, const uint32_t* sq, const uint32_t* sc, uint32_t* sp,
                    uint32_t& recA, uint32_t& recB) {
        constexpr bool RAMP = decltype(ramp)::value;
        constexpr int g = decltype(gc)::value;
        constexpr int PH = g & 3;
        const int q = q0 + g;
        const uint32_t vh = sq[g];
        const uint32_t va = sc[2 * g], vb = sc[2 * g + 1];
        const uint32_t up = (uint32_t)shr1((int)vh, (int)Hp[R - 1]);
        colA = (uint32_t)shr1((int)va, (int)colA);
        colB = (uint32_t)shr1((int)vb, (int)colB);
        if (!RAMP || kC + q - lane >= 0) {
            uint32_t dcur, pt;
            if constexpr (FK)
                asm("v_perm_b32 %1, %2, %3, %4\n\tv_pk_add_f16 %0, %5, %1"
                    : "=&v"(dcur), "=&v"(pt) : "v"(colB), "v"(colA), "v"(sel[0]), "v"(prev_up));
            else
                asm("v_perm_b32 %1, %2, %3, %4\n\tv_pk_add_u16 %0, %5, %1"
                    : "=&v"(dcur), "=&v"(pt) : "v"(colB), "v"(colA), "v"(sel[0]), "v"(prev_up));
            uint32_t hu = up;
            // the bias off again: SW with the zero clamp (unsigned saturation), NW without
#define SO2_CELL_N(LAST)                                                                          \
    asm("v_perm_b32 %[dn], %[cb], %[ca], %[sn]\n\t"                                                \
        "v_pk_add_u16 %[dn], %[hp], %[dn]\n\t"                                                     \
        "v_pk_max_i16 %[t1], %[hu], %[hp]\n\t"                                                     \
        "v_pk_add_u16 %[t1], %[t1], %[g]\n\t"                                                      \
        "v_pk_max_i16 %[t1], %[t1], %[dr]\n\t" LAST                                                \
        : [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])                                         \
        : [dr] "v"(dcur), [hu] "v"(hu), [g] "s"(G128), [c] "s"(C128),                              \
          [sn] "v"(sel[r + 1 < R ? r + 1 : r]), [ca] "v"(colA), [cb] "v"(colB))
#define SO2_CELL_L(LAST)                                                                          \
    asm("v_pk_max_i16 %[t1], %[hu], %[hp]\n\t"                                                     \
        "v_pk_add_u16 %[t1], %[t1], %[g]\n\t"                                                      \
        "v_pk_max_i16 %[t1], %[t1], %[dr]\n\t" LAST                                                \
        : [t1] "=&v"(t1), [hp] "+v"(Hp[r])                                                         \
        : [dr] "v"(dcur), [hu] "v"(hu), [g] "s"(G128), [c] "s"(C128))
#define SO2_CELL_FN                                                                               \
    asm("v_perm_b32 %[dn], %[cb], %[ca], %[sn]\n\t"                                                \
        "v_pk_add_f16 %[dn], %[hp], %[dn]\n\t"                                                     \
        "v_pk_max_i16 %[t1], %[hu], %[hp]\n\t"                                                     \
        "v_pk_add_f16 %[t1], %[t1], %[g]\n\t"                                                      \
        "v_pk_maximum3_f16 %[hp], %[t1], %[dr], 0"                                                 \
        : [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])                                         \
        : [dr] "v"(dcur), [hu] "v"(hu), [g] "s"(G128),                                             \
          [sn] "v"(sel[r + 1 < R ? r + 1 : r]), [ca] "v"(colA), [cb] "v"(colB))
#define SO2_CELL_FL                                                                               \
    asm("v_pk_max_i16 %[t1], %[hu], %[hp]\n\t"                                                     \
        "v_pk_add_f16 %[t1], %[t1], %[g]\n\t"                                                      \
        "v_pk_maximum3_f16 %[hp], %[t1], %[dr], 0"                                                 \
        : [t1] "=&v"(t1), [hp] "+v"(Hp[r])                                                         \
        : [dr] "v"(dcur), [hu] "v"(hu), [g] "s"(G128))
#pragma unroll
            for (int r = 0; r < R; ++r) {
                uint32_t t1;
                if (r + 1 < R) {
                    uint32_t dn;
                    if constexpr (FK) SO2_CELL_FN;
                    else if constexpr (NWK) SO2_CELL_N("v_pk_sub_u16 %[hp], %[t1], %[c]");
                    else SO2_CELL_N("v_pk_sub_u16 %[hp], %[t1], %[c] clamp");
                    dcur = dn;
                } else {
                    if constexpr (FK) SO2_CELL_FL;
                    else if constexpr (NWK) SO2_CELL_L("v_pk_sub_u16 %[hp], %[t1], %[c]");
                    else SO2_CELL_L("v_pk_sub_u16 %[hp], %[t1], %[c] clamp");
                }
                // the lane's chunk maximum of the rows 3 mod 4 at the steps 3 mod 4: every cell of
                // the chunk has such a cell of the same lane at most 3 rows below and 3 steps later,
                // and a cell is at most its lower / right neighbour - Gap (kSoSlack, as
                // fill_so_kernel).  Valid in ramp chunks too: the cells right of the matrix edge
                // follow the recurrence (substitution -128), so the bound holds through them.
                if (!NWK && PH == 3 && (r & 7) == 7) {
                    if constexpr (FK) {   // (f16 patterns of H >= 0; a -0.0 is the smallest i16)
                        cml = pk_max_i16(cml, Hp[r - 4]);
                        cml = pk_max_i16(cml, Hp[r]);
                    } else {
                        cml = pk_max_u16(cml, Hp[r - 4]);
                        cml = pk_max_u16(cml, Hp[r]);
                    }
                }
                hu = Hp[r];
            }
#undef SO2_CELL_N
#undef SO2_CELL_L
#undef SO2_CELL_FN
#undef SO2_CELL_FL
            prev_up = up;
        }
        if constexpr (NWK) {   // (uniform) H[m][n] of a pair: lane L's row rr after column n - 1
            if (kC + q == capSA) {
                uint32_t v = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) v = r == capIA % R ? Hp[r] : v;
                capA = lane == capIA / R ? lo16(v) : capA;
                tookA = true;
            }
            if (kC + q == capSB) {
                uint32_t v = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) v = r == capIB % R ? Hp[r] : v;
                capB = lane == capIB / R ? hi16(v) : capB;
                tookB = true;
            }
        }
        // the lane's last row of each pair, pushed into its packet word (two steps per word)
        recA = __builtin_amdgcn_alignbit(Hp[R - 1], recA, 16u);
        recB = __builtin_amdgcn_perm(Hp[R - 1], recB, 0x07060302u);
        sp[g] = Hp[R - 1];
    };

    uint8_t* const dA = P.dirs + (uint64_t)sA * P.dir_slot + (uint64_t)band0 * P.band_stride;
    uint8_t* const dB = P.dirs + (uint64_t)sB * P.dir_slot + (uint64_t)band0 * P.band_stride;
    gu32* const gA = rbA + (uint64_t)(band0 > 0 ? band0 - 1 : 0) * rbs;   // the producer band's granules
    gu32* const gB = rbB + (uint64_t)(band0 > 0 ? band0 - 1 : 0) * rbs;
    gu32* const oA = rbA + (uint64_t)band0 * rbs;   // this band's
    gu32* const oB = rbB + (uint64_t)band0 * rbs;
    for (uint32_t chunk = c0; chunk < c1; ++chunk) {
        const int kC = (int)chunk * kChunk;
        // ------------------------------------------------ the chunk's lane-0 inputs
        {
            const uint32_t ln = lane_here();
            const int c = kC + (int)ln;
            const bool in = lane < kChunk;
            uint32_t wa = 0, wb = 0;
            if (in) col_pair(c, wa, wb);
            const bool wantA = in && band0 > 0 && liveA && c < nA, wantB = in && band0 > 0 && liveB && c < nB;
            gu32* const ga = gA + (uint32_t)c;
            gu32* const gb = gB + (uint32_t)c;
            // band 0: the top border (SW 0, NW H(0, c + 1) = (c + 1) Gap)
            uint32_t ha = lo16(border2(c + 1)), hb = ha;
            if (wantA) ha = __hip_atomic_load(ga, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (wantB) hb = __hip_atomic_load(gb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (band0 > 0) {   // (uniform) the producer band's granules of this chunk, this launch's
                for (uint32_t it = 0; !seg_lost; ++it) {
                    const bool st = (wantA && (ha & 0xffff0000u) != epoch16) || (wantB && (hb & 0xffff0000u) != epoch16);
                    if (__builtin_amdgcn_ballot_w64(st) == 0) break;
                    if (it >= P.wait_polls) { seg_lost = 1; break; }
                    __builtin_amdgcn_s_sleep(2);
                    if (wantA) ha = __hip_atomic_load(ga, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (wantB) hb = __hip_atomic_load(gb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (in) {
                s_step[ln] = FK ? u16x2_to_f16x2(lo16(ha) | hb << 16) : lo16(ha) | hb << 16;
                s_step[32 + 2 * ln] = wa;
                s_step[33 + 2 * ln] = wb;
            }
        }
        __syncthreads();
        // ------------------------------------------------ 32 steps, 4 packets of 8 per pair
        // (the 8 steps of a packet unrolled with compile-time indices: the packet words and the
        // lane's rows stay in fixed registers)
        auto packet = [&](auto rmp, int q0) __attribute__((always_inline)) {
            uint32_t pa[SPP / 2] = {0, 0, 0, 0}, pb[SPP / 2] = {0, 0, 0, 0};
            const uint32_t* const sq = s_step + q0;
            const uint32_t* const sc = s_step + 32 + 2 * q0;
            uint32_t* const sp = s_park + q0;
            auto st = [&](auto gc) __attribute__((always_inline)) {
                constexpr int g = decltype(gc)::value;
                step(rmp, gc, kC, q0, sq, sc, sp, pa[g / 2], pb[g / 2]);
            };
            st(std::integral_constant<int, 0>{});
            st(std::integral_constant<int, 1>{});
            st(std::integral_constant<int, 2>{});
            st(std::integral_constant<int, 3>{});
            st(std::integral_constant<int, 4>{});
            st(std::integral_constant<int, 5>{});
            st(std::integral_constant<int, 6>{});
            st(std::integral_constant<int, 7>{});
            const uint32_t po = ((uint32_t)((kC + q0) / SPP) * kWave + (uint32_t)lane) * 16u;
            if constexpr (FK) {
#pragma unroll
                for (int w = 0; w < SPP / 2; ++w) {
                    pa[w] = f16x2_to_u16x2(pa[w]);
                    pb[w] = f16x2_to_u16x2(pb[w]);
                }
            }
            if (liveA) {
                const u32x4 v4 = {pa[0], pa[1], pa[2], pa[3]};
                __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(dA + po));
            }
            if (liveB) {
                const u32x4 v4 = {pb[0], pb[1], pb[2], pb[3]};
                __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(dB + po));
            }
        };
        if (kC < kWave - 1) {   // a band's first chunks: lanes left of their first column wait
#pragma unroll 1
            for (int q0 = 0; q0 < kChunk; q0 += SPP) packet(std::true_type{}, q0);
        } else {
#pragma unroll 1
            for (int q0 = 0; q0 < kChunk; q0 += SPP) packet(std::false_type{}, q0);
        }
        // ------------------------------------------------ the band's last row to the next band
        const uint32_t ln = lane_here();
        {
            uint32_t acc = s_step[96 + (ln & 31)];   // lane q < 32: column kC + q - 63
            if constexpr (FK) acc = f16x2_to_u16x2(acc);
            const int cc = kC + (int)ln - (kWave - 1);
            if (lane < kChunk && cc >= 0) {
                if ((int)band0 + 1 < BA && cc < nA)
                    __hip_atomic_store(oA + (uint32_t)cc, epoch16 | lo16(acc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((int)band0 + 1 < BB && cc < nB)
                    __hip_atomic_store(oB + (uint32_t)cc, epoch16 | hi16(acc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        // ------------------------------------------------ chunk maxima and snapshots, per pair
        {
            const uint64_t e = (uint64_t)band0 * P.snap_nch + chunk;
            if (kC + kChunk - 1 < lane) cml = 0;   // (a lane that has not reached its first column)
            if constexpr (FK) cml = f16x2_to_u16x2(cml);   // (integers from here on)
            smax = pk_max_u16(smax, cml);
            const uint32_t wm = NWK ? 0u : wave_pk_max(cml);
            const uint32_t pup = FK ? f16x2_to_u16x2(prev_up) : prev_up;
            if (liveA && chunk < nchA) {
                if constexpr (!NWK) {
                    int32_t* const smA = P.snap_m + (uint64_t)sA * P.snap_p_slot + e * kWave;
                    smA[ln] = (int32_t)lo16(cml);
                    if (lane == kWave - 1) P.snap_c[(uint64_t)sA * P.part_bands * P.snap_nch + e] = (int32_t)lo16(wm);
                }
                if (chunk + 1 < nchA) {
                    uint32_t* const sh = P.snap_h + (uint64_t)sA * P.snap_h_slot + e * (R / 2) * kWave + ln;
#pragma unroll
                    for (int q = 0; q < R / 2; ++q) {   // (one address, immediate offsets)
                        const uint32_t w = __builtin_amdgcn_perm(Hp[2 * q + 1], Hp[2 * q], 0x05040100u);
                        sh[q * kWave] = FK ? f16x2_to_u16x2(w) : w;
                    }
                    int32_t* const spA = P.snap_p + (uint64_t)sA * P.snap_p_slot + e * kWave;
                    spA[ln] = (int32_t)lo16(pup);
                }
            }
            if (liveB && chunk < nchB) {
                if constexpr (!NWK) {
                    int32_t* const smB = P.snap_m + (uint64_t)sB * P.snap_p_slot + e * kWave;
                    smB[ln] = (int32_t)hi16(cml);
                    if (lane == kWave - 1) P.snap_c[(uint64_t)sB * P.part_bands * P.snap_nch + e] = (int32_t)hi16(wm);
                }
                if (chunk + 1 < nchB) {
                    uint32_t* const sh = P.snap_h + (uint64_t)sB * P.snap_h_slot + e * (R / 2) * kWave + ln;
#pragma unroll
                    for (int q = 0; q < R / 2; ++q) {   // (one address, immediate offsets)
                        const uint32_t w = __builtin_amdgcn_perm(Hp[2 * q + 1], Hp[2 * q], 0x07060302u);
                        sh[q * kWave] = FK ? f16x2_to_u16x2(w) : w;
                    }
                    int32_t* const spB = P.snap_p + (uint64_t)sB * P.snap_p_slot + e * kWave;
                    spB[ln] = (int32_t)hi16(pup);
                }
            }
            cml = 0;
        }
        // ------------------------------------------------ hand the lanes' state to the next segment
        if (chunk + 1 == c1 && c1 < nch2) {
            const uint64_t hoff = ((uint64_t)band0 * SEGS + seg) * (R + 1) * kWave;
            if (liveA) {
                uint32_t* const hs = P.seg_hand + (uint64_t)sA * P.seg_slot + hoff + ln;
#pragma unroll
                for (int r = 0; r < R; ++r)
                    __hip_atomic_store(hs + r * kWave, epoch16 | lo16(Hp[r]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(hs + R * kWave, epoch16 | lo16(prev_up), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (liveB) {
                uint32_t* const hs = P.seg_hand + (uint64_t)sB * P.seg_slot + hoff + ln;
#pragma unroll
                for (int r = 0; r < R; ++r)
                    __hip_atomic_store(hs + r * kWave, epoch16 | hi16(Hp[r]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(hs + R * kWave, epoch16 | hi16(prev_up), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();   // (the step buffer of the next chunk)
    }

    // ---------------------------------------------------------------------- results
    // every unit of the couple stores one word per pair {tag, lost, the unit's maximum of the pair};
    // the couple's final unit (last band, last segment) folds them and reports both pairs
    seg_lost = __builtin_amdgcn_ballot_w64(seg_lost != 0) != 0 ? 1u : 0u;
    // the unit's word of each pair: SW its maximum of the tracked cells; NW H[m][n] - delta as
    // 1 << 16 | (v ^ 0x8000) (order-preserving, above every word of a unit without it) or 0
    uint32_t wA = 0, wB = 0;
    if constexpr (NWK) {
        if (tookA) wA = 1u << 16 | (((uint32_t)__builtin_amdgcn_readlane((int)capA, capIA / R) & 0xffffu) ^ 0x8000u);
        if (tookB) wB = 1u << 16 | (((uint32_t)__builtin_amdgcn_readlane((int)capB, capIB / R) & 0xffffu) ^ 0x8000u);
    } else {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) smax = pk_max_u16(smax, (uint32_t)__shfl_xor((int)smax, off));
        wA = liveA ? lo16(smax) : 0u;
        wB = liveB ? hi16(smax) : 0u;
    }
    typedef unsigned long long __attribute__((address_space(1))) gu64p;
    gu64p* const partA = (gu64p*)(P.band_part + (uint64_t)sA * P.part_bands * SEGS);
    gu64p* const partB = (gu64p*)(P.band_part + (uint64_t)sB * P.part_bands * SEGS);
    const uint32_t me = band0 * SEGS + seg, nparts = B2 > 0 ? (uint32_t)(B2 - 1) * SEGS + last_seg : 0u;
    if (me != nparts) {
        if (lane == 0) {
            __hip_atomic_store(partA + me, (unsigned long long)epoch16 << 32 | wA | seg_lost << 31,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (hasB)
                __hip_atomic_store(partB + me, (unsigned long long)epoch16 << 32 | wB | seg_lost << 31,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    uint32_t lostA = seg_lost, lostB = seg_lost;
    uint32_t mxA = bu_fold_parts(partA, nparts, last_seg, SEGS, epoch16, P.wait_polls, lane, lostA);
    uint32_t mxB = hasB ? bu_fold_parts(partB, nparts, last_seg, SEGS, epoch16, P.wait_polls, lane, lostB) : 0u;
    mxA = max(mxA, wA);
    mxB = max(mxB, wB);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        mxA = max(mxA, (uint32_t)__shfl_xor((int)mxA, off));
        mxB = max(mxB, (uint32_t)__shfl_xor((int)mxB, off));
    }
    if (lane == 0) {
        auto report = [&](uint32_t pidx, bool bad, int Bx, int mx_, int nx_, uint32_t mx, uint32_t lost) {
            sa_result r = {};
            if (bad) {
                r.flags = SA_FLAG_BAD_SHAPE;
            } else if constexpr (NWK) {
                // SANeedlemanWunsch.h: H[m][n], the walk starts at (m, n); an empty input is the
                // border's max(m, n) Gap
                r.end_i = mx_;
                r.end_j = nx_;
                if (Bx == 0) {
                    r.score = (mx_ > nx_ ? mx_ : nx_) * G;
                } else {
                    r.score = (int)(int16_t)(uint16_t)((mx & 0xffffu) ^ 0x8000u) + D0;
                    if (!((mx >> 16) & 1u) || lost) r.flags |= kFlagRetry;   // (no unit took it: re-run)
                }
            } else if (Bx == 0) {
                r.score = INT_MIN;   // empty input: SW keeps MaxScore = INT_MIN, (MaxRow, MaxCol) = (0, 0)
            } else {
                // S >= mx and S <= mx - kSoSlack Gap: endcell_so_kernel finds S and the last
                // row-major cell
                r.score = (int)mx;
                r.reserved = 1;
                if ((int)mx - kSoSlack * G > P.retry_above) {
                    r.flags |= kFlagRetry;
                    if constexpr (FK) atomicAdd(P.ticket + (kAuxF16Flags - kAuxTicket), 1u);   // (the host's f16 policy)
                }
                if (lost) r.flags |= kFlagRetry;
            }
            P.res[pidx] = r;
        };
        report(pA, badA, BA, mA, nA, mxA, lostA);
        if (hasB) report(pB, badB, BB, mB, nB, mxB, lostB);
    }
}

hipError_t launch_fill_so2(int algo, int R, const FillParams& p, uint32_t grid, hipStream_t stream) {
    const size_t lds = (size_t)kStepBufWords * 4 + 2 * (size_t)p.so2_stage;
#define SO2_LAUNCH(A, RR, F)                                                                        \
    if (algo == (A) && R == (RR) && (p.so2_f16 != 0) == (F)) {                                      \
        hipLaunchKernelGGL((fill_so2_kernel<A, RR, F>), dim3(grid), dim3(kWave), lds, stream, p);  \
        return hipGetLastError();                                                                  \
    }
    SO2_LAUNCH(SA_SW, 32, true)
    SO2_LAUNCH(SA_SW, 16, true)
    SO2_LAUNCH(SA_SW, 32, false)
    SO2_LAUNCH(SA_SW, 16, false)
    SO2_LAUNCH(SA_NW, 32, false)
    SO2_LAUNCH(SA_NW, 16, false)
#undef SO2_LAUNCH
    return hipErrorInvalidValue;
}

}  // namespace sa
