// sa_traceback_so.hip — buildResult of SmithWatermanSA (SASmithWaterman.h:220-339) after a
// SCORE-ONLY fill (sa_fill_impl.h, SO): the fill stored no per-cell records, so the walk recomputes
// the move tags of the cells it visits, block by block, from what the fill did store:
//   * the per-chunk snapshots (every lane's R row values entering chunk c, and its diagonal input),
//   * the edge stream (every lane's last row at every step of its band, 16 bits per lane-step).
// Block (band b, lane t, chunk c) = rows r0 .. r0+R-1 (r0 = b*64R + t*R) x columns j0 .. j0+31
// (j0 = 32c - t, 0-based), the cells lane t computed during chunk c.  Its left column (j0 - 1) is
// lane t's snapshot of chunk c-1, its corner the snapshot's diagonal input, its top row the edge
// stream of the lane above (lane t-1 computed column j at step j + t - 1; for t = 0, lane 63 of
// band b-1, at step j + 63).  The recompute runs the fill's tagged 16-bit cell (4H + tag, one
// v_max_i16 chain gives value and move with the reference's tie order diag > up > left), so the
// tags are exactly those the tagged fill would have stored (sa_traceback.hip reads those).
//
// The walk only moves up and left, so once it leaves a block it never returns, and inside a block
// it needs only the rows above and the columns left of the cell it entered at: the recompute stops
// at the entry column.  One lane per pair (64 pairs per wave); lanes whose next move leaves their
// block park, and when every unfinished lane is parked they all recompute together (as
// sa_traceback.hip batches its window refills).  The tags of a block live in LDS, item-major.
#include <limits.h>

#include "sa_internal.h"

namespace sa {

typedef const void __attribute__((address_space(1)))* so_gptr;
typedef void __attribute__((address_space(3)))* so_lptr;

// LDS per wave (bytes), words item-major ([item][lane], 256 B per item):
//   tags      32 columns x RT words (RT = ceil(2R / 32)): column q, word w at item q * RT + w
//   edge      5 packets of 16 B (the top row's 32 steps), lane t's packet k at k * 1024 + 16 * lane
//   codes     R row codes then 32 column codes (8 * code, one byte each)
//   ops       kSoOps op bytes per lane per round
constexpr int kSoOps = 64;
template <int R>
struct SoLds {
    static constexpr int RT = (2 * R + 31) / 32;
    static constexpr int kTags = 0;
    static constexpr int kEdge = kTags + 32 * RT * 256;
    static constexpr int kRowCodes = kEdge + 5 * 1024;
    static constexpr int kColCodes = kRowCodes + ((R + 3) / 4) * 256;
    static constexpr int kOps = kColCodes + 8 * 256;
    static constexpr int kBytes = kOps + kSoOps * 64;
};

__device__ __forceinline__ uint32_t so_code8(uint32_t sp, uint32_t b) {
    return (b == ((sp >> 8) & 255u) ? 8u : 0u) | (b == ((sp >> 16) & 255u) ? 16u : 0u) |
           (b == (sp >> 24) ? 24u : 0u);
}

template <int R>
__global__ __launch_bounds__(64) void traceback_so_kernel(TbParams P) {
    using L = SoLds<R>;
    constexpr int RT = L::RT;
    constexpr int BAND = kWave * R;
    __shared__ __attribute__((aligned(16))) uint8_t s_so[L::kBytes];
    typedef volatile uint8_t __attribute__((address_space(3))) lds_u8;
    typedef volatile uint32_t __attribute__((address_space(3))) lds_u32;
    typedef volatile uint16_t __attribute__((address_space(3))) lds_u16;
    lds_u8* const vb = (lds_u8*)s_so;
    lds_u32* const vw = (lds_u32*)s_so;
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
    typedef uint8_t __attribute__((address_space(1))) glb_u8;
    glb_u8* ops = (glb_u8*)(P.ops + o1 + o2 + pidx);
    const uint8_t* const dir = P.dirs + (uint64_t)slot * P.dir_slot;
    const uint64_t band_stride = P.band_stride;
    const uint32_t npk = (uint32_t)(band_stride / (kWave * 16));   // edge packets per band
    const uint32_t* const sh_base = P.snap_h + (uint64_t)slot * P.snap_h_slot;
    const int32_t* const sp_base = P.snap_p + (uint64_t)slot * P.snap_p_slot;
    const uint32_t snap_nch = P.snap_nch;
    // the batch alphabet (T16: <= 4 symbols): tagged profile words 4s + 3 by row code, the symbols,
    // and match(code a, code b) as a 16-bit table (the user's match function, or equality)
    const uint32_t symp = P.prof[4];
    const uint32_t pf0 = P.prof[0], pf1 = P.prof[1], pf2 = P.prof[2], pf3 = P.prof[3];
    uint32_t mt = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t sa_ = (symp >> (8 * a)) & 255u, sb_ = (symp >> (8 * b)) & 255u;
            const bool v = P.lutbits ? ((P.lutbits[(sa_ << 3) | (sb_ >> 5)] >> (sb_ & 31u)) & 1u) != 0 : sa_ == sb_;
            mt |= (v ? 1u : 0u) << (a * 4 + b);
        }
    const bool allow = P.allow != 0;
    const int G = P.gap, MA = P.match, MI = P.mismatch;
    const uint32_t CU = (uint32_t)(-(4 * G + 2)) & 0xffffu;   // up: max(4U + 2, 0) by saturation
    const uint32_t CL = (uint32_t)(4 * G + 1) & 0xffffu;      // left: 4L + 1

    uint32_t k = 0, k0 = 0;   // ops emitted / already written to HBM
    auto emit = [&](uint8_t op) __attribute__((always_inline)) {
        const uint32_t q = k - k0;
        vb[L::kOps + (q >> 2) * 256 + lane * 4 + (q & 3)] = op;
        ++k;
    };
    auto flush = [&]() __attribute__((always_inline)) {
        for (uint32_t q = 0; q < k - k0; ++q) ops[k0 + q] = vb[L::kOps + (q >> 2) * 256 + lane * 4 + (q & 3)];
        k0 = k;
    };

    // ------------------------------------------------------------------ blocks
    int wb = -1, wt = 0, wc = 0;     // current block (band, lane, chunk)
    int cb = 0, ct = 0, cc = 0, cr = 0, cq = 0;   // cell located by locate(): block, row, column
    auto locate = [&](int i, int j) __attribute__((always_inline)) {
        const int ii = i - 1;
        cb = ii / BAND;
        const int rem = ii - cb * BAND;
        ct = rem / R;
        cr = rem - ct * R;
        const int s = j - 1 + ct;
        cc = s >> 5;
        cq = s & 31;
    };
    auto ready = [&](int i, int j) __attribute__((always_inline)) -> bool {
        if (k - k0 >= (uint32_t)kSoOps) return false;
        if (!(i > 0 && j > 0)) return true;
        locate(i, j);
        return cb == wb && ct == wt && cc == wc;
    };
    // recompute the tags of the block holding (i, j), columns up to j
    auto recompute = [&](int i, int j) __attribute__((always_inline)) {
        if (!(i > 0 && j > 0)) return;
        locate(i, j);
        wb = cb; wt = ct; wc = cc;
        const int r0 = cb * BAND + ct * R;
        const int j0 = 32 * cc - ct;
        // the top row: edge stream of lane tp of band bp, steps j + tp for j in [j0, j0 + 32)
        const bool has_top = !(cb == 0 && ct == 0);
        const int bp = ct > 0 ? cb : cb - 1, tp = ct > 0 ? ct - 1 : kWave - 1;
        const int slo = j0 + tp;                 // 32c - 1 (t > 0) or 32c + 63 (t = 0): step of column j0
        const int pk0 = slo >> 3;                // (arithmetic: -1 for slo = -1) first packet of the row
        if (has_top) {
            const uint8_t* base = dir + (uint64_t)bp * band_stride;
#pragma unroll
            for (int d = 0; d < 5; ++d) {        // steps slo .. slo + 31 lie in 5 packets of 8
                const int pk = pk0 + d;
                if (pk >= 0 && (uint32_t)pk < npk)
                    __builtin_amdgcn_global_load_lds((so_gptr)(base + ((uint64_t)pk * kWave + tp) * 16),
                                                     (so_lptr)(s_so + L::kEdge + d * 1024), 16, 0, 0);
            }
        }
        // left column (lane t entering chunk c) and corner: the snapshot of chunk c - 1, or the
        // matrix border (0) when the block starts at column 0 or before
        int Hp[R];
        int corner = 0;
        const bool has_left = cc > 0 && j0 >= 1;
        if (has_left) {
            const uint64_t e = (uint64_t)cb * snap_nch + (cc - 1);
            const uint32_t* sh = sh_base + e * (R / 2) * kWave + ct;
#pragma unroll
            for (int q = 0; q < R / 2; ++q) {
                const uint32_t w = sh[q * kWave];
                Hp[2 * q] = (int)(w & 0xffffu) << 2;
                Hp[2 * q + 1] = (int)(w >> 16) << 2;
            }
            if (r0 > 0) corner = (sp_base[e * kWave + ct] & 0xffff) << 2;
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) Hp[r] = 0;
        }
        // row profiles and codes
        uint32_t tab[R];
#pragma unroll
        for (int r = 0; r < R; r += 4) {
            uint32_t cw = 0;
#pragma unroll
            for (int e = 0; e < 4 && r + e < R; ++e) {
                const int row = r0 + r + e;
                const uint32_t c8 = row < m ? so_code8(symp, s1[row]) : 0u;
                tab[r + e] = c8 == 0 ? pf0 : c8 == 8 ? pf1 : c8 == 16 ? pf2 : pf3;
                cw |= c8 << (8 * e);
            }
            vw[(L::kRowCodes >> 2) + (r >> 2) * 64 + lane] = cw;
        }
        const int qlo = j0 < 0 ? -j0 : 0;
        const int qhi = j - 1 - j0;              // the entry column
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            uint32_t cw = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int q = 4 * w + e, jj = j0 + q;
                cw |= (q >= qlo && q <= qhi && jj < n ? so_code8(symp, s2[jj]) : 0u) << (8 * e);
            }
            vw[(L::kColCodes >> 2) + w * 64 + lane] = cw;
        }
        // the edge DMA writes LDS behind the compiler's back: wait for it, keep reads after this
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        auto top_of = [&](int q) -> int {       // 4 * H(r0 - 1, j0 + q)
            if (!has_top) return 0;
            const int s = slo + q;               // >= 0 here (q >= qlo)
            const int d = (s >> 3) - pk0;
            return (int)((lds_u16*)(s_so + L::kEdge + d * 1024 + lane * 16 + (s & 7) * 2))[0] << 2;
        };
        auto sym_of = [&](int q) -> uint32_t {
            return (vw[(L::kColCodes >> 2) + (q >> 2) * 64 + lane] >> (8 * (q & 3))) & 255u;
        };
        // tags of rows r (16 per word, row r at bits 2 (r % 16): alignbit fills from the top)
        auto put = [&](int q, int r, uint32_t& rec) __attribute__((always_inline)) {
            if ((r & 15) == 15 || r == R - 1) {
                const uint32_t wv = (r & 15) == 15 ? rec : rec >> (32 - 2 * ((r & 15) + 1));
                vw[(q * RT + (r >> 4)) * 64 + lane] = wv;
                rec = 0;
            }
        };
#define SO_CELL(P, HP, HU, DR, REC, TAB, SYM)                                                      \
    "v_add_u16 %[" #P "0], %[cl], %[" HP "]\n\t"                                                  \
    "v_bfe_i32 %[" #P "dn], %[" TAB "], %[" SYM "], 8\n\t"                                         \
    "v_add_u16 %[" #P "dn], %[" HP "], %[" #P "dn]\n\t"                                            \
    "v_sub_u16_e64 %[" #P "1], %[" HU "], %[cu] clamp\n\t"                                         \
    "v_max_i16 %[" #P "0], %[" DR "], %[" #P "0]\n\t"                                              \
    "v_max_i16 %[" #P "0], %[" #P "1], %[" #P "0]\n\t"                                             \
    "v_and_b32 %[" HP "], -4, %[" #P "0]\n\t"                                                      \
    "v_alignbit_b32 %[" REC "], %[" #P "0], %[" REC "], 2\n\t"
        // the two cells of a column pair's sub-step, instruction by instruction (A reads hb --
        // Hp[r-1] -- as its up term before B's v_and_b32 overwrites it)
#define SO_CELL2                                                                                   \
    "v_add_u16 %[a0], %[cl], %[ha]\n\t"                                                            \
    "v_add_u16 %[b0], %[cl], %[hb]\n\t"                                                            \
    "v_bfe_i32 %[adn], %[taba], %[syma], 8\n\t"                                                    \
    "v_bfe_i32 %[bdn], %[tabb], %[symb], 8\n\t"                                                    \
    "v_add_u16 %[adn], %[ha], %[adn]\n\t"                                                          \
    "v_add_u16 %[bdn], %[hb], %[bdn]\n\t"                                                          \
    "v_sub_u16_e64 %[a1], %[hb], %[cu] clamp\n\t"                                                  \
    "v_sub_u16_e64 %[b1], %[hub], %[cu] clamp\n\t"                                                 \
    "v_max_i16 %[a0], %[da], %[a0]\n\t"                                                            \
    "v_max_i16 %[b0], %[db], %[b0]\n\t"                                                            \
    "v_max_i16 %[a0], %[a1], %[a0]\n\t"                                                            \
    "v_max_i16 %[b0], %[b1], %[b0]\n\t"                                                            \
    "v_and_b32 %[ha], -4, %[a0]\n\t"                                                               \
    "v_and_b32 %[hb], -4, %[b0]\n\t"                                                               \
    "v_alignbit_b32 %[reca], %[a0], %[reca], 2\n\t"                                                \
    "v_alignbit_b32 %[recb], %[b0], %[recb], 2"
        // one column: rows 0 .. R-1 in order (the up term of row r is row r-1 of this column)
        auto column = [&](int q, int top, int ptop) __attribute__((always_inline)) {
            const uint32_t sym = sym_of(q);
            uint32_t dcur;
            asm("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(dcur) : "v"(tab[0]), "v"(sym), "v"(ptop));
            uint32_t hu = (uint32_t)top, rec = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                uint32_t a0, a1, adn;
                asm(SO_CELL(a, "hp", "hu", "dr", "rec", "tabn", "sym")
                    : [a0] "=&v"(a0), [a1] "=&v"(a1), [adn] "=&v"(adn), [hp] "+v"(Hp[r]), [rec] "+v"(rec)
                    : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL),
                      [tabn] "v"(tab[r + 1 < R ? r + 1 : r]), [sym] "v"(sym));
                dcur = adn;
                hu = (uint32_t)Hp[r];
                put(q, r, rec);
            }
        };
        // two columns q (A) and q + 1 (B) as two interleaved dependence chains, B one row behind:
        // at sub-step r, A computes row r and B row r - 1.  B's left and diagonal inputs are A's
        // values of the previous sub-steps (Hp[r - 1] holds H(r - 1, q) until B overwrites it), so
        // a lone wave issues the two chains back to back instead of stalling on each.
        auto column_pair = [&](int q, int topA, int topB, int ptop) __attribute__((always_inline)) {
            const uint32_t symA = sym_of(q), symB = sym_of(q + 1);
            uint32_t da, db;
            asm("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(da) : "v"(tab[0]), "v"(symA), "v"(ptop));
            asm("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(db) : "v"(tab[0]), "v"(symB), "v"(topA));
            uint32_t recA = 0, recB = 0;
            {   // sub-step 0: A row 0
                uint32_t a0, a1, adn;
                asm(SO_CELL(a, "hp", "hu", "dr", "rec", "tabn", "sym")
                    : [a0] "=&v"(a0), [a1] "=&v"(a1), [adn] "=&v"(adn), [hp] "+v"(Hp[0]), [rec] "+v"(recA)
                    : [dr] "v"(da), [hu] "v"((uint32_t)topA), [cu] "s"(CU), [cl] "s"(CL),
                      [tabn] "v"(tab[R > 1 ? 1 : 0]), [sym] "v"(symA));
                da = adn;
                put(q, 0, recA);
            }
#pragma unroll
            for (int r = 1; r < R; ++r) {
                // A: row r (left Hp[r], up Hp[r-1] before B writes it); B: row r-1 (left Hp[r-1],
                // up = B's row r-2, or its top)
                const uint32_t hub = r >= 2 ? (uint32_t)Hp[r - 2] : (uint32_t)topB;
                uint32_t a0, a1, adn, b0, b1, bdn;
                asm(SO_CELL2
                    : [a0] "=&v"(a0), [a1] "=&v"(a1), [adn] "=&v"(adn), [b0] "=&v"(b0), [b1] "=&v"(b1),
                      [bdn] "=&v"(bdn), [ha] "+v"(Hp[r]), [hb] "+v"(Hp[r - 1]), [reca] "+v"(recA), [recb] "+v"(recB)
                    : [da] "v"(da), [db] "v"(db), [hub] "v"(hub), [cu] "s"(CU), [cl] "s"(CL),
                      [taba] "v"(tab[r + 1 < R ? r + 1 : r]), [syma] "v"(symA), [tabb] "v"(tab[r]), [symb] "v"(symB));
                da = adn;
                db = bdn;
                put(q, r, recA);
                put(q + 1, r - 1, recB);
            }
            {   // sub-step R: B row R-1
                const uint32_t hub = R >= 2 ? (uint32_t)Hp[R - 2] : (uint32_t)topB;
                uint32_t b0, b1, bdn;
                asm(SO_CELL(b, "hp", "hu", "dr", "rec", "tabn", "sym")
                    : [b0] "=&v"(b0), [b1] "=&v"(b1), [bdn] "=&v"(bdn), [hp] "+v"(Hp[R - 1]), [rec] "+v"(recB)
                    : [dr] "v"(db), [hu] "v"(hub), [cu] "s"(CU), [cl] "s"(CL), [tabn] "v"(tab[R - 1]), [sym] "v"(symB));
                put(q + 1, R - 1, recB);
            }
        };
#undef SO_CELL
#undef SO_CELL2
        int ptop = corner;                       // 4 * H(r0 - 1, j0 + q - 1)
        int q = qlo;
        for (; q + 1 <= qhi; q += 2) {
            const int ta = top_of(q), tb = top_of(q + 1);
            column_pair(q, ta, tb, ptop);
            ptop = tb;
        }
        if (q == qhi) column(q, top_of(q), ptop);
    };
    auto tag = [&]() __attribute__((always_inline)) -> uint32_t {
        return (vw[(cq * RT + (cr >> 4)) * 64 + lane] >> (2 * (cr & 15))) & 3u;
    };
    auto cell_match = [&]() __attribute__((always_inline)) -> bool {
        const uint32_t a = (vb[L::kRowCodes + (cr >> 2) * 256 + lane * 4 + (cr & 3)] >> 3) & 3u;
        const uint32_t b = (vb[L::kColCodes + (cq >> 2) * 256 + lane * 4 + (cq & 3)] >> 3) & 3u;
        return ((mt >> (a * 4 + b)) & 1u) != 0;
    };

    // ------------------------------------------------------------------ walk (as sa_traceback.hip)
    int i = res.end_i, j = res.end_j, V = res.score;
    if (m == 0 || n == 0) { i = 0; j = 0; }
    bool fin = false, parked = true;
    for (;;) {
        if (__builtin_amdgcn_ballot_w64(!fin && !parked) == 0) {
            if (__builtin_amdgcn_ballot_w64(!fin) == 0) break;
            if (!fin) { flush(); recompute(i, j); parked = false; }
        }
        if (!fin && !parked) {
            if (!(i > 0 && j > 0) || V == 0) {   // SASmithWaterman.h: stop on an edge or at H == 0
                fin = true;
            } else if (!ready(i, j)) {
                parked = true;
            } else {
                const uint32_t f = tag();
                const bool dg = f == 3u, up = f == 2u;
                const bool v = dg && cell_match();
                emit(dg ? (v ? 'M' : (allow ? 'S' : 'X')) : (up ? 'U' : 'L'));
                V -= dg ? (v ? MA : MI) : G;
                i -= (dg || up) ? 1 : 0;
                j -= up ? 0 : 1;
            }
        }
    }
    flush();
    res.start_i = i;
    res.start_j = j;
    res.nops = k;
    P.res[pidx] = res;
}

// ------------------------------------------------------------------------------------------------
// Four lanes per pair (a quad, 16 pairs per wave).  The walk is the same, executed identically by
// the quad's four lanes (sublane 0 writes the ops); a block's recompute is split by rows: sublane k
// owns rows k*R/4 .. (k+1)*R/4 - 1 of the block and the quad sweeps the block's columns as a
// four-lane anti-diagonal wavefront (sublane k at column q at sub-step q - qlo + k, its row above
// from sublane k-1's previous sub-step by DPP quad_perm) -- the fill's own schedule on four lanes.
// A lone wave's serial recompute per block drops from 32 columns x R rows of dependent cells to
// (32 + 3) sub-steps x R/4 rows, and the wave's registers (R/4 rows of state) stay few, so the
// traceback beside the next call's fill displaces fewer of its waves.
// Lanes per pair: 4 (16 pairs per wave) for pipelined calls, whose traceback runs beside the next
// call's fill: half the waves of 8 lanes per pair, pipelined headline step 18.4 -> 17.9 ms (round 5,
// profiles/tb_lp_ab_r05.txt); 8 for a call nothing else overlaps, where the traceback alone sets the
// time (4.53 vs 4.74 ms on the headline batch, tools/so4_stats.py).  Round 4 ran 8 at R = 32
// (profiles/tb_lp_ab_r04.txt).  TbParams::so_lp chooses (run_device); $SEQALIB_TB_LP overrides.
constexpr int kSo4DefaultLp = 4;
#ifdef SA_TB_STATS
// Debug build only (-DSA_TB_STATS, tools/so4_stats.py), per wave summed: [rounds, walk-loop
// iterations, moves, wave cycles, recompute: load-wait cycles, sub-step cycles, sub-steps, waves]
__device__ unsigned long long g_so4_stats[8];
extern "C" int sa_debug_so4_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_so4_stats), sizeof(g_so4_stats)) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_so4_stats), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif
// LP lanes per pair (a "quad" of LP sublanes; LP = 8 halves the sub-steps' rows per lane and the
// pairs per wave -- twice the waves for the same batch).
template <int R, int LP>
struct So4Lds {
    static constexpr int kPairs = kWave / LP;                 // pairs per wave
    // [quad][column q][row r] bytes (1 KiB per quad, the cell's tag in bits 0-1); 64 B of pad in
    // front: the walk reads the three cells up-left of its cell, also from a block's first row
    // quads are 1 KiB + 32 B apart so the quads' tag stores land on different banks (at 1 KiB the
    // same column's stores of every quad of the wave hit the same 8 banks)
    static constexpr int kTags = 64;
    static constexpr int kQuad = 1024 + 32;
    static constexpr int kEdge = kTags + kPairs * kQuad;       // [lane] 16 B: packet (sub) of the quad
    static constexpr int kEdge2 = kEdge + 64 * 16;            // LP = 4: [lane] 16 B: packet 4 (sublane 0)
    static constexpr int kRowC = kEdge2 + (LP < 5 ? 64 * 16 : 0);   // [quad][32] row codes (8 x code)
    static constexpr int kColC = kRowC + kPairs * 32;         // [quad][32] column codes
    static constexpr int kBytes = kColC + kPairs * 32;
};

// ALG: SA_SW (SASmithWaterman.h:220-339, from the end cell, stops at H == 0) or SA_NW
// (SANeedlemanWunsch.h:155-231: from (m, n) to (0, 0); the recompute's borders are the NW borders
// i * Gap / j * Gap, the fill's values H - t16_delta, and the cell has no zero clamp).
template <int ALG, int R, int LP>
__global__ __launch_bounds__(64) void traceback_so4_kernel(TbParams P) {
    constexpr bool NWK = ALG == SA_NW;
    using L = So4Lds<R, LP>;
    constexpr int RS = R / LP;   // rows per sublane
    constexpr int BAND = kWave * R;
    static_assert((LP == 4 || LP == 8) && R >= LP && R % LP == 0 && RS <= 16, "LP sublanes of <= 16 rows");
    __shared__ __attribute__((aligned(16))) uint8_t s_so[L::kBytes];
    typedef volatile uint8_t __attribute__((address_space(3))) lds_u8;
    typedef volatile uint32_t __attribute__((address_space(3))) lds_u32;
    typedef volatile uint16_t __attribute__((address_space(3))) lds_u16;
    typedef volatile uint64_t __attribute__((address_space(3))) lds_u64;
    lds_u8* const vb = (lds_u8*)s_so;
    lds_u32* const vw = (lds_u32*)s_so;
    const int lane = threadIdx.x, quad = lane / LP, sub = lane % LP;
    const uint32_t slot = blockIdx.x * L::kPairs + quad;
    // a quad whose pair is not walked here leaves as a whole (the four lanes agree)
    bool live = slot < P.count;
    const uint32_t pidx = P.pair_base + (live ? slot : 0);
    sa_result res = P.res[pidx];
    if (live && !(res.flags & SA_FLAG_BAD_SHAPE) && !tb_mine(P, res.flags)) {
        if (sub == 0) tb_release(P, &P.res[pidx], res.flags);
        live = false;
    }
    live = live && !(res.flags & SA_FLAG_BAD_SHAPE);
    if (__builtin_amdgcn_ballot_w64(live) == 0) return;
    res.flags &= tb_clear_mask(P);
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    typedef uint8_t __attribute__((address_space(1))) glb_u8;
    glb_u8* ops = (glb_u8*)(P.ops + o1 + o2 + pidx);
    const uint8_t* const dir = P.dirs + (uint64_t)(live ? slot : 0) * P.dir_slot;
    const uint64_t band_stride = P.band_stride;
    const uint32_t npk = (uint32_t)(band_stride / (kWave * 16));
    const uint32_t* const sh_base = P.snap_h + (uint64_t)(live ? slot : 0) * P.snap_h_slot;
    const int32_t* const sp_base = P.snap_p + (uint64_t)(live ? slot : 0) * P.snap_p_slot;
    const uint32_t snap_nch = P.snap_nch;
    const uint32_t symp = P.prof[4];
    const uint32_t pf0 = P.prof[0], pf1 = P.prof[1], pf2 = P.prof[2], pf3 = P.prof[3];
    uint32_t mt = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t sa_ = (symp >> (8 * a)) & 255u, sb_ = (symp >> (8 * b)) & 255u;
            const bool v = P.lutbits ? ((P.lutbits[(sa_ << 3) | (sb_ >> 5)] >> (sb_ & 31u)) & 1u) != 0 : sa_ == sb_;
            mt |= (v ? 1u : 0u) << (a * 4 + b);
        }
    const bool allow = P.allow != 0;
    const int G = P.gap, MA = P.match, MI = P.mismatch;
    // up term: SW max(4U + 2, 0) by unsigned saturation, NW 4U + 2 (no clamp)
    const uint32_t CU = (uint32_t)(NWK ? 4 * G + 2 : -(4 * G + 2)) & 0xffffu;
    const uint32_t CL = (uint32_t)(4 * G + 1) & 0xffffu;
    const int D0 = P.t16_delta;
    auto border = [&](int x) __attribute__((always_inline)) -> int {   // NW: 4 (H - delta) of a border cell x * Gap
        return 4 * (x * G - D0);
    };

    uint32_t k = 0;
    auto emit = [&](uint8_t op) __attribute__((always_inline)) {
        if (sub == 0) ops[k] = op;   // (a store in flight costs the walk nothing)
        ++k;
    };
    int cb = 0, ct = 0, cc = 0, cr = 0, cq = 0;
    auto locate = [&](int i, int j) __attribute__((always_inline)) {
        const int ii = i - 1;
        cb = ii / BAND;
        const int rem = ii - cb * BAND;
        ct = rem / R;
        cr = rem - ct * R;
        const int s = j - 1 + ct;
        cc = s >> 5;
        cq = s & 31;
    };
    // the walk's view of the block: the quad's R row codes and 32 column codes (2 bits each) in
    // registers; the move tags stay in LDS ([column q][lane] words, sublane r / RS, bits 2 (r % RS))
    uint64_t rowc = 0, colc = 0;
    auto pack_codes = [&](int base) __attribute__((always_inline)) -> uint64_t {   // 32 bytes of 8 x code
        uint64_t c = 0;
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            uint32_t x = (vw[(base >> 2) + d] >> 3) & 0x03030303u;   // four codes, one per byte
            x = (x | (x >> 6)) & 0x000f000fu;
            x = (x | (x >> 12)) & 0xffu;
            c |= (uint64_t)x << (8 * d);
        }
        return c;
    };
    // recompute the block holding (i, j), columns up to j; every lane of a live quad takes part
    // (a finished or dead quad runs the same sub-step loop on a zero-width column range)
#ifdef SA_TB_STATS
    unsigned long long st_rounds = 0, st_iters = 0, st_wait = 0, st_sub = 0, st_nsub = 0;
    const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();
    unsigned long long st_a = 0;
#endif
    auto recompute = [&](bool act, int i, int j) __attribute__((always_inline)) {
#ifdef SA_TB_STATS
        st_a = __builtin_amdgcn_s_memtime();
#endif
        int r0 = 0, j0 = 0, qlo = 0, qhi = -1, slo = 0, pk0 = 0, bp = 0, tp = 0;
        bool has_top = false, has_left = false;
        if (act) {
            locate(i, j);
            r0 = cb * BAND + ct * R;
            j0 = 32 * cc - ct;
            qlo = j0 < 0 ? -j0 : 0;
            qhi = j - 1 - j0;
            has_top = !(cb == 0 && ct == 0);
            bp = ct > 0 ? cb : cb - 1;
            tp = ct > 0 ? ct - 1 : kWave - 1;
            slo = j0 + tp;
            pk0 = slo >> 3;
            has_left = cc > 0 && j0 >= 1;
            if (has_top) {   // the top row's five packets: sublane k loads packet k (LP = 4: sublane 0 also packet 4)
                const uint8_t* base = dir + (uint64_t)bp * band_stride;
                const int pk = pk0 + sub;
                if (sub < 5 && pk >= 0 && (uint32_t)pk < npk)
                    __builtin_amdgcn_global_load_lds((so_gptr)(base + ((uint64_t)pk * kWave + tp) * 16),
                                                     (so_lptr)(s_so + L::kEdge), 16, 0, 0);
                if constexpr (LP < 5) {
                    const int pk4 = pk0 + 4;
                    if (sub == 0 && pk4 >= 0 && (uint32_t)pk4 < npk)
                        __builtin_amdgcn_global_load_lds((so_gptr)(base + ((uint64_t)pk4 * kWave + tp) * 16),
                                                         (so_lptr)(s_so + L::kEdge2), 16, 0, 0);
                }
            }
        }
        // this sublane's rows: left column, corner (the row above its first row, column j0 - 1)
        int Hp[RS];
        int corner = 0;
        uint32_t tab[RS];
#pragma unroll
        for (int r = 0; r < RS; ++r) { Hp[r] = 0; tab[r] = pf0; }
        if (act) {
            const int rs0 = sub * RS;   // block-relative first row
            // Every load of the block's inputs is issued before any value is used, so a round pays one
            // memory round trip, not one per load (round 5: 9.4K -> ? cycles of load wait per round)
            // (unconditional loads at clamped addresses: a recompute runs only for a cell (i, j) >= (1,
            // 1), so m, n >= 1; without a left column the snapshot words are read from the slot's first)
            uint32_t w[RS], b1[RS], b2[32 / LP];
            const uint64_t e = has_left ? (uint64_t)cb * snap_nch + (cc - 1) : 0;
            const uint32_t* sh = sh_base + e * (R / 2) * kWave + ct;
#pragma unroll
            for (int r = 0; r < RS; ++r) w[r] = sh[((rs0 + r) >> 1) * kWave];
            const uint32_t wc = sh[(rs0 > 0 ? (rs0 - 1) >> 1 : 0) * kWave];
            const int32_t pc = sp_base[e * kWave + ct];
#pragma unroll
            for (int r = 0; r < RS; ++r) b1[r] = s1[min(r0 + rs0 + r, m - 1)];
#pragma unroll
            for (int x = 0; x < 32 / LP; ++x) b2[x] = s2[min(max(j0 + sub * (32 / LP) + x, 0), n - 1)];
            if constexpr (NWK) {
                // NW borders (SANeedlemanWunsch.h:59-62): the left column j0 <= 0 is column 0 (row i
                // holds i * Gap), the corner of a first row r0 = 0 is H(0, j0) = j0 * Gap
                if (!has_left) {
#pragma unroll
                    for (int r = 0; r < RS; ++r) Hp[r] = border(r0 + rs0 + r + 1);
                    corner = border(r0 + rs0);
                } else if (rs0 == 0 && r0 == 0) {
                    corner = border(j0);
                }
            }
            if (has_left) {
#pragma unroll
                for (int r = 0; r < RS; ++r) Hp[r] = (int)(((rs0 + r) & 1) ? (w[r] >> 16) : (w[r] & 0xffffu)) << 2;
                if (rs0 > 0) corner = (int)(((rs0 - 1) & 1) ? (wc >> 16) : (wc & 0xffffu)) << 2;
                else if (r0 > 0) corner = (pc & 0xffff) << 2;
            }
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                const uint32_t c8 = r0 + rs0 + r < m ? so_code8(symp, b1[r]) : 0u;
                tab[r] = c8 == 0 ? pf0 : c8 == 8 ? pf1 : c8 == 16 ? pf2 : pf3;
                vb[L::kRowC + quad * 32 + rs0 + r] = (uint8_t)c8;
            }
#pragma unroll
            for (int x = 0; x < 32 / LP; ++x) {
                const int q = sub * (32 / LP) + x, jj = j0 + q;
                vb[L::kColC + quad * 32 + q] = (uint8_t)(q >= qlo && q <= qhi && jj < n ? so_code8(symp, b2[x]) : 0u);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the edge DMA and the code stores
#ifdef SA_TB_STATS
        {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            st_wait += t - st_a;
            st_a = t;
        }
#endif
        // sub-steps: sublane k at column qlo + u - k; its row above from sublane k-1 (DPP).  The
        // column codes come from the quad's packed 2-bit codes (registers), sublane 0's top-row value
        // of the next sub-step is read one sub-step ahead from an always-valid LDS address, so a
        // sub-step neither branches round an LDS read nor waits for one.
        if (act) colc = pack_codes(L::kColC + quad * 32);   // (in-order LDS: the codes stored above)
        int hl = Hp[RS - 1];
        int prev_up = corner;
        int nmax = qhi - qlo + 1 + (LP - 1);   // sub-steps of this quad; the wave runs the most of any
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) nmax = max(nmax, __shfl_xor(nmax, off));
        auto rd_top = [&](int q) __attribute__((always_inline)) -> int {   // (used by sublane 0 only)
            const int s = slo + q;
            const int d = min(max((s >> 3) - pk0, 0), 4);
            const int off = (LP >= 5 || d < 4) ? L::kEdge + (quad * LP + d) * 16 : L::kEdge2 + quad * 64;
            const int v = (int)((lds_u16*)(s_so + off + (s & 7) * 2))[0] << 2;
            return has_top ? v : NWK ? border(j0 + q + 1) : 0;   // row 0: H(0, j) = j * Gap (NW), 0 (SW)
        };
        int ntop = rd_top(qlo);
        for (int u = 0; u < nmax; ++u) {
            const int q = qlo + u - sub;
            const int top = ntop;
            ntop = rd_top(qlo + u + 1);
            const uint32_t sym = (uint32_t)((colc >> (2 * (q & 31))) & 3u) << 3;
            // the row above from sublane k-1: quad_perm [0,0,1,2] (LP = 4) / row_shr:1 (LP = 8; the
            // sublane 0 lanes, which take lane 7 of the previous group, use the top row instead)
            int up_h = LP == 4 ? __builtin_amdgcn_mov_dpp(hl, 0x90, 0xf, 0xf, false)
                               : __builtin_amdgcn_mov_dpp(hl, 0x111, 0xf, 0xf, false);
            const bool on = act && q >= qlo && q <= qhi;
            if (sub == 0) up_h = top;
            if (on) {
                uint32_t dcur;
                asm("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(dcur) : "v"(tab[0]), "v"(sym), "v"(prev_up));
                uint32_t hu = (uint32_t)up_h;
                uint32_t rec[(RS + 3) / 4];   // row r's tagged value, low byte, at byte r % 4 of word r / 4
#pragma unroll
                for (int w = 0; w < (RS + 3) / 4; ++w) rec[w] = 0;
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    uint32_t a0, a1, adn;
                    // v_perm_b32 selector: byte r % 4 from a0's byte 0, the others kept
                    const uint32_t kSel = (r % 4 == 0) ? 0x03020104u : (r % 4 == 1) ? 0x03020400u
                                            : (r % 4 == 2) ? 0x03040100u : 0x04020100u;
#define SO4_CELL(UP)                                                                               \
    asm("v_add_u16 %[a0], %[cl], %[hp]\n\t"                                                         \
        "v_bfe_i32 %[adn], %[tabn], %[sym], 8\n\t"                                                  \
        "v_add_u16 %[adn], %[hp], %[adn]\n\t" UP                                                   \
        "v_max_i16 %[a0], %[dr], %[a0]\n\t"                                                         \
        "v_max_i16 %[a0], %[a1], %[a0]\n\t"                                                         \
        "v_and_b32 %[hp], -4, %[a0]\n\t"                                                            \
        "v_perm_b32 %[rec], %[a0], %[rec], %[sel]"                                                 \
        : [a0] "=&v"(a0), [a1] "=&v"(a1), [adn] "=&v"(adn), [hp] "+v"(Hp[r]), [rec] "+v"(rec[r / 4]) \
        : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL),                                 \
          [tabn] "v"(tab[r + 1 < RS ? r + 1 : r]), [sym] "v"(sym), [sel] "s"(kSel))
                    if constexpr (NWK) SO4_CELL("v_add_u16 %[a1], %[cu], %[hu]\n\t");
                    else SO4_CELL("v_sub_u16_e64 %[a1], %[hu], %[cu] clamp\n\t");
#undef SO4_CELL
                    dcur = adn;
                    hu = (uint32_t)Hp[r];
                }
                // the sublane's RS rows of column q: contiguous bytes of the quad's column
                const uint32_t tpo = (uint32_t)(L::kTags + quad * L::kQuad + q * 32 + sub * RS);
                if constexpr (RS == 1) vb[tpo] = (uint8_t)rec[0];
                else if constexpr (RS == 2) *(lds_u16*)(s_so + tpo) = (uint16_t)rec[0];
                else if constexpr (RS == 4) *(lds_u32*)(s_so + tpo) = rec[0];
                else if constexpr (RS == 8) *(lds_u64*)(s_so + tpo) = (uint64_t)rec[1] << 32 | rec[0];
                else {
#pragma unroll
                    for (int w = 0; w < RS / 4; ++w) ((lds_u32*)(s_so + tpo))[w] = rec[w];
                }
                prev_up = up_h;
                hl = Hp[RS - 1];
            }
        }
#ifdef SA_TB_STATS
        st_sub += __builtin_amdgcn_s_memtime() - st_a;
        st_nsub += (unsigned long long)nmax;
#endif
        if (act) rowc = pack_codes(L::kRowC + quad * 32);
    };

    int i = res.end_i, j = res.end_j, V = res.score;
    if (!NWK && (m == 0 || n == 0)) { i = 0; j = 0; }
    bool fin = !live, parked = true;
    // the tag of block cell (r, q): byte [quad][q][r] of the tags (bits 0-1)
    const uint32_t tag_base = (uint32_t)(L::kTags + quad * L::kQuad);
    auto tag_at = [&](int r, int q) __attribute__((always_inline)) -> uint32_t {
        return (uint32_t)vb[tag_base + (uint32_t)q * 32u + (uint32_t)r] & 3u;
    };
    // Rounds: recompute the block of every unfinished walk (all lanes: the sub-steps use DPP across
    // the quad), then each quad's sublane 0 walks its block alone, one move per iteration from the
    // tags in LDS.  The three cells a move can reach next (up, left, diagonal) are read while the
    // current move is decided, so an iteration waits for one LDS round trip at most, not for the
    // quad's LP tag words of a whole column.
    const int lead = quad * LP;
    for (;;) {
        // the walk's state lives in sublane 0: the quad's other lanes take it for the recompute
        i = __shfl(i, lead);
        j = __shfl(j, lead);
        fin = __shfl((int)fin, lead) != 0;
        parked = __shfl((int)parked, lead) != 0;
        if (__builtin_amdgcn_ballot_w64(!fin && !parked) == 0) {
            if (__builtin_amdgcn_ballot_w64(!fin) == 0) break;
#ifdef SA_TB_STATS
            ++st_rounds;
#endif
            recompute(!fin && i > 0 && j > 0, i, j);   // (a walk that stops at once needs no block)
            if (!fin) parked = false;
        }
        if (sub != 0 || fin || parked) continue;
        // (cr, cq): the walk's cell in the block (recompute located it); a move that takes either
        // below 0 leaves the block.  One exit test per move, no branch inside (sublane 0 only runs here).
        uint32_t f = tag_at(max(cr, 0), max(cq, 0));
        for (;;) {
#ifdef SA_TB_STATS
            ++st_iters;
#endif
            // SASmithWaterman.h: an edge or H == 0; NW: the walk leaves the interior (border moves below)
            if (!((i > 0) & (j > 0) & (NWK | (V != 0)) & (cr >= 0) & (cq >= 0))) break;
            // the three cells the next move may reach, from one address: diagonal (r - 1, q - 1) at
            // +0, left (r, q - 1) at +1, up (r - 1, q) at +32 (a move out of the block parks; the pad
            // in front of the tags keeps those reads inside the LDS allocation)
            const uint32_t a3 = tag_base + (uint32_t)(cq * 32 + cr) - 33u;
            const uint32_t fd = (uint32_t)vb[a3] & 3u, fl = (uint32_t)vb[a3 + 1] & 3u, fu = (uint32_t)vb[a3 + 32] & 3u;
            const bool dg = f == 3u, up = f == 2u;
            const uint32_t ca = (uint32_t)(rowc >> (2 * cr)) & 3u, cb2 = (uint32_t)(colc >> (2 * cq)) & 3u;
            const bool v = dg & (((mt >> (ca * 4 + cb2)) & 1u) != 0);
            ops[k++] = dg ? (v ? 'M' : (allow ? 'S' : 'X')) : (up ? 'U' : 'L');
            V -= dg ? (v ? MA : MI) : G;
            const int di = (dg | up) ? 1 : 0, dj = up ? 0 : 1;
            i -= di;
            j -= dj;
            cr -= di;
            cq -= dj;
            f = dg ? fd : up ? fu : fl;
        }
        if (!((i > 0) & (j > 0) & (NWK | (V != 0)))) fin = true;
        else parked = true;
    }
#ifdef SA_TB_STATS
    if (lane == __builtin_amdgcn_readfirstlane(lane)) {
        atomicAdd(&g_so4_stats[0], st_rounds);
        atomicAdd(&g_so4_stats[1], st_iters);
        atomicAdd(&g_so4_stats[3], __builtin_amdgcn_s_memtime() - st_t0);
        atomicAdd(&g_so4_stats[4], st_wait);
        atomicAdd(&g_so4_stats[5], st_sub);
        atomicAdd(&g_so4_stats[6], st_nsub);
        atomicAdd(&g_so4_stats[7], 1ull);
    }
    if (live && sub == 0) atomicAdd(&g_so4_stats[2], (unsigned long long)k);
#endif
    if constexpr (NWK) {
        // on the border the reference moves up while i > 0 (H[i][0] == H[i-1][0] + Gap), then left
        // (SANeedlemanWunsch.h:216-229)
        if (live) {
            for (; i > 0; --i) emit('U');
            for (; j > 0; --j) emit('L');
        }
    }
    if (live) {
        if (sub == 0) {
            res.start_i = i;
            res.start_j = j;
            res.nops = k;
            P.res[pidx] = res;
        }
    }
}

// SEQALIB_TB_SO=1: one lane per pair (traceback_so_kernel); default four lanes per pair.
// ------------------------------------------------------------------------------------------------
// Score-only LocalGotoh / GlobalGotoh (sa_fill_impl.h, the SO affine cell): buildResult
// (SALocalGotoh.h:275-470, SAGlobalGotoh.h:235-421) on flags recomputed block by block.  Four lanes
// per pair (16 pairs per wave), sublane k owning rows k R/4 .. of the block, swept as a four-lane
// anti-diagonal wavefront as in traceback_so4_kernel.  The recompute runs the tagged affine cell of
// the T16 fill (8 V + class / extend bits: one v_max_i16 chain per state gives the value and the
// reference's tie order -- diag, then Ix, then Iy; extend before open), from the fill's exact
// unscaled M, B = Iy - (GO + GE) and A = Ix - (GO + GE): the left column and corner from the chunk
// snapshot, the top row (M and A of the lane above) from the 32-bit edge stream.  Per cell it keeps
// the four flags of the int32 records (bit 3 M == diag, bit 2 M == Ix, bit 1 Ix extends, bit 0 Iy
// extends; sa_layout.h t16a_flags) and the walk is sa_traceback.hip's three-state machine.
template <int ALG, int R>
__global__ __launch_bounds__(64) void traceback_soa_kernel(TbParams P) {
    constexpr int LP = 4, RS = R / LP, BAND = kWave * R;
    constexpr bool LG = ALG == SA_LOCAL_GOTOH;
    static_assert(R >= 4 && R <= 16 && R % LP == 0, "R in {4, 8, 16}");
    // LDS: flags [column q][lane] words (RS rows x 4 bits); the top row's <= 9 edge packets in three
    // regions of 64 lanes x 16 B (sublane k loads packets k, k + 4, k + 8); row / column codes
    constexpr int kTags = 0, kEdge = kTags + 32 * 64 * 4, kRowC = kEdge + 3 * 1024, kColC = kRowC + 16 * 32;
    constexpr int kBytes = kColC + 16 * 32;
    __shared__ __attribute__((aligned(16))) uint8_t s_so[kBytes];
    typedef volatile uint8_t __attribute__((address_space(3))) lds_u8;
    typedef volatile uint32_t __attribute__((address_space(3))) lds_u32;
    lds_u8* const vb = (lds_u8*)s_so;
    lds_u32* const vw = (lds_u32*)s_so;
    const int lane = threadIdx.x, quad = lane / LP, sub = lane % LP;
    const uint32_t slot = blockIdx.x * (kWave / LP) + quad;
    bool live = slot < P.count;
    const uint32_t pidx = P.pair_base + (live ? slot : 0);
    sa_result res = P.res[pidx];
    if (live && !(res.flags & SA_FLAG_BAD_SHAPE) && !tb_mine(P, res.flags)) {
        if (sub == 0) tb_release(P, &P.res[pidx], res.flags);
        live = false;
    }
    live = live && !(res.flags & SA_FLAG_BAD_SHAPE);
    if (__builtin_amdgcn_ballot_w64(live) == 0) return;
    res.flags &= tb_clear_mask(P);
    uint32_t flags = res.flags;
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    typedef uint8_t __attribute__((address_space(1))) glb_u8;
    glb_u8* ops = (glb_u8*)(P.ops + o1 + o2 + pidx);
    const uint8_t* const dir = P.dirs + (uint64_t)(live ? slot : 0) * P.dir_slot;
    const uint64_t band_stride = P.band_stride;
    const uint32_t npk = (uint32_t)(band_stride / (kWave * 16));   // edge packets (4 steps each) per band
    const uint32_t* const sh_base = P.snap_h + (uint64_t)(live ? slot : 0) * P.snap_h_slot;
    const int32_t* const sp_base = P.snap_p + (uint64_t)(live ? slot : 0) * P.snap_p_slot;
    const uint32_t snap_nch = P.snap_nch;
    const uint32_t symp = P.prof[4];
    const uint32_t pf0 = P.prof[0], pf1 = P.prof[1], pf2 = P.prof[2], pf3 = P.prof[3];
    uint32_t mt = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t sa_ = (symp >> (8 * a)) & 255u, sb_ = (symp >> (8 * b)) & 255u;
            const bool v = P.lutbits ? ((P.lutbits[(sa_ << 3) | (sb_ >> 5)] >> (sb_ & 31u)) & 1u) != 0 : sa_ == sb_;
            mt |= (v ? 1u : 0u) << (a * 4 + b);
        }
    const bool allow = P.allow != 0;
    const int MA = P.match, MI = P.mismatch, GO = P.gap_open, GE = P.gap_extend, GOE = GO + GE;
    const int D0 = LG ? 0 : P.t16_delta;
    const int SENT = P.t16_sent;   // the tagged Ix / Iy border (below every candidate)
    // the tagged affine cell's constants (sa_fill_impl.h, T16 affine)
    const uint32_t CXO = (uint32_t)(LG ? -(8 * GOE + 4) : 8 * GOE + 4) & 0xffffu;
    const uint32_t CXE = (uint32_t)(8 * GE + 1) & 0xffffu;
    const uint32_t CYO = (uint32_t)(8 * GOE + 2) & 0xffffu;
    // 8 (M - delta) of a border cell with index x (row i of column 0, or column j of row 0)
    auto mb = [&](int x) __attribute__((always_inline)) -> int { return LG ? 0 : 8 * ((x < 1 ? 0 : GO + x * GE) - D0); };

    uint32_t k = 0;
    auto emit = [&](uint8_t op) __attribute__((always_inline)) {
        if (sub == 0) ops[k] = op;
        ++k;
    };
    int cb = 0, ct = 0, cc = 0, cr = 0, cq = 0;
    auto locate = [&](int i, int j) __attribute__((always_inline)) {
        const int ii = i - 1;
        cb = ii / BAND;
        const int rem = ii - cb * BAND;
        ct = rem / R;
        cr = rem - ct * R;
        const int s = j - 1 + ct;
        cc = s >> 5;
        cq = s & 31;
    };
    auto recompute = [&](bool act, int i, int j) __attribute__((always_inline)) {
        int r0 = 0, j0 = 0, qlo = 0, qhi = -1, slo = 0, pk0 = 0, bp = 0, tp = 0;
        bool has_top = false, has_left = false;
        if (act) {
            locate(i, j);
            r0 = cb * BAND + ct * R;
            j0 = 32 * cc - ct;
            qlo = j0 < 0 ? -j0 : 0;
            qhi = j - 1 - j0;
            has_top = !(cb == 0 && ct == 0);
            bp = ct > 0 ? cb : cb - 1;
            tp = ct > 0 ? ct - 1 : kWave - 1;
            slo = j0 + tp;
            pk0 = slo >> 2;   // (arithmetic)
            has_left = cc > 0 && j0 >= 1;
            if (has_top) {
                const uint8_t* base = dir + (uint64_t)bp * band_stride;
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    const int pk = pk0 + sub + 4 * d;
                    if (sub + 4 * d < 9 && pk >= 0 && (uint32_t)pk < npk)
                        __builtin_amdgcn_global_load_lds((so_gptr)(base + ((uint64_t)pk * kWave + tp) * 16),
                                                         (so_lptr)(s_so + kEdge + d * 1024), 16, 0, 0);
                }
            }
        }
        const int rs0 = sub * RS;   // block-relative first row of this sublane
        int Mp[RS], Yp[RS];
        uint32_t tab[RS];
        int corner = 0;
#pragma unroll
        for (int r = 0; r < RS; ++r) { Mp[r] = 0; Yp[r] = SENT; tab[r] = pf0; }
        if (act) {
            if (has_left) {
                const uint64_t e = (uint64_t)cb * snap_nch + (cc - 1);
                const uint32_t* sh = sh_base + e * (R + 1) * kWave + ct;
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    const int rr = rs0 + r;
                    const uint32_t w = sh[(rr >> 1) * kWave], y = sh[(R / 2 + (rr >> 1)) * kWave];
                    const int mv = (int)((rr & 1) ? (w >> 16) : (w & 0xffffu));
                    const int bv = (int)(int16_t)((rr & 1) ? (y >> 16) : (y & 0xffffu));
                    Mp[r] = mv << 3;                  // 8 (M - delta)
                    Yp[r] = ((bv + GOE) << 3) + 2;    // 8 (Iy - delta) + class 1
                }
                if (rs0 > 0) {
                    const uint32_t w = sh[((rs0 - 1) >> 1) * kWave];
                    corner = (int)(((rs0 - 1) & 1) ? (w >> 16) : (w & 0xffffu)) << 3;
                } else if (r0 > 0) {
                    corner = (sp_base[e * kWave + ct] & 0xffff) << 3;
                } else {
                    corner = mb(j0);                  // M(0, j0)
                }
            } else {
#pragma unroll
                for (int r = 0; r < RS; ++r) Mp[r] = mb(r0 + rs0 + r + 1);   // M(i, 0)
                corner = mb(r0 + rs0);
            }
#pragma unroll
            for (int r = 0; r < RS; ++r) {
                const int row = r0 + rs0 + r;
                const uint32_t c8 = row < m ? so_code8(symp, s1[row]) : 0u;
                tab[r] = c8 == 0 ? pf0 : c8 == 8 ? pf1 : c8 == 16 ? pf2 : pf3;
                vb[kRowC + quad * 32 + rs0 + r] = (uint8_t)c8;
            }
#pragma unroll
            for (int e = 0; e < 32 / LP; ++e) {
                const int q = sub * (32 / LP) + e, jj = j0 + q;
                vb[kColC + quad * 32 + q] = (uint8_t)(q >= qlo && q <= qhi && jj < n ? so_code8(symp, s2[jj]) : 0u);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the edge DMA and the code stores
        int hl = Mp[RS - 1], xl = SENT;
        int prev_up = corner;
        int nmax = qhi - qlo + 1 + (LP - 1);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) nmax = max(nmax, __shfl_xor(nmax, off));
        for (int u = 0; u < nmax; ++u) {
            const int q = qlo + u - sub;
            const bool on = act && q >= qlo && q <= qhi;
            // the row above: from sublane k - 1 (quad_perm [0,0,1,2]); sublane 0: the top row
            int up_h = __builtin_amdgcn_mov_dpp(hl, 0x90, 0xf, 0xf, false);
            int up_x = __builtin_amdgcn_mov_dpp(xl, 0x90, 0xf, 0xf, false);
            if (sub == 0) {
                up_h = 0;
                up_x = SENT;
                if (on) {
                    if (!has_top) {
                        up_h = mb(j0 + q + 1);    // M(0, j)
                    } else {
                        const int st = slo + q;
                        const int p = (st >> 2) - pk0;
                        const uint32_t w = vw[(kEdge >> 2) + (p >> 2) * 256 + (quad * LP + (p & 3)) * 4 + (st & 3)];
                        up_h = (int)(w & 0xffffu) << 3;
                        up_x = (((int)(int16_t)(w >> 16) + GOE) << 3) + 4;   // 8 (Ix - delta) + class 2
                    }
                }
            }
            if (on) {
                const uint32_t sym = vb[kColC + quad * 32 + q];
                uint32_t dcur;
                asm("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(dcur) : "v"(tab[0]), "v"(sym), "v"(prev_up));
                uint32_t hu = (uint32_t)up_h, xu = (uint32_t)up_x, rec = 0;
#pragma unroll
                for (int r = 0; r < RS; ++r) {
                    uint32_t t0, t1, xr, yr, dn;
                    const uint32_t tabn = tab[r + 1 < RS ? r + 1 : r];
                    if constexpr (LG) asm("v_sub_u16_e64 %[t0], %[hu], %[cxo] clamp" : [t0] "=v"(t0) : [hu] "v"(hu), [cxo] "s"(CXO));
                    else asm("v_add_u16 %[t0], %[cxo], %[hu]" : [t0] "=v"(t0) : [hu] "v"(hu), [cxo] "s"(CXO));
                    asm("v_add_u16 %[t1], %[cyo], %[hp]\n\t"
                        "v_add_u16 %[xr], %[cxe], %[xu]\n\t"
                        "v_add_u16 %[yr], %[cxe], %[yp]\n\t"
                        "v_max_i16 %[xr], %[t0], %[xr]\n\t"
                        "v_max_i16 %[yr], %[t1], %[yr]\n\t"
                        "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\t"
                        "v_add_u16 %[dn], %[hp], %[dn]\n\t"
                        "v_max_i16 %[t1], %[dr], %[xr]\n\t"
                        "v_max_i16 %[t1], %[yr], %[t1]"
                        : [t1] "=&v"(t1), [xr] "=&v"(xr), [yr] "=&v"(yr), [dn] "=&v"(dn)
                        : [t0] "v"(t0), [hp] "v"(Mp[r]), [xu] "v"(xu), [yp] "v"(Yp[r]), [dr] "v"(dcur),
                          [cxe] "s"(CXE), [cyo] "s"(CYO), [tabn] "v"(tabn), [sym] "v"(sym));
                    const uint32_t cls = (t1 >> 1) & 3u;
                    rec |= ((cls == 3u ? 8u : 0u) | (cls == 2u ? 4u : 0u) | ((xr & 1u) << 1) | (yr & 1u)) << (4 * r);
                    xu = xr & ~1u;            // Ix keeps its class bits (8 Ix + 4)
                    Yp[r] = (int)(yr & ~1u);  // 8 Iy + 2
                    Mp[r] = (int)(t1 & ~7u);  // 8 M
                    hu = (uint32_t)Mp[r];
                    dcur = dn;
                }
                vw[q * 64 + lane] = rec;
                prev_up = up_h;
                hl = Mp[RS - 1];
                xl = (int)xu;
            }
        }
    };
    auto flag_of = [&](int r, int q) __attribute__((always_inline)) -> uint32_t {
        return (vw[q * 64 + quad * LP + r / RS] >> (4 * (r % RS))) & 15u;
    };
    auto match_of = [&](int r, int q) __attribute__((always_inline)) -> bool {
        const uint32_t a = (vb[kRowC + quad * 32 + r] >> 3) & 3u, b = (vb[kColC + quad * 32 + q] >> 3) & 3u;
        return ((mt >> (a * 4 + b)) & 1u) != 0;
    };

    int i, j, V = 0, st = 0;
    if constexpr (LG) { i = res.end_i; j = res.end_j; V = res.score; }
    else { i = m; j = n; }
    bool fin = !live, parked = true;
    for (;;) {
        if (__builtin_amdgcn_ballot_w64(!fin && !parked) == 0) {
            if (__builtin_amdgcn_ballot_w64(!fin) == 0) break;
            recompute(!fin, i, j);   // every lane: the sub-step loop uses DPP across the quad
            if (!fin) parked = false;
        }
        if (fin || parked) continue;
        if (!(i > 0 && j > 0)) { fin = true; continue; }     // LG: an edge ends the walk; GG: the edge tail below
        if (LG && st == 0 && V <= 0) { fin = true; continue; }   // M == max(D, 0) <= 0
        if (cr < 0 || cq < 0) { parked = true; continue; }     // the walk left the block
        const uint32_t f = flag_of(cr, cq);
        if (st == 0) {
            if (f & 8u) {
                const bool v = match_of(cr, cq);
                emit(v ? 'M' : (allow ? 'S' : 'X'));
                V -= v ? MA : MI;
                --i; --j; --cr; --cq;
            } else {
                st = (f & 4u) ? 1 : 2;   // M == Ix, else M == Iy (the same value)
            }
        } else if (st == 1) {
            if constexpr (LG) {
                if (f & 2u) { emit('U'); V -= GE; --i; --cr; }
                else if (V > 0) { emit('U'); V -= GOE; --i; --cr; st = 0; }
                else if (V == 0) { emit('u'); fin = true; }
                else { flags |= SA_FLAG_DIVERGED; fin = true; }
            } else {
                emit('U'); --i; --cr;
                if (!(f & 2u)) st = 0;   // gap open: Ix == M[i-1][j] + GO + GE
            }
        } else {
            if constexpr (LG) {
                if (f & 1u) { emit('L'); V -= GE; --j; --cq; }
                else if (V > 0) { emit('L'); V -= GOE; --j; --cq; st = 0; }
                else if (V == 0) { emit('l'); fin = true; }
                else { flags |= SA_FLAG_DIVERGED; fin = true; }
            } else {
                emit('L'); --j; --cq;
                if (!(f & 1u)) st = 0;
            }
        }
    }
    if constexpr (!LG) {
        // SAGlobalGotoh.h:312-319, :370-377: on the edge j == 0 the walk moves up, on i == 0 left,
        // whatever its state
        if (live) {
            for (; i > 0; --i) emit('U');
            for (; j > 0; --j) emit('L');
        }
    }
    if (live && sub == 0) {
        res.start_i = i;
        res.start_j = j;
        res.nops = k;
        res.flags = flags;
        P.res[pidx] = res;
    }
}

template <int ALG>
hipError_t launch_so4(int R, int lp, dim3 grid, dim3 block, const TbParams& p, hipStream_t stream) {
    if (lp == 8) {
        switch (R) {
            case 8: hipLaunchKernelGGL((traceback_so4_kernel<ALG, 8, 8>), grid, block, 0, stream, p); break;
            case 16: hipLaunchKernelGGL((traceback_so4_kernel<ALG, 16, 8>), grid, block, 0, stream, p); break;
            case 32: hipLaunchKernelGGL((traceback_so4_kernel<ALG, 32, 8>), grid, block, 0, stream, p); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (R) {
        case 4: hipLaunchKernelGGL((traceback_so4_kernel<ALG, 4, 4>), grid, block, 0, stream, p); break;
        case 8: hipLaunchKernelGGL((traceback_so4_kernel<ALG, 8, 4>), grid, block, 0, stream, p); break;
        case 16: hipLaunchKernelGGL((traceback_so4_kernel<ALG, 16, 4>), grid, block, 0, stream, p); break;
        case 32: hipLaunchKernelGGL((traceback_so4_kernel<ALG, 32, 4>), grid, block, 0, stream, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_traceback_so(int algo, int R, const TbParams& p, hipStream_t stream) {
    const dim3 block(64);
    if (algo == SA_LOCAL_GOTOH || algo == SA_GLOBAL_GOTOH) {   // four lanes per pair
        const dim3 grid((p.count + 15) / 16);
#define SA_TB_SOA(RR)                                                                                       \
    case RR:                                                                                                \
        if (algo == SA_LOCAL_GOTOH) hipLaunchKernelGGL((traceback_soa_kernel<SA_LOCAL_GOTOH, RR>), grid, block, 0, stream, p); \
        else hipLaunchKernelGGL((traceback_soa_kernel<SA_GLOBAL_GOTOH, RR>), grid, block, 0, stream, p);     \
        break;
        switch (R) {
            SA_TB_SOA(4)
            SA_TB_SOA(8)
            SA_TB_SOA(16)
            default: return hipErrorInvalidValue;
        }
#undef SA_TB_SOA
        return hipGetLastError();
    }
    if (algo != SA_SW && algo != SA_NW) return hipErrorInvalidValue;
    const char* e = getenv("SEQALIB_TB_SO");
    if (algo == SA_SW && e && e[0] == '1') {   // (the one-lane walker is SW only)
        const dim3 grid((p.count + 63) / 64);
        switch (R) {
            case 4: hipLaunchKernelGGL(traceback_so_kernel<4>, grid, block, 0, stream, p); break;
            case 8: hipLaunchKernelGGL(traceback_so_kernel<8>, grid, block, 0, stream, p); break;
            case 16: hipLaunchKernelGGL(traceback_so_kernel<16>, grid, block, 0, stream, p); break;
            case 32: hipLaunchKernelGGL(traceback_so_kernel<32>, grid, block, 0, stream, p); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    // lanes per pair: $SEQALIB_TB_LP (4 or 8), else kSo4DefaultLp (16 lanes per pair, round 5:
    // 5 % fewer cycles per walk but twice the waves, traceback 6.01 -> 6.29 ms and pipelined step
    // 18.9 -> 20.4 ms)
    int lp = p.so_lp == 8 && R >= 8 ? 8 : kSo4DefaultLp;
    if (const char* l = getenv("SEQALIB_TB_LP")) lp = (atoi(l) == 8 && R >= 8) ? 8 : 4;
    const uint32_t ppw = (uint32_t)(kWave / lp);
    const dim3 grid((p.count + ppw - 1) / ppw);
    return algo == SA_SW ? launch_so4<SA_SW>(R, lp, grid, block, p, stream) : launch_so4<SA_NW>(R, lp, grid, block, p, stream);
}

}  // namespace sa
