// sa_traceback_wave.hip — buildResult of the four reference aligners for FEW pairs: one whole
// wave per pair (sa_traceback.hip walks one pair per lane, which suits big batches).
//
// The walk itself is the reference's loop restated exactly as in sa_traceback.hip (same flags,
// same carried score, same op stream):
//   SW  SASmithWaterman.h:232-334   NW  SANeedlemanWunsch.h:167-230
//   LG  SALocalGotoh.h:285-470      GG  SAGlobalGotoh.h:245-421
// but it is wave-uniform: position, score and state live in scalar registers and every lane
// executes the same move.  A lone wave issues about one instruction per 4 cycles, so the cost of
// a walk is its instruction count:
//   * the flags around the walk are decoded cooperatively into an LDS WINDOW laid out by
//     diagonal: kTwD = 16 diagonals d = j - i around the anchor's, kTwP = 128 rows each, one byte
//     per cell = flag nibble (T16 tags mapped to fD/fU) | match(Seq1[i-1], Seq2[j-1]) << 4.  Four
//     lanes share a diagonal, 32 cells each, all loads issued before one wait;
//   * a diagonal move stays on its window row (p + 1), so the walker keeps 8 cells of its diagonal
//     in two SGPRs, and a RUN of diagonal moves inside them is taken at once with 64-bit scalar
//     bit arithmetic (find-first-zero of the fD bits, popcount of the match bits for the score,
//     the run's op bytes stored by one lane each) whenever the carried score cannot reach 0
//     inside the run; up / left moves and runs near a stop take the literal per-move path;
//   * when the walk leaves the window (128 rows, or 8 diagonals of drift) the wave decodes a new
//     one around the current cell.
// Ops go straight to HBM (fire-and-forget byte stores).
#include <limits.h>

#include "sa_internal.h"

namespace sa {

constexpr int kTwD = 16;                   // window diagonals
constexpr int kTwP = 128;                  // window rows (positions along a diagonal)
constexpr int kTwPPL = kTwP * kTwD / 64;   // positions decoded per lane
constexpr int kTwMid = kTwD / 2 - 1;       // window row of the anchor's diagonal
constexpr int kTwS1 = kTwP;                // Seq1 window bytes
constexpr int kTwS2 = kTwP + kTwD;         // Seq2 window bytes
static_assert(64 % kTwD == 0 && kTwPPL % 4 == 0 && kTwP % 8 == 0, "window geometry");

#ifdef SA_TB_STATS
// Debug build only: [windows, decode ticks, kernel ticks, moves, waves, runs, run moves]
__device__ unsigned long long g_tbw_stats[8];
extern "C" int sa_debug_tbw_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tbw_stats), sizeof(g_tbw_stats)) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tbw_stats), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif

typedef uint8_t __attribute__((address_space(3))) tw_u8;
typedef uint32_t __attribute__((address_space(3))) tw_u32;

// Decode the window anchored at (i0, j0): window row L = diagonal (j0 - i0) - kTwMid + L, cell p
// of a row = row i0 - p.  Lane = (L, quarter): 32 cells of one row.  Out of line: the walk loop
// keeps its few scalars in registers instead of sharing an allocation with this unrolled body.
// Every load is unconditional (addresses clamped into the matrix / sequences, cells outside the
// matrix masked to 0 afterwards), so the wave waits once for all of them.
template <int ALG, int R, bool LUT>
__device__ __attribute__((noinline)) void tw_decode(const uint8_t* dir, const uint8_t* s1, const uint8_t* s2, int m,
                                                    int n, uint32_t max_m, uint32_t max_n, int tagged, bool vrec, int i0,
                                                    int j0, tw_u8* win, tw_u8* sq1, tw_u8* sq2,
                                                    const tw_u32* lut) {
    constexpr int BPC = bits_per_cell(ALG);   // flag bits (records may pad above them: record_bpc)
    constexpr uint32_t FMASK = (1u << BPC) - 1u;
    constexpr int NS1 = (kTwS1 + 63) / 64, NS2 = (kTwS2 + 63) / 64;
    const int lane = threadIdx.x;
    const Geom g = make_geom(ALG, R, max_m, max_n, tagged);
    const int jb = j0 - kTwP - kTwMid;   // smallest j-1 of the window (may be < 0)
    {
        uint8_t a[NS1], b[NS2];
#pragma unroll
        for (int q = 0; q < NS1; ++q) a[q] = s1[min(max(i0 - 1 - (lane + 64 * q), 0), m - 1)];
#pragma unroll
        for (int q = 0; q < NS2; ++q) b[q] = s2[min(max(jb + lane + 64 * q, 0), n - 1)];
#pragma unroll
        for (int q = 0; q < NS1; ++q)
            if (lane + 64 * q < kTwS1) sq1[lane + 64 * q] = a[q];
#pragma unroll
        for (int q = 0; q < NS2; ++q)
            if (lane + 64 * q < kTwS2) sq2[lane + 64 * q] = b[q];
    }
    const int L = lane % kTwD, p0 = (lane / kTwD) * kTwPPL;
    const int d = (j0 - i0) - kTwMid + L;
    uint32_t raw[kTwPPL];
#pragma unroll
    for (int q = 0; q < kTwPPL; ++q) {
        const int p = p0 + q;
        const int i = max(i0 - p, 1), j = min(max(i0 - p + d, 1), n);
        int sh;
        const uint64_t off = cell_byte(g, (uint32_t)i, (uint32_t)j, &sh);
        raw[q] = (uint32_t)dir[off] >> sh;
    }
    uint32_t packed[kTwPPL / 4];
#pragma unroll
    for (int w = 0; w < kTwPPL / 4; ++w) packed[w] = 0;
#pragma unroll
    for (int q = 0; q < kTwPPL; ++q) {
        const int p = p0 + q;
        const int i = i0 - p, j = i + d;
        const uint32_t ok = (uint32_t)(i >= 1) & (uint32_t)(j >= 1) & (uint32_t)(j <= n);
        uint32_t f = raw[q] & FMASK;
        if (BPC == 2 && tagged) f = (f == 3u) ? 2u : (uint32_t)(f == 2u);
        if (BPC == 4 && tagged) f = t16a_flags(raw[q] & 0xffu);   // tagged affine byte
        const int jq = min(max(j - 1 - jb, 0), kTwS2 - 1);
        const uint32_t a = sq1[p], b = sq2[jq];
        uint32_t mt;
        if (vrec) mt = BPC == 2 ? ((f >> 1) & f & 1u) : ((f >> 3) & (f >> 2) & 1u);   // under fD only
        else if constexpr (LUT) mt = (lut[(a << 3) | (b >> 5)] >> (b & 31)) & 1u;
        else mt = (uint32_t)(a == b);
        packed[q / 4] |= ((f | mt << 4) & (0u - ok)) << ((q % 4) * 8);
    }
    tw_u32* row = reinterpret_cast<tw_u32*>(win + L * kTwP + p0);
#pragma unroll
    for (int w = 0; w < kTwPPL / 4; ++w) row[w] = packed[w];
}

template <int ALG, int R, bool LUT>
__global__ __launch_bounds__(64) void traceback_wave_kernel(TbParams P) {
    constexpr bool SCORED = (ALG == SA_SW || ALG == SA_LOCAL_GOTOH);   // the walk carries the score
    constexpr bool AFF = is_affine(ALG);
    constexpr uint32_t FD = AFF ? 8u : 2u;                               // fD bit of a cell byte
    __shared__ __attribute__((aligned(16))) uint8_t s_win[kTwD * kTwP];
    __shared__ __attribute__((aligned(16))) uint8_t s_seq1[kTwS1];
    __shared__ __attribute__((aligned(16))) uint8_t s_seq2[kTwS2];
    __shared__ uint32_t s_lut[LUT ? 2048 : 1];

    const int lane = threadIdx.x;
    const uint32_t slot = blockIdx.x;
    if (slot >= P.count) return;
    const uint32_t pidx = P.pair_base + slot;
    sa_result res = P.res[pidx];
    if (res.flags & SA_FLAG_BAD_SHAPE) return;
    if (!tb_mine(P, res.flags)) {
        if (lane == 0) tb_release(P, &P.res[pidx], res.flags);
        return;
    }
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    int seg_b = 0;
    bool recovered = false;
    if (seg_take<ALG, R>(P, res, m, n, &seg_b)) {
        // walked band-parallel by sa_traceback_seg.hip: apply the band where the walk stopped --
        // unless no band recorded the end or a consistency guard fired there (kSegErr): then this
        // wave walks the pair itself (an exact result, flagged SA_FLAG_RECOVERED), never a
        // fabricated one
        const int4 f = P.seg_fin[slot];   // preset to -1 by the host
        if (f.z >= 0 && !(f.w & 16)) {
            if (lane == 0) {
                res.flags &= tb_clear_mask(P);
                res.start_i = f.x;
                res.start_j = f.y;
                res.nops = (uint32_t)f.z;
                if (f.w & 2) res.flags |= SA_FLAG_DIVERGED;
                P.res[pidx] = res;
            }
            return;
        }
        recovered = true;
    }
    res.flags &= tb_clear_mask(P);
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    const int tagged = P.tagged;   // record layout (sa_layout.h Geom::tagged)
    const uint8_t* dir = P.dirs + (uint64_t)slot * P.dir_slot;
    uint8_t* ops = P.ops + o1 + o2 + pidx;
    const bool allow = P.allow != 0;
    const int G = P.gap, MA = P.match, MI = P.mismatch, GE = P.gap_extend;
    const int GOE = P.gap_open + P.gap_extend;
    if constexpr (LUT) {
        for (int q = lane; q < 2048; q += 64) s_lut[q] = P.lutbits[q];
    }
    // Diagonal runs in bulk: the op byte of a diagonal cell is 'M' (match) or obase; the score
    // check of the local modes is kept exact by taking a run only while the score cannot reach 0.
    const uint32_t obase = allow ? 'S' : 'X';
    constexpr int kBig = 1 << 20;
    const bool bulk = !SCORED || (allow && MA > -kBig && MA < kBig && MI > -kBig && MI < kBig);
    int maxstep = 0;
    if constexpr (SCORED) {
        if (bulk) maxstep = max(max(MA, -MA), max(MI, -MI));
    }

    uint32_t k = 0;     // ops emitted
    uint32_t flags = res.flags;
    // every lane stores the same byte: no exec-mask juggling for a single-lane store
    auto emit = [&](uint32_t op) {
        ops[k] = (uint8_t)op;
        ++k;
    };

    // ---------------------------------------------------------------- walk (uniform)
    int wi = -(1 << 30), wd = 0;     // window anchor: row i0, diagonal j0 - i0
    int cl = -1, cp8 = -1;           // cached 8-cell run: window row and p / 8
    uint32_t c_lo = 0, c_hi = 0;
    int i, j, st = 0;
    int V = 0;
    if constexpr (SCORED) {
        i = res.end_i; j = res.end_j; V = res.score;
        if (ALG == SA_SW && (m == 0 || n == 0)) { i = 0; j = 0; }
    } else {
        i = m; j = n;
    }
    i = __builtin_amdgcn_readfirstlane(i);
    j = __builtin_amdgcn_readfirstlane(j);
    V = __builtin_amdgcn_readfirstlane(V);
#ifdef SA_TB_STATS
    unsigned long long st_win = 0, st_dec = 0, st_runs = 0, st_runm = 0;
    const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();
#endif
    for (;;) {
        uint32_t c = 0;
        const bool inner = i > 0 && j > 0;
        if (inner) {
            int Lw = (j - i) - wd + kTwMid, p = wi - i;
            if ((unsigned)Lw >= (unsigned)kTwD || (unsigned)p >= (unsigned)kTwP) {
#ifdef SA_TB_STATS
                const unsigned long long t = __builtin_amdgcn_s_memtime();
#endif
                tw_decode<ALG, R, LUT>(dir, s1, s2, m, n, P.max_m, P.max_n, tagged, P.vrec != 0, i, j, (tw_u8*)s_win,
                                         (tw_u8*)s_seq1, (tw_u8*)s_seq2, (const tw_u32*)s_lut);
                __syncthreads();
#ifdef SA_TB_STATS
                st_dec += __builtin_amdgcn_s_memtime() - t;
                ++st_win;
#endif
                wi = i;
                wd = j - i;
                Lw = kTwMid;
                p = 0;
                cl = -1;
            }
            if (Lw != cl || (p >> 3) != cp8) {
                const uint2 v = *reinterpret_cast<const uint2*>(s_win + Lw * kTwP + (p & ~7));
                c_lo = __builtin_amdgcn_readfirstlane(v.x);
                c_hi = __builtin_amdgcn_readfirstlane(v.y);
                cl = Lw;
                cp8 = p >> 3;
            }
            c = (((p & 4) ? c_hi : c_lo) >> ((p & 3) * 8)) & 0xffu;
            // ---- a run of diagonal moves inside the cached 8 cells
            if (bulk && (c & FD) && (!AFF || st == 0)) {
                const int q = p & 7;
                const uint64_t C = ((((uint64_t)c_hi) << 32) | c_lo) >> (8 * q);
                uint64_t nd = ~C & (0x0101010101010101ull * FD);   // cells that are not diagonal
                if (q) nd |= (uint64_t)FD << (8 * (8 - q));         // ... or past the cached ones
                int r = nd ? (int)(__builtin_ctzll(nd) >> 3) : 8;
                if (SCORED && V <= (r - 1) * maxstep) r = 1;        // the score could reach 0
                if (r >= 2) {
                    const uint64_t keep = r >= 8 ? ~0ull : ((1ull << (8 * r)) - 1ull);
                    const uint64_t vb = (C >> 4) & 0x0101010101010101ull & keep;
                    if constexpr (SCORED) {
                        const int nm = __builtin_popcountll(vb);
                        V -= nm * MA + (r - nm) * MI;
                    }
                    const uint64_t o64 = 0x0101010101010101ull * obase - (uint64_t)(obase - 'M') * vb;
                    const int l = min(lane, r - 1);
                    ops[k + l] = (uint8_t)(o64 >> (8 * l));
                    k += r;
                    i -= r;
                    j -= r;
#ifdef SA_TB_STATS
                    ++st_runs;
                    st_runm += r;
#endif
                    continue;
                }
            }
        }
        const uint32_t f = c & 15u;
        const bool v = (c >> 4) & 1u;
        if constexpr (ALG == SA_SW || ALG == SA_NW) {
            if (ALG == SA_SW ? (!inner || V == 0) : !(i > 0 || j > 0)) break;
            uint32_t fl = 1u;   // NW edges: j == 0 -> up, i == 0 -> left
            if (inner) fl = f;
            else if (i == 0) fl = 0u;
            const bool dg = (fl & 2u) != 0, up = !dg && (fl & 1u);
            emit(dg ? (v ? 'M' : obase) : (up ? 'U' : 'L'));
            if constexpr (ALG == SA_SW) V -= dg ? (v ? MA : MI) : G;
            i -= (dg || up) ? 1 : 0;
            j -= up ? 0 : 1;
        } else if constexpr (ALG == SA_LOCAL_GOTOH) {
            // flags: bit3 = fD (M == diag), bit2 = fX (M == Ix), bit1 = Ix extends, bit0 = Iy extends
            if (!inner) break;
            if (st == 0) {
                if (V <= 0) break;                     // M == max(D, 0) <= 0
                if (f & 8u) { emit(v ? 'M' : obase); V -= v ? MA : MI; --i; --j; }
                else st = (f & 4u) ? 1 : 2;            // M == Ix, else M == Iy (same value)
            } else if (st == 1) {
                if (f & 2u) { emit('U'); V -= GE; --i; }
                else if (V > 0) { emit('U'); V -= GOE; --i; st = 0; }
                else if (V == 0) { emit('u'); break; }
                else { flags |= SA_FLAG_DIVERGED; break; }
            } else {
                if (f & 1u) { emit('L'); V -= GE; --j; }
                else if (V > 0) { emit('L'); V -= GOE; --j; st = 0; }
                else if (V == 0) { emit('l'); break; }
                else { flags |= SA_FLAG_DIVERGED; break; }
            }
        } else {  // SA_GLOBAL_GOTOH
            if (!(i > 0 || j > 0)) break;
            if (j == 0) { emit('U'); --i; continue; }   // edge rules hold in any state
            if (i == 0) { emit('L'); --j; continue; }
            if (st == 0) {
                if (f & 8u) { emit(v ? 'M' : obase); --i; --j; }
                else st = (f & 4u) ? 1 : 2;
            } else if (st == 1) {
                emit('U'); --i;
                if (!(f & 2u)) st = 0;   // gap open: Ix == M[i-1][j] + GO + GE
            } else {
                emit('L'); --j;
                if (!(f & 1u)) st = 0;
            }
        }
    }
#ifdef SA_TB_STATS
    if (lane == 0) {
        atomicAdd(&g_tbw_stats[0], st_win);
        atomicAdd(&g_tbw_stats[1], st_dec);
        atomicAdd(&g_tbw_stats[2], __builtin_amdgcn_s_memtime() - st_t0);
        atomicAdd(&g_tbw_stats[3], (unsigned long long)k);
        atomicAdd(&g_tbw_stats[4], 1ull);
        atomicAdd(&g_tbw_stats[5], st_runs);
        atomicAdd(&g_tbw_stats[6], st_runm);
    }
#endif
    if (lane == 0) {
        res.start_i = i;
        res.start_j = j;
        res.nops = k;
        res.flags = flags | (recovered ? SA_FLAG_RECOVERED : 0u);
        P.res[pidx] = res;
    }
}

hipError_t launch_traceback_wave(int algo, int R, bool lut, const TbParams& p, hipStream_t stream) {
    const dim3 block(64), grid(p.count);
#define SA_TBW(AA, RR, LL)                                                                    \
    if (algo == AA && R == RR && lut == LL) {                                                 \
        hipLaunchKernelGGL((traceback_wave_kernel<AA, RR, LL>), grid, block, 0, stream, p);   \
        return hipGetLastError();                                                             \
    }
#define SA_TBW_A(AA) SA_TBW(AA, 4, false) SA_TBW(AA, 8, false) SA_TBW(AA, 16, false) \
                     SA_TBW(AA, 4, true) SA_TBW(AA, 8, true) SA_TBW(AA, 16, true)   \
                     SA_TBW(AA, 1, false) SA_TBW(AA, 2, false) SA_TBW(AA, 1, true) SA_TBW(AA, 2, true)
    SA_TBW_A(SA_SW)
    SA_TBW_A(SA_NW)
    SA_TBW(SA_SW, 32, false) SA_TBW(SA_SW, 32, true) SA_TBW(SA_NW, 32, false) SA_TBW(SA_NW, 32, true)
    SA_TBW(SA_SW, 64, false) SA_TBW(SA_SW, 64, true) SA_TBW(SA_NW, 64, false) SA_TBW(SA_NW, 64, true)
    SA_TBW_A(SA_LOCAL_GOTOH)
    SA_TBW_A(SA_GLOBAL_GOTOH)
#undef SA_TBW_A
#undef SA_TBW
    return hipErrorInvalidValue;
}

}  // namespace sa
