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
#include <limits.h>

#include "sa_internal.h"

namespace sa {

template <bool LUT>
__device__ __forceinline__ bool tb_match(const uint32_t* lut, uint8_t a, uint8_t b) {
    if constexpr (LUT) return (lut[(a << 3) | (b >> 5)] >> (b & 31)) & 1;
    else return a == b;
}

template <int ALG, int R, bool LUT>
__global__ __launch_bounds__(64) void traceback_kernel(TbParams P) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= P.count) return;
    const uint32_t pidx = P.pair_base + slot;
    sa_result res = P.res[pidx];
    if (res.flags & SA_FLAG_BAD_SHAPE) return;
    const uint64_t o1 = P.off1[pidx], o2 = P.off2[pidx];
    const int m = (int)(P.off1[pidx + 1] - o1);
    const int n = (int)(P.off2[pidx + 1] - o2);
    const uint8_t* s1 = P.seq1 + o1;
    const uint8_t* s2 = P.seq2 + o2;
    const bool tagged = P.tagged != 0;
    const Geom g = make_geom(ALG, R, P.max_m, P.max_n, tagged);
    const uint8_t* dir = P.dirs + (uint64_t)slot * P.dir_slot;
    uint8_t* ops = P.ops + o1 + o2 + pidx;
    const bool allow = P.allow != 0;
    const int G = P.gap, MA = P.match, MI = P.mismatch, GE = P.gap_extend;
    const int GOE = P.gap_open + P.gap_extend;
    uint32_t k = 0;
    uint32_t flags = res.flags;

    auto cell = [&](int i, int j) -> uint32_t {
        int sh;
        const uint64_t off = cell_byte(g, (uint32_t)i, (uint32_t)j, &sh);
        return (uint32_t)(dir[off] >> sh);
    };
    // linear modes: flags fD (bit 1) / fU (bit 0); a T16 max tag (3 diag, 2 up, 1 left, 0 clamp)
    // says the same thing: diag wins iff H == D, else up iff H == U.
    auto lin = [&](int i, int j) -> uint32_t {
        const uint32_t f = cell(i, j) & 3u;
        return tagged ? (f == 3u ? 2u : (f == 2u ? 1u : 0u)) : f;
    };
    // diagonal move: emits the op and returns the substitution term that was added
    auto diag = [&](int i, int j) -> int {
        const bool v = tb_match<LUT>(P.lutbits, s1[i - 1], s2[j - 1]);
        ops[k++] = v ? 'M' : (allow ? 'S' : 'X');
        return v ? MA : MI;
    };

    int i, j;
    if constexpr (ALG == SA_SW) {
        // flags: bit1 = fD (H == diag term), bit0 = fU (H == up term)
        i = res.end_i; j = res.end_j;
        int H = res.score;
        if (m == 0 || n == 0) { i = 0; j = 0; }
        while (i > 0 && j > 0) {
            if (H == 0) break;        // diag test max(D,0) == H == 0 -> end of the local path
            const uint32_t f = lin(i, j);
            if (f & 2u) { H -= diag(i, j); --i; --j; }
            else if (f & 1u) { ops[k++] = 'U'; H -= G; --i; }
            else { ops[k++] = 'L'; H -= G; --j; }
        }
    } else if constexpr (ALG == SA_NW) {
        i = m; j = n;
        while (i > 0 || j > 0) {
            if (i > 0 && j > 0) {
                const uint32_t f = lin(i, j);
                if (f & 2u) { diag(i, j); --i; --j; }
                else if (f & 1u) { ops[k++] = 'U'; --i; }
                else { ops[k++] = 'L'; --j; }
            } else if (i > 0) {
                ops[k++] = 'U'; --i;   // H[i][0] == H[i-1][0] + Gap always holds
            } else {
                ops[k++] = 'L'; --j;
            }
        }
    } else if constexpr (ALG == SA_LOCAL_GOTOH) {
        // flags: bit3 = fD (M == diag), bit2 = fX (M == Ix), bit1 = Ix extends, bit0 = Iy extends
        i = res.end_i; j = res.end_j;
        int st = 0;
        int V = res.score;            // M, Ix or Iy of the current cell, by state
        while (i > 0 && j > 0) {
            const uint32_t f = cell(i, j);
            if (st == 0) {
                if (V <= 0) break;    // M == max(D, 0) <= 0
                if (f & 8u) { V -= diag(i, j); --i; --j; }
                else st = (f & 4u) ? 1 : 2;   // M == Ix, else M == Iy (same value)
            } else if (st == 1) {
                if (f & 2u) { ops[k++] = 'U'; V -= GE; --i; }
                else if (V > 0) { ops[k++] = 'U'; V -= GOE; --i; st = 0; }
                else if (V == 0) { ops[k++] = 'u'; break; }
                else { flags |= SA_FLAG_DIVERGED; break; }
            } else {
                if (f & 1u) { ops[k++] = 'L'; V -= GE; --j; }
                else if (V > 0) { ops[k++] = 'L'; V -= GOE; --j; st = 0; }
                else if (V == 0) { ops[k++] = 'l'; break; }
                else { flags |= SA_FLAG_DIVERGED; break; }
            }
        }
    } else {  // SA_GLOBAL_GOTOH
        i = m; j = n;
        int st = 0;
        while (i > 0 || j > 0) {
            if (j == 0) { ops[k++] = 'U'; --i; continue; }   // edge rules hold in any state
            if (i == 0) { ops[k++] = 'L'; --j; continue; }
            const uint32_t f = cell(i, j);
            if (st == 0) {
                if (f & 8u) { diag(i, j); --i; --j; }
                else st = (f & 4u) ? 1 : 2;
            } else if (st == 1) {
                ops[k++] = 'U'; --i;
                if (!(f & 2u)) st = 0;   // gap open: Ix == M[i-1][j] + GO + GE
            } else {
                ops[k++] = 'L'; --j;
                if (!(f & 1u)) st = 0;
            }
        }
    }
    res.start_i = i;
    res.start_j = j;
    res.nops = k;
    res.flags = flags;
    P.res[pidx] = res;
}

hipError_t launch_traceback(int algo, int R, bool lut, const TbParams& p, hipStream_t stream) {
    const dim3 block(64);
    const dim3 grid((p.count + 63) / 64);
#define SA_TB(AA, RR, LL)                                                                  \
    if (algo == AA && R == RR && lut == LL) {                                              \
        hipLaunchKernelGGL((traceback_kernel<AA, RR, LL>), grid, block, 0, stream, p);     \
        return hipGetLastError();                                                          \
    }
#define SA_TB_A(AA) SA_TB(AA, 4, false) SA_TB(AA, 8, false) SA_TB(AA, 16, false) \
                    SA_TB(AA, 4, true) SA_TB(AA, 8, true) SA_TB(AA, 16, true)
    SA_TB_A(SA_SW)
    SA_TB_A(SA_NW)
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
