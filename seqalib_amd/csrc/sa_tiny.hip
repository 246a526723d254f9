// sa_tiny.hip — the small-call path: one kernel per host call for a few short pairs (the
// reference's canonical use, one getAlignment() per pair: include/Test.cpp:98-144,
// test/Test.cpp:44-45).  A getAlignment on 11 x 8 cells through the batch path costs a fill and a
// traceback launch plus two copies (round 4: ~105 us per call, 70 of them host-side); here one
// single-wave workgroup per pair reads its inputs straight from the caller's pinned staging
// (host memory mapped into the GPU's address space), fills the int32 matrices in registers along
// the anti-diagonal wavefront, keeps every cell's traceback flags in LDS, walks the traceback in
// the same workgroup and writes the result and op stream back to pinned host memory.
//
// Recurrences and walks are the int32 kernels' (sa_fill_impl.h, sa_traceback.hip), i.e. the
// reference's, restated:
//   SW  SASmithWaterman.h:89-131 (fill, last row-major maximum :110), :220-339 (traceback)
//   NW  SANeedlemanWunsch.h:40-153, :155-231
//   LG  SALocalGotoh.h:56-272 (Ix / Iy borders -10000), :275-470
//   GG  SAGlobalGotoh.h:53-232, :235-421
// !AllowMismatch: a mismatched diagonal term is INT_MIN and never added to.
#include <limits.h>

#include "sa_internal.h"

namespace sa {

// one lane owns R consecutive rows; lane t computes column s - t at step s (as the fill)
template <int ALG, int R, bool LUT>
__global__ __launch_bounds__(64) void tiny_kernel(TinyParams P) {
    constexpr bool AFF = ALG >= SA_LOCAL_GOTOH;
    constexpr bool LOCAL = ALG == SA_SW || ALG == SA_LOCAL_GOTOH;
    constexpr int kNeg = -10000;   // the reference's Ix / Iy border (SALocalGotoh.h:77-90)
    __shared__ uint8_t s_flag[kTinyCells];     // cell (i, j), 1-based: (i - 1) * n + j - 1
    __shared__ uint8_t s_a[kTinyM], s_b[kTinyN];
    __shared__ uint32_t s_lut[LUT ? 2048 : 1];
    __shared__ uint8_t s_ops[kTinyM + kTinyN + 1];
    __shared__ int s_score;
    const int lane = threadIdx.x;
    const uint32_t p = blockIdx.x;
    const uint64_t o1 = P.off1[p], o2 = P.off2[p];
    const int m = (int)(P.off1[p + 1] - o1), n = (int)(P.off2[p + 1] - o2);
    for (int k = lane; k < m; k += kWave) s_a[k] = P.seq1[o1 + k];
    for (int k = lane; k < n; k += kWave) s_b[k] = P.seq2[o2 + k];
    if constexpr (LUT) {
        for (int k = lane; k < 2048; k += kWave) s_lut[k] = P.lutbits[k];
    }
    __syncthreads();
    auto match = [&](uint32_t x, uint32_t y) __attribute__((always_inline)) -> bool {
        if constexpr (LUT) return ((s_lut[(x << 3) | (y >> 5)] >> (y & 31u)) & 1u) != 0;
        else return x == y;
    };
    const int G = P.gap, MA = P.match, MI = P.mismatch, GO = P.gap_open, GE = P.gap_extend;
    const int GOE = GO + GE;
    const bool allow = P.allow != 0;
    // M / H of a border cell: row i of column 0 or column j of row 0
    auto border = [&](int x) __attribute__((always_inline)) -> int {
        if constexpr (ALG == SA_NW) return x * G;
        else if constexpr (ALG == SA_GLOBAL_GOTOH) return x < 1 ? 0 : GO + x * GE;
        else return 0;
    };

    int best_h = INT_MIN, best_i = 0, best_j = 0;   // local modes: the last row-major maximum
    if (m > 0 && n > 0) {
        const int row0 = lane * R;
        int a[R], Hp[R], Yp[R], bh[R], bj[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            a[r] = row0 + r < m ? s_a[row0 + r] : 0;
            Hp[r] = border(row0 + r + 1);
            Yp[r] = kNeg;
            bh[r] = INT_MIN;
            bj[r] = 0;
        }
        int prev_up = border(row0), hl = Hp[R - 1], xl = kNeg;
        const int lanes = (m + R - 1) / R;
        for (int s = 0; s < n + lanes - 1; ++s) {
            int up_h = __shfl_up(hl, 1), up_x = __shfl_up(xl, 1);
            const int j = s - lane;
            if (lane == 0) {
                up_h = border(j + 1);
                up_x = kNeg;
            }
            if (j >= 0 && j < n && row0 < m) {
                const uint32_t sym = s_b[j];
                int hd = prev_up, hu = up_h, xu = up_x;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (row0 + r < m) {
                        const bool v = match((uint32_t)a[r], sym);
                        const int D = allow ? hd + (v ? MA : MI) : (v ? hd + MA : INT_MIN);
                        int Hn;
                        uint32_t f;
                        if constexpr (!AFF) {
                            const int U = hu + G, L = Hp[r] + G;
                            Hn = max(max(D, U), L);
                            if constexpr (LOCAL) Hn = max(Hn, 0);
                            f = (Hn == D ? 2u : 0u) | (Hn == U ? 1u : 0u);
                        } else {
                            const int XE = xu + GE, X = max(hu + GOE, XE);
                            const int YE = Yp[r] + GE, Y = max(Hp[r] + GOE, YE);
                            Hn = max(max(D, X), Y);
                            if constexpr (LOCAL) Hn = max(Hn, 0);
                            f = (Hn == D ? 8u : 0u) | (Hn == X ? 4u : 0u) | (X == XE ? 2u : 0u) | (Y == YE ? 1u : 0u);
                            Yp[r] = Y;
                            xu = X;
                        }
                        s_flag[(row0 + r) * n + j] = (uint8_t)f;
                        hd = Hp[r];
                        Hp[r] = Hn;
                        hu = Hn;
                        if constexpr (LOCAL) {
                            if (Hn >= bh[r]) { bh[r] = Hn; bj[r] = j; }
                        }
                    }
                }
                prev_up = up_h;
                hl = Hp[R - 1];
                xl = xu;
            }
        }
        if constexpr (LOCAL) {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (row0 + r < m && bh[r] >= best_h) { best_h = bh[r]; best_i = row0 + r + 1; best_j = bj[r] + 1; }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                const int oh = __shfl_xor(best_h, off), oi = __shfl_xor(best_i, off), oj = __shfl_xor(best_j, off);
                if (oh > best_h || (oh == best_h && (oi > best_i || (oi == best_i && oj > best_j)))) {
                    best_h = oh; best_i = oi; best_j = oj;
                }
            }
        } else {
            if (row0 <= m - 1 && m - 1 < row0 + R) {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (row0 + r == m - 1) s_score = Hp[r];
            }
        }
    }
    __syncthreads();   // the flags and s_score

    // ---- traceback (one lane), as sa_traceback.hip walks the int32 records
    sa_result res = {};
    if (lane == 0) {
        int i, j, V = 0, st = 0;
        uint32_t flags = 0, k = 0;
        if constexpr (LOCAL) {
            if (m > 0 && n > 0) {
                res.score = best_h; i = best_i; j = best_j; V = best_h;
            } else {
                res.score = ALG == SA_SW ? INT_MIN : 0;   // SW keeps MaxScore = INT_MIN; LG reads M[0][0]
                i = 0; j = 0;
            }
        } else {
            res.score = (m > 0 && n > 0) ? s_score : border(m > n ? m : n);
            i = m; j = n;
        }
        res.end_i = i;
        res.end_j = j;
        auto flag = [&]() -> uint32_t { return s_flag[(i - 1) * n + (j - 1)]; };
        auto diag = [&]() -> int {
            const bool v = match(s_a[i - 1], s_b[j - 1]);
            s_ops[k++] = v ? 'M' : (allow ? 'S' : 'X');
            return v ? MA : MI;
        };
        for (;;) {
            if constexpr (ALG == SA_SW || ALG == SA_NW) {
                const bool inner = i > 0 && j > 0;
                if (ALG == SA_SW ? (!inner || V == 0) : !(i > 0 || j > 0)) break;
                uint32_t f = 1u;   // NW edges: j == 0 -> up, i == 0 -> left
                if (inner) f = flag();
                else if (i == 0) f = 0u;
                const bool dg = (f & 2u) != 0, up = !dg && (f & 1u);
                if (dg) V -= diag();
                else s_ops[k++] = up ? 'U' : 'L';
                if (!dg) V -= G;
                i -= (dg || up) ? 1 : 0;
                j -= up ? 0 : 1;
            } else if constexpr (ALG == SA_LOCAL_GOTOH) {
                if (!(i > 0 && j > 0)) break;
                const uint32_t f = flag();
                if (st == 0) {
                    if (V <= 0) break;   // M == max(D, 0) <= 0
                    if (f & 8u) { V -= diag(); --i; --j; }
                    else st = (f & 4u) ? 1 : 2;
                } else if (st == 1) {
                    if (f & 2u) { s_ops[k++] = 'U'; V -= GE; --i; }
                    else if (V > 0) { s_ops[k++] = 'U'; V -= GOE; --i; st = 0; }
                    else if (V == 0) { s_ops[k++] = 'u'; break; }
                    else { flags |= SA_FLAG_DIVERGED; break; }
                } else {
                    if (f & 1u) { s_ops[k++] = 'L'; V -= GE; --j; }
                    else if (V > 0) { s_ops[k++] = 'L'; V -= GOE; --j; st = 0; }
                    else if (V == 0) { s_ops[k++] = 'l'; break; }
                    else { flags |= SA_FLAG_DIVERGED; break; }
                }
            } else {   // SA_GLOBAL_GOTOH
                if (!(i > 0 || j > 0)) break;
                if (j == 0) { s_ops[k++] = 'U'; --i; continue; }   // edge rules hold in any state
                if (i == 0) { s_ops[k++] = 'L'; --j; continue; }
                const uint32_t f = flag();
                if (st == 0) {
                    if (f & 8u) { diag(); --i; --j; }
                    else st = (f & 4u) ? 1 : 2;
                } else if (st == 1) {
                    s_ops[k++] = 'U'; --i;
                    if (!(f & 2u)) st = 0;
                } else {
                    s_ops[k++] = 'L'; --j;
                    if (!(f & 1u)) st = 0;
                }
            }
            if (k >= (uint32_t)(kTinyM + kTinyN + 1)) { flags |= SA_FLAG_DIVERGED; break; }
        }
        res.start_i = i;
        res.start_j = j;
        res.nops = k;
        res.flags = flags;
        s_score = (int)k;
    }
    __syncthreads();
    const uint32_t nops = (uint32_t)s_score;
    uint8_t* const ops = P.ops + o1 + o2 + p;
    for (uint32_t q = lane; q < nops; q += kWave) ops[q] = s_ops[q];
    if (lane == 0) P.res[p] = res;
}

hipError_t launch_tiny(int algo, bool lut, int max_m, const TinyParams& p, hipStream_t stream) {
    const dim3 grid(p.npairs), block(64);
    const bool r4 = max_m > kWave;   // R = 1 row per lane up to 64 rows, else 4
#define SA_TINY(A)                                                                                            \
    case A:                                                                                                   \
        if (lut) {                                                                                            \
            if (r4) hipLaunchKernelGGL((tiny_kernel<A, 4, true>), grid, block, 0, stream, p);                   \
            else hipLaunchKernelGGL((tiny_kernel<A, 1, true>), grid, block, 0, stream, p);                      \
        } else {                                                                                              \
            if (r4) hipLaunchKernelGGL((tiny_kernel<A, 4, false>), grid, block, 0, stream, p);                  \
            else hipLaunchKernelGGL((tiny_kernel<A, 1, false>), grid, block, 0, stream, p);                     \
        }                                                                                                     \
        break;
    switch (algo) {
        SA_TINY(SA_SW)
        SA_TINY(SA_NW)
        SA_TINY(SA_LOCAL_GOTOH)
        SA_TINY(SA_GLOBAL_GOTOH)
        default: return hipErrorInvalidValue;
    }
#undef SA_TINY
    return hipGetLastError();
}

}  // namespace sa
