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
//     [0, |Seq2|) maximising Fwd[i] + Rev[|Seq2|-i] (:138-149; i never reaches |Seq2|) and the
//     host forms the two children (:151-161).
//   * leaves: everything smaller (and every base case) is finished by hb_leaf_kernel, one
//     thread per subproblem running the same recursion iteratively (explicit stack, left child
//     first), including the NW base case of :119-126 with the reference's NW traceback rules.
//   * assembly: a pair's leaves cover disjoint, increasing ranges of Seq1, so its alignment is
//     the concatenation of its leaves' forward op lists in Seq1 order; the host reverses it into
//     the engine's traceback-order op stream (include/seqalib_hip.h).
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

constexpr int kHbLeafRows = 48;   // subproblems with <= this many Seq1 rows are leaves (tuned)

struct HbSweep {       // NWScore over A (alen) x B (blen) -> rows[out .. out+blen]
    uint64_t a, b;     // index of A[0] / B[0] in seq1 / seq2 (rev: of the LAST element read first)
    int32_t alen, blen;
    int32_t rev;       // 1: A and B are both read backwards
    int32_t pad;
    uint64_t out;      // int32 index into the row buffer
};

struct HbSplit {
    uint64_t fwd, rev; // row indices of the forward / reverse last rows (blen + 1 each)
    int32_t n, top;    // |Seq2| of the subproblem; top: also report the NW score
};

struct HbLeaf {
    uint64_t a0, b0;   // Seq1 / Seq2 start (indices into seq1 / seq2)
    int32_t alen, blen;
    uint64_t scratch;  // int32 index into the leaf scratch
    uint64_t out;      // byte index into the leaf op buffer (capacity alen + blen)
    int32_t top, pad;
};

struct HbScore {
    int32_t gap, match, mismatch, allow;
};

// NW cell as NWScore computes it (:40-44 / :56-59).
__device__ __forceinline__ int32_t hb_cell(int32_t hd, int32_t hu, int32_t hl, bool v, const HbScore& s) {
    const int32_t sub = s.allow ? hd + (v ? s.match : s.mismatch) : (v ? hd + s.match : INT_MIN);
    return max(max(sub, hu + s.gap), hl + s.gap);
}

// The same cell with the match source (LUT) and AllowMismatch fixed at compile time: branch-free.
template <bool LUT, bool ALLOW>
__device__ __forceinline__ int32_t hb_cell_t(int32_t hd, int32_t hu, int32_t hl, uint32_t a, uint32_t b,
                                             const uint32_t* lut, const HbScore& s) {
    bool v;
    if constexpr (LUT) v = (lut[(a << 3) | (b >> 5)] >> (b & 31)) & 1;
    else v = a == b;
    int32_t sub;
    if constexpr (ALLOW) sub = hd + (v ? s.match : s.mismatch);
    else sub = v ? hd + s.match : INT_MIN;
    return max(max(sub, hu + s.gap), hl + s.gap);
}

// ------------------------------------------------------------------ batched NWScore sweeps
template <int R, bool LUT, bool ALLOW>
__global__ __launch_bounds__(64) void hb_sweep_kernel(const uint8_t* s1, const uint8_t* s2, const HbSweep* sweeps,
                                                      int32_t* rows, const uint32_t* lutbits, HbScore sc) {
    __shared__ uint32_t s_lut[LUT ? 2048 : 1];
    const int lane = threadIdx.x;
    const HbSweep d = sweeps[blockIdx.x];
    if constexpr (LUT) {
        for (int k = lane; k < 2048; k += 64) s_lut[k] = lutbits[k];
        __syncthreads();
    }
    const uint32_t* lut = s_lut;
    int32_t* out = rows + d.out;
    const int m = d.alen, n = d.blen, G = sc.gap;
    auto symA = [&](int k) -> uint32_t { return d.rev ? s1[d.a - k] : s1[d.a + k]; };
    auto symB = [&](int k) -> uint32_t { return d.rev ? s2[d.b - k] : s2[d.b + k]; };
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
            for (int q = 0; q < steps; ++q) {
                const int s = c0 + q;
                const int32_t up_h = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vup, q), hl, 0x138, 0xf,
                                                                 0xf, false);
                sym = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(vsym, q), sym, 0x138, 0xf, 0xf, false);
                const int j0 = s - lane;
                if (j0 >= 0 && j0 < n) {
                    int32_t hd = prev_up, hu = up_h;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int32_t h = hb_cell_t<LUT, ALLOW>(hd, hu, Hp[r], a[r], sym, lut, sc);
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
}

// ---------------------------------------------------------------------------- split
__global__ __launch_bounds__(64) void hb_split_kernel(const HbSplit* splits, const int32_t* rows, int32_t* mid2,
                                                      int32_t* score) {
    const int lane = threadIdx.x;
    const HbSplit d = splits[blockIdx.x];
    const int32_t* F = rows + d.fwd;
    const int32_t* B = rows + d.rev;
    const int n = d.n;
    int32_t best = INT_MIN;
    int idx = 0;
    for (int i = lane; i < n; i += 64) {
        const int32_t s = F[i] + B[n - i];
        if (s >= best) { best = s; idx = i; }
    }
    // lexicographic (sum, i) maximum = the reference's last maximum (S >= MaxScore, :144)
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const int32_t ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(idx, off);
        if (ob > best || (ob == best && oi > idx)) { best = ob; idx = oi; }
    }
    if (lane == 0) {
        mid2[blockIdx.x] = idx;
        if (d.top) score[blockIdx.x] = max(best, F[n] + B[0]);   // NW H[m][n] over i in [0, n]
    }
}

// ---------------------------------------------------------------------------- leaves
template <typename Row, typename Seq>
__device__ void hb_nwscore(Seq A, int alen, int arev, Seq B, int blen, int brev,
                           const uint32_t* lut, const HbScore& sc, Row& F, Row& X) {
    F[0] = 0;
    for (int j = 1; j <= blen; ++j) F[j] = F[j - 1] + sc.gap;
    for (int i = 1; i <= alen; ++i) {
        const uint32_t ai = arev ? A[alen - i] : A[i - 1];
        int32_t left = F[0] + sc.gap, diag = F[0];
        X[0] = left;
        for (int j = 1; j <= blen; ++j) {
            const uint32_t bj = brev ? B[blen - j] : B[j - 1];
            const int32_t up = F[j];
            left = hb_cell(diag, up, left, dc_match(lut, ai, bj), sc);
            X[j] = left;
            diag = up;
        }
        Row t = F; F = X; X = t;
    }
}

// NeedlemanWunschSA::getAlignment on a 1 x k or k x 1 view (:119-126): full matrix + the
// reference NW traceback (SANeedlemanWunsch.h:167-230); writes forward-order ops at out.
__device__ int hb_nw_small(const uint8_t* A, int m, const uint8_t* B, int n, const uint32_t* lut,
                           const HbScore& sc, int32_t* H, uint8_t* out) {
    const int w = n + 1;
    for (int i = 0; i <= m; ++i) H[i * w] = i * sc.gap;
    for (int j = 0; j <= n; ++j) H[j] = j * sc.gap;
    for (int i = 1; i <= m; ++i)
        for (int j = 1; j <= n; ++j)
            H[i * w + j] = hb_cell(H[(i - 1) * w + j - 1], H[(i - 1) * w + j], H[i * w + j - 1],
                                   dc_match(lut, A[i - 1], B[j - 1]), sc);
    int k = 0, i = m, j = n;
    while (i > 0 || j > 0) {
        if (i > 0 && j > 0) {
            const bool v = dc_match(lut, A[i - 1], B[j - 1]);
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
template <typename Row, typename Seq>
__device__ int hb_leaf_solve(Seq S1, Seq S2, const uint8_t* g1, const uint8_t* g2, int alen, int blen, bool top,
                             Row F, Row X, Row Cc, int32_t* Hs, uint8_t* out, int32_t* score,
                             const uint32_t* lut, const HbScore& sc) {
    if (top) {
        int32_t s;
        if (alen == 0) s = blen * sc.gap;
        else if (blen == 0) s = alen * sc.gap;
        else { hb_nwscore(S1, alen, 0, S2, blen, 0, lut, sc, F, X); s = F[blen]; }
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
            k += hb_nw_small(g1 + x0, xl, g2 + y0, yl, lut, sc, Hs, out + k);
        } else {
            const int mid = xl / 2;
            const Seq A0 = S1.shifted(x0), B0 = S2.shifted(y0), A1 = S1.shifted(x0 + mid);
            hb_nwscore(A0, mid, 0, B0, yl, 0, lut, sc, F, X);
            for (int q = 0; q <= yl; ++q) Cc[q] = F[q];
            hb_nwscore(A1, xl - mid, 1, B0, yl, 1, lut, sc, F, X);
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

constexpr int kHbLdsCols = 64;   // leaves with |Seq1|, |Seq2| <= this run with LDS rows + symbols

__global__ __launch_bounds__(64) void hb_leaf_kernel(const uint8_t* s1, const uint8_t* s2, const HbLeaf* leaves,
                                                     uint32_t nleaves, int32_t* scratch, uint8_t* outops,
                                                     int32_t* nout, int32_t* score, const uint32_t* lut,
                                                     HbScore sc) {
    __shared__ int32_t s_rows[3 * (kHbLdsCols + 1) * 64];
    __shared__ uint8_t s_seq[2 * kHbLdsCols * 64];
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= nleaves) return;
    const int t = threadIdx.x;
    const HbLeaf L = leaves[id];
    const uint8_t* g1 = s1 + L.a0;
    const uint8_t* g2 = s2 + L.b0;
    int32_t* Fg = scratch + L.scratch;
    int32_t* Hs = Fg + 3 * (L.blen + 1);        // 2 * (max(alen, blen) + 1): base-case matrix
    uint8_t* out = outops + L.out;
    int k;
    if (L.alen <= kHbLdsCols && L.blen <= kHbLdsCols) {
        dc_lds_u8* q1 = (dc_lds_u8*)s_seq + t;
        dc_lds_u8* q2 = q1 + kHbLdsCols * 64;
        for (int c = 0; c < L.alen; ++c) q1[c * 64] = g1[c];
        for (int c = 0; c < L.blen; ++c) q2[c * 64] = g2[c];
        dc_lds_i32* r0 = (dc_lds_i32*)s_rows + t;
        const LRow F{r0}, X{r0 + (kHbLdsCols + 1) * 64}, Cc{r0 + 2 * (kHbLdsCols + 1) * 64};
        k = hb_leaf_solve(LSeq{q1}, LSeq{q2}, g1, g2, L.alen, L.blen, L.top != 0, F, X, Cc, Hs, out, score + id,
                          lut, sc);
    } else {
        const GRow F{Fg}, X{Fg + (L.blen + 1)}, Cc{Fg + 2 * (L.blen + 1)};
        k = hb_leaf_solve(GSeq{g1}, GSeq{g2}, g1, g2, L.alen, L.blen, L.top != 0, F, X, Cc, Hs, out, score + id,
                          lut, sc);
    }
    nout[id] = k;
}

// ---------------------------------------------------------------------------- host driver
namespace {

struct Sub {
    uint32_t pair;
    uint64_t a0, b0;   // absolute indices into seq1 / seq2
    int32_t m, n;
    bool top;
};

template <bool LUT, bool ALLOW>
void launch_sweeps_t(int R, dim3 grid, const uint8_t* d1, const uint8_t* d2, const HbSweep* sw, int32_t* rows,
                     const uint32_t* lut, const HbScore& sc, hipStream_t st) {
    const dim3 block(64);
    switch (R) {
        case 1: hipLaunchKernelGGL((hb_sweep_kernel<1, LUT, ALLOW>), grid, block, 0, st, d1, d2, sw, rows, lut, sc); break;
        case 2: hipLaunchKernelGGL((hb_sweep_kernel<2, LUT, ALLOW>), grid, block, 0, st, d1, d2, sw, rows, lut, sc); break;
        case 4: hipLaunchKernelGGL((hb_sweep_kernel<4, LUT, ALLOW>), grid, block, 0, st, d1, d2, sw, rows, lut, sc); break;
        case 8: hipLaunchKernelGGL((hb_sweep_kernel<8, LUT, ALLOW>), grid, block, 0, st, d1, d2, sw, rows, lut, sc); break;
        case 16: hipLaunchKernelGGL((hb_sweep_kernel<16, LUT, ALLOW>), grid, block, 0, st, d1, d2, sw, rows, lut, sc); break;
        default: hipLaunchKernelGGL((hb_sweep_kernel<32, LUT, ALLOW>), grid, block, 0, st, d1, d2, sw, rows, lut, sc); break;
    }
}

hipError_t launch_sweeps(int R, uint32_t count, const uint8_t* d1, const uint8_t* d2, const HbSweep* sw,
                         int32_t* rows, const uint32_t* lut, const HbScore& sc, hipStream_t st) {
    const dim3 grid(count);
    if (lut) {
        if (sc.allow) launch_sweeps_t<true, true>(R, grid, d1, d2, sw, rows, lut, sc, st);
        else launch_sweeps_t<true, false>(R, grid, d1, d2, sw, rows, lut, sc, st);
    } else {
        if (sc.allow) launch_sweeps_t<false, true>(R, grid, d1, d2, sw, rows, lut, sc, st);
        else launch_sweeps_t<false, false>(R, grid, d1, d2, sw, rows, lut, sc, st);
    }
    return hipGetLastError();
}

}  // namespace

// Host driver: inputs on the device (offsets too), results and the traceback-order op streams
// returned in host memory (res[npairs], ops laid out at off1[p] + off2[p] + p).
int hirschberg_run(const sa_scoring* scoring, const uint8_t* d1, const uint64_t* d_o1, const uint8_t* d2,
                   const uint64_t* d_o2, uint32_t npairs, const uint32_t* d_lutbits, hipStream_t st,
                   std::vector<sa_result>& res, const uint8_t** ops, uint64_t* ops_bytes,
                   std::string* err) {
    const bool timing = getenv("SEQALIB_HB_TIMING") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto t_start = now(), t_mark = t_start;
    auto lap = [&](const char* what) {
        if (!timing) return;
        const auto t = now();
        fprintf(stderr, "[hb] %-28s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_mark).count());
        t_mark = t;
    };
    int leaf_rows = kHbLeafRows;   // tuning override: SEQALIB_HB_LEAF
    if (const char* lr = getenv("SEQALIB_HB_LEAF")) leaf_rows = std::max(2, atoi(lr));
    HbScore sc;
    sc.gap = scoring->gap;
    sc.match = scoring->match;
    sc.allow = scoring->allow_mismatch != 0;
    sc.mismatch = sc.allow ? scoring->mismatch : INT_MIN;
    static thread_local HostBuf<uint64_t> o1, o2;
    SA_DC_HIP(o1.alloc(npairs + 1));
    SA_DC_HIP(o2.alloc(npairs + 1));
    static thread_local HostBuf<uint8_t> hops;   // traceback-order op streams, returned in *ops
    SA_DC_HIP(hipMemcpyAsync(o1.data(), d_o1, 8ull * (npairs + 1), hipMemcpyDeviceToHost, st));
    SA_DC_HIP(hipMemcpyAsync(o2.data(), d_o2, 8ull * (npairs + 1), hipMemcpyDeviceToHost, st));
    SA_DC_HIP(dc_sync(st));
    lap("setup (offsets D2H)");
    res.assign(npairs, sa_result{});
    std::vector<Sub> cur, leaves;
    cur.reserve(npairs);
    for (uint32_t p = 0; p < npairs; ++p)
        cur.push_back(Sub{p, o1[p], o2[p], (int32_t)(o1[p + 1] - o1[p]), (int32_t)(o2[p + 1] - o2[p]), true});

    // device buffers persist per host thread (hipMalloc/hipFree per call would serialise)
    static thread_local DevBuf<HbSweep> dsw;
    static thread_local DevBuf<HbSplit> dsp;
    static thread_local DevBuf<int32_t> drows, dmid, dscore;
    std::vector<HbSweep> sw;
    std::vector<HbSplit> sp;
    std::vector<Sub> split, next;
    static thread_local HostBuf<int32_t> mid2, tops;
    while (!cur.empty()) {
        split.clear();
        for (const Sub& s : cur) (s.m > leaf_rows && s.n >= 2 ? split : leaves).push_back(s);
        if (split.empty()) break;
        sw.clear();
        sp.clear();
        uint64_t rowpos = 0;
        int maxa = 0;
        for (const Sub& s : split) {
            const int mid = s.m / 2;
            HbSplit d;
            d.n = s.n;
            d.top = s.top ? 1 : 0;
            d.fwd = rowpos;
            sw.push_back(HbSweep{s.a0, s.b0, mid, s.n, 0, 0, rowpos});
            rowpos += (uint64_t)s.n + 1;
            d.rev = rowpos;
            sw.push_back(HbSweep{s.a0 + (uint64_t)s.m - 1, s.b0 + (uint64_t)s.n - 1, s.m - mid, s.n, 1, 0, rowpos});
            rowpos += (uint64_t)s.n + 1;
            sp.push_back(d);
            maxa = std::max(maxa, s.m - mid);
        }
        SA_DC_HIP(dsw.alloc(sw.size()));
        SA_DC_HIP(dsp.alloc(sp.size()));
        SA_DC_HIP(drows.alloc(rowpos));
        SA_DC_HIP(dmid.alloc(sp.size()));
        SA_DC_HIP(dscore.alloc(sp.size()));
        static thread_local HostBuf<HbSweep> ssw;
        static thread_local HostBuf<HbSplit> ssp;
        SA_DC_HIP(dc_put(dsw.p, sw, ssw, st));
        lap("level: descriptors + H2D");
        SA_DC_HIP(dc_put(dsp.p, sp, ssp, st));
        int R = 1;
        while (R < 32 && 64 * R < maxa) R *= 2;
        SA_DC_HIP(launch_sweeps(R, (uint32_t)sw.size(), d1, d2, dsw.p, drows.p, d_lutbits, sc, st));
        hipLaunchKernelGGL(hb_split_kernel, dim3((uint32_t)sp.size()), dim3(64), 0, st, dsp.p, drows.p, dmid.p,
                           dscore.p);
        SA_DC_HIP(hipGetLastError());
        SA_DC_HIP(mid2.alloc(sp.size()));
        SA_DC_HIP(tops.alloc(sp.size()));
        SA_DC_HIP(hipMemcpyAsync(mid2.data(), dmid.p, sp.size() * 4, hipMemcpyDeviceToHost, st));
        SA_DC_HIP(hipMemcpyAsync(tops.data(), dscore.p, sp.size() * 4, hipMemcpyDeviceToHost, st));
        SA_DC_HIP(dc_sync(st));
        next.clear();
        for (size_t k = 0; k < split.size(); ++k) {
            const Sub& s = split[k];
            if (s.top) res[s.pair].score = tops[k];
            const int mid = s.m / 2, j = mid2[k];
            next.push_back(Sub{s.pair, s.a0, s.b0, mid, j, false});
            next.push_back(Sub{s.pair, s.a0 + (uint64_t)mid, s.b0 + (uint64_t)j, s.m - mid, s.n - j, false});
        }
        cur.swap(next);
        lap("level (sweeps + split)");
    }

    // leaves: one thread each
    std::vector<HbLeaf> lv(leaves.size());
    uint64_t scr = 0, outpos = 0;
    for (size_t k = 0; k < leaves.size(); ++k) {
        const Sub& s = leaves[k];
        lv[k] = HbLeaf{s.a0, s.b0, s.m, s.n, scr, outpos, s.top ? 1 : 0, 0};
        scr += 3ull * ((uint64_t)s.n + 1) + 2ull * ((uint64_t)std::max(s.m, s.n) + 1);
        outpos += (uint64_t)s.m + (uint64_t)s.n;
    }
    if (!lv.empty()) {
        static thread_local DevBuf<HbLeaf> dlv;
        static thread_local DevBuf<int32_t> dscr, dnout, dlscore;
        static thread_local DevBuf<uint8_t> dout;
        SA_DC_HIP(dlv.alloc(lv.size()));
        SA_DC_HIP(dscr.alloc(scr));
        SA_DC_HIP(dnout.alloc(lv.size()));
        SA_DC_HIP(dlscore.alloc(lv.size()));
        SA_DC_HIP(dout.alloc(outpos));
        static thread_local HostBuf<HbLeaf> slv;
        SA_DC_HIP(dc_put(dlv.p, lv, slv, st));
        hipLaunchKernelGGL(hb_leaf_kernel, dim3((uint32_t)((lv.size() + 63) / 64)), dim3(64), 0, st, d1, d2, dlv.p,
                           (uint32_t)lv.size(), dscr.p, dout.p, dnout.p, dlscore.p, d_lutbits, sc);
        SA_DC_HIP(hipGetLastError());
        static thread_local HostBuf<int32_t> nout, lscore;
        static thread_local HostBuf<uint8_t> lops;
        SA_DC_HIP(nout.alloc(lv.size()));
        SA_DC_HIP(lscore.alloc(lv.size()));
        SA_DC_HIP(lops.alloc(outpos));
        SA_DC_HIP(hipMemcpyAsync(nout.data(), dnout.p, lv.size() * 4, hipMemcpyDeviceToHost, st));
        SA_DC_HIP(hipMemcpyAsync(lscore.data(), dlscore.p, lv.size() * 4, hipMemcpyDeviceToHost, st));
        if (outpos) SA_DC_HIP(hipMemcpyAsync(lops.data(), dout.p, outpos, hipMemcpyDeviceToHost, st));
        SA_DC_HIP(dc_sync(st));
        lap("leaves (kernel + D2H)");
        std::vector<DcLeafRef> refs(lv.size());
        for (size_t k = 0; k < lv.size(); ++k)
            refs[k] = DcLeafRef{leaves[k].pair, leaves[k].a0, leaves[k].b0, lv[k].out, leaves[k].top};
        SA_DC_HIP(dc_assemble(npairs, o1.data(), o2.data(), refs, nout.data(), lscore.data(), lops.data(), res, hops));
        lap("assembly (host)");
    } else {
        SA_DC_HIP(hops.alloc(o1[npairs] + o2[npairs] + npairs));
        memset(hops.data(), 0, o1[npairs] + o2[npairs] + npairs);
    }
    *ops = hops.data();
    *ops_bytes = o1[npairs] + o2[npairs] + npairs;
    return 0;
}

}  // namespace sa
