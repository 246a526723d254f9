// sa_dc.hip — the device-resident level loop shared by HirschbergSA (sa_hirschberg.hip) and
// MyersMillerSA (sa_myersmiller.hip).
//
// Both recursions run breadth-first over all pairs of a batch.  Every buffer they touch is
// addressed by a subproblem's KEY = a0 + b0 (its first Seq1 index plus its first Seq2 index,
// both absolute in the concatenated inputs): the subproblems of one pair at one level, and the
// leaves of one pair, cover disjoint increasing ranges of Seq1 and of Seq2, so the key spans
// [a0 + b0, a0 + b0 + m + n) are disjoint across the whole batch.  A subproblem's sweep rows,
// a leaf's scratch and a leaf's forward op list therefore live at fixed multiples of its key,
// and no prefix sum or host round trip is needed between levels:
//   dc_init_kernel      pairs -> level-0 subproblems
//   dc_classify_kernel  per level: split / leaf, appended with one atomic per wave
//   (per algorithm)     sweeps + split write the next level's subproblems; leaves write their
//                       forward ops at stage[key] and their op count at mark[key]
//   dc_assemble_kernel  one wave per pair: walks its key range in order (= Seq1 order of the
//                       leaves), prefix-sums the counts and writes the traceback-order stream.
#include <hip/hip_runtime.h>

#include "sa_dc.h"

namespace sa {

// A pair longer than the caller's bounds (device API: max_m / max_n), or any pair of a batch
// whose key range passes key_cap, is not aligned: SA_FLAG_BAD_SHAPE, empty slot.
__global__ __launch_bounds__(64) void dc_init_kernel(const uint64_t* o1, const uint64_t* o2, uint32_t npairs,
                                                     int32_t t0, uint32_t max_m, uint32_t max_n, uint64_t key_cap,
                                                     DcSub* subs, sa_result* res) {
    const uint32_t p = blockIdx.x * 64 + threadIdx.x;
    if (p >= npairs) return;
    DcSub s;
    s.a0 = o1[p];
    s.b0 = o2[p];
    s.m = (int32_t)(o1[p + 1] - o1[p]);
    s.n = (int32_t)(o2[p + 1] - o2[p]);
    s.tb = t0;
    s.te = t0;
    s.pair = p;
    s.top = 1;
    if ((uint32_t)s.m > max_m || (uint32_t)s.n > max_n || o1[npairs] + o2[npairs] > key_cap) {
        s.m = -1;
        res[p].flags = SA_FLAG_BAD_SHAPE;
    }
    subs[p] = s;
}

// count = fixed (level 0) or mult * prev->nsplit; slots with m < 0 are empty (Myers–Miller's
// type-1 midpoints leave their third child slot empty).  kClsPer x 256 subproblems per block and
// ONE atomic per list per block: device-scope atomics on one address from every wave serialised
// the deep levels (a level of 1.28 M subproblems took ~20 k of them per list); the lists'
// order is free (the next level's slots and the leaves' outputs are placed by key).
constexpr int kClsThreads = 256, kClsPer = 4, kClsWaves = kClsThreads / 64;
__global__ __launch_bounds__(kClsThreads) void dc_classify_kernel(const DcSub* cur, uint32_t fixed, const DcLevel* prev,
                                                                  uint32_t mult, int leaf_rows, int min_n, DcLevel* lvl,
                                                                  DcSub* split, DcSub* leaves, uint32_t* nleaf) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t count = prev ? mult * prev->nsplit : fixed;
    const uint32_t base = blockIdx.x * (uint32_t)(kClsThreads * kClsPer);
    if (base >= count) return;   // (uniform over the block)
    __shared__ uint32_t s_ns[kClsPer * kClsWaves], s_nl[kClsPer * kClsWaves], s_base[2];
    DcSub s[kClsPer];
    uint64_t bs[kClsPer], bl[kClsPer];
#pragma unroll
    for (int it = 0; it < kClsPer; ++it) {
        const uint32_t k = base + it * kClsThreads + threadIdx.x;
        s[it] = DcSub{};
        bool valid = k < count;
        if (valid) {
            s[it] = cur[k];
            valid = s[it].m >= 0;
        }
        const bool is_split = valid && s[it].m > leaf_rows && s[it].n >= min_n;
        bs[it] = __ballot(is_split);
        bl[it] = __ballot(valid && !is_split);
        if (lane == 0) {
            s_ns[it * kClsWaves + wv] = (uint32_t)__popcll(bs[it]);
            s_nl[it * kClsWaves + wv] = (uint32_t)__popcll(bl[it]);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {   // exclusive offsets within the block, then one atomic per list
        uint32_t ts = 0, tl = 0;
        for (int q = 0; q < kClsPer * kClsWaves; ++q) {
            const uint32_t a = s_ns[q], b = s_nl[q];
            s_ns[q] = ts;
            s_nl[q] = tl;
            ts += a;
            tl += b;
        }
        s_base[0] = ts ? atomicAdd(&lvl->nsplit, ts) : 0u;
        s_base[1] = tl ? atomicAdd(nleaf, tl) : 0u;
    }
    __syncthreads();
    const uint64_t below = (1ull << lane) - 1;
#pragma unroll
    for (int it = 0; it < kClsPer; ++it) {
        if (bs[it] >> lane & 1) split[s_base[0] + s_ns[it * kClsWaves + wv] + __popcll(bs[it] & below)] = s[it];
        if (bl[it] >> lane & 1) leaves[s_base[1] + s_nl[it * kClsWaves + wv] + __popcll(bl[it] & below)] = s[it];
    }
}

__global__ __launch_bounds__(64) void dc_assemble_kernel(const uint64_t* o1, const uint64_t* o2, const int32_t* mark,
                                                         const uint8_t* stage, sa_result* res, uint8_t* ops) {
    const int lane = threadIdx.x;
    const uint32_t p = blockIdx.x;
    if (res[p].flags & SA_FLAG_BAD_SHAPE) return;   // not aligned (dc_init_kernel)
    const uint64_t key0 = o1[p] + o2[p];
    const int32_t m = (int32_t)(o1[p + 1] - o1[p]), n = (int32_t)(o2[p + 1] - o2[p]);
    const int32_t len = m + n;
    int32_t total = 0;
    for (int32_t i = lane; i < len; i += 64) total += mark[key0 + i];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) total += __shfl_xor(total, off);
    uint8_t* dst = ops + key0 + p;   // this pair's stream (m + n + 1 bytes)
    int32_t base = 0;
    for (int32_t c0 = 0; c0 < len; c0 += 64) {
        const int32_t i = c0 + lane;
        const int32_t cnt = i < len ? mark[key0 + i] : 0;
        int32_t incl = cnt;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t v = __shfl_up(incl, off);
            if (lane >= off) incl += v;
        }
        // forward op f of the pair lands at traceback index total - 1 - f
        const int32_t f0 = base + incl - cnt;
        const uint8_t* src = stage + key0 + i;
        for (int32_t q = 0; q < cnt; ++q) dst[total - 1 - (f0 + q)] = src[q];
        base += __shfl(incl, 63);
    }
    for (int32_t i = total + lane; i <= len; i += 64) dst[i] = 0;
    if (lane == 0) {
        res[p].end_i = m;
        res[p].end_j = n;
        res[p].nops = (uint32_t)total;
    }
}

hipError_t dc_launch_init(const uint64_t* o1, const uint64_t* o2, uint32_t npairs, int32_t t0, const DcBounds& b,
                          DcSub* subs, sa_result* res, hipStream_t st) {
    hipLaunchKernelGGL(dc_init_kernel, dim3((npairs + 63) / 64), dim3(64), 0, st, o1, o2, npairs, t0, b.max_m, b.max_n,
                       b.t1 + b.t2, subs, res);
    return hipGetLastError();
}

hipError_t dc_launch_classify(const DcSub* cur, uint32_t cap, uint32_t fixed, const DcLevel* prev, uint32_t mult,
                              int leaf_rows, int min_n, DcLevel* lvl, DcSub* split, DcSub* leaves, uint32_t* nleaf,
                              hipStream_t st) {
    if (!cap) return hipSuccess;
    constexpr uint32_t per = kClsThreads * kClsPer;
    hipLaunchKernelGGL(dc_classify_kernel, dim3((cap + per - 1) / per), dim3(kClsThreads), 0, st, cur, fixed, prev, mult, leaf_rows,
                       min_n, lvl, split, leaves, nleaf);
    return hipGetLastError();
}

hipError_t dc_launch_assemble(const uint64_t* o1, const uint64_t* o2, uint32_t npairs, const int32_t* mark,
                              const uint8_t* stage, sa_result* res, uint8_t* ops, hipStream_t st) {
    hipLaunchKernelGGL(dc_assemble_kernel, dim3(npairs), dim3(64), 0, st, o1, o2, mark, stage, res, ops);
    return hipGetLastError();
}

}  // namespace sa
