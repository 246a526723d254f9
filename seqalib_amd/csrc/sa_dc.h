// sa_dc.h — host and device pieces shared by the linear-space divide-and-conquer aligners
// (sa_hirschberg.hip: HirschbergSA, sa_myersmiller.hip: MyersMillerSA).
//
// Both run their recursion breadth-first over all pairs: device levels split subproblems with
// batched last-row sweeps, and what is left ("leaves") is finished one GPU thread per leaf,
// each writing its forward-order op list.  A pair's leaves tile its alignment path: leaf k
// starts at (a0, b0) where leaf k-1 ended, so sorting the leaves of a pair by (a0, b0) puts
// them in path order (a leaf that is empty in both sequences emits nothing and may land
// anywhere).  dc_assemble concatenates them and reverses the result into the engine's
// traceback-order op stream (include/seqalib_hip.h: pair p's ops at off1[p] + off2[p] + p).
#pragma once
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "sa_internal.h"

namespace sa {

// Device buffer that only grows; kept per host thread (static thread_local) by the drivers,
// since a hipMalloc/hipFree per call would serialise the device.
template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t alloc(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
    ~DevBuf() { if (p) (void)hipFree(p); }
};

// Pinned host staging buffer that only grows (per host thread, like DevBuf): the drivers read
// offsets, split results and leaf ops back every level, and pageable copies would stall.
template <typename T>
struct HostBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t alloc(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipHostMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = count;
        return e;
    }
    T& operator[](size_t k) { return p[k]; }
    const T& operator[](size_t k) const { return p[k]; }
    T* data() { return p; }
    ~HostBuf() { if (p) (void)hipHostFree(p); }
};

// ---- device helpers of the leaf solvers
// match(a, b): the 256x256 LUT as bits (lut_to_bits), or byte equality
__device__ __forceinline__ bool dc_match(const uint32_t* lut, uint32_t a, uint32_t b) {
    return lut ? ((lut[(a << 3) | (b >> 5)] >> (b & 31)) & 1) : a == b;
}

// Row / symbol accessors for the leaf solver: global scratch, or LDS laid out item-major
// (element k of thread t at k * 64 + t: conflict-free when the threads are in step).
typedef int32_t __attribute__((address_space(3))) dc_lds_i32;
typedef uint8_t __attribute__((address_space(3))) dc_lds_u8;
struct GRow {
    int32_t* p;
    __device__ int32_t& operator[](int k) const { return p[k]; }
};
struct LRow {
    dc_lds_i32* p;
    __device__ dc_lds_i32& operator[](int k) const { return p[k * 64]; }
};
struct GSeq {
    const uint8_t* p;
    __device__ uint32_t operator[](int k) const { return p[k]; }
    __device__ GSeq shifted(int k) const { return GSeq{p + k}; }
};
struct LSeq {
    const dc_lds_u8* p;
    __device__ uint32_t operator[](int k) const { return p[k * 64]; }
    __device__ LSeq shifted(int k) const { return LSeq{p + k * 64}; }
};

// Wait for a stream by polling: the drivers synchronise once per level, and a blocking
// hipStreamSynchronize here was observed to oversleep by ~20 ms per wait.
inline hipError_t dc_sync(hipStream_t st) {
    hipError_t e;
    while ((e = hipStreamQuery(st)) == hipErrorNotReady) __builtin_ia32_pause();
    return e;
}

// Host vector -> device through a pinned staging buffer, so the copy is a plain async DMA.
// The stage may be reused once the stream has passed the copy (the drivers wait every level).
template <typename T>
hipError_t dc_put(T* dst, const std::vector<T>& v, HostBuf<T>& stage, hipStream_t st) {
    if (v.empty()) return hipSuccess;
    if (hipError_t e = stage.alloc(v.size())) return e;
    memcpy(stage.data(), v.data(), v.size() * sizeof(T));
    return hipMemcpyAsync(dst, stage.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st);
}

#define SA_DC_HIP(call)                                                                              \
    do {                                                                                             \
        hipError_t e_ = (call);                                                                      \
        if (e_ != hipSuccess) { *err = std::string(#call) + ": " + hipGetErrorString(e_); return -1; } \
    } while (0)

struct DcLeafRef {
    uint32_t pair;
    uint64_t a0, b0;   // absolute start in seq1 / seq2
    uint64_t out;      // byte offset of the leaf's forward ops in the leaf op buffer
    bool top;          // the leaf is the pair's whole problem: its score is the pair's
};

// Fill res[p] (end cell (m, n), nops, score of a top leaf) and ops for every pair.
inline hipError_t dc_assemble(uint32_t npairs, const uint64_t* o1, const uint64_t* o2, const std::vector<DcLeafRef>& leaves,
                        const int32_t* nout, const int32_t* lscore, const uint8_t* lops, std::vector<sa_result>& res,
                        HostBuf<uint8_t>& ops) {
    if (hipError_t e = ops.alloc(o1[npairs] + o2[npairs] + npairs)) return e;
    memset(ops.data(), 0, o1[npairs] + o2[npairs] + npairs);
    // bucket leaves by pair (counting sort), then assemble pairs independently on host threads
    std::vector<uint32_t> start(npairs + 1, 0), order(leaves.size());
    for (const DcLeafRef& s : leaves) ++start[s.pair + 1];
    for (uint32_t p = 0; p < npairs; ++p) start[p + 1] += start[p];
    {
        std::vector<uint32_t> pos(start.begin(), start.end() - 1);
        for (uint32_t k = 0; k < leaves.size(); ++k) order[pos[leaves[k].pair]++] = k;
    }
    auto assemble = [&](uint32_t p0, uint32_t p1) {
        for (uint32_t p = p0; p < p1; ++p) {
            uint32_t* b0 = order.data() + start[p];
            uint32_t* b1 = order.data() + start[p + 1];
            std::sort(b0, b1, [&](uint32_t x, uint32_t y) {
                return leaves[x].a0 != leaves[y].a0 ? leaves[x].a0 < leaves[y].a0 : leaves[x].b0 < leaves[y].b0;
            });
            uint32_t total = 0;
            for (uint32_t* q = b0; q < b1; ++q) total += (uint32_t)nout[*q];
            sa_result& r = res[p];
            r.end_i = (int32_t)(o1[p + 1] - o1[p]);
            r.end_j = (int32_t)(o2[p + 1] - o2[p]);
            r.nops = total;
            // forward op f lands at traceback index total - 1 - f
            uint8_t* dst = ops.data() + o1[p] + o2[p] + p + total;
            for (uint32_t* q = b0; q < b1; ++q) {
                const uint32_t k = *q;
                if (leaves[k].top) r.score = lscore[k];
                const uint8_t* src = lops + leaves[k].out;
                for (int32_t c = 0; c < nout[k]; ++c) *--dst = src[c];
            }
        }
    };
    uint32_t cap = 16;   // host threads for assembly: SEQALIB_DC_THREADS overrides
    if (const char* t = getenv("SEQALIB_DC_THREADS")) cap = std::max(1, atoi(t));
    const uint32_t nth = std::max<uint32_t>(1, std::min<uint32_t>(cap, npairs / 64));
    std::vector<std::thread> pool;
    for (uint32_t t = 0; t < nth; ++t)
        pool.emplace_back(assemble, (uint32_t)((uint64_t)npairs * t / nth), (uint32_t)((uint64_t)npairs * (t + 1) / nth));
    for (auto& th : pool) th.join();
    return hipSuccess;
}

}  // namespace sa
