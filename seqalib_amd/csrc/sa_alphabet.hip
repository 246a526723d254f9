// sa_alphabet.hip — batch alphabet scan and the substitution profile of the T16 fill kernel.
//
// The T16 kernel (sa_fill_impl.h) codes symbols 0..3 and reads the substitution term of a cell
// from a per-row byte profile, so it applies when the whole batch uses at most four distinct
// byte values (DNA).  The host learns that from a 256-bit presence bitmap of every byte of both
// sequence sets (one streaming pass, ~HBM speed) before it plans the launch.
#include <stdlib.h>

#include "sa_internal.h"

namespace sa {

typedef unsigned int u32x4a __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void mark(uint32_t (&bm)[8], uint32_t b) {
    const uint32_t bit = 1u << (b & 31u), w = b >> 5;
#pragma unroll
    for (int k = 0; k < 8; ++k) bm[k] |= (w == (uint32_t)k) ? bit : 0u;
}
__device__ __forceinline__ void mark4(uint32_t (&bm)[8], uint32_t v) {
    mark(bm, v & 255u); mark(bm, (v >> 8) & 255u); mark(bm, (v >> 16) & 255u); mark(bm, v >> 24);
}

template <int THREADS>
__global__ __launch_bounds__(THREADS) void alphabet_scan(const uint8_t* d1, const uint64_t* o1,
                                                     const uint8_t* d2, const uint64_t* o2,
                                                     uint32_t npairs, uint32_t* bitmap) {
    __shared__ uint32_t sb[8];
    if (threadIdx.x < 8) sb[threadIdx.x] = 0;
    __syncthreads();
    uint32_t bm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    for (int set = 0; set < 2; ++set) {
        const uint8_t* d = set ? d2 : d1;
        const uint64_t* o = set ? o2 : o1;
        const uint64_t b0 = o[0], b1 = o[npairs];
        if (b1 <= b0) continue;
        const uint8_t* p0 = d + b0;
        const uint8_t* p1 = d + b1;
        // 16-byte aligned body, bytes before and after it
        const uint8_t* a0 = reinterpret_cast<const uint8_t*>((reinterpret_cast<uintptr_t>(p0) + 15) & ~(uintptr_t)15);
        const uint8_t* a1 = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p1) & ~(uintptr_t)15);
        if (a0 >= a1) { a0 = p1; a1 = p1; }
        const uint64_t head = (uint64_t)(a0 - p0), tail = (uint64_t)(p1 - a1);
        for (uint64_t k = tid; k < head; k += nth) mark(bm, p0[k]);
        for (uint64_t k = tid; k < tail; k += nth) mark(bm, a1[k]);
        const u32x4a* v = reinterpret_cast<const u32x4a*>(a0);
        const uint64_t nv = (uint64_t)(a1 - a0) / 16;
        for (uint64_t k = tid; k < nv; k += nth) {
            const u32x4a x = __builtin_nontemporal_load(v + k);
            mark4(bm, x.x); mark4(bm, x.y); mark4(bm, x.z); mark4(bm, x.w);
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (bm[k]) atomicOr(&sb[k], bm[k]);
    __syncthreads();
    if (threadIdx.x < 8 && sb[threadIdx.x]) atomicOr(&bitmap[threadIdx.x], sb[threadIdx.x]);
}

// The T16 decision, on the device (so the host never waits for the scan): with <= 4 distinct
// symbols, sym_pack = the symbols padded with absent byte values (codes stay distinct),
// prof[c] byte c' = (int8)(4 * s(sym c, sym c') + 3) -- (8 * s + 6) for the affine kernel
// (affine = 1), s itself for the 16-bit linear-space sweeps (affine = 2, sa_dc.h) --,
// s = match ? match : mismatch; sel = 1.
// More symbols: sel = 0 (the int32 kernel's launches run, the T16 ones return at once).
__global__ void decide_t16(const uint32_t* lutbits, int match, int mismatch, int affine, uint32_t* aux) {
    if (threadIdx.x != 0) return;
    uint32_t syms[4] = {0, 0, 0, 0};
    int nsym = 0;
    for (int b = 0; b < 256; ++b)
        if ((aux[b >> 5] >> (b & 31)) & 1u) {
            if (nsym < 4) syms[nsym] = (uint32_t)b;
            ++nsym;
        }
    if (nsym > 4) {
        aux[kAuxSel] = 0;
        return;
    }
    for (int b = 0; nsym < 4 && b < 256; ++b) {
        bool used = false;
        for (int q = 0; q < nsym; ++q) used |= syms[q] == (uint32_t)b;
        if (!used) syms[nsym++] = (uint32_t)b;
    }
    for (int c = 0; c < 4; ++c) {
        uint32_t w = 0;
        for (int c2 = 0; c2 < 4; ++c2) {
            const uint32_t a = syms[c], b = syms[c2];
            const bool v = lutbits ? ((lutbits[(a << 3) | (b >> 5)] >> (b & 31u)) & 1u) : (a == b);
            const int s = v ? match : mismatch;
            const int t = affine == 2 ? s : affine ? 8 * s + 6 : 4 * s + 3;
            w |= ((uint32_t)t & 255u) << (8 * c2);
        }
        aux[kAuxProf + c] = w;
    }
    aux[kAuxProf + 4] = syms[0] | syms[1] << 8 | syms[2] << 16 | syms[3] << 24;
    aux[kAuxSel] = 1;
}

hipError_t launch_alphabet_scan(const uint8_t* d1, const uint64_t* o1, const uint8_t* d2,
                                const uint64_t* o2, uint32_t npairs, uint32_t* bitmap, hipStream_t s) {
    hipError_t e = hipMemsetAsync(bitmap, 0, 32, s);
    if (e != hipSuccess) return e;
    // One-wave workgroups: queued behind a running fill (the pipelined calls' case), a workgroup
    // starts as soon as ONE fill unit's slot frees, where a 4-wave workgroup waited for four in one
    // CU (bench rocprofv3 r05: scans of up to 15.7 ms, 14 % of the summed kernel time).
    // $SEQALIB_SCAN_WG=256 restores the round-5 launch (A/B).
    const char* ev = getenv("SEQALIB_SCAN_WG");   // (read per launch: tests switch it in-process)
    const bool wide = ev && atoi(ev) == 256;
    if (wide) hipLaunchKernelGGL(alphabet_scan<256>, dim3(2048), dim3(256), 0, s, d1, o1, d2, o2, npairs, bitmap);
    else hipLaunchKernelGGL(alphabet_scan<64>, dim3(2048), dim3(64), 0, s, d1, o1, d2, o2, npairs, bitmap);
    return hipGetLastError();
}

hipError_t launch_decide_t16(const uint32_t* lutbits, int match, int mismatch, int affine, uint32_t* aux,
                             hipStream_t s) {
    hipLaunchKernelGGL(decide_t16, dim3(1), dim3(64), 0, s, lutbits, match, mismatch, affine, aux);
    return hipGetLastError();
}

}  // namespace sa
