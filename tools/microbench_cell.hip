// Register-only microbenchmark of the SW cell loop (no memory traffic in the loop), to measure
// the VALU issue efficiency of candidate instruction idioms on gfx950.  Not part of the product.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_cell.hip -o build/microbench_cell
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ int shr1(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t push_eq(uint32_t rec, int a, int b) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(a == b);
    uint32_t out; unsigned long long co;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(out), "=s"(co) : "v"(rec), "s"(m));
    return out;
}
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

// FLAGS: 0 none, 1 ballot+addc, 2 C shift-or; KEY: 0 none, 1 keyed max
template <int R, int FLAGS, int KEY, int DPP>
__global__ __launch_bounds__(256) void cells(const int* in, uint32_t* out, int steps) {
    const int lane = threadIdx.x & 63;
    int a[R], Hp[R], bh[R];
    for (int r = 0; r < R; ++r) { a[r] = (in[(threadIdx.x * 7 + r) & 1023]) & 3; Hp[r] = 0; bh[r] = 0; }
    int hl = 0, sym = lane & 3, prev_up = 0, up_seed = in[lane];
    uint32_t acc = 0;
    const int G = -1, MA = 1, MI = -1;
    for (int s = 0; s < steps; ++s) {
        int up_h, sv;
        if (DPP) {
            up_h = shr1(up_seed, hl);
            sym = shr1((s * 7) & 3, sym);
            sv = sym;
        } else {
            up_h = hl ^ s;
            sv = (sym + s) & 3;
        }
        int hd = prev_up, hu = up_h;
        uint32_t rec = 0;
        const int jkey = s + 1;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool v = a[r] == sv;
            const int D = hd + (v ? MA : MI);
            const int U = hu + G;
            const int L = Hp[r] + G;
            const int H = imax(imax(imax(D, U), L), 0);
            if (FLAGS == 1) { rec = push_eq(rec, H, D); rec = push_eq(rec, H, U); }
            if (FLAGS == 2) { rec = rec * 4 + (H == D ? 2u : 0u) + (H == U ? 1u : 0u); }
            if (KEY) bh[r] = (int)max((uint32_t)bh[r], ((uint32_t)H << 16) | (uint32_t)jkey);
            hd = Hp[r]; Hp[r] = H; hu = H;
        }
        prev_up = up_h;
        hl = Hp[R - 1];
        acc ^= rec;
    }
    for (int r = 0; r < R; ++r) acc += bh[r] + Hp[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// Tagged 16-bit cell: values scaled by 4, direction tag in the low 2 bits (diag 3 > up 2 >
// left 1 > zero 0), so the max also resolves the traceback direction with the reference's
// priority.  16-bit add/max are fast-class on gfx950.
__device__ __forceinline__ uint32_t lshl2_or(uint32_t rec, uint32_t t) {
    return (rec << 2) | t;
}
template <int R, int KEY, int SUB>
__global__ __launch_bounds__(256) void cells16(const int* in, uint32_t* out, int steps) {
    const int lane = threadIdx.x & 63;
    int a[R];
    short Hp[R];
    uint32_t bh[R];
    for (int r = 0; r < R; ++r) { a[r] = (in[(threadIdx.x * 7 + r) & 1023]) & 3; Hp[r] = 0; bh[r] = 0; }
    int hl = 0, sym = lane & 3, prev_up = 0, up_seed = in[lane];
    uint32_t acc = 0;
    const short CU = 4 * -1 + 2, CL = 4 * -1 + 1, SM = 4 * 1 + 3, SX = 4 * -1 + 3;
    for (int s = 0; s < steps; ++s) {
        const int up_h = shr1(up_seed, hl);
        sym = shr1((s * 7) & 3, sym);
        short hd = (short)prev_up, hu = (short)up_h;
        uint32_t rec = 0;
        const uint32_t jkey = s + 1;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const short S = (a[r] == sym) ? SM : SX;
            const short D = (short)(hd + S);
            const short U = (short)(hu + CU);
            const short L = (short)(Hp[r] + CL);
            short T = D > U ? D : U;
            T = T > L ? T : L;
            T = T > 0 ? T : (short)0;
            const short H4 = (short)(T & ~3);
            rec = lshl2_or(rec, (uint32_t)(T & 3));
            if (KEY) bh[r] = max(bh[r], ((uint32_t)(uint16_t)H4 << 14) | jkey);
            hd = Hp[r]; Hp[r] = H4; hu = H4;
        }
        prev_up = up_h;
        hl = Hp[R - 1];
        acc ^= rec;
    }
    for (int r = 0; r < R; ++r) acc += bh[r] + Hp[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
template <int R, int KEY, int SUB>
int run16(const char* name, int* din, uint32_t* dout, int blocks, int steps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((cells16<R, KEY, SUB>), dim3(blocks), dim3(256), 0, 0, din, dout, steps);
    CHECK(hipDeviceSynchronize());
    hipEventRecord(e0);
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL((cells16<R, KEY, SUB>), dim3(blocks), dim3(256), 0, 0, din, dout, steps);
    hipEventRecord(e1);
    CHECK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double cells = 3.0 * blocks * 256.0 * R * steps;
    printf("%-34s blocks %6d  %8.1f GCUPS  %.3f ms\n", name, blocks, cells / (ms * 1e-3) / 1e9, ms / 3);
    return 0;
}

template <int R, int FLAGS, int KEY, int DPP>
int run(const char* name, int* din, uint32_t* dout, int blocks, int steps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((cells<R, FLAGS, KEY, DPP>), dim3(blocks), dim3(256), 0, 0, din, dout, steps);
    CHECK(hipDeviceSynchronize());
    hipEventRecord(e0);
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL((cells<R, FLAGS, KEY, DPP>), dim3(blocks), dim3(256), 0, 0, din, dout, steps);
    hipEventRecord(e1);
    CHECK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double cells = 3.0 * blocks * 256.0 * R * steps;
    printf("%-34s blocks %6d  %8.1f GCUPS  %.3f ms\n", name, blocks, cells / (ms * 1e-3) / 1e9, ms / 3);
    return 0;
}

int main() {
    int* din; uint32_t* dout;
    CHECK(hipMalloc(&din, 4096 * 4));
    CHECK(hipMalloc(&dout, 1 << 24));
    int h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (i * 2654435761u) >> 7;
    CHECK(hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice));
    const int steps = 4096;
    for (int blocks : {2048, 4096}) {
        run16<16, 1, 0>("R16 tagged16 key", din, dout, blocks, steps);
        run16<16, 0, 0>("R16 tagged16 nokey", din, dout, blocks, steps);
        run<16, 1, 1, 1>("R16 addc-flags key dpp", din, dout, blocks, steps);
        run<16, 2, 1, 1>("R16 C-flags key dpp", din, dout, blocks, steps);
        run<16, 0, 1, 1>("R16 no-flags key dpp", din, dout, blocks, steps);
        run<16, 1, 0, 1>("R16 addc-flags nokey dpp", din, dout, blocks, steps);
        run<16, 0, 0, 1>("R16 H only dpp", din, dout, blocks, steps);
        run<16, 1, 1, 0>("R16 addc-flags key nodpp", din, dout, blocks, steps);
        run<8, 1, 1, 1>("R8 addc-flags key dpp", din, dout, blocks, steps);
        run<32, 1, 1, 1>("R32 addc-flags key dpp", din, dout, blocks, steps);
    }
    return 0;
}
