// Register-only microbenchmark of candidate tagged-16-bit SW cells on gfx950 (inline asm so the
// instruction mix is exact).  Not part of the product.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_cell16.hip -o build/microbench_cell16
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ int shr1(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false);
}

// SUB: 0 = v_bfe_i32 table, 1 = cmp(e64, sgpr)+cndmask(e64)
// MAX: 0 = v_max3_i16 + v_max_i16 0, 1 = 3 x v_max_i16
// KEY: 0 none, 1 lshl_or + max_u32
template <int SUB, int MAX, int KEY>
__device__ __forceinline__ void cell(uint32_t tab, uint32_t off, uint32_t& hd, uint32_t hu, uint32_t& hp,
                                     uint32_t& rec, uint32_t& bh, uint32_t jsh) {
    uint32_t S, D, U, L, T, H, k;
    if (SUB == 0) {
        asm volatile("v_bfe_i32 %0, %1, %2, 8" : "=v"(S) : "v"(tab), "v"(off));
    } else {
        asm volatile("v_cmp_eq_u32_e64 s[40:41], %1, %2\n\tv_cndmask_b32_e64 %0, -1, 7, s[40:41]"
                     : "=v"(S) : "v"(tab), "v"(off) : "s40", "s41");
    }
    asm volatile("v_add_u16 %0, %1, %2" : "=v"(D) : "v"(hd), "v"(S));
    asm volatile("v_add_u16 %0, -2, %1" : "=v"(U) : "v"(hu));
    asm volatile("v_add_u16 %0, -3, %1" : "=v"(L) : "v"(hp));
    if (MAX == 0) {
        asm volatile("v_max3_i16 %0, %1, %2, %3\n\tv_max_i16 %0, 0, %0" : "=&v"(T) : "v"(D), "v"(U), "v"(L));
    } else {
        asm volatile("v_max_i16 %0, %1, %2\n\tv_max_i16 %0, %0, %3\n\tv_max_i16 %0, 0, %0" : "=&v"(T) : "v"(D), "v"(U), "v"(L));
    }
    asm volatile("v_and_b32 %0, -4, %1" : "=v"(H) : "v"(T));
    asm volatile("v_alignbit_b32 %0, %1, %0, 2" : "+v"(rec) : "v"(T));
    if (KEY) {
        asm volatile("v_lshl_or_b32 %0, %1, 14, %2" : "=v"(k) : "v"(H), "v"(jsh));
        asm volatile("v_max_u32 %0, %0, %1" : "+v"(bh) : "v"(k));
    }
    hd = hp; hp = H;
    (void)hu;
}

template <int R, int SUB, int MAX, int KEY>
__global__ __launch_bounds__(256) void cells(const int* in, uint32_t* out, int steps) {
    const int lane = threadIdx.x & 63;
    uint32_t tab[R], Hp[R], bh[R];
    for (int r = 0; r < R; ++r) { tab[r] = in[(threadIdx.x * 7 + r) & 1023]; Hp[r] = 0; bh[r] = 0; }
    uint32_t hl = 0, sym = (lane & 3) * 8, prev_up = 0, up_seed = in[lane];
    uint32_t acc = 0;
    for (int s = 0; s < steps; ++s) {
        const uint32_t up_h = shr1(up_seed, hl);
        sym = shr1(((s * 7) & 3) * 8, sym);
        uint32_t hd = prev_up, hu = up_h;
        uint32_t rec = 0;
        const uint32_t jsh = s + 1;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            cell<SUB, MAX, KEY>(tab[r], sym, hd, hu, Hp[r], rec, bh[r], jsh);
            hu = Hp[r];
        }
        prev_up = up_h;
        hl = Hp[R - 1];
        acc ^= rec;
    }
    for (int r = 0; r < R; ++r) acc += bh[r] + Hp[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int R, int SUB, int MAX, int KEY>
int run(const char* name, int* din, uint32_t* dout, int blocks, int steps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((cells<R, SUB, MAX, KEY>), dim3(blocks), dim3(256), 0, 0, din, dout, steps);
    CHECK(hipDeviceSynchronize());
    hipEventRecord(e0);
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL((cells<R, SUB, MAX, KEY>), dim3(blocks), dim3(256), 0, 0, din, dout, steps);
    hipEventRecord(e1);
    CHECK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double cells = 3.0 * blocks * 256.0 * R * steps;
    printf("%-40s blocks %6d  %8.1f GCUPS  %.3f ms\n", name, blocks, cells / (ms * 1e-3) / 1e9, ms / 3);
    return 0;
}

// Do 16-bit VOP2 ops zero the upper half of the destination on this chip?
__global__ void hi_probe(uint32_t* out, uint32_t a) {
    uint32_t d = 0xdead0000u | (a & 0xffff), e = 0xbeef0000u, f;
    asm volatile("v_add_u16 %0, %1, 1" : "+v"(e) : "v"(d));
    asm volatile("v_max_i16 %0, %1, %2" : "=v"(f) : "v"(d), "v"(a | 0x77770000u));
    uint32_t g = 0xcafe0000u;
    asm volatile("v_max3_i16 %0, %1, %2, %3" : "+v"(g) : "v"(d), "v"(a | 0x12340000u), "v"(e));
    out[0] = e; out[1] = f; out[2] = g;
}

int main() {
    int* din; uint32_t* dout;
    CHECK(hipMalloc(&din, 4096 * 4));
    CHECK(hipMalloc(&dout, 1 << 24));
    int h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (int)((i * 2654435761u) >> 7);
    CHECK(hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(hi_probe, dim3(1), dim3(1), 0, 0, dout, 5u);
    uint32_t p[3];
    CHECK(hipMemcpy(p, dout, 12, hipMemcpyDeviceToHost));
    printf("hi-half probe: add_u16 -> %08x  max_i16 -> %08x  max3_i16 -> %08x\n", p[0], p[1], p[2]);
    const int steps = 4096;
    for (int blocks : {2048, 4096}) {
        run<16, 0, 0, 1>("R16 bfe  max3  key", din, dout, blocks, steps);
        run<16, 0, 1, 1>("R16 bfe  max16 key", din, dout, blocks, steps);
        run<16, 1, 0, 1>("R16 cmp  max3  key", din, dout, blocks, steps);
        run<16, 0, 0, 0>("R16 bfe  max3  nokey", din, dout, blocks, steps);
        run<16, 0, 1, 0>("R16 bfe  max16 nokey", din, dout, blocks, steps);
        run<8, 0, 0, 1>("R8  bfe  max3  key", din, dout, blocks, steps);
        run<32, 0, 0, 1>("R32 bfe  max3  key", din, dout, blocks, steps);
    }
    return 0;
}
