// VALU issue-rate microbenchmark on gfx950: 8 independent chains of one opcode per lane, many
// waves per SIMD.  Reports wave64 instructions per cycle per SIMD (at the measured clock).
// Not part of the product.  hipcc -O3 --offload-arch=gfx950 tools/microbench_issue.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define OPK(NAME, INSN)                                                                       \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, int iters, uint32_t seed) {    \
        uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9,  \
                 a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15, b = seed ^ 0x1234;                  \
        for (int i = 0; i < iters; ++i) {                                                     \
            asm volatile(INSN " %0, %0, %8\n\t" INSN " %1, %1, %8\n\t" INSN " %2, %2, %8\n\t"  \
                         INSN " %3, %3, %8\n\t" INSN " %4, %4, %8\n\t" INSN " %5, %5, %8\n\t"  \
                         INSN " %6, %6, %8\n\t" INSN " %7, %7, %8"                             \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                           "+v"(a7)                                                           \
                         : "v"(b));                                                           \
        }                                                                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;   \
    }

OPK(k_add_u32, "v_add_u32")
OPK(k_max_i32, "v_max_i32")
OPK(k_add_f32, "v_add_f32")
OPK(k_pk_add_u16, "v_pk_add_u16")
OPK(k_pk_max_i16, "v_pk_max_i16")
#undef OPK

// 3-operand forms
#define OPK3(NAME, INSN)                                                                      \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, int iters, uint32_t seed) {    \
        uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9,  \
                 a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15, b = seed ^ 0x1234, c = seed * 77;   \
        for (int i = 0; i < iters; ++i) {                                                     \
            asm volatile(INSN " %0, %0, %8, %9\n\t" INSN " %1, %1, %8, %9\n\t" INSN " %2, %2, %8, %9\n\t" \
                         INSN " %3, %3, %8, %9\n\t" INSN " %4, %4, %8, %9\n\t" INSN " %5, %5, %8, %9\n\t" \
                         INSN " %6, %6, %8, %9\n\t" INSN " %7, %7, %8, %9"                     \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                           "+v"(a7)                                                           \
                         : "v"(b), "v"(c));                                                   \
        }                                                                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;   \
    }
OPK3(k_max3_i32b, "v_max3_i32")
OPK3(k_fma_f32, "v_fma_f32")
OPK3(k_lshl_or, "v_lshl_or_b32")

__global__ __launch_bounds__(256) void k_pk_fma_f32(uint32_t* out, int iters, uint32_t seed) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a0 = {1.f * threadIdx.x, 2.f}, a1 = a0 * 1.1f, a2 = a0 * 1.2f, a3 = a0 * 1.3f, b = {1.0001f, 0.9999f}, c = {0.5f, 0.25f};
    for (int i = 0; i < iters; ++i) {
        asm volatile("v_pk_fma_f32 %0, %0, %4, %5\n\tv_pk_fma_f32 %1, %1, %4, %5\n\tv_pk_fma_f32 %2, %2, %4, %5\n\tv_pk_fma_f32 %3, %3, %4, %5\n\t"
                     "v_pk_fma_f32 %0, %0, %4, %5\n\tv_pk_fma_f32 %1, %1, %4, %5\n\tv_pk_fma_f32 %2, %2, %4, %5\n\tv_pk_fma_f32 %3, %3, %4, %5"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b), "v"(c));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0.x + a1.y + a2.x + a3.y);
}

// v_cmp into an SGPR pair + v_addc consuming it (the flag idiom), 4 independent pairs
__global__ __launch_bounds__(256) void k_cmp_addc(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, b = seed ^ 0x1234;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_cmp_eq_u32_e64 s[40:41], %0, %4\n\tv_cmp_eq_u32_e64 s[42:43], %1, %4\n\t"
            "v_cmp_eq_u32_e64 s[44:45], %2, %4\n\tv_cmp_eq_u32_e64 s[46:47], %3, %4\n\t"
            "v_addc_co_u32_e64 %0, s[40:41], %0, %0, s[40:41]\n\tv_addc_co_u32_e64 %1, s[42:43], %1, %1, s[42:43]\n\t"
            "v_addc_co_u32_e64 %2, s[44:45], %2, %2, s[44:45]\n\tv_addc_co_u32_e64 %3, s[46:47], %3, %3, s[46:47]"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3;
}

typedef void (*kfn)(uint32_t*, int, uint32_t);

int main() {
    uint32_t* dout;
    hipMalloc(&dout, 1 << 26);
    struct { const char* name; kfn f; int per_iter; } ks[] = {
        {"v_add_u32", k_add_u32, 8}, {"v_max_i32", k_max_i32, 8}, {"v_add_f32", k_add_f32, 8},
        {"v_pk_add_u16", k_pk_add_u16, 8}, {"v_pk_max_i16", k_pk_max_i16, 8}, {"v_max3_i32", k_max3_i32b, 8},
        {"v_fma_f32", k_fma_f32, 8}, {"v_lshl_or_b32", k_lshl_or, 8}, {"v_pk_fma_f32", k_pk_fma_f32, 8},
        {"v_cmp_e64+v_addc_e64", k_cmp_addc, 8},
    };
    int dev; hipGetDevice(&dev);
    hipDeviceProp_t prop; hipGetDeviceProperties(&prop, dev);
    const double clk = prop.clockRate * 1e3;  // kHz -> Hz (max clock)
    printf("CUs %d, max clock %.0f MHz\n", prop.multiProcessorCount, clk / 1e6);
    const int iters = 20000;
    for (auto& k : ks) {
        for (int blocks : {1024, 2048}) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, dout, 100, 1u);
            hipDeviceSynchronize();
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, dout, iters, 1u);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            const double winst = (double)blocks * 4 * iters * k.per_iter;   // wave64 instructions
            const double simd_cycles = prop.multiProcessorCount * 4.0 * (ms * 1e-3) * clk;
            printf("%-24s blocks %5d  %7.3f ms  %.3f wave-instr/cycle/SIMD (at max clock)  %.1f T lane-ops/s\n",
                   k.name, blocks, ms, winst / simd_cycles, winst * 64 / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
