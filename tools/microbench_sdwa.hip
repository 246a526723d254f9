// gfx950 VALU issue rate of SDWA / VOP3-encoded 16-bit ops next to their plain VOP2 forms.
// Same harness as microbench_ops2.hip: 8 independent chains per lane, 8 waves per SIMD.
// Question it answers: can the T16 cell take its substitution byte with one SDWA v_add_u16
// (src1_sel:BYTE_k, sext) at the fast 16-bit issue rate, instead of v_bfe_i32 + v_add_u16?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CH8(I)                                                                              \
    I("%0") I("%1") I("%2") I("%3") I("%4") I("%5") I("%6") I("%7")
#define KERNEL(NAME, BODY)                                                                  \
    __global__ __launch_bounds__(256) void k_##NAME(uint32_t* out, int iters, uint32_t seed) { \
        uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9,   \
                 a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15, b = seed ^ 0x1234, c = seed * 77;   \
        for (int i = 0; i < iters; ++i)                                                     \
            asm volatile(CH8(BODY)                                                          \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),      \
                           "+v"(a6), "+v"(a7)                                               \
                         : "v"(b), "v"(c));                                                 \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
    }

#define I_ADD16(x) "v_add_u16 " x ", " x ", %8\n\t"
#define I_ADD16_E64(x) "v_add_u16_e64 " x ", " x ", %8\n\t"
#define I_ADD16_SDWA_B1(x)                                                                  \
    "v_add_u16_sdwa " x ", " x ", sext(%8) dst_sel:WORD_0 dst_unused:UNUSED_PAD "           \
    "src0_sel:WORD_0 src1_sel:BYTE_1\n\t"
#define I_ADD16_SDWA_B3(x)                                                                  \
    "v_add_u16_sdwa " x ", " x ", sext(%8) dst_sel:WORD_0 dst_unused:UNUSED_PAD "           \
    "src0_sel:WORD_0 src1_sel:BYTE_3\n\t"
#define I_ADD16_SDWA_W(x)                                                                   \
    "v_add_u16_sdwa " x ", " x ", %8 dst_sel:WORD_0 dst_unused:UNUSED_PAD "                 \
    "src0_sel:WORD_0 src1_sel:WORD_1\n\t"
#define I_MAX16(x) "v_max_i16 " x ", " x ", %8\n\t"
#define I_MAX16_SDWA(x)                                                                     \
    "v_max_i16_sdwa " x ", " x ", %8 dst_sel:WORD_0 dst_unused:UNUSED_PAD "                 \
    "src0_sel:WORD_0 src1_sel:WORD_0\n\t"
#define I_MOV_SDWA_PRES(x)                                                                  \
    "v_mov_b32_sdwa " x ", %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\n\t"
#define I_AND_SDWA(x)                                                                       \
    "v_and_b32_sdwa " x ", " x ", %8 dst_sel:WORD_0 dst_unused:UNUSED_PAD "                 \
    "src0_sel:WORD_0 src1_sel:WORD_0\n\t"
#define I_AND(x) "v_and_b32 " x ", " x ", %8\n\t"
#define I_LSHL16(x) "v_lshlrev_b16 " x ", 2, " x "\n\t"
#define I_OR_SDWA(x)                                                                        \
    "v_or_b32_sdwa " x ", " x ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD "                   \
    "src0_sel:DWORD src1_sel:BYTE_0\n\t"
#define I_SUB16(x) "v_sub_u16 " x ", " x ", %8\n\t"
#define I_MIN16(x) "v_min_i16 " x ", " x ", %8\n\t"
#define I_SUBCLAMP(x) "v_sub_u16_e64 " x ", " x ", %8 clamp\n\t"
#define I_PERM(x)"v_perm_b32 " x ", " x ", %8, %9\n\t"

KERNEL(add_u16, I_ADD16)
KERNEL(add_u16_e64, I_ADD16_E64)
KERNEL(add_u16_sdwa_byte1_sext, I_ADD16_SDWA_B1)
KERNEL(add_u16_sdwa_byte3_sext, I_ADD16_SDWA_B3)
KERNEL(add_u16_sdwa_word1, I_ADD16_SDWA_W)
KERNEL(max_i16, I_MAX16)
KERNEL(max_i16_sdwa, I_MAX16_SDWA)
KERNEL(mov_b32_sdwa_preserve, I_MOV_SDWA_PRES)
KERNEL(and_b32, I_AND)
KERNEL(and_b32_sdwa, I_AND_SDWA)
KERNEL(or_b32_sdwa_byte0, I_OR_SDWA)
KERNEL(lshlrev_b16, I_LSHL16)
KERNEL(sub_u16, I_SUB16)
KERNEL(min_i16, I_MIN16)
KERNEL(perm_b32, I_PERM)
KERNEL(sub_u16_e64_clamp, I_SUBCLAMP)

typedef void (*kfn)(uint32_t*, int, uint32_t);
struct K { const char* name; kfn f; int per; };

int main() {
    uint32_t* dout;
    hipMalloc(&dout, 2048 * 256 * 4);
    K ks[] = {{"add_u16", k_add_u16, 8},
              {"add_u16_e64", k_add_u16_e64, 8},
              {"add_u16_sdwa_byte1_sext", k_add_u16_sdwa_byte1_sext, 8},
              {"add_u16_sdwa_byte3_sext", k_add_u16_sdwa_byte3_sext, 8},
              {"add_u16_sdwa_word1", k_add_u16_sdwa_word1, 8},
              {"max_i16", k_max_i16, 8},
              {"max_i16_sdwa", k_max_i16_sdwa, 8},
              {"mov_b32_sdwa_preserve", k_mov_b32_sdwa_preserve, 8},
              {"and_b32", k_and_b32, 8},
              {"and_b32_sdwa", k_and_b32_sdwa, 8},
              {"or_b32_sdwa_byte0", k_or_b32_sdwa_byte0, 8},
              {"lshlrev_b16", k_lshlrev_b16, 8},
              {"sub_u16", k_sub_u16, 8},
              {"min_i16", k_min_i16, 8},
              {"perm_b32", k_perm_b32, 8},
              {"sub_u16_e64_clamp", k_sub_u16_e64_clamp, 8}};
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const double clk = 2.4e9;
    const int iters = 20000;
    for (auto& k : ks) {
        float best = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k.f, dim3(2048), dim3(256), 0, 0, dout, 50, 1u);
            hipDeviceSynchronize();
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(2048), dim3(256), 0, 0, dout, iters, 1u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double winst = 2048.0 * 4 * iters * k.per;
        printf("%-28s %7.3f ms  %.3f wave-instr/cyc/SIMD@2.4GHz\n", k.name, best,
               winst / (prop.multiProcessorCount * 4.0 * best * 1e-3 * clk));
    }
    return 0;
}
