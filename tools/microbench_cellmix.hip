// Cell-level issue microbenchmark for the T16 fill (not part of the product): R = 32 rows per lane
// in registers, one DPP row-above shift per step, the exact inline-asm cell of each variant, no
// memory traffic in the loop.  argv[1] = waves per SIMD (default 2; 1024 single-wave workgroups each).
// Answers what the per-opcode additive model (tools/issue_model.py) cannot: the real issue rate
// of a MIX of fast (VOP2 16-bit) and slow (VOP3 / SDWA / 32-bit) instructions.
//   V0  previous cell: add, max, add, max, max(clamp), bfe, add, and, alignbit, max(chunk)   (10)
//   V1  SDWA cell:     add(L), sdwa add(next diag), sub_u16 clamp(U), max, max, and, alignbit,
//                      max(chunk)                                                              (8)
//   V2  V1 with bfe + add instead of the SDWA add                                    (9)
//   V3  V1 without the chunk max                                                               (7)
//   V4  V1 without the alignbit                                                                (7)
//   V5  V1 without the and (scores keep their tags: timing only)                               (7)
//   V6  V2 with one v_max3_i16 for the two maxes                                               (8)
//   V7  V6 without the chunk max (the NW / keyless form)                                       (7)
//   V8  V2 with the per-row chunk max replaced by one lane max: v_max3_u32 per two rows      (8.5)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int R = 32;

__device__ __forceinline__ uint32_t shr1(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x138, 0xf, 0xf, false);
}

template <int V>
__global__ __launch_bounds__(64) void cells(const uint32_t* in, uint32_t* out, int steps) {
    const int lane = threadIdx.x;
    uint32_t tab[R], Hp[R], cm[R], cp[R / 4];
#pragma unroll
    for (int r = 0; r < R; ++r) { tab[r] = in[(lane * 7 + r) & 1023]; Hp[r] = 0; cm[r] = 0; }
#pragma unroll
    for (int k = 0; k < R / 4; ++k) cp[k] = in[(lane * 3 + k) & 1023];
    uint32_t hl = 0, sym = (lane & 3) * 8, prev_up = 0, rec = 0, acc = 0;
    const uint32_t CU = 2, CL = 0xfffd;
    for (int s = 0; s < steps; ++s) {
        const uint32_t up_h = shr1(in[s & 1023], hl);
        sym = shr1((uint32_t)((s * 7) & 3) * 8, sym);
        uint32_t hu = up_h, dcur;
        asm volatile("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(dcur) : "v"(tab[0]), "v"(sym), "v"(prev_up));
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t t0, t1, dn = 0;
            const uint32_t tabn = tab[r + 1 < R ? r + 1 : r];
            const uint32_t pw = cp[(r + 1 < R ? r + 1 : r) / 4];
            if constexpr (V == 0) {
                asm volatile("v_add_u16 %[t1], %[cu], %[hu]\n\tv_max_i16 %[t0], %[dr], %[t1]\n\t"
                             "v_add_u16 %[t1], %[cl], %[hp]\n\tv_max_i16 %[t0], %[t1], %[t0]\n\t"
                             "v_max_i16 %[t0], 0, %[t0]\n\tv_bfe_i32 %[dn], %[tabn], %[sym], 8\n\t"
                             "v_add_u16 %[dn], %[hp], %[dn]\n\tv_and_b32 %[hp], -4, %[t0]\n\t"
                             "v_alignbit_b32 %[rec], %[t0], %[rec], 2\n\tv_max_i16 %[cm], %[cm], %[hp]"
                             : [t0] "=&v"(t0), [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r]), [rec] "+v"(rec), [cm] "+v"(cm[r])
                             : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL), [tabn] "v"(tabn), [sym] "v"(sym));
            } else if constexpr (V == 1 || V == 3 || V == 4 || V == 5) {
#define MB_HEAD "v_add_u16 %[t0], %[cl], %[hp]\n\t" \
    "v_add_u16_sdwa %[dn], %[hp], sext(%[pw]) dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:BYTE_%c[kb]\n\t" \
    "v_sub_u16_e64 %[t1], %[hu], %[cu] clamp\n\t" \
    "v_max_i16 %[t0], %[dr], %[t0]\n\tv_max_i16 %[t0], %[t1], %[t0]\n\t"
#define MB_AND "v_and_b32 %[hp], -4, %[t0]\n\t"
#define MB_ALIGN "v_alignbit_b32 %[rec], %[t0], %[rec], 2\n\t"
#define MB_CM "v_max_i16 %[cm], %[cm], %[hp]\n\t"
#define MB_OPS : [t0] "=&v"(t0), [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r]), [rec] "+v"(rec), [cm] "+v"(cm[r]) \
               : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL), [pw] "v"(pw), [kb] "i"((r + 1) & 3)
                if constexpr (V == 1) asm volatile(MB_HEAD MB_AND MB_ALIGN MB_CM MB_OPS);
                else if constexpr (V == 3) asm volatile(MB_HEAD MB_AND MB_ALIGN MB_OPS);
                else if constexpr (V == 4) asm volatile(MB_HEAD MB_AND MB_CM MB_OPS);
                else asm volatile(MB_HEAD MB_ALIGN MB_CM MB_OPS);
            } else if constexpr (V == 8) {
                asm volatile("v_add_u16 %[t0], %[cl], %[hp]\n\t"
                             "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\tv_add_u16 %[dn], %[hp], %[dn]\n\t"
                             "v_sub_u16_e64 %[t1], %[hu], %[cu] clamp\n\t"
                             "v_max_i16 %[t0], %[dr], %[t0]\n\tv_max_i16 %[t0], %[t1], %[t0]\n\t"
                             "v_and_b32 %[hp], -4, %[t0]\n\t"
                             "v_alignbit_b32 %[rec], %[t0], %[rec], 2"
                             : [t0] "=&v"(t0), [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r]), [rec] "+v"(rec)
                             : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL), [tabn] "v"(tabn), [sym] "v"(sym));
                if (r & 1) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(cm[0]) : "v"(Hp[r - 1 >= 0 ? r - 1 : 0]), "v"(Hp[r]));
            } else if constexpr (V == 6 || V == 7) {
#define MB6 "v_add_u16 %[t0], %[cl], %[hp]\n\t" \
    "v_sub_u16_e64 %[t1], %[hu], %[cu] clamp\n\t" \
    "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\tv_add_u16 %[dn], %[hp], %[dn]\n\t" \
    "v_max3_i16 %[t0], %[dr], %[t0], %[t1]\n\t" \
    "v_and_b32 %[hp], -4, %[t0]\n\t" \
    "v_alignbit_b32 %[rec], %[t0], %[rec], 2\n\t"
#define MB6_OPS : [t0] "=&v"(t0), [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r]), [rec] "+v"(rec), [cm] "+v"(cm[r]) \
               : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL), [tabn] "v"(tabn), [sym] "v"(sym)
                if constexpr (V == 6) asm volatile(MB6 "v_max_i16 %[cm], %[cm], %[hp]" MB6_OPS);
                else asm volatile(MB6 MB6_OPS);
            } else {
                asm volatile("v_add_u16 %[t0], %[cl], %[hp]\n\t"
                             "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\tv_add_u16 %[dn], %[hp], %[dn]\n\t"
                             "v_sub_u16_e64 %[t1], %[hu], %[cu] clamp\n\t"
                             "v_max_i16 %[t0], %[dr], %[t0]\n\tv_max_i16 %[t0], %[t1], %[t0]\n\t"
                             "v_and_b32 %[hp], -4, %[t0]\n\t"
                             "v_alignbit_b32 %[rec], %[t0], %[rec], 2\n\t"
                             "v_max_i16 %[cm], %[cm], %[hp]"
                             : [t0] "=&v"(t0), [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r]), [rec] "+v"(rec), [cm] "+v"(cm[r])
                             : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL), [tabn] "v"(tabn), [sym] "v"(sym));
            }
            dcur = dn;
            hu = Hp[r];
        }
        prev_up = up_h;
        hl = Hp[R - 1];
        acc ^= rec;
    }
    uint32_t x = acc ^ hl;
#pragma unroll
    for (int r = 0; r < R; ++r) x ^= cm[r] + Hp[r];
    out[blockIdx.x * 64 + lane] = x;
}

int main(int argc, char** argv) {
    const int wps = argc > 1 ? atoi(argv[1]) : 2;
    const int nblk = 1024 * wps;
    uint32_t *din, *dout;
    if (hipMalloc(&din, 4096 * 4) != hipSuccess || hipMalloc(&dout, (size_t)nblk * 64 * 4) != hipSuccess) return 1;
    if (hipMemset(din, 1, 4096 * 4) != hipSuccess) return 1;
    typedef void (*kfn)(const uint32_t*, uint32_t*, int);
    struct K { const char* name; kfn f; int ops; } ks[] = {
        {"V0 previous cell (10 ops)", cells<0>, 10}, {"V1 SDWA cell (8 ops)", cells<1>, 8},
        {"V2 bfe+add cell (9 ops)", cells<2>, 9}, {"V3 V1 - chunk max (7)", cells<3>, 7},
        {"V4 V1 - alignbit (7)", cells<4>, 7}, {"V5 V1 - and (7)", cells<5>, 7},
        {"V6 V2 with max3 (8)", cells<6>, 8}, {"V7 V6 - chunk max (7)", cells<7>, 7},
        {"V8 shipped: V2 + lane max3 (8.5)", cells<8>, 8}};
    const int steps = 4000;
    for (auto& k : ks) {
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            hipLaunchKernelGGL(k.f, dim3(nblk), dim3(64), 0, 0, din, dout, 100);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(nblk), dim3(64), 0, 0, din, dout, steps);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double cells = (double)nblk * 64 * R * steps;
        printf("%-30s %8.3f ms  %8.1f GCUPS-equivalent  %.2f cycles/lane-cell@2.4GHz\n", k.name, best,
               cells / best / 1e6, 1024 * 2.4e9 * best * 1e-3 / (cells / 64));
    }
    return 0;
}
