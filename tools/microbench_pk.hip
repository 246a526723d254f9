// Packed two-pair cell microbenchmark (not part of the product): can a lane run the T16 cell of
// TWO independent pairs at once, one per 16-bit half of each register, with VOP3P (v_pk_*) ops?
// R = 32 rows per lane in registers, one DPP row-above shift (both pairs) and two DPP column
// profile shifts per step, no memory traffic in the loop.  argv[1] = waves per SIMD (default 3).
//   S8  shipped scalar cell (V8 of microbench_cellmix.hip): 8.5 ops per cell
//   P1  packed cell per row (2 cells): perm (substitution bytes of both pairs, high byte of each
//       half) + pk_ashr 8 + pk_add (next row's diag), pk_add (left), pk_sub clamp (up),
//       2 pk_max, and (strip both tags), and (both tags) + lshl_add (record), pk_max (chunk max)
//                                                                               11 ops / 2 cells
//   P2  P1 without the chunk max                                               10 ops / 2 cells
//   P3  P1 without the pk_ashr (a signed perm would need no shift; timing only)  10 ops / 2 cells
//   P4  P1 with the record push as two v_alignbit (lo tag) / v_perm (hi) forms  timing variant
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
    uint32_t tab[R], Hp[R], sel[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        tab[r] = in[(lane * 7 + r) & 1023];
        sel[r] = 0x000c000cu | ((uint32_t)(r & 3) << 8) | ((uint32_t)(4 + ((r + lane) & 3)) << 24);
        Hp[r] = 0;
    }
    uint32_t hl = 0, sym = (lane & 3) * 8, colA = in[lane & 1023], colB = in[(lane + 5) & 1023];
    uint32_t prev_up = 0, rec = 0, acc = 0, cm = 0;
    const uint32_t CU = 0x00020002u, CL = 0xfffdfffdu, SM = 0xfffcfffcu;
    for (int s = 0; s < steps; ++s) {
        const uint32_t up_h = shr1(in[s & 1023], hl);
        uint32_t hu = up_h, dcur;
        if constexpr (V == 0) {
            sym = shr1((uint32_t)((s * 7) & 3) * 8, sym);
            asm volatile("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(dcur) : "v"(tab[0]), "v"(sym), "v"(prev_up));
        } else {
            colA = shr1(in[(s + 3) & 1023], colA);
            colB = shr1(in[(s + 9) & 1023], colB);
            asm volatile("v_perm_b32 %0, %1, %2, %3\n\tv_pk_ashrrev_i16 %0, 8, %0\n\tv_pk_add_u16 %0, %4, %0"
                         : "=&v"(dcur) : "v"(colB), "v"(colA), "v"(sel[0]), "v"(prev_up));
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t t0, t1, dn = 0;
            const uint32_t tabn = tab[r + 1 < R ? r + 1 : r];
            const uint32_t seln = sel[r + 1 < R ? r + 1 : r];
            if constexpr (V == 0) {
                asm volatile("v_add_u16 %[t0], %[cl], %[hp]\n\t"
                             "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\tv_add_u16 %[dn], %[hp], %[dn]\n\t"
                             "v_sub_u16_e64 %[t1], %[hu], %[cu] clamp\n\t"
                             "v_max_i16 %[t0], %[dr], %[t0]\n\tv_max_i16 %[t0], %[t1], %[t0]\n\t"
                             "v_and_b32 %[hp], -4, %[t0]\n\t"
                             "v_alignbit_b32 %[rec], %[t0], %[rec], 2"
                             : [t0] "=&v"(t0), [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r]), [rec] "+v"(rec)
                             : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(2u), [cl] "s"(0xfffdu), [tabn] "v"(tabn), [sym] "v"(sym));
                if (r & 1) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(cm) : "v"(Hp[r - 1 >= 0 ? r - 1 : 0]), "v"(Hp[r]));
            } else {
#define PK_LEFT "v_pk_add_u16 %[t0], %[cl], %[hp]\n\t"
#define PK_NEXT "v_perm_b32 %[dn], %[cb], %[ca], %[seln]\n\tv_pk_ashrrev_i16 %[dn], 8, %[dn]\n\tv_pk_add_u16 %[dn], %[hp], %[dn]\n\t"
#define PK_NEXT3 "v_perm_b32 %[dn], %[cb], %[ca], %[seln]\n\tv_pk_add_u16 %[dn], %[hp], %[dn]\n\t"
#define PK_UP "v_pk_sub_u16 %[t1], %[hu], %[cu] clamp\n\t"
#define PK_MAX "v_pk_max_i16 %[t0], %[dr], %[t0]\n\tv_pk_max_i16 %[t0], %[t1], %[t0]\n\t"
#define PK_TAIL "v_and_b32 %[hp], %[sm], %[t0]\n\tv_and_b32 %[t1], 0x30003, %[t0]\n\tv_lshl_add_u32 %[rec], %[rec], 2, %[t1]\n\t"
#define PK_TAIL4 "v_and_b32 %[hp], %[sm], %[t0]\n\tv_alignbit_b32 %[rec], %[t0], %[rec], 2\n\tv_perm_b32 %[t1], %[t0], %[rec], %[cu]\n\t"
#define PK_CM "v_pk_max_i16 %[cm], %[cm], %[hp]\n\t"
#define PK_OPS : [t0] "=&v"(t0), [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r]), [rec] "+v"(rec), [cm] "+v"(cm) \
               : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL), [sm] "s"(SM), [ca] "v"(colA), [cb] "v"(colB), [seln] "v"(seln)
                if constexpr (V == 1) asm volatile(PK_LEFT PK_NEXT PK_UP PK_MAX PK_TAIL PK_CM PK_OPS);
                else if constexpr (V == 2) asm volatile(PK_LEFT PK_NEXT PK_UP PK_MAX PK_TAIL PK_OPS);
                else if constexpr (V == 3) asm volatile(PK_LEFT PK_NEXT3 PK_UP PK_MAX PK_TAIL PK_CM PK_OPS);
                else asm volatile(PK_LEFT PK_NEXT PK_UP PK_MAX PK_TAIL4 PK_CM PK_OPS);
            }
            dcur = dn;
            hu = Hp[r];
        }
        prev_up = up_h;
        hl = Hp[R - 1];
        acc ^= rec;
    }
    uint32_t x = acc ^ hl ^ cm;
#pragma unroll
    for (int r = 0; r < R; ++r) x ^= Hp[r];
    out[blockIdx.x * 64 + lane] = x;
}

int main(int argc, char** argv) {
    const int wps = argc > 1 ? atoi(argv[1]) : 3;
    const int nblk = 1024 * wps;
    uint32_t *din, *dout;
    if (hipMalloc(&din, 4096 * 4) != hipSuccess || hipMalloc(&dout, (size_t)nblk * 64 * 4) != hipSuccess) return 1;
    if (hipMemset(din, 1, 4096 * 4) != hipSuccess) return 1;
    typedef void (*kfn)(const uint32_t*, uint32_t*, int);
    struct K { const char* name; kfn f; int cells_per_row; } ks[] = {
        {"S8 shipped scalar (8.5/cell)", cells<0>, 1}, {"P1 packed full (11/2 cells)", cells<1>, 2},
        {"P2 P1 - chunk max (10/2)", cells<2>, 2}, {"P3 P1 - ashr (10/2)", cells<3>, 2},
        {"P4 P1 alignbit+perm rec (11/2)", cells<4>, 2}};
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
        const double cells = (double)nblk * 64 * R * k.cells_per_row * steps;
        printf("wps=%d %-32s %8.3f ms  %8.1f GCUPS-equivalent  %.2f cycles/lane-cell@2.4GHz\n", wps, k.name, best,
               cells / best / 1e6, 1024 * 2.4e9 * best * 1e-3 / (cells / 64));
    }
    return 0;
}
