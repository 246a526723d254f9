// Cell-level issue microbenchmark for the SCORE-ONLY T16 fill (not part of the product): R rows per
// lane in registers, one DPP row-above shift per step, the exact inline-asm cell of each variant,
// no memory traffic in the loop.  argv[1] = waves per SIMD (1024 * wps single-wave workgroups).
//   S8   shipped tagged cell (record push + strip): add, bfe, add, sub clamp, max, max, and,
//        alignbit + v_max3_u32 per two rows                                                 (8.5)
//   SO   score-only: add(L), bfe + add(next diag), sub clamp(U), max, max + max3 per 2 rows (6.5)
//   SO4  SO with the lane maximum over every other row only (max3 per 4 rows)               (6.25)
//   SO0  SO without the lane maximum (lower bound)                                          (6)
//   SOB  SO + the lane's last row packed per step into a 16-bit stream (v_perm every 2 steps)
//   SG   shipped round-4 shared-gap cell: max(U, L), bfe + add (next diag), sub clamp, max      (5)
//   SD   shared-gap cell with the substitution by v_dot4_i32_i8 (profile bytes . one-hot column
//        code + Hp = next diag in one op): max, dot4, sub clamp, max                          (4)
//   SG2 / SG4  SG with 2 / 4 cells per inline-asm statement (no s_nop 0 between the cells)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ uint32_t shr1(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x138, 0xf, 0xf, false);
}

template <int V, int R>
__global__ __launch_bounds__(64) void cells(const uint32_t* in, uint32_t* out, int steps) {
    const int lane = threadIdx.x;
    uint32_t tab[R], Hp[R];
#pragma unroll
    for (int r = 0; r < R; ++r) { tab[r] = in[(lane * 7 + r) & 1023]; Hp[r] = 0; }
    uint32_t hl = 0, sym = (lane & 3) * 8, prev_up = 0, rec = 0, acc = 0, cml = 0, bot = 0, oh = 1u << ((lane & 3) * 8);
    const uint32_t CU = 2, CL = 0xfffd, CU1 = 1, CL1 = 0xffff;
    if constexpr (V == 9 || V == 10) {
        // SGS: the SG cell with the waves of a SIMD started out of phase (the same work)
        const int ph = (int)(blockIdx.x / 1024) % 4;   // (workgroups are spread over the SIMDs in launch order)
        for (int k = 0; k < ph * (V == 9 ? 8 : 40); ++k) __builtin_amdgcn_s_sleep(127);
    }
    for (int s = 0; s < steps; ++s) {
        const uint32_t up_h = shr1(in[s & 1023], hl);
        if constexpr (V == 6) oh = shr1(1u << (((s * 7) & 3) * 8), oh);
        else sym = shr1((uint32_t)((s * 7) & 3) * 8, sym);
        uint32_t hu = up_h, dcur;
        asm volatile("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(dcur) : "v"(tab[0]), "v"(sym), "v"(prev_up));
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t t0, t1, dn = 0;
            const uint32_t tabn = tab[r + 1 < R ? r + 1 : r];
            if constexpr (V == 5 || V == 9 || V == 10) {
                asm volatile("v_max_i16 %[t1], %[hu], %[hp]\n\t"
                             "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\tv_add_u16 %[dn], %[hp], %[dn]\n\t"
                             "v_sub_u16_e64 %[t1], %[t1], %[cu] clamp\n\t"
                             "v_max_i16 %[hp], %[dr], %[t1]"
                             : [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                             : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU1), [tabn] "v"(tabn), [sym] "v"(sym));
                (void)t0;
                if (r % 8 == 7 && (s & 3) == 3) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r - 4]), "v"(Hp[r]));
            } else if constexpr (V == 7 || V == 8) {
                // SG with K = 2 (V7) or 4 (V8) cells per asm statement: the compiler pads an
                // s_nop 0 between consecutive asm statements, one per cell in SG
                constexpr int K = V == 7 ? 2 : 4;
                if (r % K == 0) {
#define SG_C(HU, HP, DR, DN, TB)                                                                    \
    "v_max_i16 %[t1], " HU ", " HP "\n\t"                                                           \
    "v_bfe_i32 " DN ", " TB ", %[sym], 8\n\t"                                                       \
    "v_add_u16 " DN ", " HP ", " DN "\n\t"                                                          \
    "v_sub_u16_e64 %[t1], %[t1], %[cu] clamp\n\t"                                                   \
    "v_max_i16 " HP ", " DR ", %[t1]\n\t"
                    uint32_t d0, d1;
                    const uint32_t t1_ = tab[r + 1 < R ? r + 1 : R - 1], t2_ = tab[r + 2 < R ? r + 2 : R - 1];
                    if constexpr (K == 2) {
                        asm volatile(SG_C("%[hu]", "%[h0]", "%[dr]", "%[d0]", "%[ta]") SG_C("%[h0]", "%[h1]", "%[d0]", "%[d1]", "%[tb]")
                                     : [t1] "=&v"(t1), [d0] "=&v"(d0), [d1] "=&v"(d1), [h0] "+v"(Hp[r]), [h1] "+v"(Hp[r + 1 < R ? r + 1 : r])
                                     : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU1), [ta] "v"(t1_), [tb] "v"(t2_), [sym] "v"(sym));
                        dn = d1;
                    } else {
                        const uint32_t t3_ = tab[r + 3 < R ? r + 3 : R - 1], t4_ = tab[r + 4 < R ? r + 4 : R - 1];
                        asm volatile(SG_C("%[hu]", "%[h0]", "%[dr]", "%[d0]", "%[ta]") SG_C("%[h0]", "%[h1]", "%[d0]", "%[d1]", "%[tb]")
                                     SG_C("%[h1]", "%[h2]", "%[d1]", "%[d0]", "%[tc]") SG_C("%[h2]", "%[h3]", "%[d0]", "%[d1]", "%[td]")
                                     : [t1] "=&v"(t1), [d0] "=&v"(d0), [d1] "=&v"(d1), [h0] "+v"(Hp[r]), [h1] "+v"(Hp[(r + 1) % R]),
                                       [h2] "+v"(Hp[(r + 2) % R]), [h3] "+v"(Hp[(r + 3) % R])
                                     : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU1), [ta] "v"(t1_), [tb] "v"(t2_), [tc] "v"(t3_), [td] "v"(t4_), [sym] "v"(sym));
                        dn = d1;
                    }
#undef SG_C
                    if ((r + K) % 8 == 0 && (s & 3) == 3) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r + K - 5]), "v"(Hp[r + K - 1]));
                    dcur = dn;
                    hu = Hp[r + K - 1];
                }
                continue;
            } else if constexpr (V == 6) {
                asm volatile("v_max_i16 %[t1], %[hu], %[hp]\n\t"
                             "v_dot4_i32_i8 %[dn], %[tabn], %[oh], %[hp]\n\t"
                             "v_sub_u16_e64 %[t1], %[t1], %[cu] clamp\n\t"
                             "v_max_i16 %[hp], %[dr], %[t1]"
                             : [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                             : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU1), [tabn] "v"(tabn), [oh] "v"(oh));
                (void)t0;
                if (r % 8 == 7 && (s & 3) == 3) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r - 4]), "v"(Hp[r]));
            } else if constexpr (V == 0) {
                asm volatile("v_add_u16 %[t0], %[cl], %[hp]\n\t"
                             "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\tv_add_u16 %[dn], %[hp], %[dn]\n\t"
                             "v_sub_u16_e64 %[t1], %[hu], %[cu] clamp\n\t"
                             "v_max_i16 %[t0], %[dr], %[t0]\n\tv_max_i16 %[t0], %[t1], %[t0]\n\t"
                             "v_and_b32 %[hp], -4, %[t0]\n\t"
                             "v_alignbit_b32 %[rec], %[t0], %[rec], 2"
                             : [t0] "=&v"(t0), [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r]), [rec] "+v"(rec)
                             : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL), [tabn] "v"(tabn), [sym] "v"(sym));
                if (r & 1) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r - 1 >= 0 ? r - 1 : 0]), "v"(Hp[r]));
            } else {
                // score-only: Hp is H itself; next row's diagonal from the old Hp, then the cell
                asm volatile("v_add_u16 %[t0], %[cl], %[hp]\n\t"
                             "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\tv_add_u16 %[dn], %[hp], %[dn]\n\t"
                             "v_sub_u16_e64 %[t1], %[hu], %[cu] clamp\n\t"
                             "v_max_i16 %[t0], %[dr], %[t0]\n\tv_max_i16 %[hp], %[t1], %[t0]"
                             : [t0] "=&v"(t0), [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                             : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU1), [cl] "s"(CL1), [tabn] "v"(tabn), [sym] "v"(sym));
                if constexpr (V == 1 || V == 4) {
                    if (r & 1) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r - 1 >= 0 ? r - 1 : 0]), "v"(Hp[r]));
                } else if constexpr (V == 2) {
                    if ((r & 3) == 3) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r - 2 >= 0 ? r - 2 : 0]), "v"(Hp[r]));
                }
            }
            dcur = dn;
            hu = Hp[r];
        }
        prev_up = up_h;
        hl = Hp[R - 1];
        if constexpr (V == 4) {
            // the lane's last row, two steps per dword (v_perm once per two steps)
            if (s & 1) { asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(bot) : "v"(hl), "s"(0x05040100u)); acc ^= bot; }
            else bot = hl;
        }
        acc ^= rec;
    }
    uint32_t x = acc ^ hl ^ cml ^ oh;
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
    struct K { const char* name; kfn f; int R; } ks[] = {
        {"S8 shipped tagged R32 (8.5)", cells<0, 32>, 32},
        {"SO score-only R32 (6.5)", cells<1, 32>, 32},
        {"SO4 score-only R32 max/4 (6.25)", cells<2, 32>, 32},
        {"SO0 score-only R32 no max (6)", cells<3, 32>, 32},
        {"SOB SO + bottom-row stream R32", cells<4, 32>, 32},
        {"SG shared-gap shipped R32 (5)", cells<5, 32>, 32},
        {"SD shared-gap dot4 R32 (4)", cells<6, 32>, 32},
        {"SGS SG, waves out of phase (8 x 8K cyc)", cells<9, 32>, 32},
        {"SGT SG, waves out of phase (40 x 8K cyc)", cells<10, 32>, 32},
        {"SG2 SG, 2 cells per asm R32 (5)", cells<7, 32>, 32},
        {"SG4 SG, 4 cells per asm R32 (5)", cells<8, 32>, 32},
        {"SD shared-gap dot4 R16 (4)", cells<6, 16>, 16},
        {"SO score-only R16 (6.5)", cells<1, 16>, 16},
        {"SO score-only R64 (6.5)", cells<1, 64>, 64},
    };
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
        const double cells = (double)nblk * 64 * k.R * steps;
        printf("wps=%d %-34s %8.3f ms  %8.1f GCUPS-equivalent  %.2f cycles/lane-cell@2.4GHz\n", wps, k.name, best,
               cells / best / 1e6, 1024 * 2.4e9 * best * 1e-3 / (cells / 64));
    }
    return 0;
}
