// Cell-level issue microbenchmark (not part of the product): the shipped score-only SW cell (SG,
// one pair per lane, 5 VALU per cell: 4 16-bit VOP2 + v_bfe_i32) against a packed cell that runs
// TWO pairs per lane in the 16-bit halves of every register (PK6: 6 VOP3P/perm ops per 2 cells):
//   p  = v_perm_b32(srcB, srcA, sel_r)        s(a_r, c) + 128 of both pairs (sel_r: the row's two
//                                             symbols; srcA/B: the step's column table, 4 bytes)
//   dn = v_pk_add_u16(hp, p)                  next row's diagonal, biased +128
//   t  = v_pk_max_i16(hu, hp)                 max(U, L)
//   t  = v_pk_add_u16(t, G + 128)             max(U, L) + G, biased +128
//   h  = v_pk_max_i16(t, dr)                  max(M + G, D + s) + 128
//   hp = v_pk_sub_u16(h, 128) clamp           max(0, M + G, D + s)
//   PK4F (V = 4): f16 scaled by 2^-11 so that the add's clamp is the zero floor, and F = max(H + Gap,
//   0) kept per row beside H: dn = Hd + s, H = v_pk_maximum3_f16(dn, Fu, Fl), F = clamp(H + Gap) --
//   4 ops per 2 cells, 2R registers of state
//   PK5F (V = 3): the same cell in f16 -- sub as an f16 whose low byte is 0 (the perm's high byte),
//   one v_pk_maximum3_f16 takes max(D + s, M + G, 0): 5 ops per 2 cells
// argv[1] = waves per SIMD (1024 * wps single-wave workgroups).  Cycles are SIMD-cycles per 64
// lane-cells at 2.4 GHz (time-based, as tools/microbench_so.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ uint32_t shr1(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x138, 0xf, 0xf, false);
}

// V = 0: SG (R rows of one pair); V = 1: PK6 (R rows of two pairs); V = 2: PK6 without the clamp
// op (5 ops per 2 cells: the lower bound of a packed cell)
template <int V, int R>
__global__ __launch_bounds__(64) void cells(const uint32_t* in, uint32_t* out, int steps) {
    const int lane = threadIdx.x;
    uint32_t tab[R], Hp[R], Fr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        tab[r] = V == 0 ? in[(lane * 7 + r) & 1023]
                 : V >= 3 ? 0x0cu | (((r + lane) & 3) << 8) | 0x0c0000u | ((((r * 3 + lane) & 3) + 4) << 24)
                          : ((r + lane) & 3) | 0x0c00u | ((((r * 3 + lane) & 3) + 4) << 16) | 0x0c000000u;
        Hp[r] = 0;
        Fr[r] = 0;
    }
    uint32_t hl = 0, sym = (lane & 3) * 8, prev_up = 0, cml = 0, srcA = 0x7f7f7f81u, srcB = 0x7f817f7fu;
    const uint32_t CU1 = 1;
    const uint32_t G128 = 0x007f007fu, C128 = 0x00800080u;   // packed G + 128 (G = -1), 128
    const uint32_t GF16 = 0xbc00bc00u;                        // packed f16 -1.0
    for (int s = 0; s < steps; ++s) {
        const uint32_t up_h = shr1(in[s & 1023], hl);
        uint32_t hu = up_h, dcur;
        if constexpr (V == 0) {
            sym = shr1((uint32_t)((s * 7) & 3) * 8, sym);
            asm volatile("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(dcur) : "v"(tab[0]), "v"(sym), "v"(prev_up));
        } else {
            // the step's column tables of both pairs ride the DPP shift (lane 0: a new column)
            if constexpr (V >= 3) {   // f16 high bytes: -1.0 (0xbc) but +1.0 (0x3c) at the match
                srcA = shr1(0xbcbcbcbcu ^ (0x80u << (((s * 7) & 3) * 8)), srcA);
                srcB = shr1(0xbcbcbcbcu ^ (0x80u << (((s * 5) & 3) * 8)), srcB);
            } else {
                srcA = shr1(0x7f7f7f7fu + (2u << (((s * 7) & 3) * 8)), srcA);
                srcB = shr1(0x7f7f7f7fu + (2u << (((s * 5) & 3) * 8)), srcB);
            }
            uint32_t p;
            asm volatile("v_perm_b32 %0, %1, %2, %3\n\tv_pk_add_u16 %0, %4, %0" : "=&v"(dcur), "=&v"(p) : "v"(srcB), "v"(srcA), "v"(tab[0]), "v"(prev_up));
            (void)p;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t t1, dn = 0;
            const uint32_t tabn = tab[r + 1 < R ? r + 1 : r];
            if constexpr (V == 0) {
                asm volatile("v_max_i16 %[t1], %[hu], %[hp]\n\t"
                             "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\tv_add_u16 %[dn], %[hp], %[dn]\n\t"
                             "v_sub_u16_e64 %[t1], %[t1], %[cu] clamp\n\t"
                             "v_max_i16 %[hp], %[dr], %[t1]"
                             : [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                             : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU1), [tabn] "v"(tabn), [sym] "v"(sym));
                if (r % 8 == 7 && (s & 3) == 3) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(cml) : "v"(Hp[r - 4]), "v"(Hp[r]));
            } else if constexpr (V == 1) {
                asm volatile("v_perm_b32 %[dn], %[sb], %[sa], %[tabn]\n\t"
                             "v_pk_add_u16 %[dn], %[hp], %[dn]\n\t"
                             "v_pk_max_i16 %[t1], %[hu], %[hp]\n\t"
                             "v_pk_add_u16 %[t1], %[t1], %[g]\n\t"
                             "v_pk_max_i16 %[t1], %[t1], %[dr]\n\t"
                             "v_pk_sub_u16 %[hp], %[t1], %[c] clamp"
                             : [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                             : [dr] "v"(dcur), [hu] "v"(hu), [g] "s"(G128), [c] "s"(C128), [tabn] "v"(tabn), [sa] "v"(srcA),
                               [sb] "v"(srcB));
                if (r % 8 == 7 && (s & 3) == 3) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(cml) : "v"(Hp[r]));
            } else if constexpr (V == 3) {
                asm volatile("v_perm_b32 %[dn], %[sb], %[sa], %[tabn]\n\t"
                             "v_pk_add_f16 %[dn], %[hp], %[dn]\n\t"
                             "v_pk_max_i16 %[t1], %[hu], %[hp]\n\t"
                             "v_pk_add_f16 %[t1], %[t1], %[g]\n\t"
                             "v_pk_maximum3_f16 %[hp], %[t1], %[dr], 0"
                             : [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                             : [dr] "v"(dcur), [hu] "v"(hu), [g] "s"(GF16), [tabn] "v"(tabn), [sa] "v"(srcA), [sb] "v"(srcB));
                if (r % 8 == 7 && (s & 3) == 3) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(cml) : "v"(Hp[r]));
            } else if constexpr (V == 4) {
                // PK4F: scaled f16 (H / 2048, clamp = the zero floor), F = max(H + Gap, 0) kept per row:
                // dn = Hd + s; H = max3(dn, Fu, Fl); F = clamp(H + Gap)
                asm volatile("v_perm_b32 %[dn], %[sb], %[sa], %[tabn]\n\t"
                             "v_pk_add_f16 %[dn], %[hp], %[dn]\n\t"
                             "v_pk_maximum3_f16 %[hp], %[dr], %[fu], %[fl]\n\t"
                             "v_pk_add_f16 %[fl], %[hp], %[g] clamp"
                             : [dn] "=&v"(dn), [hp] "+v"(Hp[r]), [fl] "+v"(Fr[r])
                             : [dr] "v"(dcur), [fu] "v"(hu), [g] "s"(GF16), [tabn] "v"(tabn), [sa] "v"(srcA), [sb] "v"(srcB));
                if (r % 8 == 7 && (s & 3) == 3) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(cml) : "v"(Hp[r]));
                dcur = dn;
                hu = Fr[r];
                continue;
            } else {
                asm volatile("v_perm_b32 %[dn], %[sb], %[sa], %[tabn]\n\t"
                             "v_pk_add_u16 %[dn], %[hp], %[dn]\n\t"
                             "v_pk_max_i16 %[t1], %[hu], %[hp]\n\t"
                             "v_pk_add_u16 %[t1], %[t1], %[g]\n\t"
                             "v_pk_max_i16 %[hp], %[t1], %[dr]"
                             : [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r])
                             : [dr] "v"(dcur), [hu] "v"(hu), [g] "s"(G128), [tabn] "v"(tabn), [sa] "v"(srcA), [sb] "v"(srcB));
                if (r % 8 == 7 && (s & 3) == 3) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(cml) : "v"(Hp[r]));
            }
            dcur = dn;
            hu = Hp[r];
        }
        prev_up = up_h;
        hl = Hp[R - 1];
    }
    uint32_t x = hl ^ cml ^ srcA ^ srcB;
#pragma unroll
    for (int r = 0; r < R; ++r) x ^= Hp[r] ^ Fr[r];
    out[blockIdx.x * 64 + lane] = x;
}

int main(int argc, char** argv) {
    const int wps = argc > 1 ? atoi(argv[1]) : 4;
    const int nblk = 1024 * wps;
    uint32_t *din, *dout;
    if (hipMalloc(&din, 4096 * 4) != hipSuccess || hipMalloc(&dout, (size_t)nblk * 64 * 4) != hipSuccess) return 1;
    if (hipMemset(din, 1, 4096 * 4) != hipSuccess) return 1;
    typedef void (*kfn)(const uint32_t*, uint32_t*, int);
    // cells per lane-step: R (SG) or 2R (packed)
    struct K { const char* name; kfn f; int cells; } ks[] = {
        {"SG  shipped, 1 pair, R32 (5 / cell)", cells<0, 32>, 32},
        {"PK6 2 pairs packed, R32 (6 / 2 cells)", cells<1, 32>, 64},
        {"PK6 2 pairs packed, R16 (6 / 2 cells)", cells<1, 16>, 32},
        {"PK5 packed without clamp, R32 (bound)", cells<2, 32>, 64},
        {"PK5F f16 with maximum3 floor, R32", cells<3, 32>, 64},
        {"PK5F f16 with maximum3 floor, R16", cells<3, 16>, 32},
        {"PK4F scaled f16, F kept, R16", cells<4, 16>, 32},
        {"PK4F scaled f16, F kept, R32", cells<4, 32>, 64},
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
        const double cells = (double)nblk * 64 * k.cells * steps;
        printf("wps=%d %-40s %8.3f ms  %8.1f GCUPS-equivalent  %.2f cycles/64 cells@2.4GHz\n", wps, k.name, best,
               cells / best / 1e6, 1024 * 2.4e9 * best * 1e-3 / (cells / 64));
    }
    return 0;
}
