// Lone-wave step microbenchmark (not part of the product): what one wave ALONE on its SIMD pays
// per anti-diagonal step -- the unit cost of the few-pairs (SPLIT) plans, where one pair offers at
// most ~64 bands of work and every wave has a SIMD to itself.  1024 single-wave workgroups with
// 40 KiB of LDS each (<= 4 per CU, one per SIMD), register-only loops; cycles at 2.4 GHz.
//   I  independent v_add_u16, 8 chains            (lone-wave issue cost of a fast VOP2 op)
//   J  independent v_alignbit_b32, 8 chains       (lone-wave issue cost of a VOP3 op)
//   D  one dependent v_add_u16 chain              (dependent VALU latency)
//   S1 T16 SW step, R = 1: LDS row-above (old operand of a DPP shift), LDS column symbol,
//      8-op cell, lane chunk max, DPP hand-off accumulator          (the proposed SPLIT step)
//   S2 the same with R = 2 rows per lane (chained)
//   S4 the same with R = 4 rows per lane (chained; the round-1 SPLIT T16 step)
//   A1 int32 affine (Gotoh) step, R = 1, equality flags              (the LocalGotoh SPLIT step)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ uint32_t shr1(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t shl1(uint32_t old, uint32_t src) {   // wave_shl:1
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x130, 0xf, 0xf, false);
}

template <int V>
__global__ __launch_bounds__(64) void lone(const uint32_t* in, uint32_t* out, int steps) {
    __shared__ uint32_t lds[10240];   // 40 KiB: at most 4 workgroups per CU
    const int lane = threadIdx.x;
    for (int k = lane; k < 10240; k += 64) lds[k] = in[k & 1023];
    __syncthreads();
    uint32_t acc = 0, cml = 0, rec = 0, res = 0;
    if constexpr (V == 0 || V == 1) {
        uint32_t c0 = lane, c1 = lane + 1, c2 = lane + 2, c3 = lane + 3, c4 = lane + 4, c5 = lane + 5,
                 c6 = lane + 6, c7 = lane + 7;
        for (int s = 0; s < steps; ++s) {
            if constexpr (V == 0)
                asm volatile("v_add_u16 %0, 3, %0\n\tv_add_u16 %1, 3, %1\n\tv_add_u16 %2, 3, %2\n\tv_add_u16 %3, 3, %3\n\t"
                             "v_add_u16 %4, 3, %4\n\tv_add_u16 %5, 3, %5\n\tv_add_u16 %6, 3, %6\n\tv_add_u16 %7, 3, %7"
                             : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7));
            else
                asm volatile("v_alignbit_b32 %0, %0, %0, 3\n\tv_alignbit_b32 %1, %1, %1, 3\n\tv_alignbit_b32 %2, %2, %2, 3\n\t"
                             "v_alignbit_b32 %3, %3, %3, 3\n\tv_alignbit_b32 %4, %4, %4, 3\n\tv_alignbit_b32 %5, %5, %5, 3\n\t"
                             "v_alignbit_b32 %6, %6, %6, 3\n\tv_alignbit_b32 %7, %7, %7, 3"
                             : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7));
        }
        res = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
    } else if constexpr (V == 2) {
        uint32_t c = lane;
        for (int s = 0; s < steps; ++s)
            asm volatile("v_add_u16 %0, 3, %0\n\tv_add_u16 %0, 3, %0\n\tv_add_u16 %0, 3, %0\n\tv_add_u16 %0, 3, %0\n\t"
                         "v_add_u16 %0, 3, %0\n\tv_add_u16 %0, 3, %0\n\tv_add_u16 %0, 3, %0\n\tv_add_u16 %0, 3, %0"
                         : "+v"(c));
        res = c;
    } else if constexpr (V >= 3 && V <= 5) {
        constexpr int R = V == 3 ? 1 : V == 4 ? 2 : 4;
        uint32_t tab[R], Hp[R];
#pragma unroll
        for (int r = 0; r < R; ++r) { tab[r] = in[(lane * 7 + r) & 1023]; Hp[r] = 0; }
        uint32_t hl = 0, prev_up = 0;
        const uint32_t CU = 6, CL = 0xfffd;
        const uint32_t base = (lane * 5) & 8191;
        uint32_t sym = 0;
        for (int s0 = 0; s0 < steps; s0 += 32) {
            // as the fill: a chunk's lane-0 inputs and column symbols land in one VGPR each (lane q
            // = step q), broadcast per step with v_readlane and shifted in by DPP
            const uint32_t bch = lds[(s0 + lane) & 8191];
            const uint32_t symc = (uint32_t)((const uint8_t*)lds)[(base + s0 + lane) & 32767] & 24u;
#pragma unroll
            for (int q = 0; q < 32; ++q) {
                const uint32_t up_h = shr1(__builtin_amdgcn_readlane(bch, q), hl);
                sym = shr1(__builtin_amdgcn_readlane(symc, q), sym);
                uint32_t hu = up_h, dcur;
                asm volatile("v_bfe_i32 %0, %1, %2, 8\n\tv_add_u16 %0, %3, %0" : "=&v"(dcur) : "v"(tab[0]), "v"(sym), "v"(prev_up));
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    uint32_t t0, t1;
                    if (r + 1 < R) {
                        uint32_t dn;
                        asm volatile("v_add_u16 %[t0], %[cl], %[hp]\n\t"
                                     "v_bfe_i32 %[dn], %[tabn], %[sym], 8\n\tv_add_u16 %[dn], %[hp], %[dn]\n\t"
                                     "v_sub_u16_e64 %[t1], %[hu], %[cu] clamp\n\t"
                                     "v_max_i16 %[t0], %[dr], %[t0]\n\tv_max_i16 %[t0], %[t1], %[t0]\n\t"
                                     "v_and_b32 %[hp], -4, %[t0]\n\tv_alignbit_b32 %[rec], %[t0], %[rec], 2"
                                     : [t0] "=&v"(t0), [t1] "=&v"(t1), [dn] "=&v"(dn), [hp] "+v"(Hp[r]), [rec] "+v"(rec)
                                     : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL),
                                       [tabn] "v"(tab[r + 1 < R ? r + 1 : r]), [sym] "v"(sym));
                        dcur = dn;
                    } else {
                        asm volatile("v_add_u16 %[t0], %[cl], %[hp]\n\t"
                                     "v_sub_u16_e64 %[t1], %[hu], %[cu] clamp\n\t"
                                     "v_max_i16 %[t0], %[dr], %[t0]\n\tv_max_i16 %[t0], %[t1], %[t0]\n\t"
                                     "v_and_b32 %[hp], -4, %[t0]\n\tv_alignbit_b32 %[rec], %[t0], %[rec], 2"
                                     : [t0] "=&v"(t0), [t1] "=&v"(t1), [hp] "+v"(Hp[r]), [rec] "+v"(rec)
                                     : [dr] "v"(dcur), [hu] "v"(hu), [cu] "s"(CU), [cl] "s"(CL));
                    }
                    hu = Hp[r];
                }
                asm volatile("v_max_u32 %0, %0, %1" : "+v"(cml) : "v"(Hp[R - 1]));
                prev_up = up_h;
                hl = Hp[R - 1];
                acc = shl1(hl, acc);
            }
        }
        res = acc + cml + rec + prev_up;
    } else if constexpr (V == 6) {
        // int32 affine step, R = 1: X = max(hu+GOE, xu+GE), Y = max(hl+GOE, yl+GE), D = hd + s,
        // M = max(D, X, Y, 0), 4 equality flags via compare + carry shift-in
        int Hp = 0, Yp = -10000, hl = 0, xl = 0, prev_up = 0;
        const int GOE = -4, GE = -1, MA = 1, MI = -1;
        const uint32_t base = (lane * 5) & 8191;
        const int a0 = in[lane & 1023] & 3;
        int sym = 0;
        for (int s0 = 0; s0 < steps; s0 += 32) {
            const uint32_t bch = lds[(s0 + lane) & 8191];
            const uint32_t symc = (uint32_t)((const uint8_t*)lds)[(base + s0 + lane) & 32767] & 3u;
#pragma unroll
            for (int q = 0; q < 32; ++q) {
                const int inp = __builtin_amdgcn_readlane((int)bch, q);
                sym = (int)shr1((uint32_t)__builtin_amdgcn_readlane((int)symc, q), (uint32_t)sym);
                const int hu = (int)shr1((uint32_t)inp, (uint32_t)hl);
                const int xu = (int)shr1((uint32_t)inp, (uint32_t)xl);
                const int D = prev_up + (a0 == sym ? MA : MI);
                const int XE = xu + GE, X = max(hu + GOE, XE);
                const int YE = Yp + GE, Y = max(Hp + GOE, YE);
                int M = max(max(D, X), max(Y, 0));
                uint32_t f = (M == D ? 8u : 0u) | (M == X ? 4u : 0u) | (X == XE ? 2u : 0u) | (Y == YE ? 1u : 0u);
                rec = (rec << 4) | f;
                Yp = Y;
                Hp = M;
                cml = max(cml, (uint32_t)M);
                prev_up = hu;
                hl = M;
                xl = X;
                acc = shl1((uint32_t)hl, acc);
            }
        }
        res = acc + cml + rec;
    }
    out[blockIdx.x * 64 + lane] = res;
}

template <int V>
float run(const uint32_t* din, uint32_t* dout, int steps, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(lone<V>, dim3(blocks), dim3(64), 0, 0, din, dout, 64);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(lone<V>, dim3(blocks), dim3(64), 0, 0, din, dout, steps);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 1024;
    const int steps = 1 << 16;
    uint32_t* din;
    uint32_t* dout;
    hipMalloc(&din, 1024 * 4);
    hipMalloc(&dout, (size_t)blocks * 64 * 4);
    uint32_t h[1024];
    for (int k = 0; k < 1024; ++k) h[k] = (k * 2654435761u) & 0x3fff;
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    const double clk = 2.4e9;
    struct { const char* name; float ms; int per; } rows[] = {
        {"I  8 independent v_add_u16 / step", run<0>(din, dout, steps, blocks), 8},
        {"J  8 independent v_alignbit_b32 / step", run<1>(din, dout, steps, blocks), 8},
        {"D  8 dependent v_add_u16 / step", run<2>(din, dout, steps, blocks), 8},
        {"S1 T16 SW step R=1", run<3>(din, dout, steps, blocks), 1},
        {"S2 T16 SW step R=2", run<4>(din, dout, steps, blocks), 2},
        {"S4 T16 SW step R=4", run<5>(din, dout, steps, blocks), 4},
        {"A1 int32 affine step R=1", run<6>(din, dout, steps, blocks), 1},
    };
    printf("# lone-wave microbenchmark: %d single-wave workgroups (40 KiB LDS each), %d steps, best of 3\n", blocks, steps);
    for (auto& r : rows) {
        const double cyc = r.ms * 1e-3 * clk / steps;   // cycles per step of one wave
        printf("%-42s %8.3f ms  %7.1f cycles/step  %6.2f cycles per instr-or-row\n", r.name, r.ms, cyc, cyc / r.per);
    }
    return 0;
}
