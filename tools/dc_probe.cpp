// tools/dc_probe.cpp — time sa_align_batch_device for HirschbergSA (4) / MyersMillerSA (5) from C++
// (no Python): 1000 pairs of 4096 x 4096 synthetic DNA resident in HBM, 5 calls.
//   g++ -O2 -std=c++17 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/dc_probe.cpp \
//       -o build/dc_probe -Lseqalib_amd/lib -lseqalib_hip -L/opt/rocm/lib -lamdhip64 \
//       -Wl,-rpath,$PWD/seqalib_amd/lib    &&  build/dc_probe 5
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "seqalib_hip.h"
int main(int argc, char** argv) {
    const int algo = argc > 1 ? atoi(argv[1]) : SA_MYERS_MILLER;
    const uint32_t P = 1000, L = 4096;
    std::vector<uint8_t> s1((size_t)P * L), s2((size_t)P * L);
    std::vector<uint64_t> o1(P + 1), o2(P + 1);
    for (uint32_t p = 0; p <= P; ++p) o1[p] = o2[p] = (uint64_t)p * L;
    for (uint32_t p = 0; p < P; ++p) { sa_synth_dna(1000 + 2 * p, L, &s1[(size_t)p * L]); sa_synth_dna(1001 + 2 * p, L, &s2[(size_t)p * L]); }
    uint8_t *d1, *d2, *dops; uint64_t *do1, *do2; sa_result* dres;
    (void)hipMalloc(&d1, s1.size()); (void)hipMalloc(&d2, s2.size());
    (void)hipMalloc(&do1, 8 * (P + 1)); (void)hipMalloc(&do2, 8 * (P + 1));
    (void)hipMalloc(&dres, sizeof(sa_result) * P); (void)hipMalloc(&dops, 2 * s1.size() + P);
    (void)hipMemcpy(d1, s1.data(), s1.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(d2, s2.data(), s2.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(do1, o1.data(), 8 * (P + 1), hipMemcpyHostToDevice);
    (void)hipMemcpy(do2, o2.data(), 8 * (P + 1), hipMemcpyHostToDevice);
    sa_ctx* c; sa_create(0, &c);
    sa_scoring sc = {-1, 2, -1, -3, -1, 1};
    if (algo == SA_MYERS_MILLER) { sc.match = 1; sc.mismatch = -1; }
    for (int k = 0; k < 5; ++k) {
        auto t0 = std::chrono::steady_clock::now();
        int rc = sa_align_batch_device(c, algo, &sc, d1, do1, d2, do2, P, L, L, nullptr, dres, dops, nullptr);
        auto t1 = std::chrono::steady_clock::now();
        printf("algo %d call %d: rc=%d %.2f ms\n", algo, k, rc, std::chrono::duration<double, std::milli>(t1 - t0).count());
    }
    sa_destroy(c);
    return 0;
}
