// sa_synth.cpp — synthetic DNA inputs for the bench and the tests.
// A self-contained std::mt19937_64 (parameters fixed by the C++ standard, [rand.predef]), so
// inputs are identical to what the reference-side generator (oracle/ref_harness.cpp) makes with
// <random>; tests/test_synth.py pins the two against each other.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/seqalib_hip.h"

namespace {

struct Mt64 {
    static constexpr int N = 312, M = 156;
    uint64_t s[N];
    int i;
    explicit Mt64(uint64_t seed) {
        s[0] = seed;
        for (i = 1; i < N; ++i) s[i] = 6364136223846793005ULL * (s[i - 1] ^ (s[i - 1] >> 62)) + (uint64_t)i;
    }
    void twist() {
        const uint64_t UM = 0xFFFFFFFF80000000ULL, LM = 0x7FFFFFFFULL, A = 0xB5026F5AA96619E9ULL;
        for (int k = 0; k < N; ++k) {
            const uint64_t x = (s[k] & UM) | (s[(k + 1) % N] & LM);
            s[k] = s[(k + M) % N] ^ (x >> 1) ^ ((x & 1) ? A : 0);
        }
        i = 0;
    }
    uint64_t operator()() {
        if (i >= N) twist();
        uint64_t x = s[i++];
        x ^= (x >> 29) & 0x5555555555555555ULL;
        x ^= (x << 17) & 0x71D67FFFEDA60000ULL;
        x ^= (x << 37) & 0xFFF7EEE000000000ULL;
        x ^= x >> 43;
        return x;
    }
};

const char kAcgt[4] = {'A', 'C', 'G', 'T'};

void gen(uint64_t seed, uint32_t len, uint8_t* out) {
    Mt64 g(seed);
    for (uint32_t k = 0; k < len; ++k) out[k] = (uint8_t)kAcgt[g() & 3];
}

}  // namespace

extern "C" {

int sa_synth_dna(uint64_t seed, uint32_t len, uint8_t* out) {
    if (!out && len) return SA_ERR_ARG;
    gen(seed, len, out);
    return SA_OK;
}

int sa_synth_mutate(const uint8_t* src, uint32_t len, uint64_t seed, uint8_t* out, uint32_t cap,
                    uint32_t* out_len) {
    if ((!src && len) || !out_len) return SA_ERR_ARG;
    Mt64 g(seed);
    uint32_t k = 0;
    auto put = [&](uint8_t c) {
        if (k < cap && out) out[k] = c;
        ++k;
    };
    for (uint32_t p = 0; p < len; ++p) {
        const uint64_t r = g() % 100;
        if (r < 10) {
            put((uint8_t)kAcgt[g() & 3]);
        } else if (r < 12) {
            put((uint8_t)kAcgt[g() & 3]);
            put(src[p]);
        } else if (r < 14) {
            // deletion
        } else {
            put(src[p]);
        }
    }
    *out_len = k;
    return k <= cap ? SA_OK : SA_ERR_CAPACITY;
}

int sa_synth_dna_batch(uint64_t base, uint32_t npairs, uint32_t len1, uint32_t len2, uint8_t* seq1,
                       uint64_t* off1, uint8_t* seq2, uint64_t* off2, int threads) {
    if ((npairs && (!seq1 || !seq2)) || !off1 || !off2) return SA_ERR_ARG;
    for (uint32_t p = 0; p <= npairs; ++p) {
        off1[p] = (uint64_t)p * len1;
        off2[p] = (uint64_t)p * len2;
    }
    int T = std::max(1, std::min(threads, 64));
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t) {
        pool.emplace_back([=]() {
            for (uint32_t p = (uint32_t)t; p < npairs; p += (uint32_t)T) {
                gen(base + 2ull * p + 1, len1, seq1 + (uint64_t)p * len1);
                gen(base + 2ull * p + 2, len2, seq2 + (uint64_t)p * len2);
            }
        });
    }
    for (auto& th : pool) th.join();
    return SA_OK;
}

}  // extern "C"
