// 2-bit transfer codecs of the host API (seqalib_amd/csrc/sa_codec.cpp), both packing paths,
// against a byte-by-byte restatement: every length 0..300 and a few large ones, every byte value
// at every position of a 64-byte buffer (only A / C / G / T pack), and the op-letter expansion.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

namespace sa {
bool dna2_pack(uint8_t* dst, const uint8_t* src, uint64_t n);
bool dna2_pack_scalar(uint8_t* dst, const uint8_t* src, uint64_t n);
bool dna2_pack_avx2(uint8_t* dst, const uint8_t* src, uint64_t n);
void ops2_unpack(uint8_t* dst, const uint8_t* src, uint32_t n, const uint32_t* lut);
}

static int code_of(uint8_t b) { return b == 'A' ? 0 : b == 'C' ? 1 : b == 'T' ? 2 : b == 'G' ? 3 : -1; }

static bool check(const std::vector<uint8_t>& src, bool (*pack)(uint8_t*, const uint8_t*, uint64_t), const char* name) {
    const uint64_t n = src.size();
    std::vector<uint8_t> dst((n + 3) / 4 + 8, 0xee);
    const bool ok = pack(dst.data(), src.data(), n);
    bool valid = true;
    for (uint8_t b : src) valid &= code_of(b) >= 0;
    if (ok != valid) {
        fprintf(stderr, "%s: n=%llu returned %d, expected %d\n", name, (unsigned long long)n, ok, valid);
        return false;
    }
    if (!valid) return true;
    for (uint64_t i = 0; i < n; ++i) {
        const int c = (dst[i / 4] >> (2 * (i % 4))) & 3;
        if (c != code_of(src[i])) {
            fprintf(stderr, "%s: n=%llu symbol %llu code %d expected %d\n", name, (unsigned long long)n,
                    (unsigned long long)i, c, code_of(src[i]));
            return false;
        }
    }
    if (dst[(n + 3) / 4] != 0xee) {
        fprintf(stderr, "%s: n=%llu wrote past ceil(n / 4)\n", name, (unsigned long long)n);
        return false;
    }
    return true;
}

int main() {
    std::mt19937_64 rng(7);
    const char* acgt = "ACGT";
    int bad = 0;
    auto all = [&](const std::vector<uint8_t>& v) {
        bad += !check(v, sa::dna2_pack_scalar, "scalar");
        if (__builtin_cpu_supports("avx2")) bad += !check(v, sa::dna2_pack_avx2, "avx2");
        bad += !check(v, sa::dna2_pack, "dispatch");
    };
    std::vector<uint64_t> lens;
    for (uint64_t n = 0; n <= 300; ++n) lens.push_back(n);
    for (uint64_t n : {1ull << 20, (1ull << 20) + 7, 3000001ull}) lens.push_back(n);
    for (uint64_t n : lens) {
        std::vector<uint8_t> v(n);
        for (auto& b : v) b = acgt[rng() & 3];
        all(v);
    }
    for (int pos = 0; pos < 64; ++pos)
        for (int x = 0; x < 256; ++x) {
            std::vector<uint8_t> v(64);
            for (auto& b : v) b = acgt[rng() & 3];
            v[pos] = (uint8_t)x;
            all(v);
        }
    // op letters: M 0, S 1, U 2, L 3
    const uint8_t lt[4] = {'M', 'S', 'U', 'L'};
    uint32_t lut[256];
    for (uint32_t b = 0; b < 256; ++b)
        lut[b] = lt[b & 3] | (uint32_t)lt[(b >> 2) & 3] << 8 | (uint32_t)lt[(b >> 4) & 3] << 16 | (uint32_t)lt[b >> 6] << 24;
    for (uint32_t n = 0; n < 200; ++n) {
        std::vector<uint8_t> codes(n), packed((n + 3) / 4, 0), out(n + 8, 0xee);
        for (uint32_t i = 0; i < n; ++i) {
            codes[i] = (uint8_t)(rng() & 3);
            packed[i / 4] |= (uint8_t)(codes[i] << (2 * (i % 4)));
        }
        sa::ops2_unpack(out.data(), packed.data(), n, lut);
        for (uint32_t i = 0; i < n; ++i)
            if (out[i] != lt[codes[i]]) { fprintf(stderr, "ops2_unpack n=%u i=%u\n", n, i); ++bad; break; }
        if (out[n] != 0xee) { fprintf(stderr, "ops2_unpack n=%u wrote past n\n", n); ++bad; }
    }
    printf("%s\n", bad ? "FAIL" : "ok");
    return bad ? 1 : 0;
}
