// sa_codec.cpp — host side of the 2-bit transfer codecs of the host API (sa_api.hip align_host).
//
// PCIe is the host API's bottleneck outside the kernels: the headline batch moves 82 MB of
// sequences up and 46 MB of op streams down per call (1.55 + 0.94 ms at ~53 GB/s).  Both are 4-symbol
// alphabets in the common case, so both travel at 2 bits per symbol when they can:
//  * sequences: a piece whose bytes are all in {A, C, G, T} is packed here (code = (b >> 1) & 3:
//    A 0, C 1, T 2, G 3 -- a bijection on those four bytes) and unpacked on the device
//    (dna2_unpack in sa_api.hip); any other byte sends that piece as bytes;
//  * op streams: the device packs every pair's ops (M 0, S or X 1, U 2, L 3) unless a call holds
//    both S and X or another letter, and ops2_unpack expands them into the caller's layout.
#include <stdint.h>
#include <string.h>

#include <immintrin.h>

namespace sa {

namespace {

// 8 bytes -> 16 bits of codes; false if a byte is not A, C, G or T.  A byte's code is (b >> 1) & 3;
// the byte is valid iff re-deriving it from its code gives it back: 0x41 + 2c, plus 0x0f for c = 2.
inline bool pack8(uint64_t w, uint16_t* out) {
    const uint64_t c = (w >> 1) & 0x0303030303030303ull;
    const uint64_t e = c ^ 0x0202020202020202ull;                  // zero byte where c == 2
    const uint64_t isz = ~(e | (e >> 1)) & 0x0101010101010101ull;
    const uint64_t expect = 0x4141414141414141ull + (c << 1) + isz * 0x0f;
    const uint64_t x = c | (c >> 6) | (c >> 12) | (c >> 18);      // 4 codes in the low byte of each half
    *out = (uint16_t)((x & 0xff) | ((x >> 24) & 0xff00));
    return expect == w;
}

bool pack_scalar(uint8_t* dst, const uint8_t* src, uint64_t n) {
    bool ok = true;
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, src + i, 8);
        uint16_t o;
        ok &= pack8(w, &o);
        memcpy(dst + i / 4, &o, 2);
    }
    if (i < n) {   // tail: pad with 'A' (code 0)
        uint8_t t[8];
        memset(t, 'A', 8);
        memcpy(t, src + i, n - i);
        uint64_t w;
        memcpy(&w, t, 8);
        uint16_t o;
        ok &= pack8(w, &o);
        memcpy(dst + i / 4, &o, (n - i + 3) / 4);
    }
    return ok;
}

__attribute__((target("avx2"))) bool pack_avx2(uint8_t* dst, const uint8_t* src, uint64_t n) {
    const __m256i kA = _mm256_set1_epi8('A'), k2 = _mm256_set1_epi8(2), k3 = _mm256_set1_epi8(3),
                  k15 = _mm256_set1_epi8(15);
    const __m256i w01 = _mm256_set1_epi16(0x0401);          // c0 + 4 c1 per 16 bits
    const __m256i w0123 = _mm256_set1_epi32(0x00100001);    // (c0 + 4 c1) + 16 (c2 + 4 c3) per 32 bits
    // byte 0 of each dword to the low 4 bytes of each 128-bit lane
    const __m256i gather = _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                                            0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
    __m256i bad = _mm256_setzero_si256();
    uint64_t i = 0;
    for (; i + 32 <= n; i += 32) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i c = _mm256_and_si256(_mm256_srli_epi16(v, 1), k3);
        // valid iff v == 0x41 + 2c (+ 0x0f for c == 2), as pack8
        const __m256i t = _mm256_and_si256(_mm256_cmpeq_epi8(c, k2), k15);
        bad = _mm256_or_si256(bad, _mm256_xor_si256(v, _mm256_add_epi8(_mm256_add_epi8(kA, _mm256_add_epi8(c, c)), t)));
        const __m256i p = _mm256_madd_epi16(_mm256_maddubs_epi16(c, w01), w0123);
        const __m256i g = _mm256_permutevar8x32_epi32(_mm256_shuffle_epi8(p, gather), _mm256_setr_epi32(0, 4, 1, 1, 1, 1, 1, 1));
        _mm_storel_epi64(reinterpret_cast<__m128i*>(dst + i / 4), _mm256_castsi256_si128(g));
    }
    bool good = _mm256_testz_si256(bad, bad);
    if (i < n) good &= pack_scalar(dst + i / 4, src + i, n - i);
    return good;
}

}  // namespace

// Packs n bytes of src to ceil(n / 4) bytes of 2-bit codes at dst; false if a byte is not A, C, G, T
// (dst then holds garbage for those bytes).  src + 0 must start a group of 4 codes.
bool dna2_pack(uint8_t* dst, const uint8_t* src, uint64_t n) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    return avx2 ? pack_avx2(dst, src, n) : pack_scalar(dst, src, n);
}

#ifdef SA_CODEC_TEST   // tests/cpp/codec_test.cpp: both paths
bool dna2_pack_scalar(uint8_t* dst, const uint8_t* src, uint64_t n) { return pack_scalar(dst, src, n); }
bool dna2_pack_avx2(uint8_t* dst, const uint8_t* src, uint64_t n) { return pack_avx2(dst, src, n); }
#endif

// n op letters from ceil(n / 4) bytes of 2-bit codes; lut[b] = the four letters of code byte b.
void ops2_unpack(uint8_t* dst, const uint8_t* src, uint32_t n, const uint32_t* lut) {
    uint32_t k = 0;
    for (; k + 4 <= n; k += 4) memcpy(dst + k, &lut[src[k / 4]], 4);
    if (k < n) memcpy(dst + k, &lut[src[k / 4]], n - k);
}

}  // namespace sa
