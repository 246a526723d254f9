// sa_dc.h — host and device pieces shared by the linear-space divide-and-conquer aligners
// (sa_hirschberg.hip: HirschbergSA, sa_myersmiller.hip: MyersMillerSA).
//
// Both run their recursion breadth-first over all pairs, entirely on the device (sa_dc.hip):
// device levels split subproblems with batched last-row sweeps, and what is left ("leaves") is
// finished one GPU thread per leaf, each writing its forward-order op list at its key
// a0 + b0.  A pair's leaves tile its alignment path in Seq1 order, so dc_assemble_kernel walks
// the pair's key range, concatenates them and reverses the result into the engine's
// traceback-order op stream (include/seqalib_hip.h: pair p's ops at off1[p] + off2[p] + p).
#pragma once
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "sa_internal.h"

namespace sa {

// Device buffer that only grows; kept per context (sa_ctx::dc) by the drivers, since a
// hipMalloc/hipFree per call would serialise the device.
template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;              // owning: a copy's destructor would free p
    DevBuf& operator=(const DevBuf&) = delete;
    void swap(DevBuf& o) { std::swap(p, o.p); std::swap(n, o.n); }
    hipError_t alloc(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DevBuf() { reset(); }
};

// Pinned host staging buffer that only grows (per context, like DevBuf): pageable copies stall.
template <typename T>
struct HostBuf {
    T* p = nullptr;
    size_t n = 0;
    HostBuf() = default;
    HostBuf(const HostBuf&) = delete;
    HostBuf& operator=(const HostBuf&) = delete;
    hipError_t alloc(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipHostMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = count;
        return e;
    }
    T& operator[](size_t k) { return p[k]; }
    const T& operator[](size_t k) const { return p[k]; }
    T* data() { return p; }
    void reset() {   // give the pinned pages back (sa_trim)
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
    ~HostBuf() { reset(); }
};

// 8 x the code of byte b in a 16-bit sweep's alphabet (sym_pack sp: byte c = the symbol of code c,
// distinct; decide_t16, sa_alphabet.hip)
__device__ __forceinline__ uint32_t dc_code8(uint32_t sp, uint32_t b) {
    return (b == ((sp >> 8) & 255u) ? 8u : 0u) | (b == ((sp >> 16) & 255u) ? 16u : 0u) | (b == (sp >> 24) ? 24u : 0u);
}
// the low 16 bits of a 16-bit sweep register, sign-extended, plus the offset
__device__ __forceinline__ int32_t dc_unpack16(int32_t v, int32_t delta) { return (int32_t)(int16_t)(v & 0xffff) + delta; }

// f(std::integral_constant<int, K>{}) for the (wave-uniform) register index k in [0, N): a band's
// handed-on row is a register picked at compile time.  Every index has its own case -- round 3's
// hand-written switch sent every k >= 7 to register 7, so R = 16 sweeps parked the wrong row.
template <int N, int K = 0, class F>
__device__ __forceinline__ void dc_row_dispatch(int k, F&& f) {
    if constexpr (K < N) {
        if (k == K) f(std::integral_constant<int, K>{});
        else dc_row_dispatch<N, K + 1>(k, f);
    }
}

// ---- match sources
// match(a, b): the 256x256 LUT as bits (lut_to_bits), or byte equality
__device__ __forceinline__ bool dc_match(const uint32_t* lut, uint32_t a, uint32_t b) {
    return lut ? ((lut[(a << 3) | (b >> 5)] >> (b & 31)) & 1) : a == b;
}
// Byte symbols: LUT bits (or NULL = equality), decided at run time (leaf solvers).
struct DcLutMatch {
    const uint32_t* lut;
    __device__ bool operator()(uint32_t a, uint32_t b) const { return dc_match(lut, a, b); }
};
// Generic-Ty path (sa_align_batch_bits): the "symbols" a kernel carries are the pair-local
// indices i (Seq1) and j (Seq2) themselves, and match(i, j) is bit j % 32 of word
// [i * wn + j / 32] of the pair's m x n bitmap (the reference's cacheAllMatches packed to bits,
// SAHirschberg.h:31 / :73 call the MatchFnTy per cell, SAMyersMiller.h:24-37 cache it).
struct DcBitsMatch {
    const uint32_t* row0;   // the pair's bitmap
    uint32_t wn;            // words per row = ceil(n / 32)
    __device__ bool operator()(uint32_t i, uint32_t j) const { return (row0[(uint64_t)i * wn + (j >> 5)] >> (j & 31)) & 1u; }
};
// Symbols and match of one sweep (whole-wave and packed sweep kernels): bytes of the batch with
// byte equality / the LDS copy of the LUT bits, or (kMatchBits) pair-local indices and the pair's
// bitmap.  a(x) / b(x): the symbol at absolute Seq1 / Seq2 index x.
struct DcBits;
template <int MM>
struct DcSrc {
    const uint8_t* s1;
    const uint8_t* s2;
    const uint32_t* lut;   // kMatchLut: LDS copy of the LUT bits
    DcBitsMatch bm;        // kMatchBits
    uint64_t base1, base2;
    __device__ uint32_t a(uint64_t x) const {
        if constexpr (MM == kMatchBits) return (uint32_t)(x - base1);
        else return s1[x];
    }
    __device__ uint32_t b(uint64_t x) const {
        if constexpr (MM == kMatchBits) return (uint32_t)(x - base2);
        else return s2[x];
    }
    __device__ bool match(uint32_t x, uint32_t y) const {
        if constexpr (MM == kMatchBits) return bm(x, y);
        else if constexpr (MM == kMatchLut) return (lut[(x << 3) | (y >> 5)] >> (y & 31)) & 1u;
        else return x == y;
    }
};
// Device pointers of the bitmap path (all NULL on the byte-symbol path).
struct DcBits {
    const uint32_t* mbits;
    const uint64_t* mbits_off;
    const uint64_t* o1;
    const uint64_t* o2;
    // pair p: its bitmap, and the absolute Seq1 / Seq2 index of its first symbol (local = abs - base)
    __device__ DcBitsMatch of(uint32_t p, uint64_t* base1, uint64_t* base2) const {
        *base1 = o1[p];
        *base2 = o2[p];
        return DcBitsMatch{mbits + mbits_off[p], (uint32_t)((o2[p + 1] - o2[p] + 31) >> 5)};
    }
    // the match source of a sweep of pair p (valid: false for an idle lane of a packed sweep)
    template <int MM>
    __device__ DcSrc<MM> src(const uint8_t* s1, const uint8_t* s2, const uint32_t* lut, uint32_t p, bool valid) const {
        DcSrc<MM> r{s1, s2, lut, DcBitsMatch{nullptr, 0}, 0, 0};
        if constexpr (MM == kMatchBits) {
            if (valid) r.bm = of(p, &r.base1, &r.base2);
        }
        return r;
    }
};

// Row / symbol accessors for the leaf solver: global scratch, or LDS laid out item-major
// (element k of thread t at k * 64 + t: conflict-free when the threads are in step).
typedef int32_t __attribute__((address_space(3))) dc_lds_i32;
typedef uint8_t __attribute__((address_space(3))) dc_lds_u8;
struct GRow {
    int32_t* p;
    __device__ int32_t& operator[](int k) const { return p[k]; }
};
struct LRow {
    dc_lds_i32* p;
    __device__ dc_lds_i32& operator[](int k) const { return p[k * 64]; }
};
struct GSeq {
    const uint8_t* p;
    __device__ uint32_t operator[](int k) const { return p[k]; }
    __device__ GSeq shifted(int k) const { return GSeq{p + k}; }
};
struct LSeq {
    const dc_lds_u8* p;
    __device__ uint32_t operator[](int k) const { return p[k * 64]; }
    __device__ LSeq shifted(int k) const { return LSeq{p + k * 64}; }
};
// Bitmap path: symbol k of a subproblem is its pair-local index base + k.
struct ISeq {
    uint32_t base;
    __device__ uint32_t operator[](int k) const { return base + (uint32_t)k; }
    __device__ ISeq shifted(int k) const { return ISeq{base + (uint32_t)k}; }
};

// Wait for a stream by polling: the drivers synchronise once per level, and a blocking
// hipStreamSynchronize here was observed to oversleep by ~20 ms per wait.
inline hipError_t dc_sync(hipStream_t st) {
    hipError_t e;
    while ((e = hipStreamQuery(st)) == hipErrorNotReady) __builtin_ia32_pause();
    return e;
}

#define SA_DC_HIP(call)                                                                              \
    do {                                                                                             \
        hipError_t e_ = (call);                                                                      \
        if (e_ != hipSuccess) { *err = std::string(#call) + ": " + hipGetErrorString(e_); return -1; } \
    } while (0)

// One subproblem of a level (or a leaf).  m < 0 marks an empty slot.  tb / te: Myers–Miller's
// boundary gap opens (unused by Hirschberg).
struct DcSub {
    uint64_t a0, b0;   // absolute start in seq1 / seq2; key = a0 + b0
    int32_t m, n;
    int32_t tb, te;
    uint32_t pair;
    int32_t top;       // the pair's whole problem: its score is the pair's
};

struct DcLevel {
    uint32_t nsplit;   // subproblems split at this level (the next level has mult * nsplit slots)
    uint32_t pad;
};

// sa_dc.hip
struct DcBounds;
hipError_t dc_launch_init(const uint64_t* o1, const uint64_t* o2, uint32_t npairs, int32_t t0, const DcBounds& b,
                          DcSub* subs, sa_result* res, hipStream_t st);
hipError_t dc_launch_classify(const DcSub* cur, uint32_t cap, uint32_t fixed, const DcLevel* prev, uint32_t mult,
                              int leaf_rows, int min_n, DcLevel* lvl, DcSub* split, DcSub* leaves, uint32_t* nleaf,
                              hipStream_t st);
hipError_t dc_launch_assemble(const uint64_t* o1, const uint64_t* o2, uint32_t npairs, const int32_t* mark,
                              const uint8_t* stage, sa_result* res, uint8_t* ops, hipStream_t st);

// Host-side sizes of a batch: grid bounds of the level loop and the key range (keys are
// absolute a0 + b0 < t1 + t2).  From the host offsets (host API), or from the device API's
// max_m / max_n (t1 <= npairs * max_m): no read of the device offsets, no wait.
struct DcBounds {
    uint64_t t1 = 0, t2 = 0;   // Seq1 / Seq2 symbol totals (upper bounds)
    uint32_t max_m = 0, max_n = 0;
};

// Device work buffers of one level loop (grow-only, one set per context: sa_ctx::dc).  Bounds: a split
// subproblem has > leaf_rows rows and the subproblems of a level have disjoint Seq1 ranges, so
// a level splits at most t1 / (leaf_rows + 1) + 1 of them; leaves have >= 1 row (or are a whole
// empty pair), so there are at most t1 + npairs of them.
struct DcWork {
    DevBuf<uint32_t> aux;   // 16-bit sweeps: alphabet bitmap, profile and decision (sa_internal.h kAux*)
    DevBuf<DcSub> cur, next, split, leaves;
    DevBuf<DcLevel> lvl;
    DevBuf<int32_t> rows, scratch, mark;
    DevBuf<uint8_t> stage;
    uint64_t max_splits = 0, leaf_cap = 0;
    int levels = 0;
    uint32_t* nleaf() { return &lvl.p[levels + 1].nsplit; }   // lvl[0..levels]: the levels
    void release() {
        aux.reset(); cur.reset(); next.reset(); split.reset(); leaves.reset(); lvl.reset();
        rows.reset(); scratch.reset(); mark.reset(); stage.reset();
    }
    // prev: the context's last call (its kernels may still read these buffers on another
    // stream); waited for on the host before any buffer is reallocated.
    hipError_t prepare(const DcBounds& b, uint32_t npairs, int leaf_rows, uint32_t mult, uint32_t rows_per_key,
                       uint32_t scratch_per_key, hipStream_t st, hipEvent_t prev) {
        max_splits = b.t1 / (uint64_t)(leaf_rows + 1) + 1;
        uint64_t cap = npairs, total = npairs;
        levels = 0;
        for (int m = (int)b.max_m; m > leaf_rows; m = (m + 1) / 2) {
            cap = mult * std::min<uint64_t>(cap, max_splits);
            total += cap;
            ++levels;
        }
        leaf_cap = std::min<uint64_t>(total, b.t1 + npairs);
        const uint64_t sub_cap = std::max<uint64_t>(npairs, mult * max_splits);
        const uint64_t keys = b.t1 + b.t2 + 1;
        hipError_t e;
        const bool grow = cur.n < sub_cap || next.n < sub_cap || split.n < std::min(sub_cap, max_splits) ||
                          leaves.n < leaf_cap || lvl.n < (size_t)levels + 2 || rows.n < rows_per_key * keys ||
                          scratch.n < scratch_per_key * keys || mark.n < keys || stage.n < keys;
        if (grow && prev && (e = hipEventSynchronize(prev))) return e;
        if ((e = cur.alloc(sub_cap)) || (e = next.alloc(sub_cap)) || (e = split.alloc(std::min(sub_cap, max_splits))) ||
            (e = leaves.alloc(leaf_cap)) || (e = lvl.alloc(levels + 2)) || (e = rows.alloc(rows_per_key * keys)) ||
            (e = scratch.alloc(scratch_per_key * keys)) || (e = mark.alloc(keys)) || (e = stage.alloc(keys)))
            return e;
        if ((e = hipMemsetAsync(lvl.p, 0, sizeof(DcLevel) * (levels + 2), st))) return e;
        return hipMemsetAsync(mark.p, 0, sizeof(int32_t) * keys, st);
    }
};

// 16-bit whole-wave sweeps (sa_hirschberg.hip, sa_myersmiller.hip).  When the batch has at most four
// distinct symbols (decided on the device: alphabet_scan + decide_t16 with a plain profile) and the
// host proves every value a sweep can produce lies within 2^15 of an offset `delta`, the sweeps keep
// their rows as 16-bit values v - delta and run 16-bit VOP2 adds / maxes (twice the issue rate of
// the 32-bit integer max / compare ops on gfx950) with the substitution score from a per-row byte
// profile: one v_bfe_i32 per cell.  !AllowMismatch runs with mismatch' = 2 * Gap - 1
// (2 * (GapOpen + GapExtend) - 1 for Myers-Miller), which never wins a max -- the same argument as
// the fill's T16 kernels -- so the rows are the reference's exactly.
struct Dc16 {
    const uint32_t* aux = nullptr;   // NULL: int32 sweeps only
    int32_t delta = 0;
    int32_t mismatch = 0;            // the profile's mismatch score
    int32_t park = 1;                // steady chunks park the handed-on row in LDS and store it per
                                     // chunk (SEQALIB_DC16_PARK=0: a lane-masked store per step)
    int32_t seg16 = 0;               // this launch's 16-bit sweeps run in a two-per-wave kernel
};
// Grid cap of the whole-wave int32 sweep kernels launched beside a seg16 kernel: they usually
// return at once, and otherwise grid-stride over the level's sweeps.
constexpr uint32_t kDcSkipGrid = 8192;
// Lanes per split in the midpoint kernels (hb_split_kernel / mm_split_kernel), from the level's
// bound on the split rows: 64 (one per wave) for long rows, 16 or 8 at the deep levels.
inline int dc_split_lanes(int maxm) { return maxm >= 256 ? 64 : maxm >= 64 ? 16 : 8; }
// Host: is the 16-bit sweep exact for the batch's shapes and scoring?  lo / hi: bounds of every
// row value and candidate of any sweep of at most max_m x max_n.
inline Dc16 dc16_plan(bool affine, const sa_scoring* sc, uint32_t max_m, uint32_t max_n) {
    Dc16 d;
    if (const char* e = getenv("SEQALIB_DC16")) if (e[0] == '0') return d;
    const int64_t m = max_m, n = max_n, k = std::min(m, n);
    const int64_t MA = sc->match;
    const int64_t G = affine ? (int64_t)sc->gap_open : (int64_t)sc->gap;
    const int64_t H = affine ? (int64_t)sc->gap_extend : 0;
    int64_t MI = sc->mismatch;
    if (!sc->allow_mismatch) MI = affine ? 2 * (G + H) - 1 : 2 * G - 1;
    if (MA < -127 || MA > 127 || MI < -128 || MI > 127 || G > 0 || H > 0 || MI > MA) return d;
    if (MA < 0) return d;
    int64_t lo, hi;
    if (affine) {   // C, D, e >= the all-gap path (>= 3g + (m + n)h), each candidate one step below
        lo = 3 * G + (m + n) * H + std::min<int64_t>(std::min(G + H, MI), 0) + H;
        hi = k * MA + MA;
    } else {        // H >= the all-gap path (m + n) G; candidates one step below
        lo = (m + n) * G + std::min<int64_t>(std::min(G, MI), 0);
        hi = k * MA + MA;
    }
    const int64_t delta = (hi + lo) / 2;
    if (hi - delta > 32000 || lo - delta < -32000) return d;
    d.aux = reinterpret_cast<const uint32_t*>(1);   // placeholder: set to the device aux by the driver
    d.delta = (int32_t)delta;
    d.mismatch = (int32_t)MI;
    if (const char* e = getenv("SEQALIB_DC16_PARK")) d.park = e[0] != '0';
    return d;
}

// Inputs of a batch: byte symbols (d1 / d2 with the LUT bits, or NULL for equality) or, when
// bits.mbits != NULL, per-pair match bitmaps (the generic-Ty path; d1 / d2 are then not read).
struct DcInputs {
    const uint8_t* d1;
    const uint64_t* o1;
    const uint8_t* d2;
    const uint64_t* o2;
    uint32_t npairs;
    const uint32_t* lutbits;
    DcBits bits;
};

// HirschbergSA / MyersMillerSA drivers (sa_hirschberg.hip, sa_myersmiller.hip): device inputs,
// device outputs (results, op streams at o1[p] + o2[p] + p), enqueued on st with no host wait
// (grid bounds from b), work buffers from w (prev: see DcWork::prepare).  Return 0, or -1 with
// *err set.
int hirschberg_run(DcWork& w, hipEvent_t prev, const sa_scoring* scoring, const DcInputs& in, const DcBounds& b,
                   hipStream_t st, sa_result* d_res, uint8_t* d_ops, std::string* err);
int myersmiller_run(DcWork& w, hipEvent_t prev, const sa_scoring* scoring, const DcInputs& in, const DcBounds& b,
                    hipStream_t st, sa_result* d_res, uint8_t* d_ops, std::string* err);

}  // namespace sa
