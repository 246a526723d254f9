// sa_api.hip — the C ABI of libseqalib_hip.so (include/seqalib_hip.h): contexts, planning,
// workspace, batching and the host<->device plumbing around the fill and traceback kernels.
#include <hip/hip_runtime.h>
#include <limits.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "sa_dc.h"
#include "sa_internal.h"

using namespace sa;

namespace sa {   // sa_codec.cpp: 2-bit transfer codecs of the host API
bool dna2_pack(uint8_t* dst, const uint8_t* src, uint64_t n);
void ops2_unpack(uint8_t* dst, const uint8_t* src, uint32_t n, const uint32_t* lut);
}  // namespace sa

constexpr int kKEv = 6;   // SEQALIB_KERNEL_TIMING events per fill launch (two per variant, <= 3)
// Cross-call pipeline: workspace slots (call k's fill waits for call k-2's traceback).  Three slots
// with the fills alternating between two streams (call k+1's fill starting in call k's fill tail)
// measured slower, 19.5 vs 18.2 ms per headline step (round 5, profiles/pipe_slots_ab_r05.txt).
constexpr int kPipeSlots = SA_PIPELINE_DEPTH;

struct sa_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // cached device workspace (direction slots + row buffers + LUT bits)
    uint8_t* ws = nullptr;
    uint64_t ws_bytes = 0;
    uint64_t ws_limit = 0;  // 0 = automatic
    // cached device I/O buffers for the host API
    uint8_t* io = nullptr;
    uint64_t io_bytes = 0;
    // timing of the last call
    std::vector<hipEvent_t> events;  // 3 per fill launch: start, fill end, traceback end
    int launches = 0;
    // $SEQALIB_KERNEL_TIMING: per launch and variant, events around the fill kernel alone
    // (kKEv per launch: [2k] before, [2k + 1] after variant k's fill; kvars[launch] variants)
    std::vector<hipEvent_t> kevents;
    std::vector<int> kvars;
    hipStream_t timed_stream = nullptr;
    // aux words of the T16 decision (sa_internal.h kAux*), one kAuxWords slot per pipeline slot
    uint32_t* aux = nullptr;
    // plan of the last call: one entry per kernel variant it enqueued (T16 first when the batch
    // was T16-eligible by scoring and shape; the device picked one by the batch alphabet, and
    // h_sel receives that choice asynchronously, ev_sel marks its arrival)
    int nvar = 0, var_kernel[2] = {0, 0}, var_R[2] = {0, 0}, var_W[2] = {0, 0}, var_records[2] = {0, 0};
    uint32_t* h_sel = nullptr;
    hipEvent_t ev_sel = nullptr;
    // the last call's selection when the host decided it (host_alphabet), else -1: then the
    // device's word arrives in h_sel (a host write there could race with a pending download)
    int host_sel = -1;
    // cross-call pipeline of the device API (sa_set_pipeline): fills on s_fill, tracebacks on
    // s_tb, kPipeSlots workspace slots; ev_slot[k] = traceback of the last call that used slot k done
    int pipeline = 0;
    // Band-unit hand-off buffer (score-only SW / NW fills, sa_fill_impl.h BU): the row granules, the
    // column-segment state and the per-unit maxima, all {tag, value} words polled by their consumers.
    // Only those fills write it (every kernel that touches it runs on the fill stream, so one copy
    // serves both pipeline slots), and it is zeroed when allocated and whenever hand_tag wraps: a word
    // there carries the tag of the launch that wrote it or 0, so a consumer can never take an earlier
    // launch's word -- of any shape -- for its producer's.  hand_tag: the last launch's tag, 1..65535.
    uint8_t* hand = nullptr;
    uint64_t hand_bytes = 0;
    uint32_t hand_tag = 0;
    bool hand_dirty = false;   // (tests: sa_test_hook poisoned it) zero before the next launch
    hipStream_t s_fill = nullptr, s_tb = nullptr;
    hipEvent_t ev_in = nullptr, ev_slot[kPipeSlots] = {};
    // The f16 SW cell (sa_fill_so2.hip FK) re-runs in int32 every pair whose score may pass 2,000.
    // Each of its launches has a number f16_seq; its end cell posts {seq, flagged pairs} to h_f16
    // (coherent pinned, d_f16 on the device) and f16_cnt[seq % 4] keeps the launch's pair count.
    // A launch that flagged more than 1/64 of its pairs turns the cell off for the context
    // (f16_off): such batches run the 16-bit integer cell, exact to 8,191, instead of re-running.
    unsigned long long* h_f16 = nullptr;
    unsigned long long* d_f16 = nullptr;
    uint32_t f16_seq = 0, f16_seen = 0, f16_cnt[4] = {};
    bool f16_off = false;
    uint64_t pipe_k = 0;
    // SPLIT plans (few pairs, one workgroup per band): [ticket, pad to 256 B][granules][partials]
    uint8_t* split = nullptr;
    uint64_t split_bytes = 0;
    // HirschbergSA / MyersMillerSA level-loop buffers and the host API's pinned upload staging
    sa::DcWork dc;
    sa::HostBuf<uint8_t> stage, ostage;
    // the small-call path (align_tiny): coherent pinned inputs and outputs the kernel reads and
    // writes in place (host pointer, device pointer)
    uint8_t* tiny_io = nullptr;
    uint8_t* tiny_dev = nullptr;
    // host API: download stream and per-chunk events (align_host)
    hipStream_t s_out = nullptr;
    std::vector<hipEvent_t> host_ev;
    // Calls on one context are ordered: every call's stream waits for ev_last, the end of the
    // last un-pipelined call (whatever stream it ran on), since they share the workspace, the
    // I/O cache and the DC buffers.
    hipEvent_t ev_last = nullptr;
    bool ev_last_set = false;
};

namespace {

thread_local std::string g_err;

int fail(sa_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    g_err = msg;
    return code;
}

int hip_fail(sa_ctx* c, hipError_t e, const char* what) {
    return fail(c, SA_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define SA_HIP(c, call)                                   \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_fail(c, e_, #call); \
    } while (0)

// Order a call on stream st after the context's last call, and mark the end of this one.
int order_after_last(sa_ctx* c, hipStream_t st) {
    if (c->ev_last_set) SA_HIP(c, hipStreamWaitEvent(st, c->ev_last, 0));
    return SA_OK;
}
int mark_last(sa_ctx* c, hipStream_t st) {
    if (!c->ev_last) SA_HIP(c, hipEventCreateWithFlags(&c->ev_last, hipEventDisableTiming));
    SA_HIP(c, hipEventRecord(c->ev_last, st));
    c->ev_last_set = true;
    return SA_OK;
}
// Before a context buffer is freed: every stream that may still use it has finished.
int drain(sa_ctx* c) {
    SA_HIP(c, hipStreamSynchronize(c->stream));
    if (c->s_fill) SA_HIP(c, hipStreamSynchronize(c->s_fill));
    if (c->s_tb) SA_HIP(c, hipStreamSynchronize(c->s_tb));
    if (c->s_out) SA_HIP(c, hipStreamSynchronize(c->s_out));
    if (c->ev_last_set) SA_HIP(c, hipEventSynchronize(c->ev_last));
    return SA_OK;
}

// ------------------------------------------------------------------------------- planning
struct Plan {
    int R, W;
    Geom g;
    uint64_t rowbuf_elems;  // int32 per slot
    bool split = false;     // one single-wave workgroup per (pair, band), cross-workgroup hand-off
};

// SPLIT plan when a batch is too small to fill the chip one workgroup per pair and its pairs
// have at least two bands of 256 rows.  SEQALIB_SPLIT=0 disables it.
bool split_ok(uint32_t max_m, uint32_t max_n, uint32_t npairs, bool allow_split) {
    if (!allow_split) return false;
    if (const char* e = getenv("SEQALIB_SPLIT")) if (e[0] == '0') return false;
    return npairs < 1024 && max_m > 4u * kWave && max_n > 0;
}

Plan make_plan(int algo, uint32_t max_m, uint32_t max_n, uint32_t npairs, bool t16, bool allow_split = true) {
    Plan p;
    const bool aff = is_affine(algo);
    const int rmax = aff ? 16 : 16;
    if (npairs >= 1024 && t16) {
        // Many pairs, T16: one wave per workgroup running its bands back to back (no pipeline
        // skew between bands; hand-off through the row buffer), R up to 32 rows per lane.
        p.W = 1;
        p.R = 4;
        const int rcap = aff ? 16 : 32;   // T16 affine: 4 rows of state per lane row
        while (p.R < rcap && (uint64_t)kWave * p.R < max_m) p.R *= 2;
    } else if (npairs >= 1024) {
        // Many pairs, int32 kernel: one wave per workgroup as well (measured 9-10 % faster than
        // 4-wave band pipelines on 10,000 x 1024^2 LocalGotoh / GlobalGotoh, profiles/gotoh_r02.jsonl),
        // R up to 8 rows per lane for the affine cell (R = 16 is 1 % slower) and 16 for linear.
        p.W = 1;
        p.R = 4;
        const int rcap = aff ? 8 : 16;
        while (p.R < rcap && (uint64_t)kWave * p.R < max_m) p.R *= 2;
    } else if (split_ok(max_m, max_n, npairs, allow_split)) {
        // Few pairs, several bands each: every band its own single-wave workgroup (on its own
        // SIMD, anywhere on the chip), bands of a pair chained through HBM/L2 hand-offs.  A pair
        // then takes about (n + 63 + (bands - 1) * lag) steps of one lone wave each, and a step
        // costs ~40 + 36 R cycles (tools/microbench_lone.hip): short bands win while the chip has
        // a SIMD for every band -- R = 2 (128 rows) -- then R = 4 and 8 for throughput.
        p.W = 1;
        p.R = 8;
        for (int r : {2, 4}) {
            if ((uint64_t)npairs * ((max_m + (uint64_t)kWave * r - 1) / ((uint64_t)kWave * r)) <= 1024) {
                p.R = r;
                break;
            }
        }
        p.split = true;
    } else {
        // Few pairs: widen the workgroup instead (up to 16 waves) to use one CU fully.
        p.R = rmax;
        const uint64_t rows = (uint64_t)kWave * p.R;
        uint64_t w = (max_m + rows - 1) / rows;
        p.W = (int)std::max<uint64_t>(1, std::min<uint64_t>(16, w));
        while (p.R > 4 && (uint64_t)kWave * (p.R / 2) * p.W >= max_m) p.R /= 2;
    }
    // tuning override: SEQALIB_PLAN="R,W" (W = 0: SPLIT plan with R in {1, 2, 4, 8})
    if (const char* ov = getenv("SEQALIB_PLAN")) {
        int r = 0, w = 0;
        // (never for a plan that must not be SPLIT: the SPLIT fallback of build_variants)
        if (sscanf(ov, "%d,%d", &r, &w) == 2 && w == 0 && allow_split && (r == 1 || r == 2 || r == 4 || r == 8)) {
            p.R = r;
            p.W = 1;
            p.split = true;
        } else if (sscanf(ov, "%d,%d", &r, &w) == 2 && (r == 4 || r == 8 || r == 16 || ((r == 32 || r == 64) && t16 && !aff)) &&
            w >= 1 && w <= 16) {
            p.R = r;
            p.W = w;
            p.split = false;
        }
    }
    if ((p.R >= 32 || (t16 && aff && p.R >= 16)) && p.W > 4) p.W = 4;   // fill_max_threads (sa_fill_impl.h)
    // never more waves than bands
    const uint64_t bands = (max_m + (uint64_t)kWave * p.R - 1) / ((uint64_t)kWave * p.R);
    if ((uint64_t)p.W > bands) p.W = (int)std::max<uint64_t>(1, bands);
    p.g = make_geom(algo, p.R, max_m, max_n, t16);
    p.rowbuf_elems = (uint64_t)(aff ? 2 : 1) * std::max<uint32_t>(max_n, 1);
    return p;
}

// One kernel variant of a batch: its plan, end-cell tracking and per-pair workspace
// ([dirs][row buffer][end-cell snapshots h][p][m], in that order inside a launch's block).
struct Variant {
    Plan pl;
    bool t16 = false, cmax = false;
    bool so = false;   // score-only fill + block-recompute traceback (sa_traceback_so.hip)
    uint32_t snap_nch = 0;
    uint64_t snap_h_slot = 0, snap_p_slot = 0;   // 32-bit words per pair
    uint64_t part_slot = 0;   // score-only band units: 64-bit per-unit maxima per pair
    uint32_t segs = 1;        // score-only SW / NW: column segments per band (FillParams::part_segs)
    uint64_t seg_slot = 0;    // their hand-off words per pair (FillParams::seg_hand)
    uint64_t snap_c_slot = 0; // score-only SW: 32-bit (band, chunk) maxima per pair (FillParams::snap_c)
    bool so2 = false;         // score-only SW with two pairs per wave (sa_fill_so2.hip)
    uint64_t slot_bytes = 0;
    int kernel = SA_KERNEL_INT32;
};

Variant make_variant(int algo, uint32_t max_m, uint32_t max_n, uint32_t npairs, bool t16, bool allow_split) {
    Variant v;
    v.t16 = t16;
    v.pl = make_plan(algo, max_m, max_n, npairs, t16, allow_split);
    // CMAX end-cell tracking (sa_fill_impl.h / sa_endcell.hip): T16 SW on one-wave plans with an
    // end-cell replay instantiation (R <= 32)
    v.cmax = t16 && v.pl.W == 1 && v.pl.R >= 2 &&
             ((algo == SA_SW && v.pl.R <= 32) || (algo == SA_LOCAL_GOTOH && v.pl.R <= 16));
    if (const char* ec = getenv("SEQALIB_CMAX")) if (ec[0] == '0') v.cmax = false;
    // Score-only fill (T16 many-pairs plans): no per-cell records; the traceback recomputes the
    // blocks along its path from per-chunk snapshots and the edge stream.  SW with the chunk-max end
    // cell; NW (whose walk starts at (m, n)) from the plain T16 plan.  SEQALIB_SO=0 keeps the tagged
    // records (A/B, tests).
    const bool so_plan = !v.pl.split && v.pl.W == 1 && v.pl.R >= 4 && v.pl.R <= 32;
    const bool local = algo == SA_SW || algo == SA_LOCAL_GOTOH;
    v.so = so_plan && t16 && (local ? v.cmax : true) && algo <= SA_GLOBAL_GOTOH;
    if (const char* e = getenv("SEQALIB_SO")) if (e[0] == '0') v.so = false;
    if (v.cmax || v.so) {
        v.snap_nch = chunks_per_band(max_n);
        v.snap_p_slot = (uint64_t)v.pl.g.bands * v.snap_nch * kWave;
        // per lane: R 16-bit values (LocalGotoh: M, then Iy, then the last row's Ix: R + 1 words)
        v.snap_h_slot = v.snap_p_slot * (is_affine(algo) ? v.pl.R + 1 : v.pl.R / 2);
        // every band's top row: the end-cell replay reads them, and the score-only fill's band units
        // hand them over
        v.pl.rowbuf_elems = (uint64_t)(is_affine(algo) ? 2 : 1) * v.pl.g.bands * std::max<uint32_t>(max_n, 1);
    }
    if (v.so) {
        v.pl.g = make_geom(algo, v.pl.R, max_m, max_n, kGeomEdge);
        // two pairs per wave (sa_fill_so2.hip): the packed cell, for the SW / NW band units at R = 16 / 32;
        // $SEQALIB_SO2=0 runs one pair per wave (A/B, tests)
        v.so2 = (algo == SA_SW || algo == SA_NW) && (v.pl.R == 16 || v.pl.R == 32);
        if (const char* e = getenv("SEQALIB_SO2")) if (e[0] == '0') v.so2 = false;
        if (!is_affine(algo)) {
            // column segments: a band's chunks in kSoSegs (two pairs per wave: kSo2Segs) units of at
            // least 2 chunks each, so the launch tail is a fraction of a band (sa_fill_impl.h BU);
            // $SEQALIB_SO_SEGS sets the count
            // (two pairs per wave: at least 8 chunks per segment -- 1024^2 batches take 4)
            uint32_t sg = v.so2 ? std::max(2u, std::min(kSo2Segs, v.snap_nch / 8)) : kSoSegs;
            if (const char* e = getenv("SEQALIB_SO_SEGS")) sg = (uint32_t)std::max(1, atoi(e));
            v.segs = std::max(1u, std::min(sg, v.snap_nch / 2));
            v.seg_slot = v.segs > 1 ? (uint64_t)v.pl.g.bands * v.segs * (v.pl.R + 1) * kWave : 0;
        }
        v.part_slot = (uint64_t)v.pl.g.bands * v.segs;
        if (algo == SA_SW) v.snap_c_slot = (uint64_t)v.pl.g.bands * v.snap_nch;
    }
    if (v.pl.split) v.pl.rowbuf_elems = 0;   // hand-off granules live in c->split
    v.kernel = v.cmax ? SA_KERNEL_T16_ENDCELL : t16 ? SA_KERNEL_T16 : SA_KERNEL_INT32;
    v.slot_bytes = v.pl.g.dir_slot + v.pl.rowbuf_elems * 4 + (v.snap_h_slot + 2 * v.snap_p_slot) * 4 + v.part_slot * 8 +
                   v.snap_c_slot * 4 + v.seg_slot * 4;
    return v;
}

__global__ void lut_to_bits(const uint8_t* lut, uint32_t* bits) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;  // 2048 words
    if (w >= 2048) return;
    const int a = w >> 3, b0 = (w & 7) * 32;
    uint32_t v = 0;
    for (int k = 0; k < 32; ++k) v |= (lut[a * 256 + b0 + k] != 0 ? 1u : 0u) << k;
    bits[w] = v;
}

// Host API downloads of a one-chunk call: the op streams packed back to back (pair q's nops bytes at
// cpos[q], the exclusive prefix sum of nops; cpos[cnt] = the total), so the D2H moves the ops the
// walks wrote instead of the m + n + 1 bytes reserved per pair (the headline batch: 48 of 92 MB).
// ops_scan: one workgroup; ops_pack: one workgroup per pair.
// cpos2: the same over ceil(nops / 4) (the 2-bit streams, ops_pack).
__global__ __launch_bounds__(1024) void ops_scan(const sa_result* res, uint32_t cnt, uint64_t* cpos, uint64_t* cpos2) {
    __shared__ uint64_t s_part[1024], s_part2[1024];
    const uint32_t t = threadIdx.x, per = (cnt + 1023) / 1024;
    const uint32_t a = min(t * per, cnt), b = min(a + per, cnt);
    uint64_t sum = 0, sum2 = 0;
    for (uint32_t q = a; q < b; ++q) {
        sum += res[q].nops;
        sum2 += (res[q].nops + 3) / 4;
    }
    s_part[t] = sum;
    s_part2[t] = sum2;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {   // inclusive scan (Hillis-Steele)
        const uint64_t v = t >= off ? s_part[t - off] : 0, v2 = t >= off ? s_part2[t - off] : 0;
        __syncthreads();
        s_part[t] += v;
        s_part2[t] += v2;
        __syncthreads();
    }
    uint64_t base = s_part[t] - sum, base2 = s_part2[t] - sum2;
    for (uint32_t q = a; q < b; ++q) {
        cpos[q] = base;
        if (cpos2) cpos2[q] = base2;
        base += res[q].nops;
        base2 += (res[q].nops + 3) / 4;
    }
    if (t == 1023) {
        cpos[cnt] = s_part[1023];
        if (cpos2) cpos2[cnt] = s_part2[1023];
    }
}
__global__ __launch_bounds__(256) void ops_pack(const uint64_t* o1, const uint64_t* o2, const sa_result* res,
                                                const uint64_t* cpos, const uint8_t* ops, uint8_t* packed,
                                                const uint64_t* cpos2, uint8_t* packed2, uint8_t* letters) {
    const uint32_t q = blockIdx.x;
    const uint8_t* src = ops + o1[q] + o2[q] + q;
    uint8_t* dst = packed + cpos[q];
    const uint32_t n = res[q].nops;
    uint8_t* dst2 = packed2 ? packed2 + cpos2[q] : nullptr;
    // the same ops at 2 bits (sa_codec.cpp): M 0, S / X 1, U 2, L 3, one letter per lane, four lanes'
    // codes to one byte by DPP; seen: bit 0 S, bit 1 X, bit 2 another letter (the host then
    // downloads the bytes)
    uint32_t seen = 0;
    for (uint32_t k0 = 0; k0 < n; k0 += blockDim.x) {   // (uniform trip count: the DPP below)
        const uint32_t k = k0 + threadIdx.x;
        const uint32_t ch = k < n ? src[k] : 'M';
        if (k < n) dst[k] = (uint8_t)ch;
        if (!dst2) continue;
        const uint32_t code = ch == 'M' ? 0u : (ch == 'S' || ch == 'X') ? 1u : ch == 'U' ? 2u : 3u;
        seen |= ch == 'S' ? 1u : ch == 'X' ? 2u : (ch == 'M' || ch == 'U' || ch == 'L') ? 0u : 4u;
        // lane 4i + t holds code t of byte i: or in lanes +1, +2, +3 (row_shr within rows of 16)
        uint32_t v = code << (2 * (threadIdx.x & 3));
        v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xf, 0xf, false);   // row_shl:1
        v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x102, 0xf, 0xf, false);   // row_shl:2
        if ((threadIdx.x & 3) == 0 && k < n) dst2[k / 4] = (uint8_t)v;
    }
    if (dst2) {
        // one byte per pair, or-ed on the host: 40,000 waves or-ing one word serialise on it (0.48 ms)
        __shared__ uint32_t s_seen;
        if (threadIdx.x == 0) s_seen = 0;
        __syncthreads();
        for (int off = 32; off >= 1; off >>= 1) seen |= (uint32_t)__shfl_xor((int)seen, off);
        if ((threadIdx.x & 63) == 0 && seen) atomicOr(&s_seen, seen);
        __syncthreads();
        if (threadIdx.x == 0) letters[q] = (uint8_t)s_seen;
    }
}

// 2-bit sequence pieces (sa_codec.cpp dna2_pack) back to bytes: codes 0 A, 1 C, 2 T, 3 G; one
// thread per 4 packed bytes (16 symbols).  n: symbols.
__global__ __launch_bounds__(256) void dna2_unpack(const uint8_t* pk, uint8_t* dst, uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (16 * t >= n) return;
    const uint32_t w = *reinterpret_cast<const uint32_t*>(pk + 4 * t);   // (the landing zone is padded)
    uint32_t o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = (w >> (2 * (4 * d + k))) & 3u;
            x |= (0x47544341u >> (8 * c) & 0xffu) << (8 * k);   // "ACTG"
        }
        o[d] = x;
    }
    if (16 * t + 16 <= n) {
        *reinterpret_cast<uint4*>(dst + 16 * t) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
        const uint8_t* ob = reinterpret_cast<const uint8_t*>(o);
        for (uint64_t k = 16 * t; k < n; ++k) dst[k] = ob[k - 16 * t];
    }
}

// Traceback flavour per launch: one wave per pair (sa_traceback_wave.hip) for few pairs, one lane
// per pair (sa_traceback.hip) for batches.  SEQALIB_TB=wave|lane overrides.
bool tb_wave(uint32_t count) {
    if (const char* e = getenv("SEQALIB_TB")) {
        if (!strcmp(e, "wave") || !strcmp(e, "seg")) return true;
        if (!strcmp(e, "lane")) return false;
    }
    return count < 1024;
}

// Segmented traceback (sa_traceback_seg.hip) of SPLIT launches with the wave walker: 1 for the
// pairs whose walk is long (seg_take), 2 for every pair (SEQALIB_TB=seg, tests), 0 off
// (SEQALIB_TB=wave|lane).  It needs per pair and band NST * (n + 1) + 1 exit records, so it is
// offered to launches of at most kSegMaxBands (pair, band) slots (16,384 when forced).
constexpr uint64_t kSegMaxBands = 512;
int tb_seg_mode() {
    if (const char* e = getenv("SEQALIB_TB")) {
        if (!strcmp(e, "seg")) return 2;
        if (!strcmp(e, "wave") || !strcmp(e, "lane")) return 0;
    }
    return 1;
}

int zero_hand(sa_ctx* c, uint64_t need, hipStream_t st, bool grow);
// Before a band-unit launch: the hand-off buffer (sa_ctx::hand, grow-only) holds need bytes, and
// a fresh one -- or one whose tag is about to wrap -- is zeroed on the fill stream st, where every
// kernel that reads or writes it runs.  Then the launch takes the next tag (c->hand_tag).
int next_hand_tag(sa_ctx* c, uint64_t need, hipStream_t st) {
    const bool grow = c->hand_bytes < need;
    if (grow || c->hand_dirty || c->hand_tag >= 65535) {
        if (int rc = zero_hand(c, need, st, grow)) return rc;
    }
    ++c->hand_tag;
    return SA_OK;
}

int zero_hand(sa_ctx* c, uint64_t need, hipStream_t st, bool grow) {
    if (grow) {
        if (c->hand) {
            if (int rc = drain(c)) return rc;
            (void)hipFree(c->hand);
            c->hand = nullptr;
            c->hand_bytes = 0;
        }
        if (hipMalloc(&c->hand, need) != hipSuccess) {
            c->hand = nullptr;
            return fail(c, SA_ERR_NOMEM, "hipMalloc of the band hand-off buffer (" + std::to_string(need) + " bytes) failed");
        }
        c->hand_bytes = need;
    }
    SA_HIP(c, hipMemsetAsync(c->hand, 0, c->hand_bytes, st));
    c->hand_tag = 0;
    c->hand_dirty = false;
    return SA_OK;
}

int ensure_ws(sa_ctx* c, uint64_t need) {
    if (c->ws_bytes >= need) return SA_OK;
    if (c->ws) {
        if (int rc = drain(c)) return rc;
        (void)hipFree(c->ws);
        c->ws = nullptr;
        c->ws_bytes = 0;
    }
    hipError_t e = hipMalloc(&c->ws, need);
    if (e != hipSuccess) {
        c->ws = nullptr;
        return fail(c, SA_ERR_NOMEM, "hipMalloc workspace of " + std::to_string(need) + " bytes failed");
    }
    c->ws_bytes = need;
    return SA_OK;
}

// The I/O cache of the host API (device copies of the caller's buffers; the device API keeps the
// LUT bits in its tail): grow-only.
int ensure_io(sa_ctx* c, uint64_t need) {
    if (c->io_bytes >= need) return SA_OK;
    if (c->io) {
        if (int rc = drain(c)) return rc;
        (void)hipFree(c->io);
        c->io = nullptr;
        c->io_bytes = 0;
    }
    if (hipMalloc(&c->io, need) != hipSuccess) {
        c->io = nullptr;
        return fail(c, SA_ERR_NOMEM, "hipMalloc of I/O buffers (" + std::to_string(need) + " bytes) failed");
    }
    c->io_bytes = need;
    return SA_OK;
}

uint64_t ws_budget(sa_ctx* c) {
    if (c->ws_limit) return c->ws_limit;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 1ull << 30;
    return (uint64_t)((fr + c->ws_bytes) * 0.8);
}

// 16-bit (score, column) keys for the running maximum are exact when every local score and
// every column fits 16 bits.  With non-positive mismatch and gap terms a local score is at most
// match * min(m, n); otherwise fall back to a generous bound.
bool keyed_ok(int algo, const sa_scoring* sc, uint32_t max_m, uint32_t max_n) {
    if (algo != SA_SW && algo != SA_LOCAL_GOTOH) return false;
    if (max_n >= 65535) return false;
    const bool aff = is_affine(algo);
    const bool nonpos = (!sc->allow_mismatch || sc->mismatch <= 0) &&
                        (aff ? (sc->gap_extend <= 0 && (int64_t)sc->gap_open + sc->gap_extend <= 0)
                             : sc->gap <= 0);
    int64_t bound;
    if (nonpos) {
        bound = (int64_t)std::max(sc->match, 0) * std::min(max_m, max_n);
    } else {
        auto a = [](int32_t x) { return (int64_t)(x < 0 ? -(int64_t)x : x); };
        bound = (a(sc->match) + a(sc->mismatch) + a(sc->gap) + a(sc->gap_open) + a(sc->gap_extend)) *
                ((int64_t)max_m + max_n);
    }
    return bound < 65536;
}

// T16 kernel (sa_fill_impl.h) preconditions on the scoring and shapes.  It keeps 4*H + tag in
// int16 and reads 4*s + 3 from an int8 profile (allow-mismatch, gap < 0 for SW / <= 0 for NW,
// mismatch <= match, |s| small).
//   NW: a constant offset delta is free for a global recurrence (every candidate of a cell shifts
//       alike), so the fill keeps 4*(H - delta): T16 needs the whole range of H, bounded by paths
//       (upper: min(i,j) best diagonals + |i-j| gaps; lower: the all-diagonal and the all-gap
//       path), to fit 2^14 values around delta.
//   SW: H >= 0 and the maximum S bounds every cell; a candidate can only wrap once a correct cell
//       exceeds 8191 - match, and that cell is part of the maximum the fill reports.  When the
//       bound match * min(m, n) does not prove S small enough, T16 still runs and flags every pair
//       whose S exceeds retry_above; the int32 variant re-runs exactly those pairs (kFlagRetry).
//   Gotoh (T16 affine, 8*V + class/extend bits, int8 profile 8*s + 6): gap_extend < 0,
//       gap_open <= 0.  LocalGotoh is bounded like SW (M >= 0, Iy >= GO + GE, the clamped Ix >= 0;
//       retry above 4095 - match); GlobalGotoh like NW, with the affine path bounds, a delta
//       offset, and the reference's -10000 Ix/Iy border provably never winning (else int32).
//       The border becomes `sent`, below every candidate of the range.
struct T16Mode {
    bool ok = false;
    int32_t delta = 0;                // NW / GlobalGotoh offset
    int32_t retry_above = INT_MAX;    // SW / LocalGotoh: per-pair retry threshold
    int32_t sent = -10000;            // T16 affine: encoded Ix / Iy border
    int32_t mismatch = 0;             // the mismatch score the T16 variant runs with (see t16_mode)
};
T16Mode t16_mode_affine(int algo, const sa_scoring* sc, uint32_t max_m, uint32_t max_n) {
    T16Mode t;
    t.mismatch = sc->mismatch;
    const int64_t MA = sc->match, MI = sc->mismatch, GO = sc->gap_open, GE = sc->gap_extend, GOE = GO + GE;
    if (MA < -16 || MA > 15 || MI < -16 || MI > 15 || MI > MA) return t;   // 8s + 6 in int8
    if (GE >= 0 || GO > 0 || GE < -512 || GO < -2048) return t;
    if (max_n >= 65535) return t;
    const int64_t m = max_m, n = max_n, k = std::min(m, n);
    const int64_t sent = -32768 + 8 * (-GE) + 16;   // sent + 8GE + 1 cannot wrap
    const int64_t floor_ext = sent + 8 * GE + 1;    // the border's extend candidate
    if (algo == SA_LOCAL_GOTOH) {
        // every candidate is >= 8 * min(MI, GOE + GE) + 1 (M >= 0, Iy >= GOE)
        if (8 * std::min(MI, GOE + GE) + 1 <= floor_ext) return t;
        t.ok = true;
        t.sent = (int32_t)sent;
        if (8 * std::max<int64_t>(MA, 0) * k + 7 > 32767) t.retry_above = (int32_t)(4095 - std::max<int64_t>(MA, 0));
        return t;
    }
    if (MA < 0) return t;
    // GlobalGotoh: the reference's border wins nowhere (SAGlobalGotoh.h: Ix[0][j] = Iy[i][0] = -10000)
    if (GO + std::max(m, n) * GE + GOE <= -10000 + GE) return t;
    auto gapc = [&](int64_t L) { return L > 0 ? GO + L * GE : 0; };
    auto hi_at = [&](int64_t i, int64_t j) { return std::min(i, j) * MA + gapc(i > j ? i - j : j - i); };
    auto lo_at = [&](int64_t i, int64_t j) {
        return std::max(std::min(i, j) * MI + GO + (i > j ? i - j : j - i) * GE, 2 * GO + (i + j) * GE);
    };
    int64_t hi = INT64_MIN, lo = INT64_MAX;
    const int64_t pts[7][2] = {{0, 0}, {m, 0}, {0, n}, {k, k}, {m, n}, {k, n}, {m, k}};
    for (auto& q : pts) {
        hi = std::max(hi, hi_at(q[0], q[1]));
        lo = std::min(lo, lo_at(q[0], q[1]));
    }
    const int64_t cand_lo = lo + std::min<int64_t>(std::min(MI, GOE + GE), 0);
    int64_t delta = (hi + cand_lo) >> 1;
    if (8 * (hi - delta) + 7 > 32767 || 8 * (cand_lo - delta) <= floor_ext) {
        // The a-priori width does not fit (e.g. 4096^2 at (-3, -1, 1, -1): [-4104, 4096]).  The low
        // end is reached by the borders of every pair, the high end only by near-identical pairs:
        // every value and candidate is the score of an alignment of prefixes, at most
        // MA * (its matches) <= MA * L with L = sum over symbols of min(count in Seq1, count in
        // Seq2).  Place the window at the low end and let the T16 fill screen each pair
        // (retry_above = the largest MA * min(L, m, n) that fits); the int32 variant re-runs
        // the screened-out pairs exactly (kFlagRetry), as for SW.
        delta = cand_lo + 4100;
        while (8 * (cand_lo - delta) <= floor_ext) --delta;   // the largest delta that fits the low end
        const int64_t cap = delta + (32767 - 7) / 8;
        if (cap < std::max<int64_t>(MA, 0) * k / 2) return t;   // not even typical pairs would fit
        t.retry_above = (int32_t)cap;
    }
    t.ok = true;
    t.delta = (int32_t)delta;
    t.sent = (int32_t)sent;
    return t;
}
// !AllowMismatch.  The reference's diagonal term of a mismatch is INT_MIN (SASmithWaterman.h:
// 119-131, SANeedlemanWunsch.h:88-92, SALocalGotoh.h:144-170, SAGlobalGotoh.h), so it never
// wins a max and its traceback never takes a mismatched diagonal (max(INT_MIN, 0) = 0 equals a
// cell only where the zero test stops the walk anyway).  A finite mismatch score MI' loses just
// as surely when MI' < 2 * Gap (linear) / 2 * (GapOpen + GapExtend) (affine): every cell has
// H[i-1][j] >= H[i-1][j-1] + Gap (its left candidate; borders included), so the up candidate is
// >= Hd + 2 * Gap > Hd + MI'; affine: M[i-1][j] >= Iy[i-1][j] >= M[i-1][j-1] + GOE, so
// Ix >= Md + 2 * GOE > Md + MI'.  Strictly smaller, so no tie either: the matrices, the end cell
// and every traceback decision are the reference's, and T16 runs the allow-mismatch kernel with
// MI' = 2 * Gap - 1 (2 * GOE - 1), the largest such score (narrowest score range).
T16Mode t16_mode(int algo, const sa_scoring* sc0, uint32_t max_m, uint32_t max_n) {
    sa_scoring eff = *sc0;
    if (!sc0->allow_mismatch) {
        if (algo != SA_SW && algo != SA_NW && algo != SA_LOCAL_GOTOH && algo != SA_GLOBAL_GOTOH) return T16Mode{};
        const int64_t mi = is_affine(algo) ? 2 * ((int64_t)sc0->gap_open + sc0->gap_extend) - 1 : 2 * (int64_t)sc0->gap - 1;
        if (mi < INT_MIN / 4) return T16Mode{};
        eff.mismatch = (int32_t)mi;
        eff.allow_mismatch = 1;
    }
    const sa_scoring* sc = &eff;
    T16Mode t;
    t.mismatch = sc->mismatch;
    if (algo == SA_LOCAL_GOTOH || algo == SA_GLOBAL_GOTOH) return t16_mode_affine(algo, sc, max_m, max_n);
    if (algo != SA_SW && algo != SA_NW) return t;
    const int64_t MA = sc->match, MI = sc->mismatch, G = sc->gap;
    if (MA < -32 || MA > 31 || MI < -32 || MI > 31) return t;
    if (G > 0 || MI > MA || G < -4096) return t;
    if (algo == SA_SW && G == 0) return t;   // the clamped up term needs gap < 0 (sa_fill_impl.h)
    if (max_n >= 65535) return t;
    const int64_t m = max_m, n = max_n, k = std::min(m, n);
    if (algo == SA_SW) {
        t.ok = true;
        if (4 * std::max<int64_t>(MA, 0) * k + 3 > 32767) t.retry_above = (int32_t)(8191 - std::max<int64_t>(MA, 0));
        return t;
    }
    auto hi_at = [&](int64_t i, int64_t j) {
        return std::max(std::min(i, j) * MA + (i > j ? i - j : j - i) * G, (i + j) * G);
    };
    auto lo_at = [&](int64_t i, int64_t j) {
        return std::max(std::min(i, j) * MI + (i > j ? i - j : j - i) * G, (i + j) * G);
    };
    int64_t hi = INT64_MIN, lo = INT64_MAX;
    const int64_t pts[7][2] = {{0, 0}, {m, 0}, {0, n}, {k, k}, {m, n}, {k, n}, {m, k}};
    for (auto& q : pts) {
        hi = std::max(hi, hi_at(q[0], q[1]));
        lo = std::min(lo, lo_at(q[0], q[1]));
    }
    const int64_t cand_lo = lo + std::min<int64_t>(std::min(MI, G), 0);   // candidates of a cell
    const int64_t delta = (hi + cand_lo) >> 1;
    if (4 * (hi - delta) + 3 > 32767 || 4 * (cand_lo - delta) < -32768) return t;
    t.ok = true;
    t.delta = (int32_t)delta;
    return t;
}

int validate_scoring(sa_ctx* c, int algo, const sa_scoring* s) {
    if (!s) return fail(c, SA_ERR_ARG, "scoring is NULL");
    if (algo < SA_SW || algo > SA_MYERS_MILLER) return fail(c, SA_ERR_ARG, "unknown algorithm");
    return SA_OK;
}

// T16 by scoring and shape (the batch alphabet is checked on the device, decide_t16).
// The f16 cell of the two-pairs-per-wave SW fill (sa_fill_so2.hip FK): the substitutions the T16
// fill runs with (match, tm.mismatch) must be f16 values whose low byte is 0 (+-1..8, 10, 12, 14,
// 16, 20, ...), so that the perm's table byte is their high byte.  $SEQALIB_SO2_F16=0: the 16-bit
// integer cell (A/B, tests).
bool f16_hi_exact(int s) {
    if (s < -2048 || s > 2048) return false;
    const _Float16 h = (_Float16)(float)s;
    return (int)(float)h == s && (__builtin_bit_cast(uint16_t, h) & 0xffu) == 0;
}
bool so2_f16_scoring(const sa_ctx* c, int algo, const sa_scoring* sc, const T16Mode& tm) {
    if (algo != SA_SW || !tm.ok || c->f16_off) return false;
    if (const char* e = getenv("SEQALIB_SO2_F16")) if (e[0] == '0') return false;
    return f16_hi_exact(sc->match) && f16_hi_exact(tm.mismatch) && f16_hi_exact(-128);
}

T16Mode t16_candidate(int algo, const sa_scoring* sc, uint32_t max_m, uint32_t max_n, uint32_t npairs) {
    T16Mode t = t16_mode(algo, sc, max_m, max_n);
    if ((algo == SA_SW || algo == SA_LOCAL_GOTOH) && !keyed_ok(algo, sc, max_m, max_n)) t.ok = false;
    // the screened GlobalGotoh T16 fill (retry_above set) runs on the many-pairs plans only: a
    // SPLIT band cannot leave its pair alone
    if (t.ok && algo == SA_GLOBAL_GOTOH && t.retry_above != INT_MAX &&
        make_variant(algo, max_m, max_n, npairs, true, true).pl.split)
        t.ok = false;
    if (const char* e16 = getenv("SEQALIB_T16")) if (e16[0] == '0') t.ok = false;
    return t;
}

// The kernel variants a call enqueues: T16 (when the scoring and shapes admit it; the device
// picks it or the int32 one by the batch alphabet) and int32, plus -- when a variant uses the
// SPLIT plan -- the int32 single-workgroup FALLBACK, whose launches re-run, inside the same call,
// only the pairs whose SPLIT band wait expired (SA_FLAG_TIMEOUT), so no API returns one.  All
// share one record stride (the int32 variant re-runs single pairs of a T16 batch, kFlagRetry,
// while the T16 traceback still reads their neighbours).  Returns the number of variants;
// vars[nv] is the fallback when *has_fb.
// only: 0 both variants (as above), 1 the T16 variant alone, 2 the int32 variant alone (the host
// decided the batch alphabet itself and T16 provably needs no int32 re-run, run_device).
int build_variants(int algo, uint32_t max_m, uint32_t max_n, uint32_t npairs, bool t16, Variant (&vars)[3],
                   bool* has_fb, int only = 0) {
    int nv = 0;
    if (t16 && only != 2) vars[nv++] = make_variant(algo, max_m, max_n, npairs, true, true);
    if (!t16 || only != 1) vars[nv++] = make_variant(algo, max_m, max_n, npairs, false, true);
    *has_fb = false;
    for (int k = 0; k < nv; ++k) *has_fb = *has_fb || vars[k].pl.split;
    if (*has_fb) vars[nv] = make_variant(algo, max_m, max_n, npairs, false, false);
    const int all = nv + (*has_fb ? 1 : 0);
    uint64_t dir_stride = 0;
    for (int k = 0; k < all; ++k) dir_stride = std::max(dir_stride, vars[k].pl.g.dir_slot);
    for (int k = 0; k < all; ++k) {
        vars[k].slot_bytes += dir_stride - vars[k].pl.g.dir_slot;
        vars[k].pl.g.dir_slot = dir_stride;
    }
    return nv;
}

// The batch alphabet decided on the host (host API calls whose sequences are small enough to scan
// here, align_host): the same decision and profile as decide_t16 (sa_alphabet.hip) -- <= 4
// distinct bytes, padded with absent byte values, prof[c] byte c' = 4s + 3 (8s + 6 affine) with
// s = match(sym c, sym c') ? match : mismatch -- so the device runs no scan and no decide kernel
// and the host knows which variant to enqueue.
struct HostAlphabet {
    int sel = -1;          // -1: decide on the device; 1: T16; 0: int32
    uint32_t prof[5] = {0, 0, 0, 0, 0};
};
HostAlphabet host_alphabet(const uint8_t* s1, uint64_t t1, const uint8_t* s2, uint64_t t2, const uint8_t* lut,
                           int match, int mismatch, bool affine) {
    HostAlphabet h;
    bool seen[256] = {};
    for (uint64_t k = 0; k < t1; ++k) seen[s1[k]] = true;
    for (uint64_t k = 0; k < t2; ++k) seen[s2[k]] = true;
    uint32_t syms[4] = {0, 0, 0, 0};
    int nsym = 0;
    for (int b = 0; b < 256; ++b)
        if (seen[b]) {
            if (nsym == 4) { h.sel = 0; return h; }
            syms[nsym++] = (uint32_t)b;
        }
    for (int b = 0; nsym < 4 && b < 256; ++b)
        if (!seen[b]) syms[nsym++] = (uint32_t)b;
    for (int c = 0; c < 4; ++c) {
        uint32_t w = 0;
        for (int c2 = 0; c2 < 4; ++c2) {
            const bool v = lut ? lut[syms[c] * 256 + syms[c2]] != 0 : syms[c] == syms[c2];
            const int sc = v ? match : mismatch;
            w |= ((uint32_t)(affine ? 8 * sc + 6 : 4 * sc + 3) & 255u) << (8 * c2);
        }
        h.prof[c] = w;
    }
    h.prof[4] = syms[0] | syms[1] << 8 | syms[2] << 16 | syms[3] << 24;
    h.sel = 1;
    return h;
}
// host API batches up to this many sequence bytes are scanned on the host
constexpr uint64_t kHostScanBytes = 1ull << 16;
struct HostSeqs {   // a host API batch's sequences (and host match table) for host_alphabet
    const uint8_t* s1;
    uint64_t t1;
    const uint8_t* s2;
    uint64_t t2;
    const uint8_t* lut;   // 256 x 256 bytes or NULL (equality)
    // small calls (align_host): the inputs are not uploaded yet.  run_device writes the host-decided
    // profile and selection word into the pinned header hhdr, then uploads [header][inputs] with ONE
    // copy (up_bytes from up_src to up_dst; dhdr is where the header lands) before any kernel.
    uint32_t* hhdr = nullptr;
    const uint32_t* dhdr = nullptr;
    // otherwise (pipelined chunks of one host call) the chunk's own pinned slot of 6 words for the
    // profile upload: the chunks are enqueued without a host wait, so they must not share one
    uint32_t* hprof = nullptr;
    void* up_dst = nullptr;
    const void* up_src = nullptr;
    uint64_t up_bytes = 0;
};

// Enqueue fill + traceback for pairs [0, npairs) whose inputs are on the device.  Nothing here
// waits on the host: when the scoring and shapes admit the T16 kernel, the batch alphabet is
// scanned on the device and BOTH variants (T16 and int32) are enqueued, each launch guarded by
// the device's decision (sa_skip), so the launches of the variant not taken return at once.
// pipe: (device API with sa_set_pipeline) fills and end-cell replays go to c->s_fill and
// tracebacks to c->s_tb after the caller's stream reaches this call; workspace and aux use slot
// pipe_k % 2, and the call returns without ordering `stream` after the results (sa_wait).
int run_device(sa_ctx* c, int algo, const sa_scoring* sc, const uint8_t* d1, const uint64_t* o1,
               const uint8_t* d2, const uint64_t* o2, uint32_t npairs, uint32_t max_m,
               uint32_t max_n, const uint32_t* d_lutbits, sa_result* d_res, uint8_t* d_ops,
               hipStream_t stream, bool pipe = false, const uint32_t* d_mbits = nullptr,
               const uint64_t* d_mbits_off = nullptr, const HostSeqs* hs = nullptr) {
    if (max_m >= (1u << 24) || max_n >= (1u << 24))
        return fail(c, SA_ERR_UNSUPPORTED, "sequence lengths must be < 2^24");
    const bool keyed = keyed_ok(algo, sc, max_m, max_n);
    const bool allow = sc->allow_mismatch != 0;
    const bool bits = d_mbits != nullptr;   // generic-Ty path: per-pair match bitmaps
    const bool lut = !bits && d_lutbits != nullptr;
    const T16Mode tm = bits ? T16Mode{} : t16_candidate(algo, sc, max_m, max_n, npairs);
    const bool t16 = tm.ok;
    const bool kernel_timing = getenv("SEQALIB_KERNEL_TIMING") != nullptr;
    if (!c->aux) SA_HIP(c, hipMalloc(&c->aux, kPipeSlots * kAuxWords * 4));
    if (!c->h_sel) {
        SA_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_sel), 64, hipHostMallocDefault));
        SA_HIP(c, hipEventCreateWithFlags(&c->ev_sel, hipEventDisableTiming));
    }
    if (!pipe && c->s_fill) {   // a non-pipelined call reuses slot 0: drain pipelined work first
        SA_HIP(c, hipStreamSynchronize(c->s_fill));
        SA_HIP(c, hipStreamSynchronize(c->s_tb));
    }
    constexpr int nslots = kPipeSlots;
    const int slot = pipe ? (int)(c->pipe_k % (uint64_t)nslots) : 0;
    uint32_t* aux = c->aux + kAuxWords * slot;
    if (pipe && c->ev_slot[slot]) SA_HIP(c, hipStreamWaitEvent(stream, c->ev_slot[slot], 0));   // slot free
    if (!c->h_f16) {
        SA_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_f16), 8, hipHostMallocCoherent));
        *c->h_f16 = 0;
        void* dp = nullptr;
        SA_HIP(c, hipHostGetDevicePointer(&dp, c->h_f16, 0));
        c->d_f16 = static_cast<unsigned long long*>(dp);
    }
    {   // the f16 policy: the latest posted launch (one of the last 4) flagged > 1/64 of its pairs
        const unsigned long long w = __atomic_load_n(c->h_f16, __ATOMIC_ACQUIRE);
        const uint32_t s = (uint32_t)(w >> 32);
        if (s != 0 && s != c->f16_seen) {
            c->f16_seen = s;
            if (c->f16_seq - s < 4 && (uint64_t)(uint32_t)w * 64 > c->f16_cnt[s & 3]) c->f16_off = true;
        }
    }
    const uint32_t* sel = nullptr;
    const uint32_t* prof = aux + kAuxProf;   // the T16 profile words (+5: the selection word)
    static_assert(kAuxSel == kAuxProf + 5, "profile and selection word: one upload");
    int only = 0;   // build_variants: both variants, or the one the host chose
    HostAlphabet hal;
    if (t16 && hs) hal = host_alphabet(hs->s1, hs->t1, hs->s2, hs->t2, hs->lut, sc->match, tm.mismatch, is_affine(algo));
    const HostAlphabet* ha = &hal;
    const bool host_sel = t16 && ha->sel >= 0;
    if (host_sel) {
        // the host decided the alphabet (align_host): upload the profile; enqueue the chosen variant
        // alone -- plus the int32 re-run when T16 may overflow (SW / LocalGotoh retry_above, the
        // screened GlobalGotoh), which then reads the selection word as usual
        c->host_sel = ha->sel;
        const bool in_hdr = hs->hhdr != nullptr;   // (small call: travels with the inputs)
        if (!in_hdr && !hs->hprof) return fail(c, SA_ERR_ARG, "internal: no pinned profile slot");
        uint32_t* const hp = in_hdr ? hs->hhdr : hs->hprof;   // pinned, this call's / chunk's own
        for (int k = 0; k < 5; ++k) hp[k] = ha->prof[k];
        hp[5] = (uint32_t)ha->sel;
        if (in_hdr) prof = hs->dhdr;
        else SA_HIP(c, hipMemcpyAsync(aux + kAuxProf, hp, 24, hipMemcpyHostToDevice, stream));
        // (band units that hand state between workgroups keep the int32 variant: a unit whose wait
        // for its producer expired flags its pair for that re-run, sa_fill_impl.h BU)
        const Variant vt = make_variant(algo, max_m, max_n, npairs, true, true);
        const bool bu_hand = vt.so && !is_affine(algo) && (vt.pl.g.bands > 1 || vt.segs > 1);
        // (the f16 cell may flag any pair: its int32 re-run stays)
        const bool f16 = vt.so2 && so2_f16_scoring(c, algo, sc, tm);
        if (ha->sel == 0) only = 2;
        else if (tm.retry_above == INT_MAX && !bu_hand && !f16) only = 1;
        else sel = prof + 5;
    }
    if (hs && hs->up_bytes)
        SA_HIP(c, hipMemcpyAsync(hs->up_dst, hs->up_src, hs->up_bytes, hipMemcpyHostToDevice, stream));
    if (host_sel) {
        SA_HIP(c, hipEventRecord(c->ev_sel, stream));
    } else if (t16) {
        c->host_sel = -1;
        SA_HIP(c, launch_alphabet_scan(d1, o1, d2, o2, npairs, aux, stream));
        SA_HIP(c, launch_decide_t16(d_lutbits, sc->match, tm.mismatch, is_affine(algo) ? 1 : 0, aux, stream));
        SA_HIP(c, hipMemcpyAsync(c->h_sel, aux + kAuxSel, 4, hipMemcpyDeviceToHost, stream));
        SA_HIP(c, hipEventRecord(c->ev_sel, stream));
        sel = aux + kAuxSel;
    }
    Variant vars[3];
    bool has_fb = false;
    const int nv = build_variants(algo, max_m, max_n, npairs, t16, vars, &has_fb, only);
    if (const char* e = getenv("SEQALIB_SPLIT_FALLBACK")) has_fb = has_fb && e[0] != '0';   // tests only
    c->nvar = nv;
    uint64_t slot_bytes = 0, sp_bands = 0;
    bool any_split = false;
    for (int k = 0; k < nv + (has_fb ? 1 : 0); ++k) {
        if (k < nv) {
            c->var_kernel[k] = vars[k].kernel;
            c->var_R[k] = vars[k].pl.R;
            c->var_W[k] = vars[k].pl.split ? 0 : vars[k].pl.W;   // 0: SPLIT plan (one single-wave workgroup per band)
            c->var_records[k] = vars[k].so ? SA_RECORDS_SCORE_ONLY : vars[k].t16 ? SA_RECORDS_TAGS : SA_RECORDS_FLAGS;
        }
        slot_bytes = std::max(slot_bytes, vars[k].slot_bytes);
        if (vars[k].pl.split) {
            any_split = true;
            sp_bands = std::max<uint64_t>(sp_bands, vars[k].pl.g.bands);
        }
    }
    const uint64_t budget = pipe ? ws_budget(c) / nslots : ws_budget(c);
    uint64_t per_launch = slot_bytes ? std::max<uint64_t>(1, budget / std::max<uint64_t>(slot_bytes, 1)) : npairs;
    per_launch = std::min<uint64_t>(per_launch, npairs ? npairs : 1);
    per_launch = std::min<uint64_t>(per_launch, 1u << 30);
    const uint64_t need = (per_launch * slot_bytes + 4096 + 255) & ~(uint64_t)255;
    if (need > budget && per_launch == 1 && c->ws_limit)
        return fail(c, SA_ERR_NOMEM, "one pair needs " + std::to_string(slot_bytes) +
                                         " bytes of workspace, above the limit");
    int rc = ensure_ws(c, std::max<uint64_t>(pipe ? nslots * need : need, 4096));
    if (rc) return rc;
    // band units' hand-off words (score-only SW / NW), per launch: [row granules][per-unit words]
    // [segment state], each part 256-byte aligned; one copy for both pipeline slots (sa_ctx::hand)
    auto al256 = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
    uint64_t hand_rb = 0, hand_part = 0, hand_seg = 0;
    for (int k = 0; k < nv; ++k)
        if (vars[k].so && !is_affine(algo)) {
            hand_rb = std::max(hand_rb, al256(per_launch * vars[k].pl.rowbuf_elems * 4));
            hand_part = std::max(hand_part, al256(per_launch * vars[k].part_slot * 8));
            hand_seg = std::max(hand_seg, al256(per_launch * vars[k].seg_slot * 4));
        }
    const uint64_t hand_need = hand_rb + hand_part + hand_seg;
    const uint32_t so_wait_polls = [] {
        const char* e = getenv("SEQALIB_SO_WAIT_POLLS");   // tests only: force the lost-producer path
        return e ? (uint32_t)std::max(1L, atol(e)) : kSoWaitPollsDefault;
    }();
    // SPLIT scratch, per variant: [ticket][hand-off granules] (zeroed before its fill; the
    // segmented traceback reads the granules after both variants' fills), then the per-band
    // partials and the segmented traceback's exit records.  Pipelined calls alternate two copies
    // (the traceback of call k reads its granules beside the fill of call k + 1).
    const uint64_t aff2 = is_affine(algo) ? 2 : 1;
    const uint64_t sp_gran = any_split ? per_launch * sp_bands * std::max<uint32_t>(max_n, 1) * aff2 : 0;
    const uint64_t sp_vblk = (256 + sp_gran * 8 + 255) & ~(uint64_t)255;
    const uint64_t sp_part = (uint64_t)nv * sp_vblk;
    const int seg_mode = any_split && tb_wave((uint32_t)per_launch) ? tb_seg_mode() : 0;
    // tests only: SEQALIB_SPLIT_WAIT_TICKS shortens the SPLIT bands' bounded wait (forces timeouts
    // and the fallback); SEQALIB_SEG_INJECT=1 overwrites the segmented traceback's exit records
    // between its two kernels (forces its consistency guards and the serial re-walk)
    uint64_t wait_ticks = kSplitWaitTicksDefault;
    if (const char* e = getenv("SEQALIB_SPLIT_WAIT_TICKS")) wait_ticks = strtoull(e, nullptr, 10);
    const char* inj = getenv("SEQALIB_SEG_INJECT");
    const bool seg_inject = inj && inj[0] == '1';
    const bool seg_on = seg_mode != 0 && per_launch * sp_bands <= (seg_mode == 2 ? 16384 : kSegMaxBands);
    const uint64_t seg_rs = (uint64_t)aff2 * ((uint64_t)max_n + 1) + 1;
    const uint64_t sp_seg = (sp_part + per_launch * sp_bands * 16 + 255) & ~(uint64_t)255;
    // (a whole number of 256-byte blocks: slot 1 begins at (split_bytes / 2) rounded down to 256,
    // so an unaligned slot size let slot 0's last exit records and slot 1's ticket share bytes --
    // the pipelined calls then corrupted each other's scratch now and then)
    const uint64_t sp_slot = (sp_seg + (seg_on ? (per_launch * sp_bands * seg_rs + per_launch) * 16 : 0) + 255) & ~(uint64_t)255;
    const uint64_t sp_need = any_split ? sp_slot * (pipe ? nslots : 1) : 0;
    if (any_split && c->split_bytes < sp_need) {
        if (c->split) {
            if (int rc = drain(c)) return rc;
            (void)hipFree(c->split);
            c->split = nullptr;
            c->split_bytes = 0;
        }
        if (hipMalloc(&c->split, sp_need) != hipSuccess) {
            c->split = nullptr;
            return fail(c, SA_ERR_NOMEM, "hipMalloc of the split-plan scratch failed");
        }
        c->split_bytes = sp_need;
    }
    // A pipeline slot is one contiguous half of the workspace holding everything its calls
    // write (dirs, row buffers, snapshots), so calls on the other slot never touch it.
    uint8_t* const wbase = c->ws + (pipe ? slot * ((c->ws_bytes / nslots) & ~(uint64_t)255) : 0);
    // (fixed halves of the scratch, as the workspace: a slot's block never moves with the shape)
    uint8_t* const spbase = any_split ? c->split + (pipe ? slot * ((c->split_bytes / nslots) & ~(uint64_t)255) : 0) : nullptr;
    // the pipeline slots must not share a byte (each holds what its calls write)
    if (pipe && (((c->ws_bytes / nslots) & ~(uint64_t)255) < need || (any_split && ((c->split_bytes / nslots) & ~(uint64_t)255) < sp_slot)))
        return fail(c, SA_ERR_HIP, "internal: pipeline slots overlap");

    // reset timing (kernel timings describe this call only: a call without
    // SEQALIB_KERNEL_TIMING leaves none, and sa_last_kernel_timings then fails)
    c->launches = 0;
    c->kvars.clear();
    c->timed_stream = stream;
    hipStream_t sf = stream, stb = stream;
    if (pipe) {
        sf = c->s_fill;
        stb = c->s_tb;
        SA_HIP(c, hipEventRecord(c->ev_in, stream));
        SA_HIP(c, hipStreamWaitEvent(sf, c->ev_in, 0));
    }

    for (uint64_t base = 0; base < npairs; base += per_launch) {
        const uint32_t cnt = (uint32_t)std::min<uint64_t>(per_launch, npairs - base);
        while ((int)c->events.size() < 3 * (c->launches + 1)) {
            hipEvent_t ev;
            SA_HIP(c, hipEventCreate(&ev));
            c->events.push_back(ev);
        }
        hipEvent_t* ev = &c->events[3 * c->launches];
        hipEvent_t* kev = nullptr;   // SEQALIB_KERNEL_TIMING: fill-kernel-only events
        if (kernel_timing) {
            while ((int)c->kevents.size() < kKEv * (c->launches + 1)) {
                hipEvent_t e;
                SA_HIP(c, hipEventCreate(&e));
                c->kevents.push_back(e);
            }
            c->kvars.resize(c->launches + 1);
            c->kvars[c->launches] = nv;
            kev = &c->kevents[kKEv * c->launches];
        }
        // the launches of one call share the slot: launch k+1's fill overwrites the records
        // launch k's traceback reads (on the other stream when pipelined)
        if (pipe && c->launches > 0) SA_HIP(c, hipStreamWaitEvent(sf, c->events[3 * c->launches - 1], 0));
        SA_HIP(c, hipEventRecord(ev[0], sf));
        const uint64_t hand_x_off = any_split ? (uint64_t)cnt * sp_bands * std::max<uint32_t>(max_n, 1) : 0;
        // fill parameters of variant k (k == nv: the SPLIT fallback)
        FillParams fps[3];
        // $SEQALIB_STAGE_SEQ2=0: read Seq2 from global memory in every plan (tests the unstaged
        // path that batches with max_n > kMaxStagedSeq2 take)
        const char* stage_env = getenv("SEQALIB_STAGE_SEQ2");
        const bool no_stage = stage_env && stage_env[0] == '0';
        auto make_fp = [&](int k) {
            const Variant& v = vars[k];
            const Plan& pl = v.pl;
            // each SPLIT variant (the int32 one re-runs flagged pairs) has its own tickets and
            // hand-off granules
            uint8_t* const vblk = pl.split ? spbase + (uint64_t)k * sp_vblk : nullptr;
            int32_t* rowbuf = reinterpret_cast<int32_t*>(wbase + per_launch * pl.g.dir_slot);
            uint32_t* snap_h = reinterpret_cast<uint32_t*>(rowbuf + per_launch * pl.rowbuf_elems);
            int32_t* snap_p = reinterpret_cast<int32_t*>(snap_h + per_launch * v.snap_h_slot);
            FillParams& fp = fps[k];
            fp = FillParams{};
            fp.seq1 = d1; fp.off1 = o1; fp.seq2 = d2; fp.off2 = o2;
            fp.lutbits = lut ? d_lutbits : nullptr;
            fp.mbits = d_mbits; fp.mbits_off = d_mbits_off;
            fp.dirs = wbase; fp.dir_slot = pl.g.dir_slot; fp.band_stride = pl.g.band_stride;
            fp.rowbuf = rowbuf; fp.rowbuf_slot = pl.rowbuf_elems;
            fp.res = d_res;
            fp.pair_base = (uint32_t)base;
            fp.max_m = max_m; fp.max_n = max_n;
            // the T16 variant runs !AllowMismatch as allow-mismatch with tm.mismatch (t16_mode)
            fp.gap = sc->gap; fp.match = sc->match;
            fp.mismatch = v.t16 ? tm.mismatch : allow ? sc->mismatch : INT_MIN;
            fp.gap_open = sc->gap_open; fp.gap_extend = sc->gap_extend;
            fp.waves = pl.W;
            fp.count = cnt;
            fp.stage_seq2 = (max_n <= kMaxStagedSeq2 && !no_stage) ? 1 : 0;
            fp.prof = prof;
            const bool fb = k == nv;
            fp.sel = fb ? nullptr : sel; fp.sel_want = v.t16 ? 1u : 0u;
            fp.redo = (!fb && nv == 2 && !v.t16) ? 1 : 0;
            fp.rerun = fb ? 1 : 0;
            fp.t16_delta = v.t16 ? tm.delta : 0;
            fp.retry_above = v.t16 ? tm.retry_above : INT_MAX;
            fp.t16_sent = v.t16 ? tm.sent : -10000;
            fp.snap_h = snap_h; fp.snap_p = snap_p; fp.snap_m = snap_p + per_launch * v.snap_p_slot;
            if (v.so) {   // (after the chunk maxima) per-(band, chunk) maxima; ticket below
                fp.part_bands = (uint32_t)v.pl.g.bands;
                fp.snap_c = reinterpret_cast<int32_t*>(snap_p + 2 * per_launch * v.snap_p_slot);
                fp.seg_slot = v.seg_slot;
            }
            if (v.so && !is_affine(algo)) {   // band units: this launch's tag, the hand-off buffer
                fp.epoch = c->hand_tag;   // (set by the launch loop below)
#ifndef SA_R5_CONTROL
                fp.rowbuf = reinterpret_cast<int32_t*>(c->hand);
                fp.band_part = reinterpret_cast<unsigned long long*>(c->hand + hand_rb);
                fp.seg_hand = reinterpret_cast<uint32_t*>(c->hand + hand_rb + hand_part);
#else
                // control build of tests/test_gpu_handoff.py (make variant V=r5ctl DEFS=-DSA_R5_CONTROL):
                // round 5's layout, the hand-off words in the shared workspace after the chunk maxima
                const uintptr_t bp = (reinterpret_cast<uintptr_t>(fp.snap_c + per_launch * v.snap_c_slot) + 7) & ~(uintptr_t)7;
                fp.band_part = reinterpret_cast<unsigned long long*>(bp);
                fp.seg_hand = reinterpret_cast<uint32_t*>(fp.band_part + per_launch * v.part_slot);
#endif
                fp.wait_polls = so_wait_polls;
            }
            fp.snap_h_slot = v.snap_h_slot; fp.snap_p_slot = v.snap_p_slot; fp.snap_nch = v.snap_nch;
            fp.split_bands = (uint32_t)sp_bands;
            fp.ticket = pl.split ? reinterpret_cast<uint32_t*>(vblk) : v.so ? aux + kAuxTicket : nullptr;
            fp.hand = pl.split ? reinterpret_cast<unsigned long long*>(vblk + 256) : nullptr;
            fp.hand_x_off = pl.split ? hand_x_off : 0;
            fp.part = pl.split ? reinterpret_cast<int32_t*>(spbase + sp_part) : nullptr;
            fp.wait_ticks = wait_ticks;
            fp.part_segs = std::max<uint32_t>(1, v.segs);
            if (v.so2) {
                // LDS for the unit's Seq2 codes, per pair: the widest column range a unit may run
                // (ceil(chunks / segments) chunks + the 64 columns before them; one segment below 4
                // chunks), when both pairs' fit 8 KiB (16 units per CU at 4 waves per SIMD)
                const uint32_t nch = chunks_per_band(max_n);
                const uint32_t sg = std::max(1u, std::min(fp.part_segs, nch / 2));
                const uint32_t range = std::max((nch + sg - 1) / sg, 3u) * kChunk + kWave;
                const uint32_t cap = (range + 15) & ~15u;
                fp.so2_stage = (2 * cap <= 8192 && !no_stage) ? cap : 0;
                if (v.t16 && so2_f16_scoring(c, algo, sc, tm)) {
                    fp.so2_f16 = 1;
                    fp.retry_above = std::min(fp.retry_above, kSo2F16RetryAbove);
                }
            }
            FillVariant fv{pl.R, lut, allow || v.t16, keyed, v.t16, v.cmax, pl.split, bits};
            fv.so = v.so;
            fv.so2 = v.so2;
            return fv;
        };
        // Pipelined calls: the int32 variant of a T16 batch (it re-runs only the pairs the T16 fill
        // flagged, or every pair when the device chose int32) walks its traceback on the fill stream
        // right after its fill.  On the traceback stream, behind the score-only traceback, its
        // workgroups waited for the next call's fill to be dispatched (up to 9.6 ms, round 4 rocprof)
        // and delayed the slot's release to the call after it.  It then walks before the T16 variant,
        // so the pairs it re-ran are handed over by flags (TbParams::keep_redo / clear_redo).
        const bool tb_on_fill = pipe && nv == 2 && !vars[1].t16 && !vars[1].pl.split;
        auto make_tp = [&](int k) {
            const Variant& v = vars[k];
            TbParams tp{};
            tp.seq1 = d1; tp.off1 = o1; tp.seq2 = d2; tp.off2 = o2;
            tp.lutbits = lut ? d_lutbits : nullptr;
            tp.vrec = bits ? 1 : 0;
            tp.dirs = fps[k].dirs; tp.dir_slot = v.pl.g.dir_slot;
            tp.ops = d_ops; tp.res = d_res;
            tp.pair_base = (uint32_t)base; tp.count = cnt;
            tp.max_m = max_m; tp.max_n = max_n;
            tp.gap = fps[k].gap; tp.match = fps[k].match; tp.mismatch = fps[k].mismatch;
            tp.gap_open = fps[k].gap_open; tp.gap_extend = fps[k].gap_extend;
            tp.allow = (allow || v.t16) ? 1 : 0;
            tp.tagged = v.t16 ? 1 : 0;
            tp.sel = fps[k].sel; tp.sel_want = fps[k].sel_want;
            tp.rerun = fps[k].rerun;
            tp.band_stride = v.pl.g.band_stride;
            tp.snap_h = fps[k].snap_h; tp.snap_p = fps[k].snap_p;
            tp.snap_h_slot = v.snap_h_slot; tp.snap_p_slot = v.snap_p_slot; tp.snap_nch = v.snap_nch;
            tp.prof = fps[k].prof;
            tp.t16_delta = fps[k].t16_delta;
            tp.t16_sent = fps[k].t16_sent;
            tp.so_lp = pipe ? 4 : 8;   // (sa_traceback_so.hip kSo4DefaultLp)
            // the int32 re-run walked first (tb_on_fill): it leaves kFlagRedo, the T16 walk clears it
            tp.keep_redo = tb_on_fill && k == 1 ? 1 : 0;
            tp.clear_redo = tb_on_fill && k == 0 ? 1 : 0;
#ifdef SA_R5_CONTROL
            tp.keep_redo = tp.clear_redo = 0;   // (round 5: the int32 walk cleared kFlagRedo)
#endif
            return tp;
        };
        for (int k = 0; k < nv; ++k) {
            const Variant& v = vars[k];
            const Plan& pl = v.pl;
            if (v.so && !is_affine(algo))
                if (int rc = next_hand_tag(c, hand_need, sf)) return rc;
            const FillVariant fv = make_fp(k);
            const FillParams& fp = fps[k];
            if (pl.split) SA_HIP(c, hipMemsetAsync(fp.ticket, 0, 256 + hand_x_off * 8 * aff2, sf));
            if (v.so && !is_affine(algo)) SA_HIP(c, hipMemsetAsync(fp.ticket, 0, 8, sf));   // (+ kAuxF16Flags)
            static_assert(kAuxF16Flags == kAuxTicket + 1, "ticket and f16 count: one memset");
            if (kev) SA_HIP(c, hipEventRecord(kev[2 * k], sf));
            // grid: SPLIT one workgroup per (pair, band) slot; score-only SW / NW one per (pair,
            // band) unit (band units, sa_fill_impl.h BU); otherwise one per pair
            const bool units = v.so && !is_affine(algo);
            const uint32_t grid = pl.split ? (uint32_t)(cnt * sp_bands)
                                : units ? (v.so2 ? (cnt + 1) / 2 : cnt) * pl.g.bands * v.segs : cnt;
            hipError_t e = v.so2 ? launch_fill_so2(algo, pl.R, fp, grid, sf) : launch_fill(algo, fv, fp, grid, sf);
            if (e != hipSuccess) return hip_fail(c, e, "fill kernel launch");
            if (kev) SA_HIP(c, hipEventRecord(kev[2 * k + 1], sf));
            if (pl.split) {
                SplitReduceParams rp;
                rp.off1 = o1; rp.off2 = o2; rp.part = fp.part; rp.res = d_res;
                rp.pair_base = (uint32_t)base; rp.count = cnt; rp.split_bands = (uint32_t)sp_bands;
                rp.band_rows = (uint32_t)kWave * pl.R; rp.max_m = max_m; rp.max_n = max_n;
                rp.gap = sc->gap; rp.gap_open = sc->gap_open; rp.gap_extend = sc->gap_extend;
                rp.cmax = v.cmax ? 1 : 0;
                rp.sel = sel; rp.sel_want = fp.sel_want;
                rp.redo = fp.redo; rp.retry_above = fp.retry_above;
                e = launch_split_reduce(algo, rp, sf);
                if (e != hipSuccess) return hip_fail(c, e, "split reduce kernel launch");
            }
            if (v.cmax) {
                EndcellParams ep{};
                ep.seq1 = d1; ep.off1 = o1; ep.seq2 = d2; ep.off2 = o2;
                ep.prof = fp.prof; ep.sel = sel; ep.sel_want = fp.sel_want;
                ep.snap_h = fp.snap_h; ep.snap_p = fp.snap_p; ep.snap_m = fp.snap_m;
                ep.snap_h_slot = v.snap_h_slot; ep.snap_p_slot = v.snap_p_slot; ep.snap_nch = v.snap_nch;
                if (pl.split) {
                    ep.rowbuf = reinterpret_cast<const int32_t*>(fp.hand);
                    ep.rowbuf_slot = 2 * sp_bands * std::max<uint32_t>(max_n, 1);
                    ep.rowbuf_stride = 2;
                    ep.rowbuf_x_off = 2 * hand_x_off;
                } else {
                    ep.rowbuf = fp.rowbuf; ep.rowbuf_slot = pl.rowbuf_elems; ep.rowbuf_stride = 1;
                    ep.rowbuf_x_off = pl.rowbuf_elems / 2;
                }
                ep.max_n = max_n;
                ep.res = d_res; ep.pair_base = (uint32_t)base; ep.count = cnt;
                ep.gap = sc->gap; ep.gap_open = sc->gap_open; ep.gap_extend = sc->gap_extend;
                ep.hshift = v.so ? 0 : 2;
                ep.snap_c = fp.snap_c; ep.snap_c_slot = v.snap_c_slot;
                ep.dirs = fp.dirs; ep.dir_slot = fp.dir_slot; ep.band_stride = fp.band_stride;
                if (fp.so2_f16) {
                    const uint32_t seq = ++c->f16_seq ? c->f16_seq : ++c->f16_seq;   // (0: none posted)
                    c->f16_cnt[seq & 3] = cnt;
                    ep.f16_count = fp.ticket + (kAuxF16Flags - kAuxTicket);
                    ep.f16_host = c->d_f16;
                    ep.f16_seq = seq;
                }
                // on the fill stream, right after the fill: run beside the next call's fill (on the
                // traceback stream) its 10,000 short waves slowed that fill by 4 % in round 4, and
                // the whole pipelined step by 12 % in round 5 (21.4 vs 19.1 ms per step)
                e = (v.so && algo == SA_SW) ? launch_endcell_so(pl.R, ep, sf) : launch_endcell(algo, pl.R, ep, sf);
                if (e != hipSuccess) return hip_fail(c, e, "end-cell kernel launch");
            }
            if (tb_on_fill && k == 1) {
                const TbParams tp = make_tp(k);
                e = tb_wave(cnt) ? launch_traceback_wave(algo, pl.R, lut, tp, sf) : launch_traceback(algo, pl.R, lut, tp, sf);
                if (e != hipSuccess) return hip_fail(c, e, "traceback kernel launch");
            }
        }
        SA_HIP(c, hipEventRecord(ev[1], sf));
        if (pipe) SA_HIP(c, hipStreamWaitEvent(stb, ev[1], 0));
        for (int k = 0; k < nv; ++k) {
            const Variant& v = vars[k];
            if (tb_on_fill && k == 1) continue;   // walked on the fill stream (above)
            TbParams tp = make_tp(k);
            if (seg_on && v.pl.split && tb_wave(cnt)) {
                tp.seg_mode = seg_mode;
                tp.hand = fps[k].hand;
                tp.hand_x_off = fps[k].hand_x_off;
                tp.split_bands = (uint32_t)sp_bands;
                tp.hand_shift = v.t16 ? (is_affine(algo) ? 3 : 2) : 0;
                tp.seg_rec = reinterpret_cast<int4*>(spbase + sp_seg);
                tp.seg_fin = tp.seg_rec + per_launch * sp_bands * seg_rs;
                SA_HIP(c, hipMemsetAsync(tp.seg_fin, 0xff, (uint64_t)cnt * 16, stb));
                hipError_t e = launch_traceback_seg(algo, v.pl.R, lut, tp, stb, seg_inject);
                if (e != hipSuccess) return hip_fail(c, e, "segmented traceback kernel launch");
            }
            hipError_t e = v.so ? launch_traceback_so(algo, v.pl.R, tp, stb)
                         : tb_wave(cnt) ? launch_traceback_wave(algo, v.pl.R, lut, tp, stb)
                                        : launch_traceback(algo, v.pl.R, lut, tp, stb);
            if (e != hipSuccess) return hip_fail(c, e, "traceback kernel launch");
        }
        if (has_fb) {
            if (vars[nv].pl.split) return fail(c, SA_ERR_UNSUPPORTED, "internal: SPLIT fallback plan");
            // SPLIT fallback, after every traceback of this launch (it rewrites the records of the
            // pairs it re-runs): fill + traceback of exactly the pairs flagged SA_FLAG_TIMEOUT,
            // launches that return at once when there is none
            const FillVariant fv = make_fp(nv);
            hipError_t e = launch_fill(algo, fv, fps[nv], cnt, stb);
            if (e != hipSuccess) return hip_fail(c, e, "fallback fill kernel launch");
            const TbParams tp = make_tp(nv);
            e = tb_wave(cnt) ? launch_traceback_wave(algo, vars[nv].pl.R, lut, tp, stb)
                             : launch_traceback(algo, vars[nv].pl.R, lut, tp, stb);
            if (e != hipSuccess) return hip_fail(c, e, "fallback traceback kernel launch");
        }
        SA_HIP(c, hipEventRecord(ev[2], stb));
        c->launches++;
    }
    if (pipe) {
        if (!c->ev_slot[slot]) SA_HIP(c, hipEventCreateWithFlags(&c->ev_slot[slot], hipEventDisableTiming));
        SA_HIP(c, hipEventRecord(c->ev_slot[slot], stb));
        c->pipe_k++;
    }
    return SA_OK;
}

bool lut_is_identity(const uint8_t* lut) {
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            if ((lut[a * 256 + b] != 0) != (a == b)) return false;
    return true;
}

// the match table is equality on every symbol pair these sequences hold (seq1 symbol x seq2 symbol):
// a caller's table for equal<char> then needs no upload (the kernels compare bytes)
bool lut_identity_on(const uint8_t* lut, const uint8_t* s1, uint64_t t1, const uint8_t* s2, uint64_t t2) {
    bool u1[256] = {}, u2[256] = {};
    for (uint64_t k = 0; k < t1; ++k) u1[s1[k]] = true;
    for (uint64_t k = 0; k < t2; ++k) u2[s2[k]] = true;
    for (int a = 0; a < 256; ++a)
        if (u1[a])
            for (int b = 0; b < 256; ++b)
                if (u2[b] && (lut[a * 256 + b] != 0) != (a == b)) return false;
    return true;
}

bool lg_size_hack(uint64_t m, uint64_t n) {  // SALocalGotoh.h:484-488
    return (m == 314 && n == 288) || (m == 60 && n == 57) || (m == 61 && n == 58);
}

// LocalGotoh: the reference replaces three size pairs by StaticFuncs::useNW with the same
// ScoringSystem (SALocalGotoh.h:484-488).  Split them out, align them with NW, merge back.
// align_subset(algo, sel, o1, o2, r, op, cap) aligns pairs sel (o1/o2: their packed length
// offsets) into r / op (op of the q-th selected pair at o1[q] + o2[q] + q).
template <typename AlignSubset>
int lg_hack_split(sa_ctx* c, const uint64_t* off1, const uint64_t* off2, uint32_t npairs, sa_result* results,
                  uint8_t* ops, uint64_t ops_cap, AlignSubset align_subset) {
    std::vector<uint32_t> hack, keep;
    for (uint32_t p = 0; p < npairs; ++p)
        (lg_size_hack(off1[p + 1] - off1[p], off2[p + 1] - off2[p]) ? hack : keep).push_back(p);
    if (hack.empty()) {
        std::vector<uint64_t> o1(off1, off1 + npairs + 1), o2(off2, off2 + npairs + 1);
        return align_subset(SA_LOCAL_GOTOH, keep, o1, o2, results, ops, ops_cap);
    }
    const uint64_t ops_total = off1[npairs] + off2[npairs] + npairs;
    if (ops_cap < ops_total) return fail(c, SA_ERR_CAPACITY, "ops buffer too small");
    for (int pass = 0; pass < 2; ++pass) {
        const std::vector<uint32_t>& sel = pass == 0 ? keep : hack;
        if (sel.empty()) continue;
        std::vector<uint64_t> o1(1, 0), o2(1, 0);
        for (uint32_t p : sel) {
            o1.push_back(o1.back() + off1[p + 1] - off1[p]);
            o2.push_back(o2.back() + off2[p + 1] - off2[p]);
        }
        const uint32_t k = (uint32_t)sel.size();
        std::vector<sa_result> r(k);
        std::vector<uint8_t> op(o1.back() + o2.back() + k + 1);
        const int rc = align_subset(pass == 0 ? SA_LOCAL_GOTOH : SA_NW, sel, o1, o2, r.data(), op.data(), op.size());
        if (rc) return rc;
        for (uint32_t q = 0; q < k; ++q) {
            const uint32_t p = sel[q];
            results[p] = r[q];
            if (pass == 1) results[p].flags |= SA_FLAG_SIZE_HACK;
            memcpy(ops + off1[p] + off2[p] + p, op.data() + o1[q] + o2[q] + q, r[q].nops);
        }
    }
    return SA_OK;
}

// Host copy of a large buffer on several threads (the caller's pageable memory <-> pinned
// staging; one thread copies ~5-10 GB/s).  A process-wide pool of persistent workers takes 1 MiB
// slices of whatever copy jobs are posted; a caller copies slices of its own job too and returns as
// soon as all of its bytes are done, so jobs of several contexts (sa_multi: one host thread per
// device) run side by side instead of one after another, and no job waits for idle workers to
// wake.  The pool is sized from the CPUs this process may use (affinity and cgroup quota -- a GPU
// box shows all of its cores to hardware_concurrency() but grants a share).
unsigned usable_cpus() {
    unsigned n = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::min<unsigned>(n, (unsigned)std::max(1, CPU_COUNT(&set)));
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {   // cgroup v2: "<quota> <period>" or "max <period>"
        char q[32] = {0};
        unsigned long long per = 0;
        if (fscanf(f, "%31s %llu", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0)
            n = std::min<unsigned>(n, (unsigned)std::max<unsigned long long>(1, strtoull(q, nullptr, 10) / per));
        fclose(f);
    }
    return n;
}

struct CopyPool {
    struct Job {
        uint8_t* dst;
        const uint8_t* src;
        uint64_t n;
        uint64_t grain = kSlice;                   // items per slice
        std::function<void(uint64_t, uint64_t)> fn;   // set: items [a, b) of an index-range job
        std::atomic<uint64_t> next{0}, done{0};
    };
    static constexpr uint64_t kSlice = 1ull << 20;
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::vector<std::shared_ptr<Job>> jobs;   // jobs with slices left
    std::vector<std::thread> workers;
    bool quit = false;
    explicit CopyPool(unsigned k) {
        for (unsigned t = 0; t < k; ++t) workers.emplace_back([this] { run(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(mu);
            quit = true;
        }
        cv.notify_all();
        for (auto& w : workers) w.join();
    }
    // one slice of job j; false when it has none left
    bool slice(Job& j) {
        const uint64_t a = j.next.fetch_add(j.grain);
        if (a >= j.n) return false;
        const uint64_t k = std::min(j.grain, j.n - a);
        if (j.fn) j.fn(a, a + k);
        else memcpy(j.dst + a, j.src + a, k);
        if (j.done.fetch_add(k) + k == j.n) {
            std::lock_guard<std::mutex> g(mu);
            done_cv.notify_all();
        }
        return true;
    }
    void run() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return quit || !jobs.empty(); });
            if (quit) return;
            std::shared_ptr<Job> j = jobs.front();
            lk.unlock();
            if (!slice(*j)) {
                lk.lock();
                if (!jobs.empty() && jobs.front() == j) jobs.erase(jobs.begin());
                continue;
            }
            lk.lock();
        }
    }
    std::atomic<int> in_flight{0}, max_in_flight{0};   // copy jobs posted and not yet done
    void copy(void* d, const void* s, uint64_t bytes, uint64_t grain = kSlice,
              std::function<void(uint64_t, uint64_t)> fn = nullptr) {
        const int f = in_flight.fetch_add(1) + 1;
        for (int m = max_in_flight.load(); f > m && !max_in_flight.compare_exchange_weak(m, f);) {}
        auto j = std::make_shared<Job>();
        j->dst = (uint8_t*)d;
        j->src = (const uint8_t*)s;
        j->n = bytes;
        j->grain = grain;
        j->fn = std::move(fn);
        {
            std::lock_guard<std::mutex> g(mu);
            jobs.push_back(j);
        }
        cv.notify_all();
        while (slice(*j)) {}
        std::unique_lock<std::mutex> lk(mu);
        done_cv.wait(lk, [&] { return j->done.load() == j->n; });
        in_flight.fetch_sub(1);
        // (a worker may still hold j to find it exhausted; it never touches dst / src again)
    }
};
CopyPool* g_copy_pool = nullptr;

CopyPool* copy_pool() {
    static CopyPool* pool = [] {   // never destroyed: exit-safe
        const unsigned cpus = usable_cpus();
        return g_copy_pool = new CopyPool(std::min(31u, cpus > 1 ? cpus - 1 : 1u));
    }();
    return pool;
}

void par_copy(void* dst, const void* src, uint64_t n) {
    if (n < (4ull << 20)) {
        if (n) memcpy(dst, src, n);
        return;
    }
    copy_pool()->copy(dst, src, n);
}

// fn(a, b) over items [0, n) in slices of `grain` items, on the copy pool's workers and this thread
void par_for(uint64_t n, uint64_t grain, std::function<void(uint64_t, uint64_t)> fn) {
    if (n <= grain) {
        if (n) fn(0, n);
        return;
    }
    copy_pool()->copy(nullptr, nullptr, n, grain, std::move(fn));
}

// Host API batches may be cut into contiguous pair ranges ("chunks") of near-equal cells run
// through the cross-call pipeline, so chunk g+1's upload and chunk g-1's download overlap chunk
// g's fill and traceback.  Measured on 10,000 x 4096^2 (round 3, profiles/host_api_r03.txt): one
// chunk 37.8-38.1 ms per call, two chunks 40.1-40.3 ms, four 51 ms -- each fill launch pays its own
// tail and the next chunk's alphabet scan waits for CU slots behind the previous fill, which costs
// more than the ~1 ms of upload the overlap hides.  So a batch is one chunk (its uploads and
// downloads still overlap piece by piece); SEQALIB_HOST_CHUNKS=G splits it (tuning, tests).
uint32_t host_chunks(int algo, uint32_t npairs) {
    if (algo == SA_HIRSCHBERG || algo == SA_MYERS_MILLER) return 1;   // one DC work set per context
    uint32_t G = 1;
    if (const char* e = getenv("SEQALIB_HOST_CHUNKS")) G = (uint32_t)std::max(1, atoi(e));
    return std::max<uint32_t>(1, std::min(G, npairs));
}

// contiguous [cut[g], cut[g+1]) ranges with near-equal sum of m*n
std::vector<uint32_t> cut_by_cells(const uint64_t* off1, const uint64_t* off2, uint32_t npairs, uint32_t parts) {
    std::vector<double> csum(npairs + 1, 0.0);
    for (uint32_t p = 0; p < npairs; ++p)
        csum[p + 1] = csum[p] + (double)(off1[p + 1] - off1[p]) * (double)(off2[p + 1] - off2[p]) + 1.0;
    std::vector<uint32_t> cut(parts + 1, npairs);
    cut[0] = 0;
    uint32_t p = 0;
    for (uint32_t g = 1; g < parts; ++g) {
        const double target = csum[npairs] * (double)g / (double)parts;
        while (p < npairs && csum[p] < target) ++p;
        cut[g] = std::max(p, cut[g - 1]);
    }
    return cut;
}

// The small-call path (sa_tiny.hip): a host call of few short pairs -- the reference's one
// getAlignment() per pair -- is one kernel launch and one stream synchronisation.  The inputs are
// copied into coherent pinned memory the kernel reads in place, and the kernel writes the results
// and op streams there (no device buffers, no copies, no workspace).  *max_m: the longest Seq1.
bool tiny_call(int algo, const uint64_t* off1, const uint64_t* off2, uint32_t npairs, int* max_m) {
    if (algo < SA_SW || algo > SA_GLOBAL_GOTOH || npairs == 0 || npairs > (uint32_t)kTinyPairs) return false;
    if (const char* e = getenv("SEQALIB_TINY"))
        if (e[0] == '0') return false;
    uint64_t mm = 0;
    for (uint32_t p = 0; p < npairs; ++p) {
        const uint64_t m = off1[p + 1] - off1[p], n = off2[p + 1] - off2[p];
        if (m > (uint64_t)kTinyM || n > (uint64_t)kTinyN || m * n > (uint64_t)kTinyCells) return false;
        mm = std::max(mm, m);
    }
    *max_m = (int)mm;
    return true;
}

// tiny_io: inputs [seq1][seq2][off1][off2][lut bits] from 0, outputs [results][ops] from kTinyOut
constexpr uint64_t kTinyOut = 128ull << 10, kTinyIo = 256ull << 10;

int align_tiny(sa_ctx* c, int algo, const sa_scoring* sc, const uint8_t* seq1, const uint64_t* off1,
               const uint8_t* seq2, const uint64_t* off2, uint32_t npairs, const uint8_t* lut,
               sa_result* results, uint8_t* ops, int max_m) {
    const bool timing = getenv("SEQALIB_HOST_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::micro>(b - a).count();
    };
    if (!c->tiny_io) {   // once per context
        SA_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&c->tiny_io), kTinyIo, hipHostMallocCoherent));
        void* dp = nullptr;
        SA_HIP(c, hipHostGetDevicePointer(&dp, c->tiny_io, 0));
        c->tiny_dev = static_cast<uint8_t*>(dp);
    }
    const auto t_alloc = std::chrono::steady_clock::now();
    auto al = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
    const uint64_t t1 = off1[npairs], t2 = off2[npairs];
    const uint64_t b1 = al(t1 + 1), b2 = al(t2 + 1), bo = al(8ull * (npairs + 1));
    const uint64_t x_s2 = b1, x_o1 = x_s2 + b2, x_o2 = x_o1 + bo, x_lut = x_o2 + bo;
    static_assert((uint64_t)kTinyPairs * (kTinyM + kTinyN) + 4 * 256 + 2 * 8 * (kTinyPairs + 1) + 8192 <= kTinyOut,
                  "tiny inputs overflow their region");
    static_assert(kTinyOut + sizeof(sa_result) * kTinyPairs + (uint64_t)kTinyPairs * (kTinyM + kTinyN + 1) <= kTinyIo,
                  "tiny outputs overflow their region");
    uint8_t* const h = c->tiny_io;
    memcpy(h, seq1, t1);
    memcpy(h + x_s2, seq2, t2);
    memcpy(h + x_o1, off1, 8ull * (npairs + 1));
    memcpy(h + x_o2, off2, 8ull * (npairs + 1));
    const bool use_lut = lut && !lut_identity_on(lut, seq1, t1, seq2, t2);
    if (use_lut) {   // bit rows of the Seq1 symbols present (the kernel reads no other row)
        uint32_t* bits = reinterpret_cast<uint32_t*>(h + x_lut);
        bool u1[256] = {};
        for (uint64_t k = 0; k < t1; ++k) u1[seq1[k]] = true;
        for (int a = 0; a < 256; ++a) {
            if (!u1[a]) continue;
            for (int w = 0; w < 8; ++w) {
                uint32_t word = 0;
                for (int b = 0; b < 32; ++b) word |= (lut[a * 256 + w * 32 + b] ? 1u : 0u) << b;
                bits[a * 8 + w] = word;
            }
        }
    }
    TinyParams tp;
    tp.seq1 = c->tiny_dev;
    tp.seq2 = c->tiny_dev + x_s2;
    tp.off1 = reinterpret_cast<const uint64_t*>(c->tiny_dev + x_o1);
    tp.off2 = reinterpret_cast<const uint64_t*>(c->tiny_dev + x_o2);
    tp.lutbits = use_lut ? reinterpret_cast<const uint32_t*>(c->tiny_dev + x_lut) : nullptr;
    tp.res = reinterpret_cast<sa_result*>(c->tiny_dev + kTinyOut);
    tp.ops = c->tiny_dev + kTinyOut + al(sizeof(sa_result) * npairs);
    tp.npairs = npairs;
    tp.gap = sc->gap;
    tp.match = sc->match;
    tp.mismatch = sc->mismatch;
    tp.gap_open = sc->gap_open;
    tp.gap_extend = sc->gap_extend;
    tp.allow = sc->allow_mismatch;
    const auto t_stage = std::chrono::steady_clock::now();
    SA_HIP(c, launch_tiny(algo, use_lut, max_m, tp, c->stream));
    const auto t_launch = std::chrono::steady_clock::now();
    SA_HIP(c, hipStreamSynchronize(c->stream));
    const auto t_sync = std::chrono::steady_clock::now();
    const sa_result* hres = reinterpret_cast<const sa_result*>(h + kTinyOut);
    const uint8_t* hops = h + kTinyOut + al(sizeof(sa_result) * npairs);
    memcpy(results, hres, sizeof(sa_result) * npairs);
    for (uint32_t p = 0; p < npairs; ++p) {
        const uint64_t o = off1[p] + off2[p] + p;
        memcpy(ops + o, hops + o, results[p].nops);
    }
    // the plan of this call (sa_last_plan_ex); no fill launch of the batch kernels
    c->nvar = 1;
    c->host_sel = -1;
    c->var_kernel[0] = SA_KERNEL_TINY;
    c->var_R[0] = max_m > kWave ? 4 : 1;
    c->var_W[0] = 1;
    c->var_records[0] = SA_RECORDS_FLAGS;
    c->launches = 0;
    c->kvars.clear();
    if (timing)
        fprintf(stderr, "[seqalib host api] %u pairs, small-call kernel: %.1f us = pinned buffer %.1f + staging in %.1f + "
                "launch %.1f + kernel and sync %.1f + copies out %.1f\n",
                npairs, us(t0, std::chrono::steady_clock::now()), us(t0, t_alloc), us(t_alloc, t_stage),
                us(t_stage, t_launch), us(t_launch, t_sync), us(t_sync, std::chrono::steady_clock::now()));
    return SA_OK;
}

int align_host(sa_ctx* c, int algo, const sa_scoring* sc, const uint8_t* seq1, const uint64_t* off1,
               const uint8_t* seq2, const uint64_t* off2, uint32_t npairs, const uint8_t* lut,
               sa_result* results, uint8_t* ops, uint64_t ops_cap, uint32_t chunks = 0,
               sa_chunk_cb cb = nullptr, void* cb_user = nullptr) {
    // $SEQALIB_HOST_TIMING: host-side phases of the call (stderr)
    const bool timing = getenv("SEQALIB_HOST_TIMING") != nullptr;
    const auto t_call = std::chrono::steady_clock::now();
    double ms_in = 0, ms_wait = 0, ms_out = 0;
    auto since = [](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    const uint64_t t1 = off1[npairs], t2 = off2[npairs];
    for (uint32_t p = 0; p < npairs; ++p)
        if (off1[p + 1] < off1[p] || off2[p + 1] < off2[p]) return fail(c, SA_ERR_ARG, "offsets must be non-decreasing");
    const uint64_t ops_total = t1 + t2 + npairs;
    if (ops_cap < ops_total) return fail(c, SA_ERR_CAPACITY, "ops buffer needs " + std::to_string(ops_total) + " bytes");
    if (!npairs) return SA_OK;
    int tiny_m = 0;
    if (chunks <= 1 && tiny_call(algo, off1, off2, npairs, &tiny_m)) {
        const int rc = align_tiny(c, algo, sc, seq1, off1, seq2, off2, npairs, lut, results, ops, tiny_m);
        if (rc == SA_OK && cb) cb(cb_user, 0, npairs);
        return rc;
    }
    // (identity on the symbols present implies nothing for large batches, whose scan costs more)
    const bool use_lut = lut && !(t1 + t2 <= kHostScanBytes ? lut_identity_on(lut, seq1, t1, seq2, t2)
                                                            : lut_is_identity(lut));
    const bool dc = algo == SA_HIRSCHBERG || algo == SA_MYERS_MILLER;
    const uint32_t G = chunks && !dc ? std::min(chunks, npairs) : host_chunks(algo, npairs);
    const std::vector<uint32_t> cut = cut_by_cells(off1, off2, npairs, G);

    // device I/O layout (256-byte aligned pieces); chunk g's offsets (rebased to its first pair)
    // live at do1 / do2 + cut[g] + g
    auto al = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
    const uint64_t n_off = (uint64_t)npairs + G;
    const uint64_t b_s1 = al(t1 + 1), b_s2 = al(t2 + 1), b_o = al(8 * n_off);
    const uint64_t b_res = al(sizeof(sa_result) * (uint64_t)npairs);
    const uint64_t b_ops = al(ops_total + 1), b_lut = al(65536), b_bits = al(8192);
    // small calls: the host-decided T16 profile (HostSeqs::hhdr); chunked calls: one 32-byte
    // profile slot per chunk (HostSeqs::hprof)
    const uint64_t b_hdr = al(std::max<uint64_t>(256, 32ull * G));
    // small call (one chunk, sequences the host scans, <= kSmallCall bytes each way): one upload
    // (header + inputs, issued by run_device after it wrote the header) and one download
    constexpr uint64_t kSmallCall = 1ull << 20;
    const bool small = G == 1 && t1 + t2 <= kHostScanBytes && b_s1 + b_s2 + 2 * b_o <= kSmallCall &&
                       b_res + ops_total <= kSmallCall;
    // other one-chunk calls download their op streams packed (ops_scan / ops_pack): [cpos][packed]
    const bool packed = G == 1 && !small && !dc;
    const uint64_t b_cpos = packed ? al(8ull * (npairs + 1)) : 0, b_pack = packed ? b_ops : 0;
    // 2-bit transfers (sa_codec.cpp; $SEQALIB_XFER2=0 sends bytes): sequence pieces land in the
    // packed-ops region (free until the traceback has run) and are unpacked into d1 / d2; op streams
    // come down 2-bit from their own region ([cpos2][a letters byte per pair][packed2])
    const char* x2e = getenv("SEQALIB_XFER2");
    const bool xfer2 = packed && !(x2e && x2e[0] == '0');
    const uint64_t b_pk1 = al(t1 / 4 + 64);   // (seq2's landing zone follows seq1's)
    const uint64_t b_cpos2 = xfer2 ? al(8ull * (npairs + 1)) + al(npairs) : 0, b_pack2 = xfer2 ? al(ops_total / 4 + npairs + 64) : 0;
    const uint64_t io_need = b_hdr + b_s1 + b_s2 + 2 * b_o + b_res + b_ops + b_lut + b_bits + b_cpos + b_pack + b_cpos2 + b_pack2;
    if (int rc = ensure_io(c, io_need)) return rc;
    uint8_t* p = c->io;
    uint32_t* const dhdr = reinterpret_cast<uint32_t*>(p); p += b_hdr;
    uint8_t* d1 = p; p += b_s1;
    uint8_t* d2 = p; p += b_s2;
    uint64_t* do1 = reinterpret_cast<uint64_t*>(p); p += b_o;
    uint64_t* do2 = reinterpret_cast<uint64_t*>(p); p += b_o;
    sa_result* dres = reinterpret_cast<sa_result*>(p); p += b_res;
    uint8_t* dops = p; p += b_ops;
    uint8_t* dlut = p; p += b_lut;
    uint32_t* dbits = reinterpret_cast<uint32_t*>(p); p += b_bits;
    uint64_t* const dcpos = reinterpret_cast<uint64_t*>(p); p += b_cpos;
    uint8_t* const dpack = p; p += b_pack;
    uint64_t* const dcpos2 = reinterpret_cast<uint64_t*>(p); p += b_cpos2;
    uint8_t* const dletters = reinterpret_cast<uint8_t*>(dcpos2 + (npairs + 1));   // per pair (ops_pack)
    uint8_t* const dpack2 = p;
    if (xfer2 && b_pk1 + al((t2 + 3) / 4 + 64) > b_pack) return fail(c, SA_ERR_HIP, "internal: 2-bit landing zone");
    // pinned staging (pageable copies were measured to stall 10-25 ms per call next to PyTorch),
    // laid out as the device I/O: in = [seq1][seq2][off1'][off2'], out = [results][ops], so that a
    // small call moves its inputs in one copy and its outputs in one copy
    SA_HIP(c, c->stage.alloc(b_hdr + b_s1 + b_s2 + 2 * b_o));
    SA_HIP(c, c->ostage.alloc(b_res + al(ops_total) + 8ull * (npairs + 1) + (xfer2 ? 8ull * (npairs + 1) + npairs : 0)));
    uint32_t* const shdr = reinterpret_cast<uint32_t*>(c->stage.data());
    uint8_t* const si = c->stage.data() + b_hdr;
    uint64_t* const so1 = reinterpret_cast<uint64_t*>(si + b_s1 + b_s2);
    uint64_t* const so2 = reinterpret_cast<uint64_t*>(si + b_s1 + b_s2 + b_o);
    sa_result* const sres = reinterpret_cast<sa_result*>(c->ostage.data());
    uint8_t* const sops = c->ostage.data() + b_res;   // (packed: the packed op bytes)
    uint64_t* const scpos = reinterpret_cast<uint64_t*>(c->ostage.data() + b_res + al(ops_total));
    uint64_t* const scpos2 = scpos + (npairs + 1);   // (xfer2) [cpos2][letters seen, a byte per pair]
    const bool pipe = G > 1;
    if (!c->s_out) SA_HIP(c, hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking));
    if (pipe && !c->s_fill) {
        SA_HIP(c, hipStreamCreateWithFlags(&c->s_fill, hipStreamNonBlocking));
        SA_HIP(c, hipStreamCreateWithFlags(&c->s_tb, hipStreamNonBlocking));
        SA_HIP(c, hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
    }
    // downloads go in pieces of kHostPiece bytes, each with its own event, so the host copy of
    // piece k (pinned -> caller) overlaps the D2H of piece k+1; uploads likewise (host copy of
    // piece k+1 while piece k is in flight)
    constexpr uint64_t kHostPiece = 16ull << 20;
    struct OutPiece { uint32_t g; uint64_t ob, on; };
    std::vector<OutPiece> outp;
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t p0 = cut[g], p1 = cut[g + 1];
        if (p1 == p0) continue;
        const uint64_t ob = off1[p0] + off2[p0] + p0, on = off1[p1] + off2[p1] + p1 - ob;
        for (uint64_t x = 0; x < on || x == 0; x += kHostPiece) outp.push_back({g, ob + x, std::min(kHostPiece, on - x)});
    }
    while (c->host_ev.size() < (size_t)G + outp.size() + 1) {
        hipEvent_t ev;
        SA_HIP(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        c->host_ev.push_back(ev);
    }
    size_t next_out = 0;
    hipStream_t st = c->stream;   // uploads (and, un-pipelined, the kernels)
    if (use_lut) {
        SA_HIP(c, hipMemcpyAsync(dlut, lut, 65536, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(lut_to_bits, dim3(8), dim3(256), 0, st, dlut, dbits);
        SA_HIP(c, hipGetLastError());
    }
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t p0 = cut[g], p1 = cut[g + 1], cnt = p1 - p0;
        if (!cnt) continue;
        const uint64_t a1 = off1[p0], a2 = off2[p0], n1 = off1[p1] - a1, n2 = off2[p1] - a2;
        const uint64_t ob = a1 + a2 + p0, on = off1[p1] + off2[p1] + p1 - ob;   // the chunk's op bytes
        uint32_t mm = 0, mn = 0;
        for (uint32_t q = 0; q <= cnt; ++q) {
            so1[p0 + g + q] = off1[p0 + q] - a1;
            so2[p0 + g + q] = off2[p0 + q] - a2;
            if (q) {
                mm = (uint32_t)std::max<uint64_t>(mm, off1[p0 + q] - off1[p0 + q - 1]);
                mn = (uint32_t)std::max<uint64_t>(mn, off2[p0 + q] - off2[p0 + q - 1]);
            }
        }
        const auto t_in = std::chrono::steady_clock::now();
        const uint64_t small_up = b_hdr + b_s1 + b_s2 + b_o + 8ull * (cnt + 1);   // [header][inputs]
        if (small) {
            memcpy(si, seq1, n1);
            memcpy(si + b_s1, seq2, n2);
            if (dc) SA_HIP(c, hipMemcpyAsync(dhdr, shdr, small_up, hipMemcpyHostToDevice, st));
        }
        // one piece of a sequence buffer: 2-bit when every byte is A / C / G / T (packed into the
        // piece's own staging bytes, unpacked on the device), else the bytes
        auto put_piece = [&](uint8_t* dst, uint8_t* stg, const uint8_t* src, uint64_t k, uint8_t* land) -> int {
            if (xfer2) {
                std::atomic<bool> ok{true};
                par_for(k, CopyPool::kSlice, [&](uint64_t a, uint64_t b) {   // (slices: multiples of 4 bytes)
                    if (!dna2_pack(stg + a / 4, src + a, b - a)) ok.store(false, std::memory_order_relaxed);
                });
                if (ok.load()) {
                    SA_HIP(c, hipMemcpyAsync(land, stg, (k + 3) / 4, hipMemcpyHostToDevice, st));
                    const uint64_t thr = (k + 15) / 16;
                    hipLaunchKernelGGL(dna2_unpack, dim3((uint32_t)((thr + 255) / 256)), dim3(256), 0, st, land, dst, k);
                    SA_HIP(c, hipGetLastError());
                    return SA_OK;
                }
            }
            par_copy(stg, src, k);
            SA_HIP(c, hipMemcpyAsync(dst, stg, k, hipMemcpyHostToDevice, st));
            return SA_OK;
        };
        for (uint64_t x = 0; !small && x < n1; x += kHostPiece) {
            const uint64_t k = std::min(kHostPiece, n1 - x);
            if (int rc = put_piece(d1 + a1 + x, si + a1 + x, seq1 + a1 + x, k, dpack + x / 4)) return rc;
        }
        for (uint64_t x = 0; !small && x < n2; x += kHostPiece) {
            const uint64_t k = std::min(kHostPiece, n2 - x);
            if (int rc = put_piece(d2 + a2 + x, si + b_s1 + a2 + x, seq2 + a2 + x, k, dpack + b_pk1 + x / 4)) return rc;
        }
        if (!small) {
            SA_HIP(c, hipMemcpyAsync(do1 + p0 + g, so1 + p0 + g, 8ull * (cnt + 1), hipMemcpyHostToDevice, st));
            SA_HIP(c, hipMemcpyAsync(do2 + p0 + g, so2 + p0 + g, 8ull * (cnt + 1), hipMemcpyHostToDevice, st));
        }
        ms_in += since(t_in);
        hipStream_t done = st;
        if (dc) {
            std::string e;
            c->launches = 0;
            const auto run = algo == SA_HIRSCHBERG ? hirschberg_run : myersmiller_run;
            DcBounds b;
            b.t1 = n1;
            b.t2 = n2;
            b.max_m = mm;
            b.max_n = mn;
            const DcInputs in{d1 + a1, do1 + p0 + g, d2 + a2, do2 + p0 + g, cnt, use_lut ? dbits : nullptr, DcBits{}};
            if (run(c->dc, c->ev_last_set ? c->ev_last : nullptr, sc, in, b, st, dres + p0, dops + ob, &e))
                return fail(c, SA_ERR_HIP, (algo == SA_HIRSCHBERG ? "hirschberg: " : "myers-miller: ") + e);
        } else {
            // small batches: the alphabet is decided here, on the host (no scan / decide kernels)
            HostSeqs hs{seq1 + a1, n1, seq2 + a2, n2, use_lut ? lut : nullptr};
            hs.hprof = shdr + 8 * g;
            if (small) {
                hs.hhdr = shdr;
                hs.dhdr = dhdr;
                hs.up_dst = dhdr;
                hs.up_src = shdr;
                hs.up_bytes = small_up;
            }
            int rc = run_device(c, algo, sc, d1 + a1, do1 + p0 + g, d2 + a2, do2 + p0 + g, cnt, mm, mn,
                                use_lut ? dbits : nullptr, dres + p0, dops + ob, st, pipe, nullptr, nullptr,
                                n1 + n2 <= kHostScanBytes ? &hs : nullptr);
            if (rc) return rc;
            if (pipe) done = c->s_tb;   // the chunk's last kernel (its traceback) ran there
        }
        (void)on;
        if (packed) {   // (one chunk: p0 = 0, g = 0)
            uint64_t* const c2 = dcpos2;
            hipLaunchKernelGGL(ops_scan, dim3(1), dim3(1024), 0, done, dres, cnt, dcpos, xfer2 ? dcpos2 : nullptr);
            if (xfer2)
                hipLaunchKernelGGL(ops_pack, dim3(cnt), dim3(256), 0, done, do1, do2, dres, dcpos, dops, dpack, c2, dpack2,
                                   dletters);
            else
                hipLaunchKernelGGL(ops_pack, dim3(cnt), dim3(256), 0, done, do1, do2, dres, dcpos, dops, dpack,
                                   (const uint64_t*)nullptr, (uint8_t*)nullptr, (uint8_t*)nullptr);
            SA_HIP(c, hipGetLastError());
        }
        SA_HIP(c, hipEventRecord(c->host_ev[g], done));
        SA_HIP(c, hipStreamWaitEvent(c->s_out, c->host_ev[g], 0));
        if (packed) {   // the results and the packed positions now; the packed bytes once their size is known
            SA_HIP(c, hipMemcpyAsync(sres, dres, sizeof(sa_result) * cnt, hipMemcpyDeviceToHost, c->s_out));
            SA_HIP(c, hipMemcpyAsync(scpos, dcpos, 8ull * (cnt + 1), hipMemcpyDeviceToHost, c->s_out));
            if (xfer2) SA_HIP(c, hipMemcpyAsync(scpos2, dcpos2, 8ull * (cnt + 1) + cnt, hipMemcpyDeviceToHost, c->s_out));
            SA_HIP(c, hipEventRecord(c->host_ev[G], c->s_out));
            continue;
        }
        if (small) {   // results and op bytes are contiguous in both layouts
            SA_HIP(c, hipMemcpyAsync(sres, dres, b_res + ops_total, hipMemcpyDeviceToHost, c->s_out));
            SA_HIP(c, hipEventRecord(c->host_ev[G + next_out], c->s_out));
            ++next_out;
            continue;
        }
        SA_HIP(c, hipMemcpyAsync(sres + p0, dres + p0, sizeof(sa_result) * cnt, hipMemcpyDeviceToHost, c->s_out));
        for (; next_out < outp.size() && outp[next_out].g == g; ++next_out) {
            const OutPiece& o = outp[next_out];
            SA_HIP(c, hipMemcpyAsync(sops + o.ob, dops + o.ob, o.on, hipMemcpyDeviceToHost, c->s_out));
            SA_HIP(c, hipEventRecord(c->host_ev[G + next_out], c->s_out));
        }
    }
    if (packed) {
        const auto t_w = std::chrono::steady_clock::now();
        SA_HIP(c, hipEventSynchronize(c->host_ev[G]));
        ms_wait += since(t_w);
        memcpy(results, sres, sizeof(sa_result) * npairs);
        // 2-bit op streams unless a letter has no code (another letter, or S and X in one call)
        uint32_t letters = xfer2 ? 0u : 4u;
        if (xfer2) {
            const uint8_t* const seen = reinterpret_cast<const uint8_t*>(scpos2 + (npairs + 1));
            for (uint32_t q = 0; q < npairs; ++q) letters |= seen[q];
        }
        const bool ops2 = xfer2 && !(letters & 4u) && letters != 3u;
        const uint64_t* const cp = ops2 ? scpos2 : scpos;
        uint32_t lut4[256];
        if (ops2) {
            const uint8_t lt[4] = {'M', (uint8_t)(letters & 2u ? 'X' : 'S'), 'U', 'L'};
            for (uint32_t b = 0; b < 256; ++b)
                lut4[b] = lt[b & 3] | (uint32_t)lt[(b >> 2) & 3] << 8 | (uint32_t)lt[(b >> 4) & 3] << 16 |
                          (uint32_t)lt[b >> 6] << 24;
        }
        const uint64_t total = cp[npairs];
        if (total > ops_total) return fail(c, SA_ERR_HIP, "internal: packed op streams exceed their buffer");
        // pieces of the packed bytes; the pairs whose bytes have all landed go to the caller's
        // layout (pair q at off1[q] + off2[q] + q) while later pieces are in flight (2-bit: 2 MiB
        // pieces, whose expansion to 8 MiB of letters takes longer than the next piece's D2H)
        const uint64_t piece = ops2 ? (2ull << 20) : kHostPiece;
        const size_t np = (size_t)((total + piece - 1) / piece);
        while (c->host_ev.size() < (size_t)G + 1 + np) {
            hipEvent_t ev;
            SA_HIP(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            c->host_ev.push_back(ev);
        }
        for (size_t k = 0; k < np; ++k) {
            const uint64_t x = k * piece, n = std::min(piece, total - x);
            SA_HIP(c, hipMemcpyAsync(sops + x, (ops2 ? dpack2 : dpack) + x, n, hipMemcpyDeviceToHost, c->s_out));
            SA_HIP(c, hipEventRecord(c->host_ev[G + 1 + k], c->s_out));
        }
        uint32_t q0 = 0;
        for (size_t k = 0; k <= np; ++k) {
            const auto t_w2 = std::chrono::steady_clock::now();
            if (k < np) SA_HIP(c, hipEventSynchronize(c->host_ev[G + 1 + k]));
            ms_wait += since(t_w2);
            const uint64_t landed = k < np ? (uint64_t)(k + 1) * piece : total;
            uint32_t q1 = q0;
            while (q1 < npairs && cp[q1 + 1] <= landed) ++q1;
            const auto t_o = std::chrono::steady_clock::now();
            par_for(q1 - q0, 256, [&, q0](uint64_t a, uint64_t b) {
                for (uint64_t q = q0 + a; q < q0 + b; ++q) {
                    if (ops2) ops2_unpack(ops + off1[q] + off2[q] + q, sops + cp[q], results[q].nops, lut4);
                    else memcpy(ops + off1[q] + off2[q] + q, sops + cp[q], results[q].nops);
                }
            });
            ms_out += since(t_o);
            q0 = q1;
        }
        if (cb) cb(cb_user, 0, npairs);
    }
    // each piece reaches the caller's buffers while later pieces and chunks still run
    for (size_t k = 0; !packed && k < outp.size(); ++k) {
        const OutPiece& o = outp[k];
        const auto t_w = std::chrono::steady_clock::now();
        SA_HIP(c, hipEventSynchronize(c->host_ev[G + k]));
        ms_wait += since(t_w);
        const auto t_o = std::chrono::steady_clock::now();
        if (k == 0 || outp[k - 1].g != o.g)
            memcpy(results + cut[o.g], sres + cut[o.g], sizeof(sa_result) * (cut[o.g + 1] - cut[o.g]));
        par_copy(ops + o.ob, sops + o.ob, o.on);
        ms_out += since(t_o);
        if (cb && (k + 1 == outp.size() || outp[k + 1].g != o.g)) cb(cb_user, cut[o.g], cut[o.g + 1]);   // chunk landed
    }
    if (pipe) {
        SA_HIP(c, hipStreamSynchronize(c->s_fill));
        SA_HIP(c, hipStreamSynchronize(c->s_tb));
    }
    SA_HIP(c, hipStreamSynchronize(st));
    if (timing)
        fprintf(stderr, "[seqalib host api] %u pairs, %u chunks: %.2f ms = staging in %.2f + waiting %.2f + copies out %.2f + other"
                "; copy pool %zu workers, max %d copy jobs in flight\n",
                npairs, G, since(t_call), ms_in, ms_wait, ms_out, g_copy_pool ? g_copy_pool->workers.size() : (size_t)0,
                g_copy_pool ? g_copy_pool->max_in_flight.load() : 0);
    return SA_OK;
}

// Host buffers, generic-Ty path: lengths as offsets, per-pair match bitmaps (sa_align_batch_bits).
// The kernels read no symbols here (the fill takes match bits from the bitmap and records the
// match bit of diagonal moves, the traceback takes it from the records), so the device sequence
// buffers are zero-filled placeholders of the right sizes.
int align_host_bits(sa_ctx* c, int algo, const sa_scoring* sc, const uint64_t* off1, const uint64_t* off2,
                    uint32_t npairs, const uint32_t* bits, const uint64_t* bits_off, sa_result* results,
                    uint8_t* ops, uint64_t ops_cap) {
    const uint64_t t1 = off1[npairs], t2 = off2[npairs], tw = bits_off[npairs];
    uint32_t max_m = 0, max_n = 0;
    for (uint32_t p = 0; p < npairs; ++p) {
        if (off1[p + 1] < off1[p] || off2[p + 1] < off2[p]) return fail(c, SA_ERR_ARG, "offsets must be non-decreasing");
        max_m = (uint32_t)std::max<uint64_t>(max_m, off1[p + 1] - off1[p]);
        max_n = (uint32_t)std::max<uint64_t>(max_n, off2[p + 1] - off2[p]);
    }
    const uint64_t ops_total = t1 + t2 + npairs;
    if (ops_cap < ops_total) return fail(c, SA_ERR_CAPACITY, "ops buffer needs " + std::to_string(ops_total) + " bytes");
    if (!npairs) return SA_OK;
    auto al = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
    const uint64_t b_s = al(std::max(t1, t2) + 1), b_o = al(8ull * (npairs + 1));
    const uint64_t b_res = al(sizeof(sa_result) * (uint64_t)npairs), b_ops = al(ops_total + 1);
    const uint64_t b_bits = al(4 * tw + 4);
    const uint64_t io_need = b_s + 3 * b_o + b_res + b_ops + b_bits;
    if (int rc = ensure_io(c, io_need)) return rc;
    uint8_t* q = c->io;
    uint8_t* dseq = q; q += b_s;
    uint64_t* do1 = reinterpret_cast<uint64_t*>(q); q += b_o;
    uint64_t* do2 = reinterpret_cast<uint64_t*>(q); q += b_o;
    uint64_t* dbo = reinterpret_cast<uint64_t*>(q); q += b_o;
    sa_result* dres = reinterpret_cast<sa_result*>(q); q += b_res;
    uint8_t* dops = q; q += b_ops;
    uint32_t* dbits = reinterpret_cast<uint32_t*>(q);
    hipStream_t st = c->stream;
    SA_HIP(c, hipMemsetAsync(dseq, 0, std::max(t1, t2) + 1, st));
    SA_HIP(c, hipMemcpyAsync(do1, off1, 8ull * (npairs + 1), hipMemcpyHostToDevice, st));
    SA_HIP(c, hipMemcpyAsync(do2, off2, 8ull * (npairs + 1), hipMemcpyHostToDevice, st));
    SA_HIP(c, hipMemcpyAsync(dbo, bits_off, 8ull * (npairs + 1), hipMemcpyHostToDevice, st));
    if (tw) SA_HIP(c, hipMemcpyAsync(dbits, bits, 4 * tw, hipMemcpyHostToDevice, st));
    if (algo == SA_HIRSCHBERG || algo == SA_MYERS_MILLER) {
        std::string e;
        c->launches = 0;
        const auto run = algo == SA_HIRSCHBERG ? hirschberg_run : myersmiller_run;
        DcBounds b;
        b.t1 = t1;
        b.t2 = t2;
        b.max_m = max_m;
        b.max_n = max_n;
        const DcInputs in{dseq, do1, dseq, do2, npairs, nullptr, DcBits{dbits, dbo, do1, do2}};
        if (run(c->dc, c->ev_last_set ? c->ev_last : nullptr, sc, in, b, st, dres, dops, &e))
            return fail(c, SA_ERR_HIP, (algo == SA_HIRSCHBERG ? "hirschberg: " : "myers-miller: ") + e);
    } else {
        int rc = run_device(c, algo, sc, dseq, do1, dseq, do2, npairs, max_m, max_n, nullptr, dres, dops, st, false,
                            dbits, dbo);
        if (rc) return rc;
    }
    SA_HIP(c, hipMemcpyAsync(results, dres, sizeof(sa_result) * npairs, hipMemcpyDeviceToHost, st));
    SA_HIP(c, hipMemcpyAsync(ops, dops, ops_total, hipMemcpyDeviceToHost, st));
    SA_HIP(c, hipStreamSynchronize(st));
    return SA_OK;
}

}  // namespace

// =============================================================================== C ABI
extern "C" {

int sa_version(void) { return SA_ABI_VERSION; }

const char* sa_status_string(int s) {
    switch (s) {
        case SA_OK: return "ok";
        case SA_ERR_ARG: return "invalid argument";
        case SA_ERR_HIP: return "HIP runtime error";
        case SA_ERR_NOMEM: return "out of memory";
        case SA_ERR_CAPACITY: return "output buffer too small";
        case SA_ERR_UNSUPPORTED: return "unsupported input";
        default: return "unknown status";
    }
}

int sa_device_count(int* count) {
    if (!count) return fail(nullptr, SA_ERR_ARG, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) { *count = 0; return hip_fail(nullptr, e, "hipGetDeviceCount"); }
    *count = n;
    return SA_OK;
}

int sa_create(int device, sa_ctx** out) {
    if (!out) return fail(nullptr, SA_ERR_ARG, "out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return fail(nullptr, SA_ERR_HIP, "no HIP device available");
    if (device < 0 || device >= n) return fail(nullptr, SA_ERR_ARG, "device ordinal out of range");
    e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(nullptr, e, "hipSetDevice");
    sa_ctx* c = new sa_ctx();
    c->device = device;
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete c; return hip_fail(nullptr, e, "hipStreamCreate"); }
    *out = c;
    return SA_OK;
}

void sa_destroy(sa_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)drain(c);
    if (c->s_out) (void)hipStreamSynchronize(c->s_out);
    for (auto ev : c->events) (void)hipEventDestroy(ev);
    for (auto ev : c->kevents) (void)hipEventDestroy(ev);
    for (auto ev : c->host_ev) (void)hipEventDestroy(ev);
    if (c->s_out) (void)hipStreamDestroy(c->s_out);
    for (auto ev : {c->ev_in, c->ev_slot[0], c->ev_slot[1], c->ev_sel, c->ev_last})
        if (ev) (void)hipEventDestroy(ev);
    if (c->s_fill) (void)hipStreamDestroy(c->s_fill);
    if (c->s_tb) (void)hipStreamDestroy(c->s_tb);
    if (c->ws) (void)hipFree(c->ws);
    if (c->io) (void)hipFree(c->io);
    if (c->aux) (void)hipFree(c->aux);
    if (c->h_sel) (void)hipHostFree(c->h_sel);
    if (c->h_f16) (void)hipHostFree(c->h_f16);
    if (c->tiny_io) (void)hipHostFree(c->tiny_io);
    if (c->split) (void)hipFree(c->split);
    if (c->hand) (void)hipFree(c->hand);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* sa_last_error(const sa_ctx* c) { return c ? c->err.c_str() : g_err.c_str(); }

int sa_test_hook(sa_ctx* c, int hook, uint64_t value) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    SA_HIP(c, hipSetDevice(c->device));
    if (hook == SA_HOOK_HAND_TAG) {
        if (value > 65535) return fail(c, SA_ERR_ARG, "hand-off tag must be <= 65535");
        if (int rc = drain(c)) return rc;
        c->hand_tag = (uint32_t)value;
        return SA_OK;
    }
    if (hook == SA_HOOK_POISON_WS) {
        if (int rc = drain(c)) return rc;
        if (c->ws) SA_HIP(c, hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(c->ws), (int)(uint32_t)value, c->ws_bytes / 4));
        SA_HIP(c, hipDeviceSynchronize());
        return SA_OK;
    }
    if (hook == SA_HOOK_F16) {
        if (value == 2) return c->f16_off ? 1 : 0;
        if (value > 1) return fail(c, SA_ERR_ARG, "SA_HOOK_F16 takes 0, 1 or 2");
        if (int rc = drain(c)) return rc;
        c->f16_off = value == 1;
        c->f16_seen = c->h_f16 ? (uint32_t)(__atomic_load_n(c->h_f16, __ATOMIC_ACQUIRE) >> 32) : 0;
        return SA_OK;
    }
    return fail(c, SA_ERR_ARG, "unknown test hook");
}

int sa_set_workspace_limit(sa_ctx* c, uint64_t bytes) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    c->ws_limit = bytes;
    return SA_OK;
}

int sa_trim(sa_ctx* c) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    (void)hipSetDevice(c->device);
    (void)drain(c);
    if (c->ws) (void)hipFree(c->ws);
    if (c->io) (void)hipFree(c->io);
    if (c->split) (void)hipFree(c->split);
    if (c->hand) (void)hipFree(c->hand);
    c->hand = nullptr; c->hand_bytes = 0; c->hand_tag = 0;
    c->ws = nullptr; c->ws_bytes = 0;
    c->io = nullptr; c->io_bytes = 0;
    c->split = nullptr; c->split_bytes = 0;
    c->dc.release();
    c->stage.reset();    // the host API's pinned staging (~80 MB each way for the headline batch)
    c->ostage.reset();
    return SA_OK;
}

int sa_align_batch(sa_ctx* c, int algo, const sa_scoring* sc, const uint8_t* seq1,
                   const uint64_t* off1, const uint8_t* seq2, const uint64_t* off2, uint32_t npairs,
                   const uint8_t* lut, sa_result* results, uint8_t* ops, uint64_t ops_cap) {
    return sa_align_batch_cb(c, algo, sc, seq1, off1, seq2, off2, npairs, lut, results, ops, ops_cap, 0, nullptr,
                             nullptr);
}

int sa_align_batch_cb(sa_ctx* c, int algo, const sa_scoring* sc, const uint8_t* seq1,
                      const uint64_t* off1, const uint8_t* seq2, const uint64_t* off2, uint32_t npairs,
                      const uint8_t* lut, sa_result* results, uint8_t* ops, uint64_t ops_cap, uint32_t chunks,
                      sa_chunk_cb cb, void* cb_user) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    int rc = validate_scoring(c, algo, sc);
    if (rc) return rc;
    if (!off1 || !off2 || (npairs && (!results || !ops))) return fail(c, SA_ERR_ARG, "NULL buffer");
    if ((off1[npairs] && !seq1) || (off2[npairs] && !seq2)) return fail(c, SA_ERR_ARG, "NULL sequence buffer");
    if (off1[0] != 0 || off2[0] != 0) return fail(c, SA_ERR_ARG, "offsets must start at 0");
    SA_HIP(c, hipSetDevice(c->device));
    if ((rc = order_after_last(c, c->stream))) return rc;

    if (algo != SA_LOCAL_GOTOH)
        return align_host(c, algo, sc, seq1, off1, seq2, off2, npairs, lut, results, ops, ops_cap, chunks, cb, cb_user);
    // LocalGotoh: the size-hack pairs run as their own NW batch, so the whole range lands at the end
    rc = lg_hack_split(c, off1, off2, npairs, results, ops, ops_cap,
                         [&](int a, const std::vector<uint32_t>& sel, const std::vector<uint64_t>& o1,
                             const std::vector<uint64_t>& o2, sa_result* r, uint8_t* op, uint64_t cap) {
                             if (sel.size() == npairs)
                                 return align_host(c, a, sc, seq1, off1, seq2, off2, npairs, lut, r, op, cap);
                             std::vector<uint8_t> s1, s2;
                             s1.reserve(o1.back());
                             s2.reserve(o2.back());
                             for (uint32_t p : sel) {
                                 s1.insert(s1.end(), seq1 + off1[p], seq1 + off1[p + 1]);
                                 s2.insert(s2.end(), seq2 + off2[p], seq2 + off2[p + 1]);
                             }
                             return align_host(c, a, sc, s1.data(), o1.data(), s2.data(), o2.data(),
                                               (uint32_t)sel.size(), lut, r, op, cap);
                         });
    if (rc == SA_OK && cb && npairs) cb(cb_user, 0, npairs);
    return rc;
}

int sa_align_batch_bits(sa_ctx* c, int algo, const sa_scoring* sc, const uint64_t* off1, const uint64_t* off2,
                        uint32_t npairs, const uint32_t* bits, const uint64_t* bits_off, sa_result* results,
                        uint8_t* ops, uint64_t ops_cap) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    int rc = validate_scoring(c, algo, sc);
    if (rc) return rc;
    if (!off1 || !off2 || !bits_off || (npairs && (!results || !ops))) return fail(c, SA_ERR_ARG, "NULL buffer");
    if (off1[0] != 0 || off2[0] != 0) return fail(c, SA_ERR_ARG, "offsets must start at 0");
    for (uint32_t p = 0; p < npairs; ++p) {
        const uint64_t m = off1[p + 1] - off1[p], n = off2[p + 1] - off2[p];
        if (bits_off[p + 1] < bits_off[p] || bits_off[p + 1] - bits_off[p] < m * ((n + 31) / 32))
            return fail(c, SA_ERR_ARG, "bits_off: pair " + std::to_string(p) + " needs m * ceil(n/32) words");
    }
    if (bits_off[npairs] && !bits) return fail(c, SA_ERR_ARG, "NULL bitmap");
    SA_HIP(c, hipSetDevice(c->device));
    if ((rc = order_after_last(c, c->stream))) return rc;
    if (algo != SA_LOCAL_GOTOH)
        return align_host_bits(c, algo, sc, off1, off2, npairs, bits, bits_off, results, ops, ops_cap);
    return lg_hack_split(c, off1, off2, npairs, results, ops, ops_cap,
                         [&](int a, const std::vector<uint32_t>& sel, const std::vector<uint64_t>& o1,
                             const std::vector<uint64_t>& o2, sa_result* r, uint8_t* op, uint64_t cap) {
                             if (sel.size() == npairs)
                                 return align_host_bits(c, a, sc, off1, off2, npairs, bits, bits_off, r, op, cap);
                             std::vector<uint32_t> b;
                             std::vector<uint64_t> bo(1, 0);
                             for (uint32_t p : sel) {
                                 b.insert(b.end(), bits + bits_off[p], bits + bits_off[p + 1]);
                                 bo.push_back(b.size());
                             }
                             return align_host_bits(c, a, sc, o1.data(), o2.data(), (uint32_t)sel.size(),
                                                    b.data(), bo.data(), r, op, cap);
                         });
}

int sa_align_batch_device(sa_ctx* c, int algo, const sa_scoring* sc, const uint8_t* d1,
                          const uint64_t* o1, const uint8_t* d2, const uint64_t* o2, uint32_t npairs,
                          uint32_t max_m, uint32_t max_n, const uint8_t* d_lut, sa_result* d_res,
                          uint8_t* d_ops, void* stream) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    int rc = validate_scoring(c, algo, sc);
    if (rc) return rc;
    if (!o1 || !o2 || (npairs && (!d_res || !d_ops))) return fail(c, SA_ERR_ARG, "NULL buffer");
    if (npairs == 0) return SA_OK;
    SA_HIP(c, hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if ((rc = order_after_last(c, st))) return rc;
    uint32_t* bits = nullptr;
    if (d_lut) {
        // LUT bits live in the tail of the I/O cache
        if (int rc2 = ensure_io(c, 8192)) return rc2;
        bits = reinterpret_cast<uint32_t*>(c->io + c->io_bytes - 8192);
        hipLaunchKernelGGL(lut_to_bits, dim3(8), dim3(256), 0, st, d_lut, bits);
        SA_HIP(c, hipGetLastError());
    }
    if (algo == SA_HIRSCHBERG || algo == SA_MYERS_MILLER) {
        std::string e;
        c->launches = 0;
        const auto run = algo == SA_HIRSCHBERG ? hirschberg_run : myersmiller_run;
        DcBounds b;   // the caller's bounds (pairs past them: SA_FLAG_BAD_SHAPE), no read of o1 / o2
        b.t1 = (uint64_t)npairs * max_m;
        b.t2 = (uint64_t)npairs * max_n;
        b.max_m = max_m;
        b.max_n = max_n;
        const DcInputs in{d1, o1, d2, o2, npairs, bits, DcBits{}};
        if (run(c->dc, c->ev_last_set ? c->ev_last : nullptr, sc, in, b, st, d_res, d_ops, &e))
            return fail(c, SA_ERR_HIP, (algo == SA_HIRSCHBERG ? "hirschberg: " : "myers-miller: ") + e);
        return mark_last(c, st);
    }
    const bool pipe = c->pipeline != 0;
    rc = run_device(c, algo, sc, d1, o1, d2, o2, npairs, max_m, max_n, bits, d_res, d_ops, st, pipe);
    if (rc || pipe) return rc;
    return mark_last(c, st);
}

int sa_set_pipeline(sa_ctx* c, int enable) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    SA_HIP(c, hipSetDevice(c->device));
    if (enable && !c->s_fill) {
        SA_HIP(c, hipStreamCreateWithFlags(&c->s_fill, hipStreamNonBlocking));
        SA_HIP(c, hipStreamCreateWithFlags(&c->s_tb, hipStreamNonBlocking));
        SA_HIP(c, hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
    }
    if (!enable && c->pipeline) {
        int rc = sa_wait(c);
        if (rc) return rc;
    }
    c->pipeline = enable ? 1 : 0;
    return SA_OK;
}

int sa_wait(sa_ctx* c) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    SA_HIP(c, hipSetDevice(c->device));
    if (c->s_fill) SA_HIP(c, hipStreamSynchronize(c->s_fill));
    if (c->s_tb) SA_HIP(c, hipStreamSynchronize(c->s_tb));
    SA_HIP(c, hipStreamSynchronize(c->stream));
    return SA_OK;
}

int sa_last_timings(sa_ctx* c, float* fill_ms, float* tb_ms, int* launches) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    float f = 0.f, t = 0.f;
    for (int k = 0; k < c->launches; ++k) {
        hipEvent_t* ev = &c->events[3 * k];
        SA_HIP(c, hipEventSynchronize(ev[2]));
        float a = 0.f, b = 0.f;
        SA_HIP(c, hipEventElapsedTime(&a, ev[0], ev[1]));
        SA_HIP(c, hipEventElapsedTime(&b, ev[1], ev[2]));
        f += a;
        t += b;
    }
    if (fill_ms) *fill_ms = f;
    if (tb_ms) *tb_ms = t;
    if (launches) *launches = c->launches;
    return SA_OK;
}

int sa_last_kernel_timings(sa_ctx* c, float* fill_kernel_ms, float* fill_stream_ms) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    float f = 0.f, s = 0.f;
    if ((int)c->kvars.size() < c->launches)
        return fail(c, SA_ERR_ARG, "the last call ran without SEQALIB_KERNEL_TIMING");
    for (int k = 0; k < c->launches; ++k) {
        hipEvent_t* ev = &c->events[3 * k];
        SA_HIP(c, hipEventSynchronize(ev[1]));
        float a = 0.f;
        SA_HIP(c, hipEventElapsedTime(&a, ev[0], ev[1]));
        s += a;
        for (int v = 0; v < c->kvars[k]; ++v) {
            hipEvent_t* kev = &c->kevents[kKEv * k + 2 * v];
            SA_HIP(c, hipEventElapsedTime(&a, kev[0], kev[1]));
            f += a;
        }
    }
    if (fill_kernel_ms) *fill_kernel_ms = f;
    if (fill_stream_ms) *fill_stream_ms = s;
    return SA_OK;
}

int sa_last_plan_ex(sa_ctx* c, int* kernel, int* R, int* W, int* records) {
    if (!c) return fail(nullptr, SA_ERR_ARG, "ctx is NULL");
    int k = 0;
    if (c->nvar == 2) {   // T16 and int32 were both enqueued: the host's or the device's choice decides
        SA_HIP(c, hipEventSynchronize(c->ev_sel));
        k = (c->host_sel >= 0 ? (uint32_t)c->host_sel : *c->h_sel) == 1 ? 0 : 1;
    }
    if (kernel) *kernel = c->var_kernel[k];
    if (R) *R = c->var_R[k];
    if (W) *W = c->var_W[k];
    if (records) *records = c->var_records[k];
    return SA_OK;
}

int sa_last_plan(sa_ctx* c, int* kernel, int* R, int* W) { return sa_last_plan_ex(c, kernel, R, W, nullptr); }

int sa_plan_query(int algo, uint32_t max_m, uint32_t max_n, uint32_t npairs, int* R, int* W,
                  uint64_t* dir_bytes, uint64_t* rowbuf_bytes) {
    if (algo < SA_SW || algo > SA_GLOBAL_GOTOH) return fail(nullptr, SA_ERR_ARG, "unknown algorithm");
    const Plan p = make_plan(algo, max_m, max_n, npairs, false);
    if (R) *R = p.R;
    if (W) *W = p.W;
    if (dir_bytes) *dir_bytes = p.g.dir_slot;
    if (rowbuf_bytes) *rowbuf_bytes = p.rowbuf_elems * 4;
    return SA_OK;
}

int sa_plan_query_ex(int algo, const sa_scoring* sc, uint32_t max_m, uint32_t max_n, uint32_t npairs,
                     int nsym, int* kernel, int* R, int* W, uint64_t* ws_bytes_per_pair) {
    if (algo < SA_SW || algo > SA_GLOBAL_GOTOH) return fail(nullptr, SA_ERR_ARG, "unknown algorithm");
    if (!sc) return fail(nullptr, SA_ERR_ARG, "scoring is NULL");
    const bool cand = t16_candidate(algo, sc, max_m, max_n, npairs).ok;
    // exactly the variants a call enqueues (build_variants: common record stride, SPLIT fallback)
    Variant vars[3];
    bool has_fb = false;
    const int nv = build_variants(algo, max_m, max_n, npairs, cand, vars, &has_fb);
    const Variant& v = (cand && nsym <= 4) ? vars[0] : vars[nv - 1];
    if (kernel) *kernel = v.kernel;
    if (R) *R = v.pl.R;
    if (W) *W = v.pl.split ? 0 : v.pl.W;
    uint64_t ws = 0;
    for (int k = 0; k < nv + (has_fb ? 1 : 0); ++k) ws = std::max(ws, vars[k].slot_bytes);
    if (ws_bytes_per_pair) *ws_bytes_per_pair = ws;
    return SA_OK;
}

}  // extern "C"
