// seqalib/detail/Engine.h — glue between the reference-shaped C++ templates and the C ABI
// (include/seqalib_hip.h): per-thread device context, symbol coding for arbitrary Ty, the match
// table built from the user's MatchFnTy, and op-stream -> AlignedSequence assembly.
#pragma once

#include <algorithm>
#include <array>
#include <sched.h>
#include <chrono>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../seqalib_hip.h"

namespace seqalib {
namespace detail {

// One HIP context per host thread (the reference's aligners are not reentrant either; separate
// instances on separate threads are independent).  Device: $SEQALIB_DEVICE or 0.
struct ThreadContext {
    sa_ctx* h = nullptr;
    ~ThreadContext() {
        if (h) sa_destroy(h);
    }
};

inline sa_ctx* context() {
    thread_local ThreadContext c;
    if (!c.h) {
        const char* env = std::getenv("SEQALIB_DEVICE");
        const int dev = env ? std::atoi(env) : 0;
        const int rc = sa_create(dev, &c.h);
        if (rc != SA_OK) {
            c.h = nullptr;
            throw std::runtime_error(std::string("seqalib: cannot open HIP device: ") + sa_last_error(nullptr));
        }
    }
    return c.h;
}

// $SEQALIB_DEVICES="0,1,..." (two or more ordinals): batches are spread over those GPUs through
// one persistent sa_multi handle per host thread (contiguous pair ranges of near-equal work,
// results in place); otherwise the single context above is used.
struct ThreadMulti {
    sa_multi* h = nullptr;
    bool checked = false;
    ~ThreadMulti() {
        if (h) sa_multi_destroy(h);
    }
};

inline sa_multi* multi_context() {
    thread_local ThreadMulti m;
    if (!m.checked) {
        m.checked = true;
        const char* env = std::getenv("SEQALIB_DEVICES");
        std::vector<int> devs;
        for (const char* q = env; q && *q;) {
            char* end = nullptr;
            const long d = std::strtol(q, &end, 10);
            if (end == q) break;
            devs.push_back((int)d);
            q = (*end == ',') ? end + 1 : end;
        }
        if (devs.size() >= 2) {
            const int rc = sa_multi_create(devs.data(), (int)devs.size(), &m.h);
            if (rc != SA_OK) {
                m.h = nullptr;
                throw std::runtime_error(std::string("seqalib: cannot open SEQALIB_DEVICES: ") + sa_multi_last_error(nullptr));
            }
        }
    }
    return m.h;
}

// Host staging buffers that are written in full before they are read: a vector whose resize()
// leaves elements default-initialised (no zero fill of ~80 MB per headline batch).
template <typename T>
struct DefaultInitAlloc : std::allocator<T> {
    template <typename U>
    struct rebind {
        using other = DefaultInitAlloc<U>;
    };
    DefaultInitAlloc() = default;
    template <typename U>
    DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
    template <typename U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
        ::new (static_cast<void*>(p)) U;
    }
    template <typename U, typename... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
template <typename T>
using raw_vector = std::vector<T, DefaultInitAlloc<T>>;

// The batch's large host buffers (coded Seq1 / Seq2 and the op streams: ~2 x 82 MB for the
// 10,000 x 4096^2 batch) are kept per host thread across calls (grow-only): allocated per call they
// came from fresh mmap'd pages, ~40 K first-touch page faults per call (round 6, tests/cpp/
// dropin_bench per-rep counters), on the threads that build the lists at the same time.
enum HostBuf { kHostSeq1, kHostSeq2, kHostOps, kHostBufs };
inline raw_vector<uint8_t>& host_buffer(int which) {
    thread_local raw_vector<uint8_t> bufs[kHostBufs];
    return bufs[which];
}

// CPUs this process may use: hardware threads, capped by its affinity mask and its cgroup CPU
// quota (a GPU box shows every core of the machine but grants a share; threads beyond the quota
// get the whole process throttled for the rest of the CFS period).
inline size_t host_cpu_share() {
    static const size_t share = [] {
        size_t n = std::max(1u, std::thread::hardware_concurrency());
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::min<size_t>(n, (size_t)std::max(1, CPU_COUNT(&set)));
        if (std::FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {   // "<quota> <period>" or "max <period>"
            char q[32] = {0};
            unsigned long long per = 0;
            if (std::fscanf(f, "%31s %llu", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0)
                n = std::min<size_t>(n, (size_t)std::max<unsigned long long>(1, std::strtoull(q, nullptr, 10) / per));
            std::fclose(f);
        }
        return n;
    }();
    return share;
}

// Host threads for per-pair work of a batch of P pairs (symbol coding, list construction): the
// CPU share (at most 16), at least 32 pairs each.
inline size_t host_threads(size_t P) {
    const size_t cpus = std::max<size_t>(1, std::min<size_t>(host_cpu_share(), 16));
    return std::max<size_t>(1, std::min<size_t>(cpus, P / 32));
}

// Runs body(t, p0, p1) over nth contiguous pair ranges [P*t/nth, P*(t+1)/nth), one host thread
// each (the caller's thread takes the first); rethrows the first exception.
template <typename Body>
void parallel_pairs(size_t P, size_t nth, Body&& body) {
    if (nth <= 1) {
        body((size_t)0, (size_t)0, P);
        return;
    }
    std::vector<std::exception_ptr> errs(nth);
    std::vector<std::thread> pool;
    for (size_t t = 1; t < nth; ++t)
        pool.emplace_back([&, t] {
            try {
                body(t, P * t / nth, P * (t + 1) / nth);
            } catch (...) {
                errs[t] = std::current_exception();
            }
        });
    try {
        body((size_t)0, (size_t)0, P / nth);
    } catch (...) {
        errs[0] = std::current_exception();
    }
    for (auto& th : pool) th.join();
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
}

// $SEQALIB_HOST_TIMING: print the host-side phases of each batch to stderr.
struct PhaseTimer {
    bool on = std::getenv("SEQALIB_HOST_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(const char* what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[seqalib host] %-22s %8.2f ms\n", what,
                     std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

inline void check(int rc, const char* what) {
    if (rc != SA_OK)
        throw std::runtime_error(std::string("seqalib: ") + what + ": " + sa_status_string(rc) + " (" +
                                 sa_last_error(context()) + ")");
}

// Maps symbols of type Ty onto byte codes.  Single-byte integral types are their own code; other
// types get codes in order of first appearance, at most 256 distinct symbols per batch -- a batch
// with more goes through the match-bitmap path instead (align_bits below).
template <typename Ty, bool Direct = (std::is_integral<Ty>::value && sizeof(Ty) == 1)>
struct SymbolCoder {
    std::vector<Ty> values;
    bool overflow = false;
    uint8_t code(const Ty& v) {
        for (size_t k = 0; k < values.size(); ++k)
            if (values[k] == v) return (uint8_t)k;
        if (values.size() == 256) {
            overflow = true;
            return 0;
        }
        values.push_back(v);
        return (uint8_t)(values.size() - 1);
    }
    size_t size() const { return values.size(); }
    const Ty& value(size_t k) const { return values[k]; }
    bool used(size_t) const { return true; }           // every code in [0, size()) is in use
    bool identity_on_equal() const { return true; }   // distinct values -> distinct codes
};

template <typename Ty>
struct SymbolCoder<Ty, true> {
    bool overflow = false;
    bool seen[256] = {};
    uint8_t code(const Ty& v) {
        const uint8_t c = (uint8_t)v;
        seen[c] = true;
        return c;
    }
    size_t size() const { return 256; }
    Ty value(size_t k) const { return (Ty)(uint8_t)k; }
    bool used(size_t k) const { return seen[k]; }
};

template <typename Ty, typename MatchFnTy, bool Direct>
std::vector<uint8_t> build_lut(SymbolCoder<Ty, Direct>& coder, MatchFnTy& fn) {
    std::vector<uint8_t> lut(65536, 0);
    const size_t k = Direct ? 256 : coder.size();
    for (size_t a = 0; a < k; ++a) {
        if (!coder.used(a)) continue;
        for (size_t b = 0; b < k; ++b) {
            if (!coder.used(b)) continue;
            lut[a * 256 + b] = fn(coder.value(a), coder.value(b)) ? 1 : 0;
        }
    }
    return lut;
}

// match(x, y) as the reference's cacheAllMatches evaluates it: the user's MatchFnTy, or == for a
// nullptr one.  (Overloads rather than if constexpr: the headers build with the reference's own
// -std=c++14, test/Makefile:2.)
template <typename MatchFnTy, typename A>
bool call_match(MatchFnTy& fn, bool has_fn, const A& x, const A& y) {
    return has_fn ? (bool)fn(x, y) : (x == y);
}
template <typename A>
bool call_match(std::nullptr_t&, bool, const A& x, const A& y) {
    return x == y;
}

// Generic-Ty path: per-pair m x n match bitmaps, built exactly as the reference's
// cacheAllMatches builds its match cache (one MatchFnTy call per cell, e.g. SASmithWaterman.h:
// 20-45; the == operator for a nullptr match fn), packed to bits for sa_align_batch_bits.
template <typename Ty, typename ContainerType, typename MatchFnTy>
void align_bits(int algo, const sa_scoring& sc, MatchFnTy& fn, bool has_fn,
                const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs, std::vector<sa_result>& res,
                raw_vector<uint8_t>& ops, std::vector<uint64_t>& ops_off) {
    PhaseTimer tm;
    const uint32_t np = (uint32_t)pairs.size();
    std::vector<uint64_t> o1(1, 0), o2(1, 0), bo(1, 0);
    for (auto& p : pairs) {
        const uint64_t m = (uint64_t)p.first->size(), n = (uint64_t)p.second->size();
        o1.push_back(o1.back() + m);
        o2.push_back(o2.back() + n);
        bo.push_back(bo.back() + m * ((n + 31) / 32));
    }
    std::vector<uint32_t> bits(bo.back() + 1, 0u);
    for (uint32_t q = 0; q < np; ++q) {
        ContainerType& a = *pairs[q].first;
        ContainerType& b = *pairs[q].second;
        const size_t m = (size_t)a.size(), n = (size_t)b.size(), wn = (n + 31) / 32;
        uint32_t* w = bits.data() + bo[q];
        for (size_t i = 0; i < m; ++i)
            for (size_t j = 0; j < n; ++j) {
                if (call_match(fn, has_fn, a[i], b[j])) w[i * wn + j / 32] |= 1u << (j % 32);
            }
    }
    tm.lap("match bitmaps");
    res.assign(np, sa_result{});
    const uint64_t cap = o1.back() + o2.back() + np + 1;
    ops.resize(cap);
    ops_off.resize(np);
    for (uint32_t p = 0; p < np; ++p) ops_off[p] = o1[p] + o2[p] + p;
    check(sa_align_batch_bits(context(), algo, &sc, o1.data(), o2.data(), np, bits.data(), bo.data(), res.data(),
                              ops.data(), cap),
          "sa_align_batch_bits");
    tm.lap("sa_align_batch_bits (GPU)");
    for (auto& r : res)
        if (r.flags & SA_FLAG_DIVERGED)
            throw std::runtime_error("seqalib: the reference traceback does not terminate for this scoring");
}

// Symbol coding of a batch into the packed byte buffers.  Byte symbols are their own codes: they
// are copied on the host threads, each marking the symbols it saw (for the match table) in a table
// of its own.  Other types get codes in order of first appearance (serial; stops on overflow).
template <typename Coder, typename ContainerType>
void code_symbols(std::true_type, Coder& coder, const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs,
                  const std::vector<uint64_t>& o1, const std::vector<uint64_t>& o2, raw_vector<uint8_t>& s1,
                  raw_vector<uint8_t>& s2) {
    const size_t nth = host_threads(pairs.size());
    std::vector<std::array<uint8_t, 256>> seen(nth);
    parallel_pairs(pairs.size(), nth, [&](size_t t, size_t p0, size_t p1) {
        std::array<uint8_t, 256>& sn = seen[t];
        sn.fill(0);
        for (size_t q = p0; q < p1; ++q) {
            ContainerType& a = *pairs[q].first;
            ContainerType& b = *pairs[q].second;
            uint8_t* d1 = s1.data() + o1[q];
            uint8_t* d2 = s2.data() + o2[q];
            for (size_t k = 0; k < (size_t)a.size(); ++k) sn[d1[k] = (uint8_t)a[k]] = 1;
            for (size_t k = 0; k < (size_t)b.size(); ++k) sn[d2[k] = (uint8_t)b[k]] = 1;
        }
    });
    using Ty = typename std::remove_reference<decltype((*pairs[0].first)[0])>::type;
    for (auto& sn : seen)
        for (int c = 0; c < 256; ++c)
            if (sn[c]) coder.code((typename std::remove_cv<Ty>::type)(uint8_t)c);
}
template <typename Coder, typename ContainerType>
void code_symbols(std::false_type, Coder& coder, const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs,
                  const std::vector<uint64_t>& o1, const std::vector<uint64_t>& o2, raw_vector<uint8_t>& s1,
                  raw_vector<uint8_t>& s2) {
    for (size_t q = 0; q < pairs.size(); ++q) {
        ContainerType& a = *pairs[q].first;
        ContainerType& b = *pairs[q].second;
        uint8_t* d1 = s1.data() + o1[q];
        uint8_t* d2 = s2.data() + o2[q];
        for (size_t k = 0; k < (size_t)a.size(); ++k) d1[k] = coder.code(a[k]);
        for (size_t k = 0; k < (size_t)b.size(); ++k) d2[k] = coder.code(b[k]);
        if (coder.overflow) break;
    }
}

// Aligns a batch of (Seq1, Seq2) pairs on the GPU.  Returns the per-pair results and the op
// streams (traceback order).  has_fn = false means the reference's nullptr match fn (equality).
// chunks > 1: the GPU call runs in that many pair ranges (sa_align_batch_cb) and on_chunk(p0, p1)
// is called, on this thread, as soon as a range's results and op streams are in res / ops (the
// other paths report the whole batch once at the end).
using ChunkFn = std::function<void(size_t, size_t)>;
inline void chunk_tramp(void* user, uint32_t p0, uint32_t p1) { (*static_cast<ChunkFn*>(user))(p0, p1); }

template <typename Ty, typename ContainerType, typename MatchFnTy>
void align(int algo, const sa_scoring& sc, MatchFnTy& fn, bool has_fn,
           const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs,
           std::vector<sa_result>& res, raw_vector<uint8_t>& ops, std::vector<uint64_t>& ops_off,
           uint32_t chunks = 0, ChunkFn on_chunk = nullptr) {
    PhaseTimer tm;
    SymbolCoder<Ty> coder;
    std::vector<uint64_t> o1(1, 0), o2(1, 0);
    o1.reserve(pairs.size() + 1);
    o2.reserve(pairs.size() + 1);
    for (auto& p : pairs) {
        o1.push_back(o1.back() + (uint64_t)p.first->size());
        o2.push_back(o2.back() + (uint64_t)p.second->size());
    }
    raw_vector<uint8_t>& s1 = host_buffer(kHostSeq1);   // (+1 below: never a NULL pointer)
    raw_vector<uint8_t>& s2 = host_buffer(kHostSeq2);
    s1.resize(o1.back() + 1);
    s2.resize(o2.back() + 1);
    constexpr bool kDirect = std::is_integral<Ty>::value && sizeof(Ty) == 1;
    code_symbols(std::integral_constant<bool, kDirect>{}, coder, pairs, o1, o2, s1, s2);
    tm.lap("symbol coding");
    if (coder.overflow) {   // more than 256 distinct symbols: the generic-Ty (bitmap) path
        align_bits<Ty>(algo, sc, fn, has_fn, pairs, res, ops, ops_off);
        if (on_chunk && !pairs.empty()) on_chunk(0, pairs.size());
        return;
    }
    std::vector<uint8_t> lut;
    if (has_fn) lut = build_lut(coder, fn);
    const uint32_t n = (uint32_t)pairs.size();
    res.assign(n, sa_result{});
    const uint64_t cap = s1.size() + s2.size() + n + 1;
    ops.resize(cap);
    ops_off.resize(n);
    for (uint32_t p = 0; p < n; ++p) ops_off[p] = o1[p] + o2[p] + p;
    tm.lap("match table + buffers");
    if (sa_multi* mg = multi_context()) {
        const int rc = sa_multi_align_batch(mg, algo, &sc, s1.data(), o1.data(), s2.data(), o2.data(), n,
                                            has_fn ? lut.data() : nullptr, res.data(), ops.data(), cap);
        if (rc != SA_OK)
            throw std::runtime_error(std::string("seqalib: sa_multi_align_batch: ") + sa_status_string(rc) + " (" +
                                     sa_multi_last_error(mg) + ")");
        if (on_chunk && n) on_chunk(0, n);
    } else {
        check(sa_align_batch_cb(context(), algo, &sc, s1.data(), o1.data(), s2.data(), o2.data(), n,
                                has_fn ? lut.data() : nullptr, res.data(), ops.data(), cap, chunks,
                                on_chunk ? chunk_tramp : nullptr, on_chunk ? &on_chunk : nullptr),
              "sa_align_batch");
    }
    tm.lap("sa_align_batch (GPU)");
    for (auto& r : res) {
        if (r.flags & SA_FLAG_DIVERGED)
            throw std::runtime_error("seqalib: the reference traceback does not terminate for this scoring");
        if (r.flags & SA_FLAG_TIMEOUT)
            throw std::runtime_error("seqalib: device band hand-off timed out; result invalid");
    }
}

}  // namespace detail
}  // namespace seqalib
