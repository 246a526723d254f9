// TEST INFRASTRUCTURE ONLY — never linked into, loaded by or called from the product path.
//
// Thin C-ABI harness around the *unmodified* reference headers in /root/reference/include
// (przemektmalon/SeqALib).  It is compiled in place by `oracle/Makefile` (target `ref`) into
// `oracle/_ref/libsaref.so`; nothing from the reference is copied into this repository.
//
// Build workarounds, all on the command line / in oracle/_ref:
//   * SequenceAlignment.h:259 includes "staticFuncs.h" but the file is StaticFuncs.h: the
//     Makefile puts a *symlink* oracle/_ref/shim/staticFuncs.h -> the real StaticFuncs.h on
//     the include path (same file, case-correct name; no stand-in content).
//   * <limits>, <cmath>, <chrono> are used but never included: `-include` them.
//   * MaxScore/MaxRow/MaxCol/Matrix are private and getAlignment() never exposes them, so this
//     TU pre-includes the std headers and then `#define private public` before the reference
//     header, and drives the same call sequence getAlignment() uses
//     (cacheAllMatches -> computeScoreMatrix -> [read members] -> buildResult -> clearAll),
//     e.g. SASmithWaterman.h:358-366, SANeedlemanWunsch.h:256-264, SALocalGotoh.h:518-526,
//     SAGlobalGotoh.h:450-459.
#include <algorithm>
#include <atomic>
#include <cassert>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <limits>
#include <list>
#include <memory>
#include <queue>
#include <random>
#include <string>
#include <thread>
#include <vector>

#define private public
#include "SequenceAlignment.h"
#undef private

namespace {

using Fn = std::function<bool(char, char)>;
using SW = SmithWatermanSA<std::string, char, '-'>;
using NW = NeedlemanWunschSA<std::string, char, '-'>;
using LG = LocalGotohSA<std::string, char, '-'>;
using GG = GlobalGotohSA<std::string, char, '-'>;
using HB = HirschbergSA<std::string, char, '-'>;
using MM = MyersMillerSA<std::string, char, '-'>;

bool equal_char(char a, char b) { return a == b; }

// nargs selects the ScoringSystem overload exactly as user code would (SequenceAlignment.h:92-118).
ScoringSystem make_scoring(int nargs, int a0, int a1, int a2, int a3, int allow) {
    if (nargs == 2) return ScoringSystem(a0, a1);
    if (nargs == 3) return ScoringSystem(a0, a1, a2);
    if (nargs == 4) return ScoringSystem(a0, a1, a2, allow != 0);
    return ScoringSystem(a0, a1, a2, a3, allow != 0);
}

struct Lut {
    const unsigned char* t;
    bool operator()(char a, char b) const { return t[(unsigned char)a * 256 + (unsigned char)b] != 0; }
};

Fn make_fn(int match_mode, const unsigned char* lut) {
    if (match_mode == 0) return nullptr;        // reference default: nullptr match fn
    if (match_mode == 1) return equal_char;     // include/Test.cpp:7-8 `equal<char>`
    return Fn(Lut{lut});                        // arbitrary user predicate over char
}

template <typename A>
void emit(AlignedSequence<char, '-'>& r, char* row0, char* bars, char* row1, int cap, int* len) {
    int k = 0;
    for (auto& e : r) {
        if (k < cap) {
            row0[k] = e.get(0);
            bars[k] = e.match() ? '|' : ' ';
            row1[k] = e.get(1);
        }
        ++k;
    }
    *len = k;
}

}  // namespace

extern "C" {

struct ref_out {
    int32_t score;      // SW/LG: MaxScore; NW/GG: H[m][n]
    int32_t max_row;    // SW/LG: MaxRow; NW/GG: m
    int32_t max_col;    // SW/LG: MaxCol; NW/GG: n
    int32_t len;        // number of Entries in the AlignedSequence
};

// Align one pair with the reference.  Returns 0, or -1 if the output did not fit in `cap`.
int ref_align(int algo, int nargs, int a0, int a1, int a2, int a3, int allow, int match_mode,
              const unsigned char* lut, const char* s1, int m, const char* s2, int n,
              ref_out* out, char* row0, char* bars, char* row1, int cap) {
    std::string q(s1, s1 + m), t(s2, s2 + n);
    ScoringSystem sc = make_scoring(nargs, a0, a1, a2, a3, allow);
    Fn fn = make_fn(match_mode, lut);
    AlignedSequence<char, '-'> res;
    if (algo == 0) {
        SW a(sc, fn);
        a.cacheAllMatches(q, t);
        a.computeScoreMatrix(q, t);
        out->score = a.MaxScore;
        out->max_row = (int)a.MaxRow;
        out->max_col = (int)a.MaxCol;
        a.buildResult(q, t, res);
        a.clearAll();
    } else if (algo == 1) {
        NW a(sc, fn);
        a.cacheAllMatches(q, t);
        a.computeScoreMatrix(q, t);
        out->score = a.Matrix[(size_t)m * (n + 1) + n];
        out->max_row = m;
        out->max_col = n;
        a.buildResult(q, t, res);
        a.clearAll();
    } else if (algo == 2) {
        LG a(sc, fn);
        a.MaxRow = 0;  // uninitialised in the reference (SALocalGotoh.h:30-31); only read for empty inputs
        a.MaxCol = 0;
        a.cacheAllMatches(q, t);
        a.computeScoreMatrix(q, t);
        out->score = a.Matrix[a.MaxRow * (n + 1) + a.MaxCol];
        out->max_row = (int)a.MaxRow;
        out->max_col = (int)a.MaxCol;
        a.buildResult(q, t, res);
        a.clearAll();
    } else if (algo == 4) {
        // HirschbergSA::getAlignment (SAHirschberg.h:172-184) exposes no score: report H[m][n] of
        // NW with the same scoring (every Hirschberg alignment is an optimal NW alignment).
        NW s(sc, fn);
        s.cacheAllMatches(q, t);
        s.computeScoreMatrix(q, t);
        out->score = s.Matrix[(size_t)m * (n + 1) + n];
        s.clearAll();
        out->max_row = m;
        out->max_col = n;
        HB a(sc, fn);
        // copy-initialise: AlignedSequence::operator= does not compile (SequenceAlignment.h:62-66)
        AlignedSequence<char, '-'> hres = a.getAlignment(q, t);
        int len = 0;
        emit<int>(hres, row0, bars, row1, cap, &len);
        out->len = len;
        return len <= cap ? 0 : -1;
    } else if (algo == 5) {
        // MyersMillerSA::getAlignment (SAMyersMiller.h:412-420) exposes no score (none reported).
        out->score = 0;
        out->max_row = m;
        out->max_col = n;
        MM a(sc, fn);
        AlignedSequence<char, '-'> mres = a.getAlignment(q, t);
        int len = 0;
        emit<int>(mres, row0, bars, row1, cap, &len);
        out->len = len;
        return len <= cap ? 0 : -1;
    } else {
        GG a(sc, fn);
        a.cacheAllMatches(q, t);
        a.computeScoreMatrix(q, t);
        out->score = a.Matrix[(size_t)m * (n + 1) + n];
        out->max_row = m;
        out->max_col = n;
        a.buildResult(q, t, res);
        a.clearAll();
    }
    int len = 0;
    emit<int>(res, row0, bars, row1, cap, &len);
    out->len = len;
    return len <= cap ? 0 : -1;
}

// Public-API path only (getAlignment), as a user would call it: used as the CPU baseline.
// Runs SmithWatermanSA<std::string,char,'-'>(ScoringSystem(gap,match,mismatch,allow), equal<char>)
// over npairs pairs on `threads` std::threads (one aligner per pair).  Writes the alignment
// length of each pair into out_len.
int ref_sw_batch(int gap, int match, int mismatch, int allow, const char* s1cat,
                 const uint64_t* off1, const char* s2cat, const uint64_t* off2, int npairs,
                 int threads, int32_t* out_len) {
    if (threads < 1) threads = 1;
    std::vector<std::thread> pool;
    std::atomic<int> next{0};
    for (int w = 0; w < threads; ++w) {
        pool.emplace_back([&]() {
            for (;;) {
                int p = next.fetch_add(1);
                if (p >= npairs) break;
                std::string q(s1cat + off1[p], s1cat + off1[p + 1]);
                std::string t(s2cat + off2[p], s2cat + off2[p + 1]);
                SW a(ScoringSystem(gap, match, mismatch, allow != 0), equal_char);
                AlignedSequence<char, '-'> r = a.getAlignment(q, t);
                out_len[p] = (int32_t)r.Data.size();
            }
        });
    }
    for (auto& th : pool) th.join();
    return 0;
}

// Per-call latency of the reference's public API, timed the way include/Test.cpp:98-107 times it:
// construct the aligner, getAlignment(seq1, seq2), with equal<char>; algo 0 SmithWatermanSA,
// 1 NeedlemanWunschSA.  Runs `reps` calls on the calling thread and returns the mean ns per call.
double ref_call_ns(int algo, int nargs, int a0, int a1, int a2, int allow, const char* s1, int m,
                   const char* s2, int n, int reps) {
    std::string q(s1, s1 + m), t(s2, s2 + n);
    const ScoringSystem sc = nargs == 2 ? ScoringSystem(a0, a1) : ScoringSystem(a0, a1, a2, allow != 0);
    size_t sink = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < reps; ++k) {
        if (algo == 0) {
            AlignedSequence<char, '-'> r = SmithWatermanSA<std::string, char, '-'>(sc, equal_char).getAlignment(q, t);
            sink += r.Data.size();
        } else {
            AlignedSequence<char, '-'> r = NeedlemanWunschSA<std::string, char, '-'>(sc, equal_char).getAlignment(q, t);
            sink += r.Data.size();
        }
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (sink == (size_t)-1) std::abort();
    return std::chrono::duration<double, std::nano>(t1 - t0).count() / (reps > 0 ? reps : 1);
}

// std::mt19937_64 DNA generator: symbol = "ACGT"[g() & 3].  Pins the
// product library's own generator (sa_synth_dna) bit for bit.
void ref_gen_dna(uint64_t seed, int len, char* out) {
    std::mt19937_64 g(seed);
    for (int i = 0; i < len; ++i) out[i] = "ACGT"[g() & 3];
}

}  // extern "C"
