// Drop-in check of the generic-Ty path with a WIDE alphabet: std::vector<int> sequences holding
// more than 256 distinct values (here ~2,000), with equality, a user predicate and a nullptr
// match fn, through the four DP aligners and the two linear-space ones (HirschbergSA,
// MyersMillerSA).  The drop-in build sends these batches down the
// match-bitmap path (sa_align_batch_bits); built against the unmodified reference
// (oracle/Makefile, target ref-dropin) the same source produced tests/golden/dropin_wide.ref.txt.
// Prints one line per alignment: Seq1 row | match bars | Seq2 row.
#include <cstdint>
#include <functional>
#include <iostream>
#include <string>
#include <vector>

#ifdef SEQALIB_REFERENCE
#include <cmath>
#include <limits>
#include "SequenceAlignment.h"
#else
#include "seqalib/SequenceAlignment.h"
#endif

template <typename Ty, Ty Blank>
static void print(AlignedSequence<Ty, Blank>& r) {
    for (auto& e : r) std::cout << e.get(0) << ',';
    std::cout << '|';
    for (auto& e : r) std::cout << (e.match() ? '1' : '0');
    std::cout << '|';
    for (auto& e : r) std::cout << e.get(1) << ',';
    std::cout << '\n';
}

static uint64_t lcg(uint64_t& s) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return s >> 33;
}

// a random sequence over `vocab` values, and a relative of it (substitutions and indels)
static std::vector<int> random_seq(uint64_t seed, int len, int vocab) {
    std::vector<int> v;
    for (int k = 0; k < len; ++k) v.push_back((int)(lcg(seed) % (uint64_t)vocab));
    return v;
}
static std::vector<int> relative(const std::vector<int>& a, uint64_t seed, int vocab) {
    std::vector<int> b;
    for (int x : a) {
        const int r = (int)(lcg(seed) % 100);
        if (r < 8) b.push_back((int)(lcg(seed) % (uint64_t)vocab));
        else if (r < 11) { b.push_back(x); b.push_back((int)(lcg(seed) % (uint64_t)vocab)); }
        else if (r < 14) continue;
        else b.push_back(x);
    }
    return b;
}

bool eq_int(int a, int b) { return a == b; }

int main() {
    std::vector<int> a = random_seq(11, 1500, 2000), b = relative(a, 12, 2000);
    std::vector<int> c = random_seq(13, 900, 3000), d = random_seq(14, 1100, 3000);
    std::function<bool(int, int)> near = [](int x, int y) { return x - y <= 1 && y - x <= 1; };
    std::function<bool(int, int)> eq = eq_int;
    using Fn = std::function<bool(int, int)>;
    {
        SmithWatermanSA<std::vector<int>, int, -1, Fn> sw(ScoringSystem(-1, 2, -1), eq);
        auto r = sw.getAlignment(a, b); print(r);
        SmithWatermanSA<std::vector<int>, int, -1, Fn> sw2(ScoringSystem(-2, 1, -1), near);
        auto r2 = sw2.getAlignment(c, d); print(r2);
    }
    {
        NeedlemanWunschSA<std::vector<int>, int, -1, Fn> nw(ScoringSystem(-1, 2, -1), eq);
        auto r = nw.getAlignment(a, b); print(r);
        NeedlemanWunschSA<std::vector<int>, int, -1, Fn> nw2(ScoringSystem(-1, 2), near);
        auto r2 = nw2.getAlignment(c, d); print(r2);
    }
    {
        LocalGotohSA<std::vector<int>, int, -1, Fn> lg(ScoringSystem(-3, -1, 2, -1), eq);
        auto r = lg.getAlignment(a, b); print(r);
        LocalGotohSA<std::vector<int>, int, -1, Fn> lg2(ScoringSystem(-3, -1, 1, -1, false), near);
        auto r2 = lg2.getAlignment(c, d); print(r2);
    }
    {
        GlobalGotohSA<std::vector<int>, int, -1, Fn> gg(ScoringSystem(-3, -1, 2, -1), eq);
        auto r = gg.getAlignment(a, b); print(r);
        GlobalGotohSA<std::vector<int>, int, -1, Fn> gg2(ScoringSystem(-3, -1, 1, -1), near);
        auto r2 = gg2.getAlignment(c, d); print(r2);
    }
    {
        // (the reference's HirschbergSA calls the match fn per cell, so it needs one)
        HirschbergSA<std::vector<int>, int, -1, Fn> hb(ScoringSystem(-1, 2, -1), eq);
        auto r = hb.getAlignment(a, b); print(r);
        HirschbergSA<std::vector<int>, int, -1, Fn> hb2(ScoringSystem(-1, 2, -1, false), near);
        auto r2 = hb2.getAlignment(c, d); print(r2);
        HirschbergSA<std::vector<int>, int, -1, Fn> hb3(ScoringSystem(-2, 1, -1), near);
        auto r3 = hb3.getAlignment(a, d); print(r3);
    }
    {
        MyersMillerSA<std::vector<int>, int, -1, Fn> mm(ScoringSystem(-3, -1, 2, -1), eq);
        auto r = mm.getAlignment(a, b); print(r);
        MyersMillerSA<std::vector<int>, int, -1, Fn> mm2(ScoringSystem(-3, -1, 1, -1, false), near);
        auto r2 = mm2.getAlignment(c, d); print(r2);
        MyersMillerSA<std::vector<int>, int, -1, Fn> mm3(ScoringSystem(-2, -1, 2, -1));   // nullptr: ==
        auto r3 = mm3.getAlignment(b, c); print(r3);
    }
    return 0;
}
