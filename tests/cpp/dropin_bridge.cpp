// Drop-in check for NW bridging: the gaps between anchors of a
// composite aligner, filled with StaticFuncs::bridgeNW (reference StaticFuncs.h:27-39).  Built
// against the unmodified reference (oracle/Makefile, target ref-dropin) every window is bridged
// by the reference's bridgeNW in order; built against the drop-in, all windows of all pairs go
// through the batched extension bridgeNWBatch in ONE GPU pass.  The printed alignments must be
// identical (tests/golden/dropin_bridge.ref.txt).
#include <cstdint>
#include <iostream>
#include <random>
#include <string>
#include <vector>

#ifdef SEQALIB_REFERENCE
#include <cmath>
#include <limits>
#include "SequenceAlignment.h"
#else
#include "seqalib/SequenceAlignment.h"
#endif

template <typename T>
bool equal(T V1, T V2) { return V1 == V2; }

using Fn = std::function<bool(char, char)>;
using SF = StaticFuncs<std::string, char, '-', Fn>;

static std::string dna(uint64_t seed, int n) {
    std::mt19937_64 g(seed);
    std::string s(n, 'A');
    for (auto& c : s) c = "ACGT"[g() & 3];
    return s;
}

int main() {
    // three sequence pairs; anchors every ~80-140 bp, gaps of varied shapes bridged by NW
    std::vector<std::string> s1, s2;
    for (int p = 0; p < 3; ++p) {
        s1.push_back(dna(100 + p, 2000 + 300 * p));
        s2.push_back(dna(200 + p, 1800 + 500 * p));
    }
    std::vector<AlignedSequence<char, '-'>> res(3);
    std::mt19937_64 g(7);
    struct W { int p, i1, i2, e1, e2; };
    std::vector<W> ws;
    for (int p = 0; p < 3; ++p) {
        int i1 = 0, i2 = 0;
        while (true) {
            const int e1 = i1 + (int)(g() % 140), e2 = i2 + (int)(g() % 140);
            if (e1 > (int)s1[p].size() || e2 > (int)s2[p].size()) break;
            ws.push_back(W{p, i1, i2, e1, e2});
            i1 = e1 + 20;   // skip an "anchor" of 20
            i2 = e2 + 20;
        }
    }
    for (int k = 0; k < 2; ++k) {   // two scorings: (-1,2,-1) with a predicate, (-2,1,-1,false)
        ScoringSystem sc = k == 0 ? ScoringSystem(-1, 2, -1) : ScoringSystem(-2, 1, -1, false);
        Fn fn = equal<char>;
        for (auto& r : res) r.Data.clear();
#ifdef SEQALIB_REFERENCE
        for (const W& w : ws) SF::bridgeNW(s1[w.p], s2[w.p], res[w.p], sc, w.i1, w.i2, w.e1, w.e2, fn);
#else
        std::vector<SF::Job> jobs;
        for (const W& w : ws) jobs.push_back(SF::Job{&s1[w.p], &s2[w.p], w.i1, w.i2, w.e1, w.e2, &res[w.p]});
        SF::bridgeNWBatch(jobs, sc, fn);
#endif
        for (auto& r : res) {
            std::string a, b, m;
            for (auto& e : r) { a += e.get(0); m += e.match() ? '|' : ' '; b += e.get(1); }
            std::cout << ws.size() << ' ' << a << '\n' << m << '\n' << b << '\n';
        }
    }
    return 0;
}
