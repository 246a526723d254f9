// Drop-in check for the generic parts of the API: non-char containers (std::vector<int>) with a
// user predicate, ArrayView windows + StaticFuncs::useNW (the NW call path of the reference's
// composite aligners), the batch extension, and SmithWatermanSA's member persistence on empty
// input (SASmithWaterman.h:14-16, :232-238).  Prints one result per line.
#include <iostream>
#include <string>
#include <vector>

#ifdef SEQALIB_REFERENCE   // built against the unmodified reference (oracle/Makefile, target ref-dropin)
#include <cmath>
#include <limits>
#include "SequenceAlignment.h"
#else
#include "seqalib/SequenceAlignment.h"
#endif

template <typename T>
bool equal(T V1, T V2) { return V1 == V2; }

template <typename Ty, Ty Blank>
static void print(AlignedSequence<Ty, Blank>& r) {
    for (auto& e : r) std::cout << e.get(0) << ',';
    std::cout << '|';
    for (auto& e : r) std::cout << (e.match() ? '1' : '0');
    std::cout << '|';
    for (auto& e : r) std::cout << e.get(1) << ',';
    std::cout << '\n';
}

int main() {
    // 1. std::vector<int>, Blank = -1, predicate "same residue class mod 3"
    std::vector<int> a = {5, 1, 7, 7, 2, 9, 4, 4, 8, 300, 12}, b = {5, 7, 7, 3, 9, 4, 8, 300, 12, 6};
    auto mod3 = [](int x, int y) { return x % 3 == y % 3; };
    SmithWatermanSA<std::vector<int>, int, -1, std::function<bool(int, int)>> sw(ScoringSystem(-1, 2, -1), mod3);
    auto r1 = sw.getAlignment(a, b);
    print(r1);
    NeedlemanWunschSA<std::vector<int>, int, -1> nw(ScoringSystem(-1, 2, -1), equal<int>);
    auto r2 = nw.getAlignment(a, b);
    print(r2);
    // 2. ArrayView + StaticFuncs::useNW over std::string
    std::string s = "AAAGAATGCAT", t = "AAACTCAT";
    AlignedSequence<char, '-'> r3;
    StaticFuncs<std::string, char, '-'>::useNW(s, t, r3, ScoringSystem(-1, 2), equal<char>);
    print(r3);
    AlignedSequence<char, '-'> r4;
    StaticFuncs<std::string, char, '-'>::bridgeNW(s, t, r4, ScoringSystem(-1, 2, -1), 2, 1, 9, 7, equal<char>);
    print(r4);
    // 3. batch extension
    std::string x1 = "AGCTTCAGGCTGA", y1 = "AGCTGGATCGATCGATG", x2 = "CTGAAGCGG", y2 = "CTCAAGCGTAGTCC";
    LocalGotohSA<std::string, char, '-'> lg(ScoringSystem(-3, -1, 1, -1, true), equal<char>);
#ifdef SEQALIB_REFERENCE
    auto rs0 = lg.getAlignment(x1, y1);
    auto rs1 = lg.getAlignment(x2, y2);
    print(rs0);
    print(rs1);
#else
    std::vector<std::pair<std::string*, std::string*>> batch = {{&x1, &y1}, {&x2, &y2}};
    auto rs = lg.getAlignments(batch);
    print(rs[0]);
    print(rs[1]);
#endif
    // 4. SW: an empty input re-uses the previous call's max cell in forceGlobal
    SmithWatermanSA<std::string, char, '-'> sw2(ScoringSystem(-1, 1, -1), equal<char>);
    std::string p = "GGTCGCGACTAC", q = "CGACTA", e = "";
    auto r5 = sw2.getAlignment(p, q);
    print(r5);
    auto r6 = sw2.getAlignment(p, e);
    print(r6);
    return 0;
}
