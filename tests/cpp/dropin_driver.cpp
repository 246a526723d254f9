// Drop-in check: the reference's user-facing API (as used by include/Test.cpp:95-144 and
// test/Test.cpp:44-45), compiled with g++ against include/seqalib/ and linked to libseqalib_hip.
// Reads one case per line:  algo nargs a0 a1 a2 a3 allow match seq1 seq2   ('.' = empty)
// and prints, per case, the three printAlignment lines and getScore(), tab-separated.
#include <iostream>
#include <sstream>
#include <string>

#include "seqalib/SequenceAlignment.h"

template <typename T>
bool equal(T V1, T V2) { return V1 == V2; }

using Fn = std::function<bool(char, char)>;

static bool purine(char a, char b) {
    auto cls = [](char c) { return c == 'A' || c == 'G' ? 0 : (c == 'C' || c == 'T' ? 1 : 2); };
    return a == b || (cls(a) != 2 && cls(a) == cls(b));
}

template <typename A>
static void emit(A& aligner, std::string& s1, std::string& s2) {
    AlignedSequence<char, '-'> r = aligner.getAlignment(s1, s2);
    std::string r0, bars, r1;
    for (auto& e : r) { r0 += e.get(0); bars += e.match() ? '|' : ' '; r1 += e.get(1); }
    std::cout << r0 << '\t' << bars << '\t' << r1 << '\t' << aligner.getScore() << '\n';
}

static ScoringSystem scoring(int nargs, int a0, int a1, int a2, int a3, int allow) {
    if (nargs == 2) return ScoringSystem(a0, a1);
    if (nargs == 3) return ScoringSystem(a0, a1, a2);
    if (nargs == 4) return ScoringSystem(a0, a1, a2, allow != 0);
    return ScoringSystem(a0, a1, a2, a3, allow != 0);
}

int main() {
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string algo, match, s1, s2;
        int nargs, a0, a1, a2, a3, allow;
        in >> algo >> nargs >> a0 >> a1 >> a2 >> a3 >> allow >> match >> s1 >> s2;
        if (s1 == ".") s1.clear();
        if (s2 == ".") s2.clear();
        ScoringSystem sc = scoring(nargs, a0, a1, a2, a3, allow);
        Fn fn = match == "equal" ? Fn(equal<char>) : match == "purine" ? Fn(purine) : Fn(nullptr);
        if (algo == "sw") { SmithWatermanSA<std::string, char, '-'> a(sc, fn); emit(a, s1, s2); }
        else if (algo == "nw") { NeedlemanWunschSA<std::string, char, '-'> a(sc, fn); emit(a, s1, s2); }
        else if (algo == "lg") { LocalGotohSA<std::string, char, '-'> a(sc, fn); emit(a, s1, s2); }
        else if (algo == "hb") { HirschbergSA<std::string, char, '-'> a(sc, fn); emit(a, s1, s2); }
        else if (algo == "mm") { MyersMillerSA<std::string, char, '-'> a(sc, fn); emit(a, s1, s2); }
        else { GlobalGotohSA<std::string, char, '-'> a(sc, fn); emit(a, s1, s2); }
    }
    return 0;
}
