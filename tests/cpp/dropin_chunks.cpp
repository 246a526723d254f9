// Chunked drop-in batch check (run() in include/seqalib/SequenceAlignment.h): a getAlignments()
// batch large enough to be aligned in several chunks, whose lists are built while later chunks are
// still on the GPU.  Pair p = synth DNA of seeds 7e9 + 2p + 1 / + 2, Seq1 length 40 + (37p mod 260),
// Seq2 the Seq1 of pair p mutated (every third pair) or its own random sequence, length
// 30 + (53p mod 270).  Prints, per pair, the FNV-1a 64 of the three printAlignment rows
// (include/Test.cpp:10-31) joined by '\n' -- tests/test_dropin_cpp.py recomputes them from the oracle.
//   dropin_chunks [pairs=4500] [sw|nw|lg]
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "seqalib/SequenceAlignment.h"

template <typename T>
bool equal(T V1, T V2) { return V1 == V2; }

static uint64_t fnv(const std::string& s) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h;
}

int main(int argc, char** argv) {
    const uint32_t P = argc > 1 ? (uint32_t)atoi(argv[1]) : 4500;
    std::vector<std::string> s1(P), s2(P);
    for (uint32_t p = 0; p < P; ++p) {
        const uint32_t m = 40 + (37 * p) % 260, n = 30 + (53 * p) % 270;
        s1[p].assign(m, 'A');
        sa_synth_dna(7000000000ull + 2 * p + 1, m, reinterpret_cast<uint8_t*>(&s1[p][0]));
        s2[p].assign(n, 'A');
        sa_synth_dna(7000000000ull + 2 * p + 2, n, reinterpret_cast<uint8_t*>(&s2[p][0]));
        if (p % 3 == 0)
            for (uint32_t k = 0; k < n && k < m; ++k) s2[p][k] = (k % 11 == 5) ? s2[p][k] : s1[p][k];
    }
    std::vector<std::pair<std::string*, std::string*>> pairs;
    for (uint32_t p = 0; p < P; ++p) pairs.push_back({&s1[p], &s2[p]});
    auto print = [&](std::vector<AlignedSequence<char, '-'>>& out) {
        for (uint32_t p = 0; p < P; ++p) {
            std::string r0, bars, r1;
            for (auto& e : out[p].Data) {
                r0 += e.get(0);
                bars += e.match() ? '|' : ' ';
                r1 += e.get(1);
            }
            printf("%016llx\n", (unsigned long long)fnv(r0 + "\n" + bars + "\n" + r1));
        }
    };
    const std::string algo = argc > 2 ? argv[2] : "sw";
    if (algo == "sw") {
        SmithWatermanSA<std::string, char, '-'> a(ScoringSystem(-1, 1, -1), equal<char>);
        auto out = a.getAlignments(pairs);
        print(out);
    } else if (algo == "nw") {
        NeedlemanWunschSA<std::string, char, '-'> a(ScoringSystem(-1, 2, -1), equal<char>);
        auto out = a.getAlignments(pairs);
        print(out);
    } else {   // LocalGotoh: the size-hack split reports the whole batch at the end
        LocalGotohSA<std::string, char, '-'> a(ScoringSystem(-3, -1, 1, -1), equal<char>);
        auto out = a.getAlignments(pairs);
        print(out);
    }
    return 0;
}
