// Single-call latency of the C++ drop-in: the reference's canonical use is one
// pair per getAlignment(), timed in microseconds (include/Test.cpp:98-107: construct the aligner,
// call getAlignment, std::chrono around both).  Same calls here, through the GPU engine:
//   * config 1: NeedlemanWunschSA<std::string,char,'-'>(ScoringSystem(-1,2), equal<char>) on
//     test/Test.cpp's pair "AAAGAATGCAT" / "AAACTCAT";
//   * one 1024 x 1024 SmithWatermanSA (default scoring) DNA pair.
// The first-call costs are reported apart: "context_us" opens the drop-in's HIP context (runtime
// start-up + stream), each call's "first_call_us" is its first getAlignment (code-object load at
// the first launch, pinned buffers); then `reps` calls are timed one by one.  With
// SEQALIB_HOST_TIMING set the library prints each call's host phases to stderr (bench.py reads
// them).  Prints one JSON line.   dropin_latency [reps=200] [nw|sw: that call only]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "seqalib/SequenceAlignment.h"

template <typename T>
bool equal(T V1, T V2) { return V1 == V2; }

template <typename Call>
void timed(const char* name, int reps, Call call, bool last) {
    const auto f0 = std::chrono::steady_clock::now();
    size_t len = call();
    const double first = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - f0).count();
    std::vector<double> us;
    for (int r = 0; r < reps; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        len += call();
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(us.begin(), us.end());
    double sum = 0;
    for (double u : us) sum += u;
    printf("\"%s\": {\"first_call_us\": %.1f, \"reps\": %d, \"median_us\": %.1f, \"mean_us\": %.1f, \"min_us\": %.1f, "
           "\"p90_us\": %.1f, \"entries\": %zu}%s",
           name, first, reps, us[us.size() / 2], sum / us.size(), us[0], us[us.size() * 9 / 10], len, last ? "" : ", ");
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    const std::string only = argc > 2 ? argv[2] : "";
    std::string a = "AAAGAATGCAT", b = "AAACTCAT";   // test/Test.cpp:29-30
    std::string x(1024, 'A'), y(1024, 'A');
    sa_synth_dna(1000000001ull, 1024, reinterpret_cast<uint8_t*>(&x[0]));   // config 1 x 1e9 seeds
    sa_synth_dna(1000000002ull, 1024, reinterpret_cast<uint8_t*>(&y[0]));
    const auto c0 = std::chrono::steady_clock::now();
    seqalib::detail::context();
    const double ctx_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count();
    printf("{\"what\": \"C++ drop-in getAlignment per call (aligner constructed per call, as include/Test.cpp:98-107)\", ");
    printf("\"context_us\": %.1f, ", ctx_us);
    if (only != "sw") timed("nw_11x8", reps, [&] {
        AlignedSequence<char, '-'> r = NeedlemanWunschSA<std::string, char, '-'>(ScoringSystem(-1, 2), equal<char>).getAlignment(a, b);
        return r.Data.size();
    }, only == "nw");
    if (only != "nw") timed("sw_1024x1024", std::max(1, reps / 4), [&] {
        AlignedSequence<char, '-'> r = SmithWatermanSA<std::string, char, '-'>(ScoringSystem(-1, 1, -1), equal<char>).getAlignment(x, y);
        return r.Data.size();
    }, true);
    printf("}\n");
    return 0;
}
