// Drop-in end-to-end timing (SURVEY.md §8(d) "end-to-end including list construction"): the C++
// header API exactly as a SeqALib user calls it — SmithWatermanSA<std::string, char, '-'> with
// equal<char> — over a batch of synthetic DNA pairs held in host std::strings.  The clock covers
// getAlignments(): symbol coding, H2D, fill, traceback, D2H and building every
// AlignedSequence's std::list.  Prints one JSON line.
//   dropin_bench [pairs=1000] [len=4096] [reps=3]
#include <chrono>
#include <cstdio>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <malloc.h>
#include <sys/resource.h>
#include <string>
#include <vector>

#include "seqalib/SequenceAlignment.h"

template <typename T>
bool equal(T V1, T V2) { return V1 == V2; }

// cgroup v2 CPU throttling counters of this process's cgroup (nr_throttled, throttled_usec)
static void cpu_stat(unsigned long long& nr, unsigned long long& us) {
    nr = us = 0;
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.stat", "r")) {
        char k[64];
        unsigned long long v;
        while (fscanf(f, "%63s %llu", k, &v) == 2) {
            if (!strcmp(k, "nr_throttled")) nr = v;
            if (!strcmp(k, "throttled_usec")) us = v;
        }
        fclose(f);
    }
}

int main(int argc, char** argv) {
    const uint32_t P = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000;
    const uint32_t L = argc > 2 ? (uint32_t)atoi(argv[2]) : 4096;
    const int reps = argc > 3 ? atoi(argv[3]) : 3;
    // argv[4] = "keep": glibc keeps freed memory instead of returning it to the kernel (no trim, no
    // mmap'd chunks), so each rep's ~48 M list nodes reuse the pages of the rep before instead of
    // faulting fresh ones in (A/B of the list-construction spread; the default is glibc's)
    if (argc > 4 && !strcmp(argv[4], "keep")) {
        mallopt(M_TRIM_THRESHOLD, INT_MAX);
        mallopt(M_MMAP_THRESHOLD, INT_MAX);
    }
    std::vector<std::string> s1(P, std::string(L, 'A')), s2(P, std::string(L, 'A'));
    for (uint32_t p = 0; p < P; ++p) {   // seeds base+2p+1 / base+2p+2, base = 3e9
        sa_synth_dna(3000000000ull + 2 * p + 1, L, reinterpret_cast<uint8_t*>(&s1[p][0]));
        sa_synth_dna(3000000000ull + 2 * p + 2, L, reinterpret_cast<uint8_t*>(&s2[p][0]));
    }
    std::vector<std::pair<std::string*, std::string*>> pairs;
    for (uint32_t p = 0; p < P; ++p) pairs.push_back({&s1[p], &s2[p]});
    SmithWatermanSA<std::string, char, '-'> sw(ScoringSystem(-1, 1, -1), equal<char>);
    size_t entries = 0;
    {
        auto warm = sw.getAlignments(pairs);   // first call: context + workspace allocation
    }
    double best = 1e30, sum = 0;
    std::string each, thr;
    for (int r = 0; r < reps; ++r) {
        unsigned long long n0, u0, n1, u1;
        cpu_stat(n0, u0);
        struct rusage ru0, ru1;
        getrusage(RUSAGE_SELF, &ru0);
        const auto t0 = std::chrono::steady_clock::now();
        auto out = sw.getAlignments(pairs);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        cpu_stat(n1, u1);
        getrusage(RUSAGE_SELF, &ru1);
        char tb[160];
        snprintf(tb, sizeof tb, "%s{\"nr_throttled\": %llu, \"throttled_ms\": %.2f, \"minor_faults\": %ld}", r ? ", " : "",
                 n1 - n0, (u1 - u0) / 1e3, ru1.ru_minflt - ru0.ru_minflt);
        thr += tb;
        best = std::min(best, s);
        sum += s;
        entries = 0;
        for (auto& a : out) entries += a.Data.size();
        char b[32];
        snprintf(b, sizeof b, "%s%.2f", r ? ", " : "", s * 1e3);
        each += b;
    }
    const double cells = (double)P * L * L;
    printf("{\"what\": \"C++ drop-in SmithWatermanSA<std::string,char,'-'>::getAlignments, end-to-end incl. "
           "std::list construction\", \"pairs\": %u, \"len\": %u, \"reps\": %d, \"ms_best\": %.2f, "
           "\"ms_mean\": %.2f, \"ms_each\": [%s], \"gcups_best\": %.1f, \"gcups_mean\": %.1f, \"entries\": %zu, "
           "\"per_rep\": [%s]}\n",
           P, L, reps, best * 1e3, sum / reps * 1e3, each.c_str(), cells / best / 1e9, cells / (sum / reps) / 1e9, entries,
           thr.c_str());
    return 0;
}
