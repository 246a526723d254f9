// Host floor of the drop-in's list construction: 10,000 std::list<Entry> of 4,845 nodes each (the
// headline batch's 48.45 M entries, push_front as build_from_ops), built in chunks over T threads,
// freed between reps as a caller's loop does.  No GPU, no library.
//   g++ -O2 -o /tmp/lbf tools/list_build_floor.cpp -lpthread && /tmp/lbf [threads=8] [chunk=2048]
#include <list>
#include <vector>
#include <thread>
#include <chrono>
#include <cstdio>
#include <cstdlib>
struct E { char a, b; bool m; E(char x, char y, bool z): a(x), b(y), m(z) {} };
int main(int argc, char** argv) {
    const int P = 10000, N = 4845, T = argc > 1 ? atoi(argv[1]) : 8, reps = 5;
    const int chunk = argc > 2 ? atoi(argv[2]) : 2048;
    for (int r = 0; r < reps; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::list<E>> out(P);
        for (int c0 = 0; c0 < P; c0 += chunk) {
            const int c1 = std::min(P, c0 + chunk);
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t) th.emplace_back([&, t] {
                const int n = c1 - c0, q0 = c0 + n * t / T, q1 = c0 + n * (t + 1) / T;
                for (int p = q0; p < q1; ++p) for (int k = 0; k < N; ++k) out[p].push_front(E('A', 'C', k & 1));
            });
            for (auto& x : th) x.join();
        }
        double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        auto t1 = std::chrono::steady_clock::now();
        out.clear(); out.shrink_to_fit();
        double d = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
        printf("build %.1f ms  free %.1f ms\n", s * 1e3, d * 1e3);
    }
}
