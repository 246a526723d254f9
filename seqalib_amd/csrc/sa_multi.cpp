// sa_multi.cpp — several GPUs of one node behind one handle (include/seqalib_hip.h, sa_multi_*).
//
// Pairs are independent, so a batch is cut into contiguous pair ranges of near-equal work
// (sum of m*n), one per device, with no collective anywhere.  Every device has
// a persistent context (its cached workspace survives across calls) and one host thread per
// call.  A contiguous range [s, e) of the batch is itself a batch whose op buffer is exactly
// ops + (off1[s] + off2[s] + s): each device writes its results and op streams straight into
// the caller's buffers at their final place, so nothing is gathered or copied afterwards.
#include <stdint.h>
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "../../include/seqalib_hip.h"

struct sa_multi {
    std::vector<sa_ctx*> ctx;
    std::string err;
};

namespace {
thread_local std::string g_multi_err;

int mfail(sa_multi* g, int code, const std::string& msg) {
    if (g) g->err = msg;
    g_multi_err = msg;
    return code;
}

// contiguous [start, end) ranges with near-equal sum of m*n (at least one pair per non-empty range)
std::vector<uint32_t> split_by_cells(const uint64_t* off1, const uint64_t* off2, uint32_t npairs, size_t parts) {
    std::vector<double> csum(npairs + 1, 0.0);
    for (uint32_t p = 0; p < npairs; ++p)
        csum[p + 1] = csum[p] + (double)(off1[p + 1] - off1[p]) * (double)(off2[p + 1] - off2[p]) + 1.0;
    std::vector<uint32_t> cut(parts + 1, 0);
    cut[parts] = npairs;
    uint32_t p = 0;
    for (size_t g = 1; g < parts; ++g) {
        const double target = csum[npairs] * (double)g / (double)parts;
        while (p < npairs && csum[p] < target) ++p;
        cut[g] = p;
    }
    for (size_t g = 1; g <= parts; ++g) cut[g] = cut[g] < cut[g - 1] ? cut[g - 1] : cut[g];
    return cut;
}
}  // namespace

extern "C" {

int sa_multi_create(const int* devices, int ndevices, sa_multi** out) {
    if (!out || !devices || ndevices <= 0) return mfail(nullptr, SA_ERR_ARG, "devices / out");
    *out = nullptr;
    sa_multi* g = new sa_multi();
    for (int k = 0; k < ndevices; ++k) {
        sa_ctx* c = nullptr;
        const int rc = sa_create(devices[k], &c);
        if (rc != SA_OK) {
            const std::string e = std::string("device ") + std::to_string(devices[k]) + ": " + sa_last_error(nullptr);
            sa_multi_destroy(g);
            return mfail(nullptr, rc, e);
        }
        g->ctx.push_back(c);
    }
    *out = g;
    return SA_OK;
}

void sa_multi_destroy(sa_multi* g) {
    if (!g) return;
    for (sa_ctx* c : g->ctx) sa_destroy(c);
    delete g;
}

const char* sa_multi_last_error(const sa_multi* g) { return g ? g->err.c_str() : g_multi_err.c_str(); }

int sa_multi_align_batch(sa_multi* g, int algo, const sa_scoring* scoring, const uint8_t* seq1,
                         const uint64_t* off1, const uint8_t* seq2, const uint64_t* off2, uint32_t npairs,
                         const uint8_t* lut, sa_result* results, uint8_t* ops, uint64_t ops_cap) {
    if (!g) return mfail(nullptr, SA_ERR_ARG, "handle is NULL");
    if (!off1 || !off2 || (npairs && (!results || !ops))) return mfail(g, SA_ERR_ARG, "NULL buffer");
    if (off1[0] != 0 || off2[0] != 0) return mfail(g, SA_ERR_ARG, "offsets must start at 0");
    for (uint32_t p = 0; p < npairs; ++p)
        if (off1[p + 1] < off1[p] || off2[p + 1] < off2[p]) return mfail(g, SA_ERR_ARG, "offsets must be non-decreasing");
    const uint64_t total = off1[npairs] + off2[npairs] + npairs;
    if (ops_cap < total) return mfail(g, SA_ERR_CAPACITY, "ops buffer needs " + std::to_string(total) + " bytes");
    const size_t G = g->ctx.size();
    const std::vector<uint32_t> cut = split_by_cells(off1, off2, npairs, G);
    std::vector<int> rc(G, SA_OK);
    auto work = [&](size_t d) {
        const uint32_t s = cut[d], e = cut[d + 1];
        if (e <= s) return;
        std::vector<uint64_t> o1(e - s + 1), o2(e - s + 1);
        for (uint32_t p = s; p <= e; ++p) {
            o1[p - s] = off1[p] - off1[s];
            o2[p - s] = off2[p] - off2[s];
        }
        const uint64_t base = off1[s] + off2[s] + s;
        const uint64_t cap = off1[e] + off2[e] + e - base;
        rc[d] = sa_align_batch(g->ctx[d], algo, scoring, seq1 ? seq1 + off1[s] : nullptr, o1.data(),
                               seq2 ? seq2 + off2[s] : nullptr, o2.data(), e - s, lut, results + s, ops + base, cap);
    };
    std::vector<std::thread> th;
    for (size_t d = 1; d < G; ++d) th.emplace_back(work, d);
    work(0);
    for (auto& t : th) t.join();
    for (size_t d = 0; d < G; ++d)
        if (rc[d] != SA_OK) return mfail(g, rc[d], "context " + std::to_string(d) + ": " + sa_last_error(g->ctx[d]));
    return SA_OK;
}

}  // extern "C"
