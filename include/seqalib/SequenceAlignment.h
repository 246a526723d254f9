// seqalib/SequenceAlignment.h — drop-in for the reference's single include
// (przemektmalon/SeqALib include/SequenceAlignment.h) for its DP hot path.
//
// Same public names and template signatures as the reference:
//   ScoreSystemType, AlignedSequence<Ty, Blank> (+ Entry), ScoringSystem,
//   SequenceAligner<ContainerType, Ty, Blank, MatchFnTy>,
//   SmithWatermanSA, NeedlemanWunschSA, LocalGotohSA, GlobalGotohSA, ArrayView, StaticFuncs.
// getAlignment() runs the DP fill and traceback on an MI355X through libseqalib_hip.so
// (include/seqalib_hip.h); the AlignedSequence list and forceGlobal are assembled here, on the
// host, exactly as the reference's buildResult does.  Link with -lseqalib_hip.
// Also provided: HirschbergSA and MyersMillerSA (linear-space, on the GPU).
// Not provided (outside the tier's hot path): FOGSAA, BLAT, MUMmer, SuffixTree and
// SequenceAligner::longestIncreasingSubsequence.
#pragma once

#include <algorithm>
#include <cassert>
#include <climits>
#include <cstdint>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <limits>
#include <list>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "detail/Engine.h"

#ifndef ScoreSystemType
#define ScoreSystemType int
#endif

// Result of an alignment: an ordered list of column pairs.
template <typename Ty, Ty Blank = Ty(0)>
class AlignedSequence {
public:
    class Entry {
        std::pair<Ty, Ty> Pair;
        bool IsMatchingPair = false;

    public:
        Entry() {}
        Entry(Ty V1, Ty V2) : Pair(V1, V2) { IsMatchingPair = !hasBlank(); }
        Entry(Ty V1, Ty V2, bool Matching) : Pair(V1, V2), IsMatchingPair(Matching) {}

        Ty get(size_t index) {
            assert((index == 0 || index == 1) && "Index out of bounds!");
            return index == 0 ? Pair.first : Pair.second;
        }
        bool empty() { return Pair.first == Blank && Pair.second == Blank; }
        bool hasBlank() { return Pair.first == Blank || Pair.second == Blank; }
        bool match() { return IsMatchingPair; }
        bool mismatch() { return !IsMatchingPair; }
        Ty getNonBlank() { return Pair.first != Blank ? Pair.first : Pair.second; }
    };

    std::list<Entry> Data;

    AlignedSequence() {}
    AlignedSequence(const AlignedSequence& Other) : Data(Other.Data) {}
    AlignedSequence(AlignedSequence&& Other) noexcept : Data(std::move(Other.Data)) {}
    AlignedSequence& operator=(const AlignedSequence& Other) {
        Data = Other.Data;
        return *this;
    }
    void append(const AlignedSequence& Other) { Data.insert(Data.end(), Other.Data.begin(), Other.Data.end()); }
    void splice(AlignedSequence& Other) { Data.splice(Data.end(), Other.Data); }
    typename std::list<Entry>::iterator begin() { return Data.begin(); }
    typename std::list<Entry>::iterator end() { return Data.end(); }
};

// Scoring parameters.  The overload used decides which fields are meaningful, as in the
// reference; fields an overload does not set are 0 here (the reference leaves them indeterminate).
class ScoringSystem {
    ScoreSystemType Gap = 0, Match = 0, Mismatch = 0, GapOpen = 0, GapExtend = 0;
    bool AllowMismatch = true;

public:
    ScoringSystem(ScoreSystemType gap, ScoreSystemType match)
        : Gap(gap), Match(match), Mismatch(std::numeric_limits<ScoreSystemType>::min()), AllowMismatch(false) {}
    ScoringSystem(ScoreSystemType gap, ScoreSystemType match, ScoreSystemType mismatch, bool allow = true)
        : Gap(gap), Match(match), Mismatch(mismatch), AllowMismatch(allow) {}
    ScoringSystem(ScoreSystemType gapOpen, ScoreSystemType gapExtend, ScoreSystemType match,
                  ScoreSystemType mismatch, bool allow = true)
        : Match(match), Mismatch(mismatch), GapOpen(gapOpen), GapExtend(gapExtend), AllowMismatch(allow) {}

    bool getAllowMismatch() { return AllowMismatch; }
    ScoreSystemType getMismatchPenalty() { return Mismatch; }
    ScoreSystemType getGapPenalty() { return Gap; }
    ScoreSystemType getMatchProfit() { return Match; }
    ScoreSystemType getGapOpenPenalty() { return GapOpen; }
    ScoreSystemType getGapExtendPenalty() { return GapExtend; }

    sa_scoring toC() const {
        sa_scoring s;
        s.gap = Gap;
        s.match = Match;
        s.mismatch = AllowMismatch ? Mismatch : std::numeric_limits<ScoreSystemType>::min();
        s.gap_open = GapOpen;
        s.gap_extend = GapExtend;
        s.allow_mismatch = AllowMismatch ? 1 : 0;
        return s;
    }
};

template <typename ContainerType, typename Ty = typename ContainerType::value_type, Ty Blank = Ty(0),
          typename MatchFnTy = std::function<bool(Ty, Ty)>>
class SequenceAligner {
    ScoringSystem Scoring;
    MatchFnTy Match;

public:
    using EntryType = typename AlignedSequence<Ty, Blank>::Entry;

    SequenceAligner(ScoringSystem Scoring, MatchFnTy Match = nullptr) : Scoring(Scoring), Match(Match) {}
    virtual ~SequenceAligner() {}

    ScoringSystem& getScoring() { return Scoring; }
    bool match(Ty Val1, Ty Val2) { return Match(Val1, Val2); }
    MatchFnTy getMatchOperation() { return Match; }
    Ty getBlank() { return Blank; }

    virtual AlignedSequence<Ty, Blank> getAlignment(ContainerType& Seq0, ContainerType& Seq1) = 0;

    // Pad a local alignment to a global one: Seq1[0, idx1) and Seq2[0, idx2) in front, the tails
    // from endIdx1 / endIdx2 behind, each against a Blank (SequenceAlignment.h:156-189 semantics).
    void forceGlobal(ContainerType& Seq1, ContainerType& Seq2, AlignedSequence<Ty, Blank>& Result, int idx1,
                     int idx2, int endIdx1, int endIdx2) {
        std::list<EntryType> out;
        for (int i = 0; i < idx1; ++i) out.push_back(EntryType(Seq1[i], Blank, false));
        for (int i = 0; i < idx2; ++i) out.push_back(EntryType(Blank, Seq2[i], false));
        out.splice(out.end(), Result.Data);
        for (int i = endIdx1; i < (int)Seq1.size(); ++i) out.push_back(EntryType(Seq1[i], Blank, false));
        for (int i = endIdx2; i < (int)Seq2.size(); ++i) out.push_back(EntryType(Blank, Seq2[i], false));
        Result.Data.clear();
        Result.Data.splice(Result.Data.end(), out);
    }
};

namespace seqalib {
namespace detail {

// Host half of buildResult: replay the op stream (traceback order) with push_front, exactly the
// order in which the reference's buildResult inserts entries.
template <typename Ty, Ty Blank, typename ContainerType>
void build_from_ops(ContainerType& Seq1, ContainerType& Seq2, const sa_result& r, const uint8_t* ops,
                    AlignedSequence<Ty, Blank>& Result) {
    using E = typename AlignedSequence<Ty, Blank>::Entry;
    auto& Data = Result.Data;
    int i = r.end_i, j = r.end_j;
    for (uint32_t k = 0; k < r.nops; ++k) {
        switch (ops[k]) {
            case 'M': Data.push_front(E(Seq1[i - 1], Seq2[j - 1], true)); --i; --j; break;
            case 'S': Data.push_front(E(Seq1[i - 1], Seq2[j - 1], false)); --i; --j; break;
            case 'X':
                Data.push_front(E(Seq1[i - 1], Blank, false));
                Data.push_front(E(Blank, Seq2[j - 1], false));
                --i; --j;
                break;
            case 'U': Data.push_front(E(Seq1[i - 1], Blank, false)); --i; break;
            case 'u': Data.push_front(E(Seq1[i - 1], Blank, false)); break;
            case 'L': Data.push_front(E(Blank, Seq2[j - 1], false)); --j; break;
            case 'l': Data.push_front(E(Blank, Seq2[j - 1], false)); break;
            default: throw std::runtime_error("seqalib: corrupt op stream");
        }
    }
}

// Pairs per chunk when a large batch is aligned in chunks (run below): the GPU call is one
// sa_align_batch_cb over the whole batch, pipelined chunk by chunk on the device, and the lists of a
// chunk are built while the GPU works on the chunks after it.  Off by default since round 6: the
// lists built beside the landing chunks faulted in fresh heap pages in bursts (0.3 K - 59 K minor
// faults per call against a steady 24 K), and those reps ran 2-3x slower; one GPU call followed by
// the lists is 103-106 ms per 10,000 x 4096^2 call, 3 % spread (profiles/dropin_spread_r06.txt).
// $SEQALIB_LIST_CHUNK_PAIRS=N turns chunking on (N pairs per chunk).
constexpr size_t kChunkPairs = SIZE_MAX;

// Shared getAlignment()/getAlignments() body of the four aligners.  Building the std::list of
// every pair (one allocation per Entry, as the reference's buildResult) dominates a large batch
// end to end, so a batch of >= 2 chunks is aligned in one chunked GPU call whose chunk
// callbacks hand each landed range to a builder thread (which fans out over the host threads).
template <int ALGO, typename Aligner, typename ContainerType, typename Ty, Ty Blank>
std::vector<AlignedSequence<Ty, Blank>> run(Aligner& self, const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs,
                                            std::vector<sa_result>& res) {
    auto fn = self.getMatchOperation();
    const bool has_fn = !(fn == nullptr);
    const sa_scoring sc = self.getScoring().toC();
    const size_t P = pairs.size();
    std::vector<AlignedSequence<Ty, Blank>> out(P);
    raw_vector<uint8_t>& ops = host_buffer(kHostOps);
    std::vector<uint64_t> off;
    auto build = [&](size_t p0, size_t p1) {
        for (size_t p = p0; p < p1; ++p) {
            const sa_result& r = res[p];
            // a diverged or timed-out pair has no valid end cell / op stream: never expand it
            // (align() throws for it once the GPU call returns)
            if (r.flags & (SA_FLAG_DIVERGED | SA_FLAG_TIMEOUT)) continue;
            build_from_ops<Ty, Blank>(*pairs[p].first, *pairs[p].second, r, ops.data() + off[p], out[p]);
            const bool local = (ALGO == SA_SW || ALGO == SA_LOCAL_GOTOH) && !(r.flags & SA_FLAG_SIZE_HACK);
            if (local)
                self.forceGlobal(*pairs[p].first, *pairs[p].second, out[p], r.start_i, r.start_j, r.end_i, r.end_j);
        }
    };
    auto build_range = [&](size_t p0, size_t p1) {
        parallel_pairs(p1 - p0, host_threads(p1 - p0), [&](size_t, size_t q0, size_t q1) { build(p0 + q0, p0 + q1); });
    };
    PhaseTimer tm;
    size_t cp = kChunkPairs;
    if (const char* e = std::getenv("SEQALIB_LIST_CHUNK_PAIRS")) cp = std::max<size_t>(1, std::strtoull(e, nullptr, 10));
    const size_t G = cp <= P / 2 ? (P + cp - 1) / cp : 1;
    if (G == 1) {
        align<Ty>(ALGO, sc, fn, has_fn, pairs, res, ops, off);
        build_range(0, P);
        tm.lap("AlignedSequence lists");
        return out;
    }
    // landed ranges, built in arrival order by one builder thread
    struct Queue {
        std::mutex mu;
        std::condition_variable cv;
        std::deque<std::pair<size_t, size_t>> q;
        bool closed = false;
        std::exception_ptr err;
    } lq;
    std::thread builder([&] {
        for (;;) {
            std::pair<size_t, size_t> r;
            {
                std::unique_lock<std::mutex> lk(lq.mu);
                lq.cv.wait(lk, [&] { return lq.closed || !lq.q.empty(); });
                if (lq.q.empty()) return;
                r = lq.q.front();
                lq.q.pop_front();
            }
            try {
                build_range(r.first, r.second);
            } catch (...) {
                std::lock_guard<std::mutex> lk(lq.mu);
                if (!lq.err) lq.err = std::current_exception();
            }
        }
    });
    auto close = [&] {
        {
            std::lock_guard<std::mutex> lk(lq.mu);
            lq.closed = true;
        }
        lq.cv.notify_one();
        builder.join();
    };
    try {
        align<Ty>(ALGO, sc, fn, has_fn, pairs, res, ops, off, (uint32_t)G, [&](size_t p0, size_t p1) {
            {
                std::lock_guard<std::mutex> lk(lq.mu);
                lq.q.emplace_back(p0, p1);
            }
            lq.cv.notify_one();
        });
    } catch (...) {
        close();
        throw;
    }
    tm.lap("GPU call (lists overlapped)");
    close();
    if (lq.err) std::rethrow_exception(lq.err);
    tm.lap("AlignedSequence lists (tail)");
    return out;
}

}  // namespace detail
}  // namespace seqalib

#include "ArrayView.h"
#include "SANeedlemanWunsch.h"
#include "StaticFuncs.h"
#include "SAHirschberg.h"
#include "SAMyersMiller.h"
#include "SASmithWaterman.h"
#include "SAGlobalGotoh.h"
#include "SALocalGotoh.h"
