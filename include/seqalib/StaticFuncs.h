// seqalib/StaticFuncs.h — NW bridging helpers used by composite aligners (reference
// StaticFuncs.h:12-40): run NeedlemanWunschSA over ArrayView windows and append the result.
#pragma once

template <typename ContainerType, typename Ty = typename ContainerType::value_type, Ty Blank = Ty(0),
          typename MatchFnTy = std::function<bool(Ty, Ty)>>
class StaticFuncs {
public:
    static void useNW(ContainerType& Seq1, ContainerType& Seq2, AlignedSequence<Ty, Blank>& Result,
                      ScoringSystem Scoring, MatchFnTy match) {
        Result.Data.clear();
        bridgeNW(Seq1, Seq2, Result, Scoring, 0, 0, (int)Seq1.size(), (int)Seq2.size(), match);
    }

    static void bridgeNW(ContainerType& Seq1, ContainerType& Seq2, AlignedSequence<Ty, Blank>& Result,
                         ScoringSystem Scoring, int idx1, int idx2, int endIdx1, int endIdx2, MatchFnTy match) {
        NeedlemanWunschSA<ArrayView<ContainerType>, Ty, Blank, MatchFnTy> NW(Scoring, match);
        ArrayView<ContainerType> a(Seq1), b(Seq2);
        a.sliceWindow(idx1, endIdx1);
        b.sliceWindow(idx2, endIdx2);
        AlignedSequence<Ty, Blank> part = NW.getAlignment(a, b);
        Result.Data.insert(Result.Data.end(), part.Data.begin(), part.Data.end());
    }

    // ---- Extension: batched bridging.  The gap fills of composite
    // aligners (SABLAT.h:399, SAMummer.h:49,75,101 call bridgeNW once per gap) become one GPU
    // pass.  Results are appended exactly as calling bridgeNW on each window in order would.
    struct Window {
        int idx1, idx2, endIdx1, endIdx2;
    };
    static void bridgeNWBatch(ContainerType& Seq1, ContainerType& Seq2, AlignedSequence<Ty, Blank>& Result,
                              ScoringSystem Scoring, const std::vector<Window>& windows, MatchFnTy match) {
        std::vector<Job> jobs;
        jobs.reserve(windows.size());
        for (const Window& w : windows) jobs.push_back(Job{&Seq1, &Seq2, w.idx1, w.idx2, w.endIdx1, w.endIdx2, &Result});
        bridgeNWBatch(jobs, Scoring, match);
    }

    // Windows of many sequence pairs, each appended to its own Result, in job order.
    struct Job {
        ContainerType* Seq1;
        ContainerType* Seq2;
        int idx1, idx2, endIdx1, endIdx2;
        AlignedSequence<Ty, Blank>* Result;
    };
    static void bridgeNWBatch(const std::vector<Job>& jobs, ScoringSystem Scoring, MatchFnTy match) {
        using View = ArrayView<ContainerType>;
        std::vector<View> v1, v2;
        v1.reserve(jobs.size());
        v2.reserve(jobs.size());
        for (const Job& j : jobs) {
            View a(*j.Seq1), b(*j.Seq2);
            a.sliceWindow(j.idx1, j.endIdx1);
            b.sliceWindow(j.idx2, j.endIdx2);
            v1.push_back(a);
            v2.push_back(b);
        }
        std::vector<std::pair<View*, View*>> pairs;
        pairs.reserve(jobs.size());
        for (size_t k = 0; k < jobs.size(); ++k) pairs.push_back({&v1[k], &v2[k]});
        NeedlemanWunschSA<View, Ty, Blank, MatchFnTy> NW(Scoring, match);
        std::vector<AlignedSequence<Ty, Blank>> parts = NW.getAlignments(pairs);
        for (size_t k = 0; k < jobs.size(); ++k)
            jobs[k].Result->Data.insert(jobs[k].Result->Data.end(), parts[k].Data.begin(), parts[k].Data.end());
    }
};
