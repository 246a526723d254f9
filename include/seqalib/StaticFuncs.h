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
};
