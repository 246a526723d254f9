// seqalib/SANeedlemanWunsch.h — NeedlemanWunschSA (linear-gap global alignment) on the MI355X engine.
// Reference behaviour restated: SANeedlemanWunsch.h:22-264 (borders i*Gap / j*Gap :59-62, fill
// :69-86, traceback from (m, n) diag > up > left :155-231, default scoring (-1,2,-1) :244-247).
#pragma once

template <typename ContainerType, typename Ty = typename ContainerType::value_type, Ty Blank = Ty(0),
          typename MatchFnTy = std::function<bool(Ty, Ty)>>
class NeedlemanWunschSA : public SequenceAligner<ContainerType, Ty, Blank, MatchFnTy> {
    using BaseType = SequenceAligner<ContainerType, Ty, Blank, MatchFnTy>;
    ScoreSystemType LastScore = 0;

public:
    static ScoringSystem getDefaultScoring() { return ScoringSystem(-1, 2, -1); }

    NeedlemanWunschSA() : BaseType(getDefaultScoring(), nullptr) {}
    NeedlemanWunschSA(ScoringSystem Scoring, MatchFnTy Match = nullptr) : BaseType(Scoring, Match) {}

    virtual AlignedSequence<Ty, Blank> getAlignment(ContainerType& Seq1, ContainerType& Seq2) {
        std::vector<std::pair<ContainerType*, ContainerType*>> one{{&Seq1, &Seq2}};
        return std::move(getAlignments(one)[0]);
    }

    std::vector<AlignedSequence<Ty, Blank>> getAlignments(const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs) {
        std::vector<sa_result> res;
        auto out = seqalib::detail::run<SA_NW, NeedlemanWunschSA, ContainerType, Ty, Blank>(*this, pairs, res);
        if (!res.empty()) LastScore = res.back().score;
        return out;
    }

    // Extension: H[m][n] of the last alignment.
    ScoreSystemType getScore() const { return LastScore; }
};
