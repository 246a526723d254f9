// seqalib/SAGlobalGotoh.h — GlobalGotohSA (affine-gap global alignment) on the MI355X engine.
// Reference behaviour restated: SAGlobalGotoh.h:33-459 (borders M = GO + i*GE, Ix = Iy = -10000
// :75-88, fill :98-126, traceback from (m, n) with j == 0 -> up, i == 0 -> left :235-422).
#pragma once

template <typename ContainerType, typename Ty = typename ContainerType::value_type, Ty Blank = Ty(0),
          typename MatchFnTy = std::function<bool(Ty, Ty)>>
class GlobalGotohSA : public SequenceAligner<ContainerType, Ty, Blank, MatchFnTy> {
    using BaseType = SequenceAligner<ContainerType, Ty, Blank, MatchFnTy>;
    ScoreSystemType LastScore = 0;

public:
    static ScoringSystem getDefaultScoring() { return ScoringSystem(-1, 2, -1); }

    GlobalGotohSA() : BaseType(getDefaultScoring(), nullptr) {}
    GlobalGotohSA(ScoringSystem Scoring, MatchFnTy Match = nullptr) : BaseType(Scoring, Match) {}

    virtual AlignedSequence<Ty, Blank> getAlignment(ContainerType& Seq1, ContainerType& Seq2) {
        std::vector<std::pair<ContainerType*, ContainerType*>> one{{&Seq1, &Seq2}};
        return std::move(getAlignments(one)[0]);
    }

    std::vector<AlignedSequence<Ty, Blank>> getAlignments(const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs) {
        std::vector<sa_result> res;
        auto out = seqalib::detail::run<SA_GLOBAL_GOTOH, GlobalGotohSA, ContainerType, Ty, Blank>(*this, pairs, res);
        if (!res.empty()) LastScore = res.back().score;
        return out;
    }

    ScoreSystemType getScore() const { return LastScore; }
};
