// seqalib/SALocalGotoh.h — LocalGotohSA (affine-gap local alignment, M/Ix/Iy) on the MI355X engine.
// Reference behaviour restated: SALocalGotoh.h:36-526 (borders M = 0, Ix = Iy = -10000 :77-90,
// fill :102-139, 3-state traceback :275-470, forceGlobal :473, and the size hack :484-488 that
// re-aligns (314,288), (60,57), (61,58) with StaticFuncs::useNW — done inside the engine).
#pragma once

template <typename ContainerType, typename Ty = typename ContainerType::value_type, Ty Blank = Ty(0),
          typename MatchFnTy = std::function<bool(Ty, Ty)>>
class LocalGotohSA : public SequenceAligner<ContainerType, Ty, Blank, MatchFnTy> {
    using BaseType = SequenceAligner<ContainerType, Ty, Blank, MatchFnTy>;
    size_t MaxRow = 0;
    size_t MaxCol = 0;
    ScoreSystemType MaxScore = 0;

public:
    // As in the reference (:509) this 3-argument default leaves the affine penalties unset (0 here).
    static ScoringSystem getDefaultScoring() { return ScoringSystem(-1, 2, -1); }

    LocalGotohSA() : BaseType(getDefaultScoring(), nullptr) {}
    LocalGotohSA(ScoringSystem Scoring, MatchFnTy Match = nullptr) : BaseType(Scoring, Match) {}

    virtual AlignedSequence<Ty, Blank> getAlignment(ContainerType& Seq1, ContainerType& Seq2) {
        std::vector<std::pair<ContainerType*, ContainerType*>> one{{&Seq1, &Seq2}};
        return std::move(getAlignments(one)[0]);
    }

    std::vector<AlignedSequence<Ty, Blank>> getAlignments(const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs) {
        std::vector<sa_result> res;
        auto out = seqalib::detail::run<SA_LOCAL_GOTOH, LocalGotohSA, ContainerType, Ty, Blank>(*this, pairs, res);
        if (!res.empty()) {
            MaxRow = res.back().end_i;
            MaxCol = res.back().end_j;
            MaxScore = res.back().score;
        }
        return out;
    }

    ScoreSystemType getScore() const { return MaxScore; }
    std::pair<size_t, size_t> getEndCell() const { return {MaxRow, MaxCol}; }
};
