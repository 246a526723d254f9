// seqalib/SAHirschberg.h — HirschbergSA (linear-space global alignment) on the MI355X engine.
// Reference behaviour restated: SAHirschberg.h:1-185 — NWScore last rows (:11-100), split at the
// last maximum of Fwd[i] + Rev[|Seq2|-i] over i < |Seq2| (:138-149), NeedlemanWunschSA base case
// for length-1 sides (:119-126), default scoring = NeedlemanWunschSA's (:166-167).  The result is
// the reference's alignment exactly (its own recursion and ties), computed batched on the GPU
// (seqalib_amd/csrc/sa_hirschberg.hip).
#pragma once

template <typename ContainerType, typename Ty = typename ContainerType::value_type, Ty Blank = Ty(0),
          typename MatchFnTy = std::function<bool(Ty, Ty)>>
class HirschbergSA : public SequenceAligner<ContainerType, Ty, Blank, MatchFnTy> {
    using BaseType = SequenceAligner<ContainerType, Ty, Blank, MatchFnTy>;
    ScoreSystemType LastScore = 0;

public:
    HirschbergSA() : BaseType(ScoringSystem(-1, 2, -1), nullptr) {}
    HirschbergSA(ScoringSystem Scoring, MatchFnTy Match = nullptr) : BaseType(Scoring, Match) {}

    virtual AlignedSequence<Ty, Blank> getAlignment(ContainerType& Seq1, ContainerType& Seq2) {
        std::vector<std::pair<ContainerType*, ContainerType*>> one{{&Seq1, &Seq2}};
        return std::move(getAlignments(one)[0]);
    }

    std::vector<AlignedSequence<Ty, Blank>> getAlignments(const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs) {
        std::vector<sa_result> res;
        auto out = seqalib::detail::run<SA_HIRSCHBERG, HirschbergSA, ContainerType, Ty, Blank>(*this, pairs, res);
        if (!res.empty()) LastScore = res.back().score;
        return out;
    }

    // Extension: NW score H[m][n] of the last alignment (the reference exposes none).
    ScoreSystemType getScore() const { return LastScore; }
};
