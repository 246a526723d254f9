// seqalib/SAMyersMiller.h — MyersMillerSA (linear-space affine global alignment) on the MI355X
// engine.  Reference behaviour restated: SAMyersMiller.h:1-421 — forward CC/DD and reverse RR/SS
// sweeps (:167-313), the first maximum of max(CC+RR, DD+SS-g) with its midpoint type (:315-340),
// type-1/type-2 children with their boundary gap opens (:358-395), the N == 0 / M == 0 / M == 1
// base cases (:57-160), top call with (GapOpen, GapOpen) (:412-420), default scoring (-1, 2, -1)
// (:406).  The result is the reference's alignment exactly, computed batched on the GPU
// (seqalib_amd/csrc/sa_myersmiller.hip).  Use a 4/5-argument ScoringSystem: the reference reads
// GapOpen/GapExtend, which the 2/3-argument forms leave unset (0 here).
#pragma once

template <typename ContainerType, typename Ty = typename ContainerType::value_type, Ty Blank = Ty(0),
          typename MatchFnTy = std::function<bool(Ty, Ty)>>
class MyersMillerSA : public SequenceAligner<ContainerType, Ty, Blank, MatchFnTy> {
    using BaseType = SequenceAligner<ContainerType, Ty, Blank, MatchFnTy>;
    ScoreSystemType LastScore = 0;

public:
    static ScoringSystem getDefaultScoring() { return ScoringSystem(-1, 2, -1); }

    MyersMillerSA() : BaseType(getDefaultScoring(), nullptr) {}
    MyersMillerSA(ScoringSystem Scoring, MatchFnTy Match = nullptr) : BaseType(Scoring, Match) {}

    virtual AlignedSequence<Ty, Blank> getAlignment(ContainerType& Seq1, ContainerType& Seq2) {
        std::vector<std::pair<ContainerType*, ContainerType*>> one{{&Seq1, &Seq2}};
        return std::move(getAlignments(one)[0]);
    }

    // Extension: many pairs in one batched GPU pass.
    std::vector<AlignedSequence<Ty, Blank>> getAlignments(const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs) {
        std::vector<sa_result> res;
        auto out = seqalib::detail::run<SA_MYERS_MILLER, MyersMillerSA, ContainerType, Ty, Blank>(*this, pairs, res);
        if (!res.empty()) LastScore = res.back().score;
        return out;
    }

    // Extension: the optimum the top call computed for the last alignment (the reference
    // exposes none).
    ScoreSystemType getScore() const { return LastScore; }
};
