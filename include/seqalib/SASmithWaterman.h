// seqalib/SASmithWaterman.h — SmithWatermanSA (linear-gap local alignment) on the MI355X engine.
// Reference behaviour restated: SASmithWaterman.h:20-366 (fill :89-117, max cell = last
// row-major maximum :110, traceback :220-339, forceGlobal :337, default scoring (-1,1,-1) :352).
#pragma once

template <typename ContainerType, typename Ty = typename ContainerType::value_type, Ty Blank = Ty(0),
          typename MatchFnTy = std::function<bool(Ty, Ty)>>
class SmithWatermanSA : public SequenceAligner<ContainerType, Ty, Blank, MatchFnTy> {
    using BaseType = SequenceAligner<ContainerType, Ty, Blank, MatchFnTy>;
    // The reference keeps the max cell in members that survive between calls (:14-16); an empty
    // input re-uses them in forceGlobal.  Kept here with the same lifetime.
    size_t MaxRow = 0;
    size_t MaxCol = 0;
    ScoreSystemType MaxScore = std::numeric_limits<ScoreSystemType>::min();

    AlignedSequence<Ty, Blank> emptyResult(ContainerType& Seq1, ContainerType& Seq2) {
        AlignedSequence<Ty, Blank> r;
        MaxScore = std::numeric_limits<ScoreSystemType>::min();
        BaseType::forceGlobal(Seq1, Seq2, r, 0, 0, (int)MaxRow, (int)MaxCol);
        return r;
    }

public:
    static ScoringSystem getDefaultScoring() { return ScoringSystem(-1, 1, -1); }

    SmithWatermanSA() : BaseType(getDefaultScoring(), nullptr) {}
    SmithWatermanSA(ScoringSystem Scoring, MatchFnTy Match = nullptr) : BaseType(Scoring, Match) {}

    virtual AlignedSequence<Ty, Blank> getAlignment(ContainerType& Seq1, ContainerType& Seq2) {
        std::vector<std::pair<ContainerType*, ContainerType*>> one{{&Seq1, &Seq2}};
        return std::move(getAlignments(one)[0]);
    }

    // Batch extension: one GPU pass over many pairs (configs 3/5 of BASELINE.json).
    std::vector<AlignedSequence<Ty, Blank>> getAlignments(const std::vector<std::pair<ContainerType*, ContainerType*>>& pairs) {
        std::vector<std::pair<ContainerType*, ContainerType*>> work;
        for (auto& p : pairs)
            if (p.first->size() && p.second->size()) work.push_back(p);
        std::vector<sa_result> res;
        std::vector<AlignedSequence<Ty, Blank>> done;
        if (!work.empty()) done = seqalib::detail::run<SA_SW, SmithWatermanSA, ContainerType, Ty, Blank>(*this, work, res);
        std::vector<AlignedSequence<Ty, Blank>> out;
        out.reserve(pairs.size());
        size_t k = 0;
        for (auto& p : pairs) {
            if (p.first->size() && p.second->size()) {
                MaxRow = res[k].end_i;
                MaxCol = res[k].end_j;
                MaxScore = res[k].score;
                out.push_back(std::move(done[k++]));
            } else {
                out.push_back(emptyResult(*p.first, *p.second));
            }
        }
        return out;
    }

    // Extensions (the reference keeps these private): score and end cell of the last alignment.
    ScoreSystemType getScore() const { return MaxScore; }
    std::pair<size_t, size_t> getEndCell() const { return {MaxRow, MaxCol}; }
};
