// seqalib/ArrayView.h — non-owning window over a random-access container.  The reference's NW
// call sites (StaticFuncs.h:12-40, SAHirschberg.h:121-125) align ArrayView<Container> slices, so
// the aligners here accept it as ContainerType too.  Interface as in the reference's ArrayView.h.
#pragma once

template <typename ArrayBaseType>
class ArrayView {
public:
    using iterator = typename ArrayBaseType::iterator;
    using reverse_iterator = typename ArrayBaseType::reverse_iterator;
    using value_type = typename ArrayBaseType::value_type;

private:
    iterator First, Last;
    reverse_iterator RFirst, RLast;
    size_t Count;

public:
    ArrayView(ArrayBaseType& Arr)
        : First(Arr.begin()), Last(Arr.end()), RFirst(Arr.rbegin()), RLast(Arr.rend()), Count(Arr.end() - Arr.begin()) {}
    ArrayView(iterator B, iterator E, reverse_iterator RB, reverse_iterator RE)
        : First(B), Last(E), RFirst(RB), RLast(RE), Count(E - B) {}

    iterator begin() { return First; }
    iterator end() { return Last; }
    reverse_iterator rbegin() { return RFirst; }
    reverse_iterator rend() { return RLast; }
    size_t size() { return Count; }

    // Narrow to [StartOffset, EndOffset) of the current window.
    void sliceWindow(size_t StartOffset, size_t EndOffset) {
        iterator b = First + StartOffset, e = First + EndOffset;
        reverse_iterator rb = RFirst + (Count - EndOffset), re = RFirst + (Count - StartOffset);
        First = b; Last = e; RFirst = rb; RLast = re;
        Count = e - b;
    }

    value_type& operator[](size_t Index) { return *(First + Index); }
};
