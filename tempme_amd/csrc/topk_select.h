// std::nth_element / std::partial_sort selection of libstdc++ restated for (value, index) pairs,
// host and device (see select.hip for why: it reproduces torch.topk's CPU tie order).  Plain
// C++ apart from the TM_HD qualifier, so tests/test_select_host.py compiles it with g++ and checks
// it against torch.topk directly.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define TM_HD __host__ __device__
#else
#define TM_HD
#endif

namespace tmk {

struct PairArr {
    float *v;
    int32_t *x;
    TM_HD inline void swap(int a, int b) {
        const float tv = v[a];
        v[a] = v[b];
        v[b] = tv;
        const int32_t tx = x[a];
        x[a] = x[b];
        x[b] = tx;
    }
};

// comp of TopKImpl.h for largest=false: (!isnan(a) && isnan(b)) || a < b
TM_HD inline bool sel_lt(float a, float b) { return (!__builtin_isnan(a) && __builtin_isnan(b)) || a < b; }

// std::__adjust_heap + std::__push_heap on [first, first+len)
TM_HD inline void adjust_heap(PairArr &A, int first, int hole, int len, float val, int32_t idx) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (sel_lt(A.v[first + second], A.v[first + second - 1])) --second;
        A.v[first + hole] = A.v[first + second];
        A.x[first + hole] = A.x[first + second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        A.v[first + hole] = A.v[first + second - 1];
        A.x[first + hole] = A.x[first + second - 1];
        hole = second - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && sel_lt(A.v[first + parent], val)) {
        A.v[first + hole] = A.v[first + parent];
        A.x[first + hole] = A.x[first + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    A.v[first + hole] = val;
    A.x[first + hole] = idx;
}

// std::__heap_select(first, middle, last): a max-heap of the middle-first smallest
TM_HD inline void heap_select(PairArr &A, int first, int middle, int last) {
    const int len = middle - first;
    if (len >= 2) {  // std::__make_heap
        for (int parent = (len - 2) / 2;; --parent) {
            adjust_heap(A, first, parent, len, A.v[first + parent], A.x[first + parent]);
            if (parent == 0) break;
        }
    }
    for (int i = middle; i < last; ++i) {
        if (sel_lt(A.v[i], A.v[first])) {  // std::__pop_heap(first, middle, i)
            const float val = A.v[i];
            const int32_t idx = A.x[i];
            A.v[i] = A.v[first];
            A.x[i] = A.x[first];
            adjust_heap(A, first, 0, len, val, idx);
        }
    }
}

// std::__insertion_sort(first, last)
TM_HD inline void insertion_sort(PairArr &A, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i < last; ++i) {
        const float val = A.v[i];
        const int32_t idx = A.x[i];
        int j = i;
        if (sel_lt(val, A.v[first])) {
            for (; j > first; --j) {
                A.v[j] = A.v[j - 1];
                A.x[j] = A.x[j - 1];
            }
        } else {
            while (sel_lt(val, A.v[j - 1])) {
                A.v[j] = A.v[j - 1];
                A.x[j] = A.x[j - 1];
                --j;
            }
        }
        A.v[j] = val;
        A.x[j] = idx;
    }
}

// std::nth_element(first, nth, last) == std::__introselect(first, nth, last, 2*__lg(last-first))
TM_HD inline void nth_element(PairArr &A, int first, int nth, int last) {
    if (first == last || nth == last) return;
    int depth = 2 * (31 - __builtin_clz((unsigned)(last - first)));
    while (last - first > 3) {
        if (depth == 0) {
            heap_select(A, first, nth + 1, last);
            A.swap(first, nth);
            return;
        }
        --depth;
        // std::__unguarded_partition_pivot: median of (first+1, mid, last-1) moved to first
        const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
        int med;
        if (sel_lt(A.v[a], A.v[b])) {
            if (sel_lt(A.v[b], A.v[c])) med = b;
            else if (sel_lt(A.v[a], A.v[c])) med = c;
            else med = a;
        } else if (sel_lt(A.v[a], A.v[c])) med = a;
        else if (sel_lt(A.v[b], A.v[c])) med = c;
        else med = b;
        A.swap(first, med);
        // std::__unguarded_partition(first + 1, last, first)
        int lo = first + 1, hi = last;
        const float pv = A.v[first];
        for (;;) {
            while (sel_lt(A.v[lo], pv)) ++lo;
            --hi;
            while (sel_lt(pv, A.v[hi])) --hi;
            if (!(lo < hi)) break;
            A.swap(lo, hi);
            ++lo;
        }
        if (lo <= nth) first = lo;
        else last = lo;
    }
    insertion_sort(A, first, last);
}

// the first k of n pairs after torch.topk(largest=False)'s selection step (ATen TopKImpl.h)
TM_HD inline void topk_smallest_select(PairArr &A, int n, int k) {
    if (k <= 0) return;
    if (k > n) k = n;
    if ((int64_t)k * 64 <= n) heap_select(A, 0, k, n);  // std::partial_sort's selection step
    else nth_element(A, 0, k - 1, n);
}

}  // namespace tmk
