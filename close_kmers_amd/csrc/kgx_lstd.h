/*
 * kgx_lstd.h -- the reference's ordering rules, written once for the device
 * kernels and for the host-side checks (tests/native/lstd_check.cpp):
 *   lstd_sort / lstd_heap_sort  libstdc++ std::sort / partial_sort(first,
 *                               last, last) replayed step by step, so that
 *                               equal elements end where the reference's
 *                               sorts leave them (OTU finalize, kguts.h:214-218)
 *   best_call_decide            find_best_call (kguts.cc:1008-1199) up to the
 *                               function names
 *   otu_finalize                KmerOtuStats otu_map + finalize()
 * Everything is __host__ __device__ and allocation-free: the caller passes
 * a workspace as long as the input.
 */
#ifndef KGX_LSTD_H
#define KGX_LSTD_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kgx.h"

namespace kgx {

/* libstdc++'s std::sort (bits/stl_algo.h, stl_heap.h: introsort with
 * median-of-three pivots, heapsort below the depth limit, final insertion
 * sort, threshold 16) replayed step by step on a[0, n), so elements that
 * compare equal end in the order the reference's std::sort leaves them.
 * The recursion on the right part becomes an explicit stack (the parts are
 * disjoint, so the order they are sorted in does not matter). */
template <class T, class C>
__host__ __device__ void lstd_push_heap(T *a, int64_t hole, int64_t top, T value, C comp)
{
    int64_t parent = (hole - 1) / 2;
    while (hole > top && comp(a[parent], value)) {
        a[hole] = a[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[hole] = value;
}

template <class T, class C>
__host__ __device__ void lstd_adjust_heap(T *a, int64_t hole, int64_t len, T value, C comp)
{
    const int64_t top = hole;
    int64_t second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (comp(a[second], a[second - 1]))
            second--;
        a[hole] = a[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        a[hole] = a[second - 1];
        hole = second - 1;
    }
    lstd_push_heap(a, hole, top, value, comp);
}

template <class T, class C> __host__ __device__ void lstd_make_heap(T *a, int64_t len, C comp)
{
    if (len < 2)
        return;
    for (int64_t parent = (len - 2) / 2;; parent--) {
        lstd_adjust_heap(a, parent, len, a[parent], comp);
        if (parent == 0)
            return;
    }
}

/* __pop_heap(first, first + len, first + result) */
template <class T, class C> __host__ __device__ void lstd_pop_heap(T *a, int64_t len, int64_t result, C comp)
{
    const T value = a[result];
    a[result] = a[0];
    lstd_adjust_heap(a, 0, len, value, comp);
}

/* __partial_sort(first, last, last): heap_select over the whole range, then sort_heap */
template <class T, class C> __host__ __device__ void lstd_heap_sort(T *a, int64_t n, C comp)
{
    lstd_make_heap(a, n, comp);
    for (int64_t last = n; last > 1;) {
        --last;
        lstd_pop_heap(a, last, last, comp);
    }
}

template <class T> __host__ __device__ inline void lstd_swap(T &x, T &y)
{
    const T t = x;
    x = y;
    y = t;
}

template <class T, class C> __host__ __device__ void lstd_unguarded_linear_insert(T *a, int64_t last, C comp)
{
    const T val = a[last];
    int64_t next = last - 1;
    while (comp(val, a[next])) {
        a[last] = a[next];
        last = next;
        --next;
    }
    a[last] = val;
}

template <class T, class C> __host__ __device__ void lstd_insertion_sort(T *a, int64_t n, C comp)
{
    for (int64_t i = 1; i < n; i++) {
        if (comp(a[i], a[0])) {
            const T val = a[i];
            for (int64_t k = i; k > 0; k--)
                a[k] = a[k - 1];
            a[0] = val;
        } else {
            lstd_unguarded_linear_insert(a, i, comp);
        }
    }
}

/* one pending __introsort_loop range */
struct LstdPart {
    int64_t first, last;
    int depth;
};

/* std::sort with the partition stack supplied by the caller (64 entries; the
 * depth limit 2 log2 n bounds the pushes): a device caller passes LDS, so a
 * persistent kernel holds no scratch for it */
template <class T, class C> __host__ __device__ void lstd_sort_on(T *a, int64_t n, C comp, LstdPart *stack)
{
    if (n <= 1)
        return;
    constexpr int64_t THRESH = 16;
    using Part = LstdPart;
    int sp = 0;
    stack[sp++] = Part{0, n, 2 * (63 - __builtin_clzll((unsigned long long)n))};
    while (sp) {
        Part p = stack[--sp];
        while (p.last - p.first > THRESH) {
            if (p.depth == 0) {
                lstd_heap_sort(a + p.first, p.last - p.first, comp);
                break;
            }
            --p.depth;
            /* __unguarded_partition_pivot */
            const int64_t mid = p.first + (p.last - p.first) / 2;
            T *r = a + p.first;
            T *x = a + p.first + 1, *y = a + mid, *z = a + p.last - 1;
            if (comp(*x, *y)) {
                if (comp(*y, *z))
                    lstd_swap(*r, *y);
                else if (comp(*x, *z))
                    lstd_swap(*r, *z);
                else
                    lstd_swap(*r, *x);
            } else if (comp(*x, *z))
                lstd_swap(*r, *x);
            else if (comp(*y, *z))
                lstd_swap(*r, *z);
            else
                lstd_swap(*r, *y);
            int64_t lo = p.first + 1, hi = p.last;
            const T pivot = a[p.first];
            while (true) {
                while (comp(a[lo], pivot))
                    ++lo;
                --hi;
                while (comp(pivot, a[hi]))
                    --hi;
                if (!(lo < hi))
                    break;
                lstd_swap(a[lo], a[hi]);
                ++lo;
            }
            stack[sp++] = Part{lo, p.last, p.depth}; /* __introsort_loop(cut, last) */
            p.last = lo;
        }
    }
    /* __final_insertion_sort */
    if (n > THRESH) {
        lstd_insertion_sort(a, THRESH, comp);
        for (int64_t i = THRESH; i < n; i++)
            lstd_unguarded_linear_insert(a, i, comp);
    } else {
        lstd_insertion_sort(a, n, comp);
    }
}

template <class T, class C> __host__ __device__ void lstd_sort(T *a, int64_t n, C comp)
{
    LstdPart stack[64];
    lstd_sort_on(a, n, comp, stack);
}

/* find_best_call's decision over calls c[0, n); m = workspace of n calls.
 * The calls are rewritten in m (every step writes at or below the index it
 * has read): collapse adjacent same-function calls (kguts.cc:1026-1041),
 * join F1|F2|F1 with a weak interior (kguts.cc:1064-1084), then a stable
 * insertion sort by function index and a run sum give the std::map<int,
 * FuncScore> totals in key order with each float sum in the reference's
 * order (kguts.cc:1108-1125).  The top two come from libstdc++'s
 * partial_sort(begin, begin + 2, end) replayed (__heap_select: make_heap of
 * two, pop_heap for every later element that beats the heap top, then
 * sort_heap), so ties and the element left at index 2 match. */
__host__ __device__ inline kgx_best_call best_call_decide(const kgx_call *c, uint32_t n, kgx_call *m)
{
    kgx_best_call r;
    r.kind = 0;
    r.fi0 = -1;
    r.fi1 = -1;
    r.score = 0.0f;
    r.weighted_score = 0.0f;
    r.score_offset = 0.0f;
    if (n == 0)
        return r;
    /* collapse */
    uint32_t nc = 0;
    for (uint32_t i = 0; i < n;) {
        kgx_call cur = c[i++];
        while (i < n && c[i].function_index == cur.function_index) {
            cur.end = c[i].end;
            cur.count += c[i].count;
            cur.weighted_hits += c[i].weighted_hits;
            i++;
        }
        m[nc++] = cur;
    }
    /* F1 | F2 | F1: interior count < 5, exterior counts >= 10 */
    uint32_t nm = 0;
    for (uint32_t i = 0; i < nc;) {
        kgx_call cur = m[i++];
        while (i + 1 < nc && m[i + 1].function_index == cur.function_index && m[i].count < 5 &&
               cur.count + m[i + 1].count >= 10) {
            cur.end = m[i + 1].end;
            cur.count += m[i + 1].count;
            cur.weighted_hits += m[i + 1].weighted_hits;
            i += 2;
        }
        m[nm++] = cur;
    }
    /* std::map<int, FuncScore>: key order is the signed function index */
    for (uint32_t i = 1; i < nm; i++) {
        const kgx_call v = m[i];
        uint32_t j = i;
        while (j > 0 && (int32_t)m[j - 1].function_index > (int32_t)v.function_index) {
            m[j] = m[j - 1];
            j--;
        }
        m[j] = v;
    }
    uint32_t nr = 0;
    for (uint32_t i = 0; i < nm;) {
        kgx_call cur = m[i++];
        while (i < nm && m[i].function_index == cur.function_index) {
            cur.count += m[i].count;
            cur.weighted_hits += m[i].weighted_hits;
            i++;
        }
        m[nr++] = cur;
    }
    /* partial_sort(vec.begin(), vec.begin() + 2, vec.end(), weighted >) */
    kgx_call v0 = m[0], v1 = v0, v2 = v0;
    if (nr > 1) {
        kgx_call h0, h1; /* the two-element heap; its top h0 is the weakest */
        const kgx_call a0 = m[0], a1 = m[1];
        if (a1.weighted_hits > a0.weighted_hits) {
            h0 = a0;
            h1 = a1;
        } else {
            h0 = a1;
            h1 = a0;
        }
        if (nr > 2)
            v2 = m[2];
        for (uint32_t i = 2; i < nr; i++) {
            const kgx_call x = m[i];
            if (x.weighted_hits > h0.weighted_hits) { /* __pop_heap(first, middle, i) */
                if (i == 2)
                    v2 = h0; /* *i = *first */
                const kgx_call t = h1;
                if (t.weighted_hits > x.weighted_hits) {
                    h0 = x;
                    h1 = t;
                } else {
                    h0 = t;
                    h1 = x;
                }
            }
        }
        v0 = h1; /* __sort_heap of two swaps them */
        v1 = h0;
    }
    r.score_offset = nr == 1 ? (float)v0.count : (float)(v0.count - v1.count);
    if (r.score_offset >= 5.0f) {
        r.kind = 1;
        r.fi0 = (int32_t)v0.function_index;
        r.score = (float)v0.count;
        r.weighted_score = v0.weighted_hits;
    } else {
        r.kind = 3;
        if (nr >= 2) {
            r.fi0 = (int32_t)v0.function_index;
            r.fi1 = (int32_t)v1.function_index;
            if (nr == 2) {
                r.kind = 2;
                r.score = (float)v0.count;
            } else {
                const float pair_offset = (float)(v1.count - v2.count);
                if (pair_offset > 5.0f) {
                    r.kind = 2;
                    r.score = (float)v0.count;
                    r.score_offset = pair_offset;
                    r.weighted_score = v0.weighted_hits;
                }
            }
        }
    }
    return r;
}

/* KmerOtuStats for one sequence: v[0, n) = the OTU of every tallied hit (in
 * any order; sorted in place).  o receives otu_map's pairs in key order, then
 * std::sort'ed by count, larger first (less_second); returns their number. */
__host__ __device__ inline int64_t otu_finalize(int32_t *v, int64_t n, kgx_otu *o)
{
    lstd_heap_sort(v, n, [](int32_t a, int32_t b) { return a < b; });
    int64_t m = 0;
    for (int64_t i = 0; i < n;) {
        int64_t j = i + 1;
        while (j < n && v[j] == v[i])
            j++;
        o[m++] = kgx_otu{v[i], (int32_t)(j - i)};
        i = j;
    }
    lstd_sort(o, m, [](const kgx_otu &lhs, const kgx_otu &rhs) { return rhs.count < lhs.count; });
    return m;
}

}  // namespace kgx

#endif
