/*
 * kgx_wave_sort.h -- libstdc++'s std::sort replayed by one wave over
 * elements in LDS (the call service's OTU pairs by count, kgx_fused.hip),
 * device only; tests/native/wave_sort_check.cpp times both variants and
 * checks them against the serial replay (kgx_lstd.h).
 */
#ifndef KGX_WAVE_SORT_H
#define KGX_WAVE_SORT_H

#include "kgx_device.h"
#include "kgx_lstd.h"

namespace kgx {

/* libstdc++'s std::sort (lstd_sort_on, kgx_lstd.h) of n <= 64 elements in
 * LDS, replayed by one wave.  Each __unguarded_partition step is done at
 * once: its left scan stops at the positions whose element is not less than
 * the pivot (L_1 < L_2 < ...), its right scan at those the pivot is not less
 * than (R_1 > R_2 > ...); the t-th swap exchanges L_t and R_t for as long as
 * L_t < R_t, and the cut is min(L_{P+1}, R_P) after P swaps (a scan that
 * runs past its last stop halts at the other's last swapped position).  So a
 * lane that holds L_t swaps iff at least t R-stops lie above it, a lane that
 * holds R_t iff at least t L-stops lie below it, and partners meet through
 * two 64-entry buffers indexed by t.  The median-of-three and the range
 * stack are uniform; a range whose depth budget runs out goes to the serial
 * heap sort (lane 0), as std::sort's does.  The final insertion sort is a
 * stable sort, so each lane places its element by counting.  comp must be a
 * strict weak order.  buf: 192 elements of scratch; stack: 64 ranges. */
template <class T, class C>
__device__ void lstd_sort_wave64(T *a, uint32_t n, C comp, T *buf, LstdPart *stack)
{
    const uint32_t lane = lane_id();
    T *bl = buf, *br = buf + 64, *bs = buf + 128;
    if (n > 16) {
        int sp = 0;
        if (lane == 0)
            stack[0] = LstdPart{0, (int64_t)n, 2 * (31 - (int)__builtin_clz(n))};
        sp = 1;
        wave_lds_sync();
        while (sp) {
            --sp;
            LstdPart p = stack[sp];
            wave_lds_sync();
            int32_t f = (int32_t)p.first, l = (int32_t)p.last, depth = p.depth;
            while (l - f > 16) {
                if (depth == 0) {
                    if (lane == 0)
                        lstd_heap_sort(a + f, l - f, comp);
                    wave_lds_sync();
                    break;
                }
                --depth;
                /* __move_median_to_first(first, first + 1, mid, last - 1) */
                const int32_t mid = f + (l - f) / 2;
                const T x = a[f + 1], y = a[mid], z = a[l - 1];
                int32_t pick;
                if (comp(x, y))
                    pick = comp(y, z) ? mid : (comp(x, z) ? l - 1 : f + 1);
                else
                    pick = comp(x, z) ? f + 1 : (comp(y, z) ? l - 1 : mid);
                const T first_v = a[f], pick_v = a[pick];
                wave_lds_sync();
                if (lane == 0) {
                    a[f] = pick_v;
                    a[pick] = first_v;
                }
                wave_lds_sync();
                const T pivot = a[f];
                const int32_t i = f + 1 + (int32_t)lane;
                const bool in = i < l;
                T v = pivot; /* (a select of the two structs went through scratch) */
                if (in)
                    v = a[i];
                const bool lf = in && !comp(v, pivot), rf = in && !comp(pivot, v);
                const uint64_t LM = __ballot(lf), RM = __ballot(rf);
                const uint32_t l_below = (uint32_t)__popcll(LM & lanes_le(lane) & ~(1ull << lane));
                const uint32_t r_above = (uint32_t)__popcll(RM & ~lanes_le(lane));
                const uint32_t rank_l = l_below + 1, rank_r = r_above + 1;
                const bool swl = lf && rank_l <= r_above, swr = rf && rank_r <= l_below;
                const uint32_t P = (uint32_t)__popcll(__ballot(swl));
                if (swl)
                    bl[rank_l - 1] = v;
                if (swr)
                    br[rank_r - 1] = v;
                wave_lds_sync();
                if (swl)
                    a[i] = br[rank_l - 1];
                else if (swr)
                    a[i] = bl[rank_r - 1];
                const uint64_t LN = __ballot(lf && rank_l == P + 1), RP = __ballot(P > 0 && rf && rank_r == P);
                const int32_t lcut = LN ? f + 1 + (int32_t)lowbit(LN) : INT32_MAX;
                const int32_t rcut = RP ? f + 1 + (int32_t)lowbit(RP) : INT32_MAX;
                const int32_t cut = min(lcut, rcut);
                wave_lds_sync();
                if (lane == 0)
                    stack[sp] = LstdPart{cut, l, depth}; /* __introsort_loop(cut, last) */
                sp++;
                l = cut;
                wave_lds_sync();
            }
        }
    }
    /* __final_insertion_sort: stable, so by counting */
    if (lane < n) {
        const T v = a[lane];
        uint32_t pos = 0;
        for (uint32_t j = 0; j < n; j++) {
            const T w = a[j];
            pos += comp(w, v) || (j < lane && !comp(v, w)) ? 1u : 0u;
        }
        bs[pos] = v;
    }
    wave_lds_sync();
    if (lane < n)
        a[lane] = bs[lane];
    wave_lds_sync();
}

/* lstd_sort_wave64 for kgx_otu pairs by count (less_second: comp(l, r) =
 * r.count < l.count) with the elements in registers: lane i holds a[i] for
 * the whole replay, so a partition step costs one LDS round trip (its swaps
 * meet through bl / br, indexed by rank, as above) instead of the reads and
 * writes of `a` around every move; the median of three, the pivot and the
 * range stack (lane k holds entry k) are lane reads; and the final insertion
 * sort -- stable -- places each element by counting over lane reads within
 * its final range of at most 16.  Same steps, so
 * the same result as lstd_sort_wave64 and the serial replay.  a: the n <= 64
 * pairs in LDS (read at the start, written at the end); bl, br: 64 elements
 * of scratch each. */
__device__ __forceinline__ kgx_otu otu_lane(const kgx_otu &v, uint32_t j)
{
    return kgx_otu{(int32_t)__builtin_amdgcn_readlane(v.otu_index, (int)j),
                   (int32_t)__builtin_amdgcn_readlane(v.count, (int)j)};
}

template <class C>
__device__ __forceinline__ void lstd_sort_wave64_reg(kgx_otu *a, uint32_t n, C comp, kgx_otu *bl, kgx_otu *br)
{
    const uint32_t lane = lane_id();
    const uint64_t le = lanes_le(lane), below = le & ~(1ull << lane);
    kgx_otu v = lane < n ? a[lane] : kgx_otu{0, 0};
    uint64_t marks = 1; /* bit f: [f, next mark) is a range the loop left (<= 16 elements) */
    bool heaped = false;
    if (n > 16) {
        /* the range stack, entry k in lane k */
        int32_t sf = 0, sl = (int32_t)n, sd = 2 * (31 - (int)__builtin_clz(n));
        uint32_t sp = 1;
        while (sp) {
            --sp;
            int32_t f = __builtin_amdgcn_readlane(sf, (int)sp);
            int32_t l = __builtin_amdgcn_readlane(sl, (int)sp);
            int32_t depth = __builtin_amdgcn_readlane(sd, (int)sp);
            while (l - f > 16) {
                if (depth == 0) { /* std::sort's heap sort of the range, serial */
                    if (lane < n)
                        a[lane] = v;
                    wave_lds_sync();
                    if (lane == 0)
                        lstd_heap_sort(a + f, l - f, comp);
                    wave_lds_sync();
                    if (lane < n)
                        v = a[lane];
                    wave_lds_sync();
                    heaped = true;
                    break;
                }
                --depth;
                /* __move_median_to_first(first, first + 1, mid, last - 1) */
                const int32_t mid = f + (l - f) / 2;
                const kgx_otu x = otu_lane(v, (uint32_t)(f + 1)), y = otu_lane(v, (uint32_t)mid),
                              z = otu_lane(v, (uint32_t)(l - 1));
                int32_t pick;
                if (comp(x, y))
                    pick = comp(y, z) ? mid : (comp(x, z) ? l - 1 : f + 1);
                else
                    pick = comp(x, z) ? f + 1 : (comp(y, z) ? l - 1 : mid);
                pick = __builtin_amdgcn_readfirstlane(pick);
                const kgx_otu first_v = otu_lane(v, (uint32_t)f), pivot = otu_lane(v, (uint32_t)pick);
                if ((int32_t)lane == f)
                    v = pivot;
                else if ((int32_t)lane == pick)
                    v = first_v;
                const bool in = (int32_t)lane > f && (int32_t)lane < l;
                const bool lf = in && !comp(v, pivot), rf = in && !comp(pivot, v);
                const uint64_t LM = __ballot(lf), RM = __ballot(rf);
                const uint32_t l_below = (uint32_t)__popcll(LM & below);
                const uint32_t r_above = (uint32_t)__popcll(RM & ~le);
                const uint32_t rank_l = l_below + 1, rank_r = r_above + 1;
                const bool swl = lf && rank_l <= r_above, swr = rf && rank_r <= l_below;
                const uint32_t P = (uint32_t)__popcll(__ballot(swl));
                if (swl)
                    bl[rank_l - 1] = v;
                if (swr)
                    br[rank_r - 1] = v;
                wave_lds_sync();
                if (swl)
                    v = br[rank_l - 1];
                else if (swr)
                    v = bl[rank_r - 1];
                const uint64_t LN = __ballot(lf && rank_l == P + 1), RP = __ballot(P > 0 && rf && rank_r == P);
                const int32_t lcut = LN ? (int32_t)lowbit(LN) : INT32_MAX;
                const int32_t rcut = RP ? (int32_t)lowbit(RP) : INT32_MAX;
                const int32_t cut = min(lcut, rcut);
                wave_lds_sync(); /* bl / br are written again by the next step */
                if (lane == sp) { /* __introsort_loop(cut, last) */
                    sf = cut;
                    sl = l;
                    sd = depth;
                }
                sp++;
                l = cut;
            }
            marks |= 1ull << f; /* [f, l) is final */
        }
    }
    /* __final_insertion_sort: stable, so by counting.  No element moves
     * across the boundary of a range the loop left (every element of an
     * earlier range is not greater than every element of a later one), so
     * each counts only within its own range of at most 16: 16 independent
     * lane reads (a register bitonic sort by (count, position) measured
     * slower, its 21 dependent exchanges 3 us even for 3 pairs).  After a
     * heap sort (a range past 16 elements, rare) every element counts over
     * all n. */
    uint32_t pos = 0;
    if (heaped || n <= 16) { /* (up to 16: n uniform lane reads beat 16 lane exchanges) */
        for (uint32_t j = 0; j < n; j++) {
            const kgx_otu w = otu_lane(v, j);
            pos += comp(w, v) || (j < lane && !comp(v, w)) ? 1u : 0u;
        }
    } else {
        const uint32_t lo = (uint32_t)hibit(marks & le);
        const uint64_t up = marks & ~le;
        const uint32_t hi = up ? min(n, lowbit(up)) : n;
        pos = lo;
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) {
            const uint32_t j = lo + k;
            const kgx_otu w{__shfl(v.otu_index, (int)min(j, 63u)), __shfl(v.count, (int)min(j, 63u))};
            pos += j < hi && (comp(w, v) || (j < lane && !comp(v, w))) ? 1u : 0u;
        }
    }
    if (lane < n)
        a[pos] = v;
    wave_lds_sync();
}

/* The same for n <= 64 S elements, 64 positions per strip (the service
 * takes it past 64 pairs; up to 64 lstd_sort_wave64 is faster: r4h, 5.2 vs
 * 3.0 us at 33-64 pairs, 0.8 vs 0.4 at 2-8).
 *
 * Each __unguarded_partition step is done at once: its left scan stops at the
 * positions whose element is not less than the pivot (L_1 < L_2 < ...), its
 * right scan at those the pivot is not less than (R_1 > R_2 > ...); the t-th
 * swap exchanges L_t and R_t for as long as L_t < R_t, and the cut is
 * min(L_{P+1}, R_P) after P swaps (a scan that runs past its last stop halts
 * at the other's last swapped position).  So an L-stop swaps iff at least t
 * R-stops lie above it, an R-stop of rank t (from the top) iff at least t
 * L-stops lie below it, and partners meet through two buffers indexed by t.
 * The median-of-three and the range stack are uniform; a range whose depth
 * budget runs out goes to the serial heap sort (lane 0), as std::sort's does.
 *
 * __final_insertion_sort is stable and never moves an element across the
 * boundary of a range the loop left behind (every element of an earlier
 * range is not greater than every element of a later one, and an insertion
 * moves an element only past strictly greater ones), so each element is
 * placed by counting within its final range, whose starts the loop marks in
 * seg.  comp must be a strict weak order.  bl, br: n elements of scratch
 * each; seg: n bytes; stack: 64 ranges. */
template <uint32_t S, class T, class C>
__device__ void lstd_sort_wave(T *a, uint32_t n, C comp, T *bl, T *br, uint8_t *seg, LstdPart *stack)
{
    const uint32_t lane = lane_id();
    const uint64_t le = lanes_le(lane), below = le & ~(1ull << lane);
    for (uint32_t i = lane; i < n; i += 64)
        seg[i] = i == 0 ? 1 : 0;
    int sp = 0;
    if (n > 16) {
        if (lane == 0)
            stack[0] = LstdPart{0, (int64_t)n, 2 * (31 - (int)__builtin_clz(n))};
        sp = 1;
    }
    wave_lds_sync();
    while (sp) {
        --sp;
        const LstdPart p = stack[sp];
        wave_lds_sync();
        const int32_t f = (int32_t)p.first;
        int32_t l = (int32_t)p.last, depth = p.depth;
        while (l - f > 16) {
            if (depth == 0) {
                if (lane == 0)
                    lstd_heap_sort(a + f, l - f, comp);
                wave_lds_sync();
                break;
            }
            --depth;
            /* __move_median_to_first(first, first + 1, mid, last - 1) */
            const int32_t mid = f + (l - f) / 2;
            const T x = a[f + 1], y = a[mid], z = a[l - 1];
            int32_t pick;
            if (comp(x, y))
                pick = comp(y, z) ? mid : (comp(x, z) ? l - 1 : f + 1);
            else
                pick = comp(x, z) ? f + 1 : (comp(y, z) ? l - 1 : mid);
            const T first_v = a[f], pick_v = a[pick];
            wave_lds_sync();
            if (lane == 0) {
                a[f] = pick_v;
                a[pick] = first_v;
            }
            wave_lds_sync();
            const T pivot = a[f];
            const uint32_t nst = (uint32_t)(l - f - 1 + 63) / 64; /* strips of the range (uniform) */
            T v[S];
            bool lf[S], rf[S];
            uint64_t LM[S], RM[S];
            uint32_t NR = 0;
#pragma unroll
            for (uint32_t s = 0; s < S; s++) {
                const int32_t i = f + 1 + (int32_t)(64 * s + lane);
                const bool in = s < nst && i < l;
                v[s] = pivot; /* (a select of the two structs went through scratch) */
                if (in)
                    v[s] = a[i];
                lf[s] = in && !comp(v[s], pivot);
                rf[s] = in && !comp(pivot, v[s]);
                LM[s] = __ballot(lf[s]);
                RM[s] = __ballot(rf[s]);
                NR += (uint32_t)__popcll(RM[s]);
            }
            uint32_t rank_l[S], rank_r[S];
            bool swl[S], swr[S];
            uint32_t Lb = 0, Rle = 0, P = 0;
#pragma unroll
            for (uint32_t s = 0; s < S; s++) {
                if (s >= nst) {
                    swl[s] = swr[s] = false;
                    rank_l[s] = rank_r[s] = 0;
                    continue;
                }
                const uint32_t lb = Lb + (uint32_t)__popcll(LM[s] & below);
                const uint32_t r_above = NR - (Rle + (uint32_t)__popcll(RM[s] & le));
                rank_l[s] = lb + 1;
                rank_r[s] = r_above + 1;
                swl[s] = lf[s] && rank_l[s] <= r_above;
                swr[s] = rf[s] && rank_r[s] <= lb;
                P += (uint32_t)__popcll(__ballot(swl[s]));
                Lb += (uint32_t)__popcll(LM[s]);
                Rle += (uint32_t)__popcll(RM[s]);
            }
#pragma unroll
            for (uint32_t s = 0; s < S; s++) {
                if (swl[s])
                    bl[rank_l[s] - 1] = v[s];
                if (swr[s])
                    br[rank_r[s] - 1] = v[s];
            }
            wave_lds_sync();
            int32_t cut = INT32_MAX;
#pragma unroll
            for (uint32_t s = 0; s < S && s < nst; s++) {
                const int32_t i = f + 1 + (int32_t)(64 * s + lane);
                if (swl[s])
                    a[i] = br[rank_l[s] - 1];
                else if (swr[s])
                    a[i] = bl[rank_r[s] - 1];
                const uint64_t LN = __ballot(lf[s] && rank_l[s] == P + 1);
                const uint64_t RP = __ballot(P > 0 && rf[s] && rank_r[s] == P);
                if (LN)
                    cut = min(cut, f + 1 + (int32_t)(64 * s + lowbit(LN)));
                if (RP)
                    cut = min(cut, f + 1 + (int32_t)(64 * s + lowbit(RP)));
            }
            wave_lds_sync();
            if (lane == 0)
                stack[sp] = LstdPart{cut, l, depth}; /* __introsort_loop(cut, last) */
            sp++;
            l = cut;
            wave_lds_sync();
        }
        if (lane == 0)
            seg[f] = 1; /* [f, l) is final */
        wave_lds_sync();
    }
    /* __final_insertion_sort: stable within each final range, so by
     * counting.  Each lane's range bounds from ballots of the range marks:
     * its start the last mark at or below it, its end the next mark above. */
    const uint32_t nst = (n + 63) / 64;
    uint32_t lo[S], hi[S];
    uint32_t carry = 0;
#pragma unroll
    for (uint32_t s = 0; s < S; s++) {
        const uint32_t i = 64 * s + lane;
        const uint64_t SM = s < nst ? __ballot(i < n && seg[i]) : 0ull;
        const int hb = hibit(SM & le);
        lo[s] = hb >= 0 ? 64 * s + (uint32_t)hb : carry;
        if (SM)
            carry = 64 * s + (uint32_t)hibit(SM);
    }
    carry = n;
#pragma unroll
    for (int s = (int)S - 1; s >= 0; s--) {
        const uint32_t i = 64 * (uint32_t)s + lane;
        const uint64_t SM = (uint32_t)s < nst ? __ballot(i < n && seg[i]) : 0ull;
        const uint64_t up = SM & ~le;
        hi[s] = up ? 64 * (uint32_t)s + lowbit(up) : carry;
        if (SM)
            carry = 64 * (uint32_t)s + lowbit(SM);
    }
#pragma unroll
    for (uint32_t s = 0; s < S && s < nst; s++) {
        const uint32_t i = 64 * s + lane;
        if (i < n) {
            const T v = a[i];
            uint32_t pos = lo[s];
            for (uint32_t j = lo[s]; j < hi[s]; j++) {
                const T w = a[j];
                pos += comp(w, v) || (j < i && !comp(v, w)) ? 1u : 0u;
            }
            bl[pos] = v;
        }
    }
    wave_lds_sync();
    for (uint32_t i = lane; i < n; i += 64)
        a[i] = bl[i];
    wave_lds_sync();
}

}  // namespace kgx

#endif
