/*
 * kgx_wave_sort.h -- libstdc++'s std::sort replayed by one wave over at most
 * 64 elements in LDS (the call service's OTU pairs by count, kgx_fused.hip),
 * device only; tests/native/wave_sort_check.cpp times it and checks it
 * against the serial replay (kgx_lstd.h).
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

}  // namespace kgx

#endif
