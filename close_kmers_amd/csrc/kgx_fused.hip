/*
 * kgx_fused.hip -- process_aa_seq for a few sequences in ONE launch.
 *
 * The reference's handlers call KmerGuts::process_aa_seq once per sequence
 * (lookup_request.cc:153-172, kguts.cc:888-908); the facade coalesces the
 * concurrent calls of a worker pool into small batches.  For such a batch
 * the general path's four launches (upload, probe, score, gather) and their
 * hand-offs through HBM are the whole cost, so here one workgroup takes one
 * sequence end to end:
 *
 *   1. its residues, read straight from the caller's pinned staging over
 *      PCIe, mapped to codes in LDS (to_amino_acid_off, kguts.cc:273-339);
 *   2. every window encoded from LDS (encoded_kmer, kguts.cc:438-455; a
 *      window with a code-20 residue is skipped, advance_past_ambig
 *      kguts.cc:682-732) and probed in the PACKED16 table, all of a thread's
 *      windows in flight at once (lookup_hash_entry, kguts.cc:585-602);
 *   3. the hits compacted in window order into LDS (ballots + a wave scan);
 *   4. the kgx_hit records stored to the caller's mapped result region while
 *      wave 0 scores the hits 64 at a time (gather_hits / process_set_of_hits,
 *      kguts.cc:734-877, the wave-parallel formulation of score_wave_kernel
 *      for one sequence: run breaks, current_fI as a segmented last-mark scan,
 *      pair switches; f32 sums serial in hit order);
 *   5. counts, then a system-scope fence and the sequence's completion token.
 *
 * Preconditions (checked by the host): PACKED16 image, order_constraint 0,
 * min_hits >= 1, want within HITS | CALLS, every sequence at most
 * FUSED_MAX_WINDOWS windows.
 */
#include <type_traits>

#include "kgx_device.h"
#include "kgx_internal.h"
#include "kgx_lstd.h"
#include "kgx_wave_sort.h"

namespace kgx {

struct FusedArgs {
    const uint8_t *res;    /* mapped: the batch's residues (NUL-cut), concatenated */
    const uint64_t *off;   /* mapped: n + 1 offsets into res */
    const uint64_t *wbase; /* mapped: n + 1 exclusive scan of the window counts */
    uint32_t n;
    uint32_t want;
    const uint4 *table; /* PACKED16 records in HBM */
    uint64_t num_sigs, magic; /* buckets; magic of num_sigs >> hs */
    uint32_t hs;              /* home = (key mod (num_sigs >> hs)) << hs (kgx_image_set_line_index) */
    kgx_params prm;
    kgx_hit *hits;    /* mapped: sequence s's hits from hits[wbase[s]] */
    kgx_call *calls;  /* mapped: sequence s's calls from calls[wbase[s]] */
    kgx_otu *otus;    /* mapped, want OTU (the call service only): s's OTU pairs from otus[wbase[s]] */
    uint32_t *counts; /* mapped: hit count of s at [s], call count at [n + s], OTU pairs at [2n + s] */
    uint32_t *done;   /* mapped: done[s] = token once s's results are visible */
    uint32_t token;
    uint64_t *dbg; /* mapped, or NULL: wall-clock stamps of workgroup 0's phases */
};

/* a batch small enough to travel in the kernel arguments themselves
 * (offsets, window bases, residues): the kernel then reads nothing over PCIe
 * before it probes */
struct FusedInline {
    uint32_t off[FUSED_INLINE_SEQ + 1];
    uint32_t wb[FUSED_INLINE_SEQ + 1];
    uint8_t res[FUSED_INLINE_RES];
};
struct FusedMapped { /* the mapped arrays instead (FusedArgs.res / off / wbase) */
};

/* FJ = windows per thread at most (the batch's longest sequence has at most
 * 256 FJ windows): 2 for proteins up to 520 aa, 8 up to FUSED_MAX_WINDOWS */
template <uint32_t FJ, class IN, bool QUAD = false>
__device__ __forceinline__ void fused_small_body(const FusedArgs &a, const IN &k, uint32_t s);

template <uint32_t FJ>
__global__ __launch_bounds__(256) void fused_small_kernel(FusedArgs a)
{
    fused_small_body<FJ>(a, FusedMapped{}, blockIdx.x);
}

template <uint32_t FJ>
__global__ __launch_bounds__(256) void fused_small_inline_kernel(FusedArgs a, FusedInline k)
{
    fused_small_body<FJ>(a, k, blockIdx.x);
}

/* one sequence in a service slot (svc_kernel): residues in the slot's mapped
 * buffer, offsets {0, len}, window bases {0, W} */
struct FusedSlot {
    const uint8_t *res;
    uint32_t len;
    uint8_t *codes; /* LDS: the residues' codes, decoded by the polling wave */
};

template <class IN> struct FusedInput;
template <> struct FusedInput<FusedMapped> {
    __device__ static uint64_t off(const FusedArgs &a, const FusedMapped &, uint32_t i) { return a.off[i]; }
    __device__ static uint64_t wb(const FusedArgs &a, const FusedMapped &, uint32_t i) { return a.wbase[i]; }
    __device__ static uint8_t res(const FusedArgs &a, const FusedMapped &, uint64_t i) { return a.res[i]; }
};
template <> struct FusedInput<FusedInline> {
    __device__ static uint64_t off(const FusedArgs &, const FusedInline &k, uint32_t i) { return k.off[i]; }
    __device__ static uint64_t wb(const FusedArgs &, const FusedInline &k, uint32_t i) { return k.wb[i]; }
    __device__ static uint8_t res(const FusedArgs &, const FusedInline &k, uint64_t i) { return k.res[i]; }
};
template <> struct FusedInput<FusedSlot> {
    __device__ static uint64_t off(const FusedArgs &, const FusedSlot &k, uint32_t i) { return i ? k.len : 0u; }
    __device__ static uint64_t wb(const FusedArgs &, const FusedSlot &, uint32_t) { return 0; }
    __device__ static uint8_t res(const FusedArgs &, const FusedSlot &k, uint64_t i) { return k.res[i]; }
};

template <uint32_t FJ, class IN, bool QUAD>
__device__ __forceinline__ void fused_small_body(const FusedArgs &a, const IN &k, const uint32_t s)
{
    typedef FusedInput<IN> In;
    const bool dbg = a.dbg && s == 0 && threadIdx.x == 0;
    /* the stamps go to LDS and out to the mapped a.dbg only before the done
     * token: a store to host memory in the middle of a phase made the next
     * wait on stores (any s_waitcnt vmcnt) wait for PCIe, inflating the
     * phase it sat in (the OTU by-count sort: 4.0 us in the service against
     * 2.3 us for the same lists alone, tests/native/wave_sort_check.cpp) */
    __shared__ uint64_t dstamp[18];
    if (dbg)
        dstamp[0] = wall_clock64();
    __shared__ uint8_t code_tab[256];
    __shared__ uint8_t codes_own[256 * FJ + 8];
    constexpr bool SLOT = std::is_same<IN, FusedSlot>::value;
    uint8_t *codes = codes_own;
    if constexpr (SLOT)
        codes = k.codes;
    __shared__ uint4 hrec[256 * FJ];
    __shared__ uint32_t hpos[256 * FJ];
    __shared__ uint32_t wave_cnt[4];
    __shared__ uint8_t oflag[256 * FJ]; /* want OTU: hit i is a counted member of an emitted call */
    __shared__ uint32_t n_otu;
    typedef HitFields<true> HF;

    const uint32_t t = threadIdx.x, lane = lane_id(), wave = t >> 6;
    const uint64_t r0 = In::off(a, k, s), len = In::off(a, k, s + 1) - r0;
    const uint64_t wb = In::wb(a, k, s);
    const uint32_t W = (uint32_t)windows_of(len);
    /* 1. residues -> codes (the service's polling wave has decoded them) */
    if constexpr (!SLOT) {
        code_tab[t] = (uint8_t)residue_code(t);
        __syncthreads();
        /* each wave reads 64 consecutive bytes per round */
        for (uint32_t i = t; i < W + 8 && i < len; i += 256)
            codes[i] = code_tab[In::res(a, k, r0 + i)];
        __syncthreads();
    }
    if (dbg)
        dstamp[1] = wall_clock64();

    uint32_t nh = 0;
    const uint32_t J = (W + 255) / 256; /* 256-window slices */
    {
        /* 2. encode + probe: thread t owns windows t + 256 j, probed RB
         * slices at a time (the LDS holds FJ slices; the registers hold RB,
         * so a long protein costs more probe rounds, not spilled registers:
         * with all FJ = 8 slices in registers the long-protein body spilled
         * 150+ SGPRs, and the service kernel that inlines it spilled in its
         * short-protein path too) */
        constexpr uint32_t RB = FJ < 2 ? FJ : 2;
        for (uint32_t jb = 0; jb < J; jb += RB) {
            uint64_t key[RB], slot[RB];
            bool pend[RB], hit[RB];
            uint4 rec[RB];
            /* window w's key (encoded_kmer) and home; pend: no code 20 in it */
            auto encode = [&](uint32_t w, uint64_t &k, uint64_t &sl, bool &pd) {
                const uint8_t *c = codes + w;
                const uint32_t cmax = max(max(max(c[0], c[1]), max(c[2], c[3])), max(max(c[4], c[5]), max(c[6], c[7])));
                const uint32_t ka = ((c[0] * 20u + c[1]) * 20u + c[2]) * 20u + c[3];
                const uint32_t kb = ((c[4] * 20u + c[5]) * 20u + c[6]) * 20u + c[7];
                k = (uint64_t)ka * 160000u + kb;
                pd = cmax < 20u;
                sl = pd ? mod_by(k, a.num_sigs >> a.hs, a.magic) << a.hs : 0;
            };
#pragma unroll
            for (uint32_t j = 0; j < RB; j++) {
                hit[j] = false;
                pend[j] = false;
                rec[j] = make_uint4(0, 0, 0, 0);
                key[j] = 0;
                slot[j] = 0;
                if constexpr (QUAD) {
                    /* lane sub of quad g takes the pass's windows g + 64 i
                     * with i = sub + 4 j (the quads' own windows, below) */
                    const uint32_t wi = (t >> 2) + 64 * ((t & 3u) + 4 * j);
                    if (wi < min(256u * RB, W - 256u * jb))
                        encode(256 * jb + wi, key[j], slot[j], pend[j]);
                } else {
                    const uint32_t w = t + 256 * (jb + j);
                    if (jb + j < J && w < W)
                        encode(w, key[j], slot[j], pend[j]);
                }
            }
            /* linear probe by 64-B lines: a round reads the rest of the line
             * holding each pending window's next bucket (the table is 256-B
             * aligned, 4 records per line), all of a thread's windows in
             * flight at once, and examines those buckets in probe order -- a
             * chain costs one round per line it touches instead of one per
             * bucket (reading the next line too, speculatively, measured
             * slower: 6.8 vs 4.6 us for one protein).  Bounded by num_sigs
             * buckets where the reference would spin forever. */
            constexpr uint32_t R = 4; /* records per round: one line */
            const uint64_t NS = a.num_sigs;
            uint32_t rounds = 0;
            if (dbg && jb == 0)
                dstamp[12] = wall_clock64(); /* keys and homes computed */
            if constexpr (QUAD) {
                /* the loads by quads (the call service): the 4 lanes of quad g
                 * read window g + 64 i's line, 16 B each, one instruction for
                 * 16 windows; lane i & 3 of the quad holds that window's key
                 * and next bucket (its register j = i >> 2) and a DPP quad
                 * broadcast hands them to the other three.  A round's lines
                 * cost one address translation each where a thread's four 16-B
                 * loads of its own line cost four, and over a table of many GB
                 * those translations bound the round (tools/tlb_probe.cpp, 293
                 * lines over 114 GB: 2.3 vs 3.2 us) */
                __shared__ uint4 qrec[256 * RB];
                __shared__ uint8_t qhit[256 * RB];
                const uint32_t g = t >> 2, sub = t & 3u, qsh = 4u * (lane >> 2);
#pragma unroll
                for (uint32_t j = 0; j < RB; j++)
                    qhit[g + 64 * (sub + 4 * j)] = 0;
                /* every bucket examined once a window has gone round the
                 * table (its first line may be partial): a miss where the
                 * reference would spin forever */
                const uint64_t turn = (NS + 3) / 4 + 1;
                for (;;) {
                    uint64_t kq[4 * RB], sl[4 * RB];
                    bool pd[4 * RB];
                    uint4 pv[4 * RB];
#pragma unroll
                    for (uint32_t i = 0; i < 4 * RB; i++) {
                        const uint32_t j = i >> 2;
                        kq[i] = quad_bcast64(key[j], i & 3);
                        sl[i] = quad_bcast64(slot[j], i & 3);
                        pd[i] = quad_bcast32(pend[j] ? 1u : 0u, i & 3) != 0;
                        const uint64_t base = sl[i] & ~3ull;
                        if (pd[i] && sub >= (uint32_t)(sl[i] & 3) && base + sub < NS)
                            pv[i] = a.table[base + sub];
                    }
                    rounds++;
                    if (dbg && rounds == 1 && jb == 0) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        dstamp[13] = wall_clock64(); /* thread 0's own loads back */
                    }
                    const bool turned = rounds >= turn;
                    bool more = false;
#pragma unroll
                    for (uint32_t i = 0; i < 4 * RB; i++) {
                        const uint32_t wi = g + 64 * i;
                        const uint64_t base = sl[i] & ~3ull;
                        const bool in = pd[i] && sub >= (uint32_t)(sl[i] & 3) && base + sub < NS;
                        const uint64_t kv = ((uint64_t)pv[i].y << 32 | pv[i].x) & PACK_KEY_MASK;
                        const bool m = in && kv == kq[i];
                        const bool stop = in && (m || kv > MAX_ENCODED);
                        /* the quad's first bucket in probe order that is the
                         * key or a stop decides the window */
                        const uint32_t sq = (uint32_t)(__ballot(stop) >> qsh) & 0xFu;
                        const uint32_t mq = (uint32_t)(__ballot(m) >> qsh) & 0xFu;
                        const uint32_t first = sq ? (uint32_t)__builtin_ctz(sq) : 4u;
                        if (sq && ((mq >> first) & 1u) && sub == first) {
                            qrec[wi] = pv[i];
                            qhit[wi] = 1;
                        }
                        const bool live = pd[i] && !sq && !turned;
                        if (sub == (i & 3)) { /* the window's own lane moves it on */
                            const uint64_t next = base + R >= NS ? 0 : base + R;
                            slot[i >> 2] = live ? next : slot[i >> 2];
                            pend[i >> 2] = live;
                        }
                        more = more || live;
                    }
                    const bool again = __syncthreads_or(more);
                    if (dbg && rounds == 1 && jb == 0)
                        dstamp[11] = wall_clock64(); /* the first round examined */
                    if (!again)
                        break;
                }
#pragma unroll
                for (uint32_t j = 0; j < RB; j++) {
                    const uint32_t wi = t + 256 * j;
                    hit[j] = qhit[wi] != 0;
                    rec[j] = hit[j] ? qrec[wi] : make_uint4(0, 0, 0, 0);
                }
            } else {
                uint64_t examined[RB];
#pragma unroll
                for (uint32_t j = 0; j < RB; j++)
                    examined[j] = 0;
                for (;;) {
                    uint4 pv[RB][R];
    #pragma unroll
                    for (uint32_t j = 0; j < RB; j++) {
                        const uint64_t base = slot[j] & ~3ull;
    #pragma unroll
                        for (uint32_t q = 0; q < R; q++)
                            if (pend[j] && q >= (uint32_t)(slot[j] & 3) && base + q < NS)
                                pv[j][q] = a.table[base + q];
                    }
                    bool more = false;
    #pragma unroll
                    for (uint32_t j = 0; j < RB; j++) {
                        const uint64_t base = slot[j] & ~3ull;
                        bool live = pend[j]; /* still searching within this line */
    #pragma unroll
                        for (uint32_t q = 0; q < R; q++) {
                            const bool in = live && q >= (uint32_t)(slot[j] & 3) && base + q < NS;
                            const uint64_t kv = ((uint64_t)pv[j][q].y << 32 | pv[j][q].x) & PACK_KEY_MASK;
                            const bool m = in && kv == key[j];
                            const bool stop = in && (m || kv > MAX_ENCODED || examined[j] + 1 >= NS);
                            rec[j].x = m ? pv[j][q].x : rec[j].x;
                            rec[j].y = m ? pv[j][q].y : rec[j].y;
                            rec[j].z = m ? pv[j][q].z : rec[j].z;
                            rec[j].w = m ? pv[j][q].w : rec[j].w;
                            hit[j] = hit[j] || m;
                            examined[j] += in ? 1u : 0u;
                            live = live && !stop;
                        }
                        /* not resolved in this line: on at the next one (wrapping
                         * at the table's end, where the round's loads stopped) */
                        const uint64_t next = base + R >= NS ? 0 : base + R;
                        pend[j] = live;
                        slot[j] = live ? next : slot[j];
                        more = more || live;
                    }
                    if (dbg && rounds == 0 && jb == 0) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        dstamp[13] = wall_clock64(); /* thread 0's own loads back */
                    }
                    const bool again = __syncthreads_or(more);
                    if (dbg && rounds++ == 0 && jb == 0)
                        dstamp[11] = wall_clock64(); /* the first round examined */
                    if (!again)
                        break;
                }
            }
            if (dbg) {
                dstamp[10] = (jb == 0 ? 0 : dstamp[10]) + rounds;
                if (jb + RB >= J)
                    dstamp[2] = wall_clock64();
            }

            /* 3. ordered compaction into LDS: slice j = windows [256 j, 256 j
             * + 256), every slice of the pass behind one barrier */
            __shared__ uint32_t slice_cnt[RB][4];
            uint64_t m[RB];
#pragma unroll
            for (uint32_t q = 0; q < RB; q++) {
                m[q] = __ballot(hit[q]); /* (no hit past the last slice) */
                if (lane == 0)
                    slice_cnt[q][wave] = (uint32_t)__popcll(m[q]);
            }
            __syncthreads();
#pragma unroll
            for (uint32_t q = 0; q < RB; q++) {
                uint32_t before = 0, total = 0;
                for (uint32_t v = 0; v < 4; v++) {
                    before += v < wave ? slice_cnt[q][v] : 0u;
                    total += slice_cnt[q][v];
                }
                if (hit[q]) {
                    const uint32_t at = nh + before + lanes_below(m[q]);
                    hrec[at] = rec[q];
                    hpos[at] = t + 256 * (jb + q);
                }
                nh += total;
            }
            __syncthreads();
        }
    }
    if (dbg)
        dstamp[3] = wall_clock64();

    const bool want_otu = (a.want & KGX_WANT_OTU) != 0;
    if (want_otu) {
        for (uint32_t i = t; i < nh; i += 256)
            oflag[i] = 0;
        __syncthreads();
    }
    /* 4a. kgx_hit records into the caller's mapped region (kguts.h:228-233) */
    if (a.want & KGX_WANT_HITS)
        for (uint32_t i = t; i < nh; i += 256) {
            const uint4 h = hrec[i];
            const uint64_t k = HF::key(h, h);
            uint4 *dst = reinterpret_cast<uint4 *>(a.hits + wb + i);
            dst[0] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), HF::otu(h, h), HF::avg(h));
            dst[1] = make_uint4(HF::fi(h), HF::wt(h), hpos[i], s);
        }

    if (dbg)
        dstamp[6] = wall_clock64(); /* thread 0's record stores issued */
    /* 4b. the run scorer, wave 0, 64 hits per step (score_wave_kernel's
     * chunk rules for a single sequence) */
    uint32_t ncalls_out = 0;
    const bool want_calls = (a.want & KGX_WANT_CALLS) != 0;
    if ((want_calls || want_otu) && wave == 0 && nh) {
        const kgx_params prm = a.prm;
        const uint32_t gap = (uint32_t)prm.max_gap;
        const float min_wh = (float)prm.min_weighted_hits;
        kgx_call *calls = a.calls + wb;
        bool o_valid = false;
        uint32_t o_cur = 0, o_cnt = 0, o_first = 0, o_last = 0, o_ncalls = 0;
        /* the open sub-run's first and last counted hit (indices), for its OTU flags */
        uint32_t o_first_idx = 0, o_last_idx = 0;
        float o_wsum = 0.0f;
        uint32_t p_pos = 0, p_fi = 0;
        float p_wt = 0.0f;
        /* flush of the open sub-run (kguts.cc:757-770) */
        auto close_open = [&]() {
            if ((int)o_cnt >= prm.min_hits && o_wsum >= min_wh) {
                /* OTU tally (kguts.cc:757-770): the run's hits of its function, first to last */
                if (want_otu)
                    for (uint32_t i = o_first_idx + lane; i <= o_last_idx; i += 64)
                        if (HF::fi(hrec[i]) == o_cur)
                            oflag[i] = 1;
                if (want_calls && lane == 0) {
                    kgx_call cl;
                    cl.start = o_first;
                    cl.end = o_last + (KMER - 1);
                    cl.count = (int32_t)o_cnt;
                    cl.function_index = o_cur;
                    cl.weighted_hits = o_wsum;
                    calls[o_ncalls] = cl;
                }
                o_ncalls++;
            }
        };
        for (uint32_t h0 = 0; h0 < nh; h0 += 64) {
            const uint32_t n = min(64u, nh - h0);
            const uint32_t k = lane;
            const bool act = k < n;
            const uint64_t ACT = n >= 64 ? ~0ull : ((1ull << n) - 1);
            const uint4 r = act ? hrec[h0 + k] : make_uint4(0, 0, 0, 0);
            const uint32_t pos = act ? hpos[h0 + k] : 0u;
            const uint32_t fi = HF::fi(r);
            const float wt = __uint_as_float(HF::wt(r));
            /* the predecessor of each hit (lane 0: the carried last hit) */
            uint32_t ppos = __shfl_up(pos, 1), pfi = __shfl_up(fi, 1);
            const bool first_hit = h0 == 0 && k == 0;
            if (k == 0) {
                ppos = p_pos;
                pfi = p_fi;
            }
            /* a run breaks at the first hit and where prev.pos + max_gap <
             * pos, unsigned (kguts.cc:821-831) */
            const bool brk = first_hit || (ppos + gap < pos);
            const bool eqp = !brk && fi == pfi;
            const uint64_t M = __ballot(act && (brk || eqp));
            const int jm = hibit(M & lanes_le(k));
            uint32_t cur = __shfl(fi, jm < 0 ? 0 : jm);
            if (jm < 0)
                cur = o_cur;
            uint32_t pcur = __shfl_up(cur, 1);
            if (k == 0)
                pcur = o_cur;
            /* pair switch (kguts.cc:852-856) */
            const bool sw = act && eqp && fi != pcur;
            const uint64_t SW = __ballot(sw);
            const uint64_t S = (__ballot(act && brk) | (SW >> 1)) & ACT; /* sub-run starts */
            const bool memb = act && (fi == cur || ((S >> k) & 1));
            const uint64_t MEMB = __ballot(memb);
            if (dbg && h0 == 0)
                dstamp[14] = wall_clock64(); /* the first chunk's runs and members */
            if (SW & 1) { /* the open run flushes; the pair (last hit, lane 0) carries */
                close_open();
                o_cur = rl32(fi, 0);
                o_cnt = 1;
                o_wsum = 0.0f + p_wt;
                o_first = p_pos;
                o_last = p_pos;
                o_first_idx = h0 - 1;
                o_last_idx = h0 - 1;
            }
            /* lanes before the first start continue the open sub-run */
            const uint32_t fs = S ? lowbit(S) : n;
            if (fs > 0) {
                uint64_t mm = MEMB & bit_range(0, fs);
                o_cnt += (uint32_t)__popcll(mm);
                if (mm) {
                    o_last = rl32(pos, (uint32_t)hibit(mm));
                    o_last_idx = h0 + (uint32_t)hibit(mm);
                }
                o_wsum = sum_lanes_in_order(o_wsum, wt, mm);
            }
            if (fs < n && o_valid)
                close_open();
            /* sub-runs that start in this chunk, one per start lane */
            const bool is_start = (S >> k) & 1;
            const uint64_t above = S & ~lanes_le(k);
            const uint32_t e_k = above ? lowbit(above) : n;
            const uint64_t msg = MEMB & bit_range(k, e_k);
            const uint32_t c_seg = (uint32_t)__popcll(msg);
            const int lm = hibit(msg);
            const uint32_t last_pos = __shfl(pos, lm < 0 ? 0 : lm);
            const bool closed = e_k < n;
            const int b_open = hibit(S);
            uint64_t SUM = __ballot(is_start && closed && (int)c_seg >= prm.min_hits);
            if (b_open >= 0)
                SUM |= 1ull << b_open;
            float ws = 0.0f;
            while (SUM) { /* f32 sums in hit order (kguts.cc:744-756) */
                const uint32_t b = lowbit(SUM);
                SUM &= SUM - 1;
                const uint64_t ab = S & ~lanes_le(b);
                const uint64_t mm = MEMB & bit_range(b, ab ? lowbit(ab) : n);
                const float acc = sum_lanes_in_order(0.0f, wt, mm);
                if (lane == b)
                    ws = acc;
            }
            if (dbg && h0 == 0)
                dstamp[15] = wall_clock64(); /* the first chunk's sums */
            const uint64_t EMIT = __ballot(is_start && closed && (int)c_seg >= prm.min_hits && ws >= min_wh);
            const uint32_t idx = o_ncalls + (uint32_t)__popcll(EMIT & bit_range(0, k));
            if (want_otu && act && ((MEMB >> k) & 1)) { /* a counted member of a sub-run emitted here */
                const int st = hibit(S & lanes_le(k));
                if (st >= 0 && ((EMIT >> st) & 1))
                    oflag[h0 + k] = 1;
            }
            if (want_calls && ((EMIT >> k) & 1)) {
                kgx_call cl;
                cl.start = pos;
                cl.end = last_pos + (KMER - 1);
                cl.count = (int32_t)c_seg;
                cl.function_index = fi;
                cl.weighted_hits = ws;
                calls[idx] = cl;
            }
            if (b_open >= 0) { /* carry the sub-run left open */
                const uint32_t b = (uint32_t)b_open;
                o_valid = true;
                o_cur = rl32(fi, b);
                o_cnt = rl32(c_seg, b);
                o_wsum = rlf(ws, b);
                o_first = rl32(pos, b);
                o_last = rl32(last_pos, b);
                o_ncalls = rl32(idx, b);
                o_first_idx = h0 + b;
                o_last_idx = h0 + (uint32_t)rl32((uint32_t)(lm < 0 ? 0 : lm), b);
            }
            p_pos = rl32(pos, n - 1);
            p_fi = rl32(fi, n - 1);
            p_wt = rlf(wt, n - 1);
            if (dbg && h0 == 0)
                dstamp[9] = wall_clock64(); /* the first 64-hit chunk scored */
        }
        if (o_valid) /* the final flush (kguts.cc:873-876) */
            close_open();
        ncalls_out = want_calls ? o_ncalls : 0u;
    }
    /* 4c. OTU tallies (KmerOtuStats::finalize, kguts.h:196-218), in LDS
     * (hpos, hrec and codes are free once the records are stored and the
     * scorer is done).  A call's hits share few OTUs, so first wave 0 collects
     * the flagged hits' distinct OTUs in its registers -- lane j holds the
     * j-th value met and its count, one ballot round per distinct value among
     * each 64 hits -- and places each value by its rank among the others (=
     * the std::map's key order).  Past 8 distinct values an LDS hash counts
     * them and the distinct pairs are sorted by value (below).  Then the
     * pairs are std::sort'ed by count: lstd_sort_wave64 / lstd_sort_on
     * replay libstdc++'s tie order.  (r4b: O(m^2) count and rank scans, 18.8
     * us at 36 OTUs per call, 6.6 at 3; r4c: the register list alone, 22.6 /
     * 1.8; r4d: the sort alone, 15.9 / 4.4.) */
    if (want_otu) {
        constexpr uint32_t KREG = 8;
        __shared__ LstdPart ostack[64];
        if (dbg)
            dstamp[7] = wall_clock64();
        kgx_otu *o = reinterpret_cast<kgx_otu *>(hrec);
        __syncthreads();
        if (wave == 0) {
            int32_t dv = 0;
            uint32_t dc = 0, dn = 0;
            bool over = false;
            for (uint32_t h0 = 0; h0 < nh && !over; h0 += 64) {
                const uint32_t i = h0 + lane;
                const bool f = i < nh && oflag[i];
                const int32_t x = f ? (int32_t)HF::otu(hrec[i], hrec[i]) : 0;
                uint64_t rem = __ballot(f);
                while (rem) {
                    const int32_t y = (int32_t)rl32((uint32_t)x, lowbit(rem));
                    const uint64_t mk = __ballot(f && x == y);
                    rem &= ~mk;
                    const uint64_t at = __ballot(lane < dn && dv == y);
                    if (at) {
                        if (lane == lowbit(at))
                            dc += (uint32_t)__popcll(mk);
                    } else if (dn < KREG) {
                        if (lane == dn) {
                            dv = y;
                            dc = (uint32_t)__popcll(mk);
                        }
                        dn++;
                    } else {
                        over = true;
                        break;
                    }
                }
            }
            if (!over) {
                uint32_t r = 0;
                for (uint32_t j = 0; j < dn; j++)
                    r += (int32_t)rl32((uint32_t)dv, j) < dv ? 1u : 0u;
                if (lane < dn)
                    o[r] = kgx_otu{dv, (int32_t)dc};
            }
            if (lane == 0)
                n_otu = over ? ~0u : dn;
        }
        __syncthreads();
        uint32_t d = n_otu;
        if (d == ~0u) {
            /* past KREG distinct values: the flagged hits' OTUs counted in an
             * LDS hash (at most 256 FJ slots: one per window at least, so it
             * never fills), the distinct (value, count) pairs compacted, then
             * sorted by value -- one wave's register bitonic network up to 64
             * pairs, a block network beyond.  (r4o: a bitonic sort of every
             * flagged hit's value, then runs -- 6.1 us of the 36-OTU tally.) */
            constexpr uint32_t H = 256 * FJ;
            /* the hash's slots: at least twice the hits (so it stays sparse),
             * at most H; its scans below cost a barrier per 256 slots */
            uint32_t Hs = 256;
            while (Hs < 2 * nh && Hs < H)
                Hs <<= 1;
            /* the records end before the hash (the second half of hrec) when
             * they fill at most half of it: the hash counts straight from
             * them.  Else the flagged values first, compacted in hit order
             * into hpos (the records in hrec are dead then), so the hash can
             * use hrec */
            const bool direct = nh <= 128 * FJ;
            int32_t *v = reinterpret_cast<int32_t *>(hpos);
            uint32_t m = 0;
            for (uint32_t j = 0; !direct && j < (nh + 255) / 256; j++) {
                const uint32_t i = t + 256 * j;
                const bool f = i < nh && oflag[i];
                const int32_t x = f ? (int32_t)HF::otu(hrec[i], hrec[i]) : 0;
                const uint64_t bm = __ballot(f);
                if (lane == 0)
                    wave_cnt[wave] = (uint32_t)__popcll(bm);
                __syncthreads();
                uint32_t before = 0, total = 0;
                for (uint32_t w = 0; w < 4; w++) {
                    before += w < wave ? wave_cnt[w] : 0u;
                    total += wave_cnt[w];
                }
                __syncthreads(); /* hpos[m + ...] may overlap hits not yet read by slower waves: read, then write */
                if (f)
                    v[m + before + lanes_below(bm)] = x;
                m += total;
                __syncthreads();
            }
            int32_t *hk = reinterpret_cast<int32_t *>(hrec) + 2 * 256 * FJ; /* past the pairs */
            uint32_t *hcnt = reinterpret_cast<uint32_t *>(hrec) + 3 * 256 * FJ;
            for (uint32_t i = t; i < Hs; i += 256) {
                hk[i] = INT32_MIN; /* OTUs are -1 .. 2^21 - 2 */
                hcnt[i] = 0;
            }
            __syncthreads();
            for (uint32_t i = t; i < (direct ? nh : m); i += 256) {
                if (direct && !oflag[i])
                    continue;
                const int32_t x = direct ? (int32_t)HF::otu(hrec[i], hrec[i]) : v[i];
                uint32_t h = ((uint32_t)x * 0x9E3779B1u) & (Hs - 1);
                for (;;) {
                    const int32_t old = atomicCAS(hk + h, INT32_MIN, x);
                    if (old == INT32_MIN || old == x)
                        break;
                    h = (h + 1) & (Hs - 1);
                }
                atomicAdd(hcnt + h, 1u);
            }
            __syncthreads();
            /* the pairs, packed (value with its sign bit flipped << 32 | count)
             * so that unsigned order is the map's key order */
            uint64_t *pk = reinterpret_cast<uint64_t *>(o);
            d = 0;
            for (uint32_t j = 0; j < Hs / 256; j++) {
                const uint32_t i = t + 256 * j;
                const bool f = hk[i] != INT32_MIN;
                const uint64_t bm = __ballot(f);
                if (lane == 0)
                    wave_cnt[wave] = (uint32_t)__popcll(bm);
                __syncthreads();
                uint32_t before = 0, total = 0;
                for (uint32_t w = 0; w < 4; w++) {
                    before += w < wave ? wave_cnt[w] : 0u;
                    total += wave_cnt[w];
                }
                if (f)
                    pk[d + before + lanes_below(bm)] = (uint64_t)((uint32_t)hk[i] ^ 0x80000000u) << 32 | hcnt[i];
                d += total;
                __syncthreads();
            }
            if (d <= 64) {
                if (wave == 0) {
                    uint64_t x = lane < d ? pk[lane] : ~0ull; /* the padding sorts last */
                    for (uint32_t k = 2; k <= 64; k <<= 1)
                        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                            const uint64_t y = (uint64_t)(uint32_t)xor_lane((int32_t)(uint32_t)x, j) |
                                               (uint64_t)(uint32_t)xor_lane((int32_t)(uint32_t)(x >> 32), j) << 32;
                            const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
                            x = keep_min ? (x < y ? x : y) : (x < y ? y : x);
                        }
                    if (lane < d)
                        pk[lane] = x;
                }
            } else {
                uint32_t P = 128;
                while (P < d)
                    P <<= 1;
                for (uint32_t i = d + t; i < P; i += 256)
                    pk[i] = ~0ull;
                __syncthreads();
                for (uint32_t k = 2; k <= P; k <<= 1)
                    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                        for (uint32_t i = t; i < P; i += 256) {
                            const uint32_t ixj = i ^ j;
                            if (ixj > i) {
                                const uint64_t x = pk[i], y = pk[ixj];
                                if ((x > y) == ((i & k) == 0)) {
                                    pk[i] = y;
                                    pk[ixj] = x;
                                }
                            }
                        }
                        __syncthreads();
                    }
            }
            __syncthreads();
            for (uint32_t i = t; i < d; i += 256) {
                const uint64_t x = pk[i];
                o[i] = kgx_otu{(int32_t)((uint32_t)(x >> 32) ^ 0x80000000u), (int32_t)(uint32_t)x};
            }
            __syncthreads();
        }
        if (dbg) {
            dstamp[8] = wall_clock64();
            dstamp[16] = __builtin_amdgcn_s_memtime();
        }
        /* std::sort by count (less_second, kguts.h:214-218): one wave replays
         * it, lstd_sort_wave64_reg up to 64 pairs (the pairs in registers),
         * lstd_sort_wave up to 64 SW
         * (their scratch past the pairs in hrec, range marks in codes),
         * thread 0 beyond.  (r4f: a 36-OTU call's pairs sort in 0.33 us; the
         * calls past 64 pairs, on the serial replay then, cost 11 us per
         * call on average.) */
        constexpr uint32_t SW = FJ * 2 < 4 ? FJ * 2 : 4;
        const auto by_count = [](const kgx_otu &lhs, const kgx_otu &rhs) { return rhs.count < lhs.count; };
        if (d > 1 && d <= 64) {
            if (wave == 0)
                lstd_sort_wave64_reg(o, d, by_count, o + 64 * SW, o + 64 * SW + 64);
        } else if (d > 64 && d <= 64 * SW) {
            if (wave == 0)
                lstd_sort_wave<SW>(o, d, by_count, o + 64 * SW, o + 128 * SW, codes, ostack);
        } else if (d > 1 && t == 0) {
            lstd_sort_on(o, (int64_t)d, by_count, ostack);
        }
        if (dbg)
            dstamp[17] = __builtin_amdgcn_s_memtime();
        if (t == 0)
            n_otu = d;
        __syncthreads();
        for (uint32_t i = t; i < d; i += 256)
            a.otus[wb + i] = o[i];
    }

    if (dbg)
        dstamp[4] = wall_clock64();
    /* 5. counts, then the token: every store above is visible to the host
     * before it sees done[s] == token */
    if (t == 0) {
        a.counts[s] = nh;
        a.counts[a.n + s] = ncalls_out;
        if (want_otu)
            a.counts[2 * a.n + s] = n_otu;
    }
    __threadfence_system();
    __syncthreads();
    if (t == 0) {
        __threadfence_system();
        if (dbg) {
            dstamp[5] = wall_clock64();
            for (int k = 0; k < 18; k++)
                a.dbg[k] = dstamp[k];
            __threadfence_system();
        }
        *reinterpret_cast<volatile uint32_t *>(a.done + s) = a.token;
    }
}

hipError_t launch_fused_small(const uint8_t *res, const uint64_t *off, const uint64_t *wbase, uint32_t n,
                              uint32_t want, const void *packed_table, uint64_t num_sigs, kgx_params prm,
                              kgx_hit *hits, kgx_call *calls, uint32_t *counts, uint32_t *done, uint32_t token,
                              uint32_t max_windows, uint64_t *dbg, const uint64_t *h_off, const uint64_t *h_wbase,
                              const uint8_t *h_res, uint32_t inline_res, hipStream_t stream, uint32_t hs)
{
    if (n == 0)
        return hipSuccess;
    if (n > FUSED_MAX_SEQ || num_sigs == 0 || !packed_table)
        return hipErrorInvalidValue;
    FusedArgs a;
    a.res = res;
    a.off = off;
    a.wbase = wbase;
    a.n = n;
    a.want = want;
    a.table = static_cast<const uint4 *>(packed_table);
    a.num_sigs = num_sigs;
    a.magic = mod_magic(num_sigs >> hs);
    a.hs = hs;
    a.prm = prm;
    a.hits = hits;
    a.calls = calls;
    a.otus = nullptr;
    a.counts = counts;
    a.done = done;
    a.token = token;
    a.dbg = dbg;
    if (max_windows > FUSED_MAX_WINDOWS)
        return hipErrorInvalidValue;
    const bool small = max_windows <= 2 * 256;
    if (inline_res) { /* offsets, window bases and residues in the kernel arguments */
        if (n > FUSED_INLINE_SEQ || inline_res > FUSED_INLINE_RES)
            return hipErrorInvalidValue;
        FusedInline k;
        for (uint32_t i = 0; i <= n; i++) {
            k.off[i] = (uint32_t)h_off[i];
            k.wb[i] = (uint32_t)h_wbase[i];
        }
        __builtin_memcpy(k.res, h_res, inline_res);
        if (small)
            hipLaunchKernelGGL(fused_small_inline_kernel<2>, dim3(n), dim3(256), 0, stream, a, k);
        else
            hipLaunchKernelGGL(fused_small_inline_kernel<FUSED_MAX_WINDOWS / 256>, dim3(n), dim3(256), 0, stream, a, k);
    } else if (small) {
        hipLaunchKernelGGL(fused_small_kernel<2>, dim3(n), dim3(256), 0, stream, a);
    } else {
        hipLaunchKernelGGL(fused_small_kernel<FUSED_MAX_WINDOWS / 256>, dim3(n), dim3(256), 0, stream, a);
    }
    return hipGetLastError();
}

/*
 * The resident call service: the same per-sequence body, served from slots in
 * mapped host memory by workgroups that stay resident, so a call costs no
 * launch (the runtime's launch path serialises a worker pool's threads:
 * ~6 us of host time per launch, 170K calls/s at T = 16 in r3g).  Workgroup
 * i owns slot i: wave 0 polls the slot's header line and its first residue
 * chunks with system-scope loads (the host wrote the residues, length, want
 * and parameters before it stored req; a chunk carries the request number it
 * belongs to) and decodes the chunks into codes, the workgroup runs the
 * sequence, and fused_small_body stores the records, the counts and done =
 * req behind a system-scope fence.  Every workgroup leaves on stop or life_ticks after
 * its start -- a bound on how long the instance holds its hardware queue; the
 * host keeps the next instance queued behind it while calls arrive
 * (kgx_svc.cpp).  There is no per-workgroup idle exit: a first version left
 * after 1 ms without a request in any slot, read from a device word every
 * pickup raised, but a workgroup on another XCD could read that word stale
 * from its own L2, leave while its slot was merely quiet, and strand the
 * slot's next request until the instance ended (0.5% of calls waited up to
 * the instance's lifetime: +40% mean latency at 16 callers).
 */
/* a 16-B load at system scope (past every cache: the host writes this memory) */
__device__ __forceinline__ uint4 load_system16(const uint4 *p)
{
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return make_uint4(v.x, v.y, v.z, v.w);
}

template <bool QUAD>
__global__ __launch_bounds__(256) void svc_kernel(const SvcSlotHdr *hdr, SvcSlotOut *out, SvcSlotDbg *dbgs,
                                                  const uint8_t *res_base, kgx_hit *hits, kgx_call *calls,
                                                  kgx_otu *otus,
                                                  const uint4 *table, uint64_t num_sigs, uint64_t magic,
                                                  uint32_t hs, uint64_t life_ticks, uint32_t poll_chunks)
{
    __shared__ uint32_t cmd[18]; /* the request's header line; [16] = go, [17] = chunks still stale */
    __shared__ uint32_t scodes[SVC_RES_CHUNKS * 3]; /* the request's residue codes, 12 per chunk */
    __shared__ uint8_t tab[256]; /* residue -> code (to_amino_acid_off, kguts.cc:273-339) */
    const uint32_t slot = blockIdx.x, t = threadIdx.x, lane = lane_id();
    const uint64_t t0 = wall_clock64();
    uint32_t last = 0;
    if (t == 0)
        last = __hip_atomic_load(&out[slot].done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    last = __shfl(last, 0);
    const uint4 *hline = reinterpret_cast<const uint4 *>(&hdr[slot]);
    const uint4 *chunks = reinterpret_cast<const uint4 *>(res_base + (uint64_t)slot * SVC_RES_STRIDE);
    tab[t] = (uint8_t)residue_code(t);
    __syncthreads();
    /* 4 residues -> their 4 codes */
    auto code4 = [&](uint32_t w) -> uint32_t {
        return (uint32_t)tab[w & 0xFFu] | (uint32_t)tab[(w >> 8) & 0xFFu] << 8 |
               (uint32_t)tab[(w >> 16) & 0xFFu] << 16 | (uint32_t)tab[w >> 24] << 24;
    };
    for (;;) {
        if (t < 64) {
            /* wave 0 polls with one 16-B load a lane: lanes 0-3 the header
             * line (its request number and fields), lanes 4-63 the first
             * SVC_POLL_CHUNKS residue chunks (12 residues and the request
             * number they belong to) -- so a protein of up to 720 aa comes in
             * with its header and costs no second round trip.  A header whose
             * copy word lags its request number was read mid-write and is
             * read again; a chunk read with its header may predate it (its
             * tag says so) and is read again, now behind the header. */
            uint32_t go = 0;
            const uint4 *src = lane < 4 ? hline + lane : chunks + (lane - 4);
            const bool polls = lane < 4 + poll_chunks;
            for (;;) {
                uint4 v = polls ? load_system16(src) : make_uint4(0, 0, 0, 0);
                const uint32_t req = rl32(v.x, 0), stop = rl32(v.y, 0), copy = rl32(v.w, 3);
                if (stop)
                    break;
                if (req != last && copy == req) {
                    go = 1;
                    const uint32_t n_chunks = (min(rl32(v.z, 0), SVC_MAX_RES) + 11) / 12;
                    const uint32_t c = lane - 4;
                    bool stale = lane >= 4 && polls && c < n_chunks && v.w != req;
                    const uint64_t t1 = wall_clock64();
                    while (__ballot(stale) && wall_clock64() - t1 < 100000000ull) { /* (1 s: a bound, not a wait) */
                        if (stale) {
                            v = load_system16(src);
                            stale = v.w != req;
                        }
                    }
                    /* past the bound with chunks still stale: the request is
                     * answered with an impossible count (the host rejects it,
                     * KGX_EDEVICE, and takes the batch path), never computed
                     * over residues of another request */
                    const bool lost = __ballot(stale) != 0;
                    if (lane == 0)
                        cmd[17] = lost ? 1u : 0u;
                    if (lane < 4) {
                        cmd[4 * lane] = v.x;
                        cmd[4 * lane + 1] = v.y;
                        cmd[4 * lane + 2] = v.z;
                        cmd[4 * lane + 3] = v.w;
                    } else if (polls && c < n_chunks) {
                        scodes[3 * c] = code4(v.x);
                        scodes[3 * c + 1] = code4(v.y);
                        scodes[3 * c + 2] = code4(v.z);
                    }
                    break;
                }
                if (wall_clock64() - t0 > life_ticks)
                    break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (lane == 0)
                cmd[16] = go;
        }
        __syncthreads();
        if (!cmd[16])
            break;
        if (cmd[17]) {
            const uint32_t req = cmd[0];
            if (t == 0) {
                out[slot].nh = 0xFFFFFFFFu;
                out[slot].nc = 0;
                out[slot].no = 0;
                __threadfence_system();
                *reinterpret_cast<volatile uint32_t *>(&out[slot].done) = req;
            }
            last = req;
            __syncthreads(); /* cmd is rewritten by the next poll */
            continue;
        }
        /* the residues the host wrote before req: no stale line in this CU's caches */
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const SvcSlotHdr *h = reinterpret_cast<const SvcSlotHdr *>(cmd);
        FusedArgs a;
        const uint32_t req = h->req, len = min(h->len, SVC_MAX_RES);
        a.res = nullptr;
        a.off = nullptr;
        a.wbase = nullptr;
        a.n = 1;
        a.want = h->want;
        a.table = table;
        a.num_sigs = num_sigs;
        a.magic = magic;
        a.hs = hs;
        a.prm = h->prm;
        a.hits = hits + (uint64_t)slot * FUSED_MAX_WINDOWS;
        a.calls = calls + (uint64_t)slot * FUSED_MAX_WINDOWS;
        a.otus = otus + (uint64_t)slot * FUSED_MAX_WINDOWS;
        a.counts = &out[slot].nh; /* nh, nc, no */
        a.done = &out[slot].done;
        a.token = req;
        a.dbg = h->debug ? dbgs[slot].stamp : nullptr;
        /* the chunks past the polled ones (proteins over 720 aa), read now
         * that the header is seen */
        for (uint32_t c = poll_chunks + t; c < (len + 11) / 12; c += 256) {
            const uint4 v = load_system16(chunks + c);
            scodes[3 * c] = code4(v.x);
            scodes[3 * c + 1] = code4(v.y);
            scodes[3 * c + 2] = code4(v.z);
        }
        const FusedSlot in{nullptr, len, reinterpret_cast<uint8_t *>(scodes)};
        __syncthreads(); /* every thread has its copy of the request and the residues before cmd can change */
        /* one body for every length (its registers probe two 256-window
         * slices at a time, its LDS holds all of them): a second, inlined
         * body for short proteins made the kernel spill ~190 SGPRs into VGPR
         * lanes, reloaded in the short path's loops too */
        fused_small_body<FUSED_MAX_WINDOWS / 256, FusedSlot, QUAD>(a, in, 0);
        last = req;
    }
    /* counted out: the host's exit hook waits for every launched instance's
     * workgroups without a runtime call (kgx_svc.cpp, stop_all_at_exit) */
    if (t == 0)
        __hip_atomic_fetch_add(&out[slot].left, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_svc(const SvcSlotHdr *hdr, SvcSlotOut *out, SvcSlotDbg *dbg, const uint8_t *res, kgx_hit *hits,
                      kgx_call *calls, kgx_otu *otus, uint32_t slots, const void *packed_table, uint64_t num_sigs,
                      uint64_t life_ticks, int quad_probe, hipStream_t stream, uint32_t hs, uint32_t poll_chunks)
{
    poll_chunks = std::min(poll_chunks, SVC_POLL_CHUNKS);
    if (slots == 0 || slots > SVC_MAX_SLOTS || num_sigs == 0 || !packed_table)
        return hipErrorInvalidValue;
    if (quad_probe)
        hipLaunchKernelGGL(svc_kernel<true>, dim3(slots), dim3(256), 0, stream, hdr, out, dbg, res, hits, calls, otus,
                           static_cast<const uint4 *>(packed_table), num_sigs, mod_magic(num_sigs >> hs), hs,
                           life_ticks, poll_chunks);
    else
        hipLaunchKernelGGL(svc_kernel<false>, dim3(slots), dim3(256), 0, stream, hdr, out, dbg, res, hits, calls,
                           otus, static_cast<const uint4 *>(packed_table), num_sigs, mod_magic(num_sigs >> hs), hs,
                           life_ticks, poll_chunks);
    return hipGetLastError();
}

}  // namespace kgx
