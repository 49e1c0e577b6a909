/*
 * kgx_kernels.hip -- gfx950 kernels for the close_kmers hot path.
 *
 *   plan   : per-sequence window / chunk bookkeeping (exclusive scans)
 *   probe  : 8-mer encode + linear-probe lookup in the HBM-resident image;
 *            one wave per chunk of PROBE_J*64 windows of one sequence,
 *            PROBE_J independent probe chains in flight per lane; hits are
 *            compacted in position order with a wave ballot
 *   score  : the gather_hits / process_set_of_hits run state machine, one
 *            lane per sequence, O(1) state (no 40000-entry buffer)
 *   gather : sparse per-sequence results -> dense CSR (host-buffer path)
 *   synth  : synthetic image builder (parallel linear-probe insert) and
 *            synthetic query generator, bit-identical to synth.py
 *
 * Reference behaviour restated here (kguts.cc line numbers):
 *   residue map            273-339     window set / rolling code  682-732, 783-871
 *   probe                  585-602     run rules                  734-781, 808-876
 */
#include "kgx_internal.h"

namespace kgx {

/* ------------------------------------------------------------------------ */
/* helpers                                                                   */
/* ------------------------------------------------------------------------ */

/* to_amino_acid_off (kguts.cc:273-339) without a table: the 20 standard
 * upper-case residues are the set bits of a 26-bit mask over 'A'..'Z'; the
 * code is the number of set bits below the letter.  Anything else -> 20. */
__device__ __forceinline__ uint32_t residue_code(uint32_t c)
{
    constexpr uint32_t kMask = (1u << 0) | (1u << 2) | (1u << 3) | (1u << 4) | (1u << 5) |
                               (1u << 6) | (1u << 7) | (1u << 8) | (1u << 10) | (1u << 11) |
                               (1u << 12) | (1u << 13) | (1u << 15) | (1u << 16) | (1u << 17) |
                               (1u << 18) | (1u << 19) | (1u << 21) | (1u << 22) | (1u << 24);
    const uint32_t idx = c - 'A';
    const bool ok = idx < 26u && ((kMask >> (idx & 31u)) & 1u);
    return ok ? (uint32_t)__popc(kMask & ((1u << (idx & 31u)) - 1u)) : 20u;
}

__device__ __forceinline__ uint32_t codes4(uint32_t bytes)
{
    return residue_code(bytes & 0xFFu) | (residue_code((bytes >> 8) & 0xFFu) << 8) |
           (residue_code((bytes >> 16) & 0xFFu) << 16) | (residue_code(bytes >> 24) << 24);
}

/* x % n for x < 2^35, n >= 1, m = floor((2^64-1)/n) */
__device__ __forceinline__ uint64_t mod_by(uint64_t x, uint64_t n, uint64_t m)
{
    uint64_t q = __umul64hi(x, m);
    uint64_t r = x - q * n;
    return r >= n ? r - n : r;
}

/* splitmix64 finaliser; rnd(seed, i) = mix64(seed ^ mix64(i)) (synth.py) */
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rnd(uint64_t seed, uint64_t i) { return mix64(seed ^ mix64(i)); }

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

/* order LDS accesses between lanes of one wave (no s_barrier needed) */
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* ------------------------------------------------------------------------ */
/* plan                                                                      */
/* ------------------------------------------------------------------------ */

__device__ __forceinline__ uint64_t windows_of(uint64_t len) { return len >= 9 ? len - 8 : 0; }

/*
 * wbase / cbase = exclusive scans of windows and chunks per sequence, in two
 * launches: plan_reduce sums each 1024-sequence tile, plan_scan adds the sums
 * of the tiles before it, scans inside the tile and fills chunk -> sequence.
 * Windows of a sequence of length L are positions 0 .. L-9 (kguts.cc:792,798:
 * the last full window is never probed).
 */
constexpr uint32_t PLAN_PER = 4;                  /* sequences per thread */
constexpr uint32_t PLAN_TILE = 256 * PLAN_PER;    /* sequences per workgroup */

struct WinChunk {
    uint64_t w, c;
};

__device__ __forceinline__ WinChunk thread_sums(const uint64_t *seq_off, uint32_t n, uint32_t s0)
{
    WinChunk a = {0, 0};
    for (uint32_t k = 0; k < PLAN_PER; k++) {
        const uint32_t s = s0 + k;
        if (s < n) {
            const uint64_t nw = windows_of(seq_off[s + 1] - seq_off[s]);
            a.w += nw;
            a.c += (nw + CHUNK - 1) / CHUNK;
        }
    }
    return a;
}

/* inclusive scan of one u64 pair over a 256-thread block */
__device__ __forceinline__ WinChunk block_scan(WinChunk v, WinChunk *lds4, WinChunk &total)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint64_t w = __shfl_up(v.w, off), c = __shfl_up(v.c, off);
        if (lane >= off) {
            v.w += w;
            v.c += c;
        }
    }
    if (lane == 63)
        lds4[wave] = v;
    __syncthreads();
    WinChunk pre = {0, 0};
    total = {0, 0};
    for (uint32_t i = 0; i < 4; i++) {
        if (i < wave) {
            pre.w += lds4[i].w;
            pre.c += lds4[i].c;
        }
        total.w += lds4[i].w;
        total.c += lds4[i].c;
    }
    v.w += pre.w;
    v.c += pre.c;
    return v;
}

__global__ __launch_bounds__(256) void plan_reduce_kernel(const uint64_t *__restrict__ seq_off,
                                                          uint32_t n, WinChunk *__restrict__ tile_sums)
{
    __shared__ WinChunk lds4[4];
    const uint32_t s0 = blockIdx.x * PLAN_TILE + threadIdx.x * PLAN_PER;
    WinChunk total;
    block_scan(thread_sums(seq_off, n, s0), lds4, total);
    if (threadIdx.x == 0)
        tile_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void plan_scan_kernel(const uint64_t *__restrict__ seq_off,
                                                        uint32_t n,
                                                        const WinChunk *__restrict__ tile_sums,
                                                        uint64_t *__restrict__ wbase,
                                                        uint64_t *__restrict__ cbase,
                                                        uint32_t *__restrict__ chunk_seq)
{
    __shared__ WinChunk lds4[4];
    __shared__ WinChunk lds_pre[4];
    /* sum of all earlier tiles */
    WinChunk p = {0, 0};
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += 256) {
        p.w += tile_sums[b].w;
        p.c += tile_sums[b].c;
    }
    WinChunk ptot;
    block_scan(p, lds_pre, ptot);
    const WinChunk before = ptot;
    __syncthreads();

    const uint32_t s0 = blockIdx.x * PLAN_TILE + threadIdx.x * PLAN_PER;
    const WinChunk mine = thread_sums(seq_off, n, s0);
    WinChunk tot;
    const WinChunk incl = block_scan(mine, lds4, tot);
    uint64_t bw = before.w + incl.w - mine.w, bc = before.c + incl.c - mine.c;
    for (uint32_t k = 0; k < PLAN_PER; k++) {
        const uint32_t s = s0 + k;
        if (s >= n)
            break;
        const uint64_t nw = windows_of(seq_off[s + 1] - seq_off[s]);
        const uint64_t nc = (nw + CHUNK - 1) / CHUNK;
        wbase[s] = bw;
        cbase[s] = bc;
        for (uint64_t c = 0; c < nc; c++)
            chunk_seq[bc + c] = s;
        bw += nw;
        bc += nc;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 255) {
        wbase[n] = before.w + tot.w;
        cbase[n] = before.c + tot.c;
    }
}

size_t plan_workspace_bytes(uint32_t n_seq)
{
    return ((size_t)n_seq / PLAN_TILE + 1) * sizeof(WinChunk);
}

hipError_t launch_plan(const uint64_t *seq_off, uint32_t n_seq, uint64_t *wbase, uint64_t *cbase,
                       uint32_t *chunk_seq, void *workspace, hipStream_t stream)
{
    const uint32_t tiles = n_seq / PLAN_TILE + 1; /* >= 1 so wbase[n] is written */
    hipLaunchKernelGGL(plan_reduce_kernel, dim3(tiles), dim3(256), 0, stream, seq_off, n_seq,
                       static_cast<WinChunk *>(workspace));
    hipLaunchKernelGGL(plan_scan_kernel, dim3(tiles), dim3(256), 0, stream, seq_off, n_seq,
                       static_cast<const WinChunk *>(workspace), wbase, cbase, chunk_seq);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* probe                                                                     */
/* ------------------------------------------------------------------------ */

constexpr int STAGE_DW = (CHUNK + KMER + 4) / 4 + 3; /* LDS dwords per wave */

/* Residue dword at absolute address `a` (4-aligned), bytes outside
 * [lo, hi) read as 0 (code 20). */
__device__ __forceinline__ uint32_t load_dword_clamped(uintptr_t a, uintptr_t lo, uintptr_t hi)
{
    if (a >= lo && a + 4 <= hi)
        return *reinterpret_cast<const uint32_t *>(a);
    uint32_t v = 0;
    for (int b = 0; b < 4; b++)
        if (a + b >= lo && a + b < hi)
            v |= (uint32_t)(*reinterpret_cast<const uint8_t *>(a + b)) << (8 * b);
    return v;
}

/*
 * One wave = one chunk: windows [w0, w1) of sequence s.  Lane l owns windows
 * w0 + l + 64 j (j < PROBE_J), so each j-slice is 64 consecutive windows and a
 * ballot over a slice is in position order.  All PROBE_J first probes of a
 * lane are issued before any is resolved.
 *   KEY_FIRST = false: every probe round loads the 8-byte key and the 16-byte
 *     payload of its bucket together (two loads per bucket examined);
 *   KEY_FIRST = true: a round loads only keys; a matching bucket's payload is
 *     loaded in the round that finds it, overlapping the other chains (one
 *     load per bucket + one per hit; the payload mostly shares the key's
 *     sector, still in L2).
 */
template <bool KEY_FIRST>
__global__ __launch_bounds__(256) void probe_kernel(
    const uint8_t *__restrict__ residues, uint64_t n_residues, const uint64_t *__restrict__ seq_off,
    const uint64_t *__restrict__ wbase, const uint64_t *__restrict__ cbase,
    const uint32_t *__restrict__ chunk_seq, uint32_t n_seq, const kgx_sig_kmer *__restrict__ table,
    uint64_t num_sigs, uint64_t magic, kgx_hit *__restrict__ hits, uint32_t *__restrict__ chunk_hits)
{
    __shared__ uint32_t stage[PROBE_WAVES][STAGE_DW];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    const uint64_t c = (uint64_t)blockIdx.x * PROBE_WAVES + wave;
    if (c >= cbase[n_seq])
        return;
    const uint32_t s = chunk_seq[c];
    const uint64_t k = c - cbase[s];
    const uint64_t seq_start = seq_off[s];
    const uint64_t nwin = windows_of(seq_off[s + 1] - seq_start);
    const uint64_t w0 = k * CHUNK;
    const uint64_t w1 = min(w0 + (uint64_t)CHUNK, nwin);
    const uint64_t out0 = wbase[s] + w0;

    /* stage residues [w0, w1 + 7) of the sequence as codes, keeping the
     * global 4-byte alignment so dword loads stay aligned */
    uint32_t *lds = stage[wave];
    const uintptr_t arr_lo = reinterpret_cast<uintptr_t>(residues);
    const uintptr_t arr_hi = arr_lo + n_residues;
    const uintptr_t g = arr_lo + seq_start + w0;
    const uintptr_t gb = g & ~(uintptr_t)3;
    const uint32_t shift = (uint32_t)(g - gb);
    const uint32_t ndw = (uint32_t)((shift + (w1 - w0) + KMER - 1 + 3) / 4);
    for (uint32_t i = lane; i < ndw; i += 64)
        lds[i] = codes4(load_dword_clamped(gb + 4 * (uintptr_t)i, arr_lo, arr_hi));
    wave_lds_sync();

    uint64_t key[PROBE_J], slot[PROBE_J], kv[PROBE_J];
    uint4 pv[PROBE_J];
    bool pend[PROBE_J], hit[PROBE_J];
    const kgx_sig_kmer *tab = table;

#pragma unroll
    for (int j = 0; j < PROBE_J; j++) {
        const uint64_t w = w0 + lane + 64 * j;
        const uint32_t o = shift + lane + 64 * j;
        const uint32_t d0 = lds[o >> 2], d1 = lds[(o >> 2) + 1], d2 = lds[(o >> 2) + 2];
        const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, o & 3);
        const uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, o & 3);
        /* a code-20 byte anywhere kills the window (advance_past_ambig) */
        const bool ok = (w < w1) && ((((lo + 0x6C6C6C6Cu) | (hi + 0x6C6C6C6Cu)) & 0x80808080u) == 0);
        /* big-endian base-20 Horner (encoded_kmer, kguts.cc:438-455) */
        const uint32_t a = (((lo & 0xFF) * 20 + ((lo >> 8) & 0xFF)) * 20 + ((lo >> 16) & 0xFF)) * 20 +
                           (lo >> 24);
        const uint32_t b = (((hi & 0xFF) * 20 + ((hi >> 8) & 0xFF)) * 20 + ((hi >> 16) & 0xFF)) * 20 +
                           (hi >> 24);
        key[j] = (uint64_t)a * 160000u + b;
        slot[j] = ok ? mod_by(key[j], num_sigs, magic) : 0;
        pend[j] = ok;
        hit[j] = false;
        kv[j] = 0;
        pv[j] = make_uint4(0, 0, 0, 0);
        if (ok) {
            const kgx_sig_kmer *e = tab + slot[j];
            kv[j] = e->which_kmer;
            if (!KEY_FIRST)
                pv[j] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(e) + 8);
        }
    }

    /* linear probe rounds (lookup_hash_entry, kguts.cc:585-602); bounded by
     * num_sigs buckets where the reference would spin forever */
    for (uint64_t round = 0;; round++) {
        bool more = false;
#pragma unroll
        for (int j = 0; j < PROBE_J; j++) {
            if (pend[j]) {
                if (kv[j] == key[j]) {
                    hit[j] = true;
                    pend[j] = false;
                    if (KEY_FIRST)
                        pv[j] = *reinterpret_cast<const uint4 *>(
                            reinterpret_cast<const char *>(tab + slot[j]) + 8);
                } else if (kv[j] > MAX_ENCODED || round + 1 >= num_sigs) {
                    pend[j] = false;
                } else {
                    slot[j] = (slot[j] + 1 == num_sigs) ? 0 : slot[j] + 1;
                    const kgx_sig_kmer *e = tab + slot[j];
                    kv[j] = e->which_kmer;
                    if (!KEY_FIRST)
                        pv[j] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(e) + 8);
                    more = true;
                }
            }
        }
        if (!__any(more))
            break;
    }

    /* ordered compaction: slice j holds windows w0+64j .. w0+64j+63 */
    uint32_t count = 0;
#pragma unroll
    for (int j = 0; j < PROBE_J; j++) {
        const uint64_t m = __ballot(hit[j]);
        if (hit[j]) {
            kgx_hit *dst = hits + out0 + count + lanes_below(m);
            uint4 *d = reinterpret_cast<uint4 *>(dst);
            d[0] = make_uint4((uint32_t)kv[j], (uint32_t)(kv[j] >> 32), pv[j].x, pv[j].y & 0xFFFFu);
            d[1] = make_uint4(pv[j].z, pv[j].w, (uint32_t)(w0 + lane + 64 * j), s);
        }
        count += (uint32_t)__popcll(m);
    }
    if (lane == 0)
        chunk_hits[c] = count;
}

hipError_t launch_probe(const uint8_t *residues, uint64_t n_residues, const uint64_t *seq_off,
                        const uint64_t *wbase, const uint64_t *cbase, const uint32_t *chunk_seq,
                        uint32_t n_seq, uint64_t max_chunks, const kgx_sig_kmer *table,
                        uint64_t num_sigs, kgx_hit *hits, uint32_t *chunk_hits, int variant,
                        hipStream_t stream)
{
    if (max_chunks == 0)
        return hipSuccess;
    const uint64_t blocks = (max_chunks + PROBE_WAVES - 1) / PROBE_WAVES;
    if (variant == PROBE_KEY_FIRST)
        hipLaunchKernelGGL(probe_kernel<true>, dim3((uint32_t)blocks), dim3(64 * PROBE_WAVES), 0,
                           stream, residues, n_residues, seq_off, wbase, cbase, chunk_seq, n_seq,
                           table, num_sigs, mod_magic(num_sigs), hits, chunk_hits);
    else
        hipLaunchKernelGGL(probe_kernel<false>, dim3((uint32_t)blocks), dim3(64 * PROBE_WAVES), 0,
                           stream, residues, n_residues, seq_off, wbase, cbase, chunk_seq, n_seq,
                           table, num_sigs, mod_magic(num_sigs), hits, chunk_hits);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* score                                                                     */
/* ------------------------------------------------------------------------ */

/*
 * The run state machine of gather_hits (kguts.cc:808-876) and
 * process_set_of_hits (kguts.cc:734-781), one lane per sequence.  The
 * reference keeps up to 40000 hits in a buffer and rescans it at every flush;
 * here the buffer is summarised by O(1) state that yields the same call:
 *   n         number of buffered hits (capped at RUN_CAP, kguts.cc:850-851)
 *   cur       current_fI
 *   cnt/wsum  count and f32 sum (in append order) of buffered hits with
 *             fI == cur -- exactly the reference's flush loop
 *   first/last position of buffer[0] / of the last buffered hit with fI == cur
 *   p1, p2    the last two buffered hits (gap rule, order constraint,
 *             pair switch and carry-over read only these)
 * Buffered hits are flagged KGX_HIT_IN_RUN, and KGX_HIT_COUNTED when their
 * function is their run's current_fI.  An emitted call records its run's hit
 * range; one forward pass then flags the COUNTED hits inside emitted ranges
 * KGX_HIT_OTU -- the hits the reference tallies into otu_map (kguts.cc:760-768).
 */
struct RunTail {
    uint32_t pos, fI, idx;
    float wt;
    uint32_t avg;
};

constexpr int SCORE_BATCH = 8;
constexpr uint32_t F_RUN = KGX_HIT_IN_RUN << 16, F_CNT = KGX_HIT_COUNTED << 16,
                   F_OTU = KGX_HIT_OTU << 16;

__global__ __launch_bounds__(256) void score_kernel(
    uint32_t n_seq, const uint64_t *__restrict__ wbase, const uint64_t *__restrict__ cbase,
    const uint32_t *__restrict__ chunk_hits, kgx_hit *__restrict__ hits, kgx_call *__restrict__ calls,
    uint2 *__restrict__ ranges, uint32_t *__restrict__ hit_count, uint32_t *__restrict__ call_count,
    kgx_params prm, uint32_t want)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_seq)
        return;
    const uint64_t base = wbase[s];
    const uint64_t c0 = cbase[s], c1 = cbase[s + 1];

    /* make the sequence's hits contiguous (chunk k wrote at base + k*CHUNK) */
    uint32_t nh = 0;
    for (uint64_t c = c0; c < c1; c++) {
        const uint32_t ch = chunk_hits[c];
        const uint64_t src = base + (c - c0) * CHUNK;
        if (src != base + nh) {
            const uint4 *from = reinterpret_cast<const uint4 *>(hits + src);
            uint4 *to = reinterpret_cast<uint4 *>(hits + base + nh);
            for (uint32_t i = 0; i < 2 * ch; i++)
                to[i] = from[i];
        }
        nh += ch;
    }
    hit_count[s] = nh;

    const bool want_calls = (want & KGX_WANT_CALLS) != 0;
    const bool want_otu = (want & KGX_WANT_OTU) != 0;
    if (!want_calls && !want_otu) {
        /* process_set_of_hits returns before doing anything (kguts.cc:737) */
        call_count[s] = 0;
        return;
    }

    uint32_t *hw = reinterpret_cast<uint32_t *>(hits + base); /* 8 dwords per hit */
    const uint32_t gap = (uint32_t)prm.max_gap;
    int n = 0;
    uint32_t cur = 0, first_pos = 0, last_pos = 0, last_idx = 0, run_start = 0;
    int cnt = 0;
    float wsum = 0.0f;
    RunTail p1 = {0, 0, 0, 0.0f, 0}, p2 = {0, 0, 0, 0.0f, 0};
    uint32_t ncalls = 0;

    auto flush = [&]() {
        if (n == 0)
            return; /* min_hits <= 0 final flush: reference UB, emit nothing */
        if (cnt >= prm.min_hits && wsum >= (float)prm.min_weighted_hits) {
            if (want_calls) {
                kgx_call cl;
                cl.start = first_pos;
                cl.end = last_pos + (KMER - 1);
                cl.count = cnt;
                cl.function_index = cur;
                cl.weighted_hits = wsum;
                calls[base + ncalls] = cl;
            }
            if (want_otu)
                ranges[base + ncalls] = make_uint2(run_start, last_idx);
            ncalls++;
        }
        if (n >= 2 && p2.fI != cur && p2.fI == p1.fI) { /* carry the pair */
            cur = p1.fI;
            n = 2;
            run_start = p2.idx;
            first_pos = p2.pos;
            cnt = 2;
            wsum = 0.0f + p2.wt;
            wsum = wsum + p1.wt;
            last_pos = p1.pos;
            last_idx = p1.idx;
            if (want_otu) {
                hw[8 * p2.idx + 3] = p2.avg | F_RUN | F_CNT;
                hw[8 * p1.idx + 3] = p1.avg | F_RUN | F_CNT;
            }
        } else {
            n = 0;
        }
    };

    /* hits are read SCORE_BATCH at a time, all loads issued before any is
     * consumed: the state machine is serial, its inputs are not */
    for (uint32_t i0 = 0; i0 < nh; i0 += SCORE_BATCH) {
        uint4 rb[SCORE_BATCH];
#pragma unroll
        for (int k = 0; k < SCORE_BATCH; k++)
            if (i0 + k < nh) /* avg|flags, fI, wt, pos */
                rb[k] = *reinterpret_cast<const uint4 *>(hw + 8 * (i0 + k) + 3);
#pragma unroll
        for (int k = 0; k < SCORE_BATCH; k++) {
            const uint32_t i = i0 + k;
            if (i >= nh)
                break;
            const uint32_t avg = rb[k].x & 0xFFFFu;
            const uint32_t fI = rb[k].y;
            const float wt = __uint_as_float(rb[k].z);
            const uint32_t pos = rb[k].w;

            /* gap rule (kguts.cc:821-831), unsigned arithmetic */
            if (n > 0 && p1.pos + gap < pos) {
                if (n >= prm.min_hits)
                    flush();
                else
                    n = 0;
            }
            if (n == 0) {
                cur = fI;
                cnt = 0;
                wsum = 0.0f;
                run_start = i;
                first_pos = pos;
            }
            bool accept = true;
            if (prm.order_constraint && n > 0) { /* kguts.cc:838-842 */
                const uint32_t d = (pos - p1.pos) - (uint32_t)((int)p1.avg - (int)avg);
                accept = (fI == p1.fI) && d <= 20u;
            }
            if (accept) {
                if (n < RUN_CAP) {
                    n++;
                    const bool counted = fI == cur;
                    if (want_otu) /* flags only feed the OTU pass */
                        hw[8 * i + 3] = avg | F_RUN | (counted ? F_CNT : 0u);
                    if (counted) {
                        cnt++;
                        wsum += wt;
                        last_pos = pos;
                        last_idx = i;
                    }
                    p2 = p1;
                    p1 = RunTail{pos, fI, i, wt, avg};
                }
                /* pair switch (kguts.cc:852-856) */
                if (n > 1 && cur != fI && p2.fI == p1.fI)
                    flush();
            }
        }
    }
    if (n >= prm.min_hits) /* kguts.cc:873-876 */
        flush();
    call_count[s] = want_calls ? ncalls : 0;

    /* OTU flags: COUNTED hits inside an emitted call's range (ranges are
     * disjoint and in order) */
    if (want_otu && ncalls > 0) {
        uint32_t ci = 0;
        uint2 rg = ranges[base];
        const uint32_t end = ranges[base + ncalls - 1].y;
        for (uint32_t i0 = rg.x; i0 <= end; i0 += SCORE_BATCH) {
            uint32_t fb[SCORE_BATCH];
#pragma unroll
            for (int k = 0; k < SCORE_BATCH; k++)
                if (i0 + k <= end)
                    fb[k] = hw[8 * (i0 + k) + 3];
#pragma unroll
            for (int k = 0; k < SCORE_BATCH; k++) {
                const uint32_t i = i0 + k;
                if (i > end)
                    break;
                while (i > rg.y) /* i <= end keeps ci < ncalls */
                    rg = ranges[base + ++ci];
                if (i >= rg.x && (fb[k] & F_CNT))
                    hw[8 * i + 3] = fb[k] | F_OTU;
            }
        }
    }
}

hipError_t launch_score(uint32_t n_seq, const uint64_t *wbase, const uint64_t *cbase,
                        const uint32_t *chunk_hits, kgx_hit *hits, kgx_call *calls, void *ranges,
                        uint32_t *hit_count, uint32_t *call_count, kgx_params params,
                        uint32_t want, hipStream_t stream)
{
    if (n_seq == 0)
        return hipSuccess;
    hipLaunchKernelGGL(score_kernel, dim3((n_seq + 255) / 256), dim3(256), 0, stream, n_seq, wbase,
                       cbase, chunk_hits, hits, calls, static_cast<uint2 *>(ranges), hit_count,
                       call_count, params, want);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* gather: sparse (window_base-indexed) -> dense CSR, one wave per sequence  */
/* ------------------------------------------------------------------------ */

__global__ __launch_bounds__(256) void gather_kernel(
    uint32_t n_seq, const uint64_t *__restrict__ wbase, const uint32_t *__restrict__ hit_count,
    const uint32_t *__restrict__ call_count, const kgx_hit *__restrict__ hits,
    const kgx_call *__restrict__ calls, const uint64_t *__restrict__ hoff,
    const uint64_t *__restrict__ coff, kgx_hit *__restrict__ hits_out, kgx_call *__restrict__ calls_out)
{
    const uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= n_seq)
        return;
    const uint32_t lane = lane_id();
    const uint64_t base = wbase[s];
    if (hits_out) {
        const uint4 *src = reinterpret_cast<const uint4 *>(hits + base);
        uint4 *dst = reinterpret_cast<uint4 *>(hits_out + hoff[s]);
        const uint32_t n = 2 * hit_count[s];
        for (uint32_t i = lane; i < n; i += 64)
            dst[i] = src[i];
    }
    if (calls_out) {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(calls + base);
        uint32_t *dst = reinterpret_cast<uint32_t *>(calls_out + coff[s]);
        const uint32_t n = 5 * call_count[s];
        for (uint32_t i = lane; i < n; i += 64)
            dst[i] = src[i];
    }
}

hipError_t launch_gather(uint32_t n_seq, const uint64_t *wbase, const uint32_t *hit_count,
                         const uint32_t *call_count, const kgx_hit *hits, const kgx_call *calls,
                         const uint64_t *hoff, const uint64_t *coff, kgx_hit *hits_out,
                         kgx_call *calls_out, hipStream_t stream)
{
    if (n_seq == 0)
        return hipSuccess;
    hipLaunchKernelGGL(gather_kernel, dim3((n_seq + 3) / 4), dim3(256), 0, stream, n_seq, wbase,
                       hit_count, call_count, hits, calls, hoff, coff, hits_out, calls_out);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* random-read ceiling of the image buffer (roofline denominator)            */
/* ------------------------------------------------------------------------ */

/* Every lane reads RR_ILP independent uniformly random buckets per round:
 * mode 0 the whole 24-byte bucket (8-byte key + 16-byte payload, as the probe
 * does), mode 1 the 8-byte key only, mode 2 one aligned 64-byte sector. */
constexpr int RR_ILP = 8;

template <int MODE>
__global__ __launch_bounds__(256) void random_read_kernel(const kgx_sig_kmer *__restrict__ t,
                                                          uint64_t n, uint64_t magic,
                                                          uint32_t rounds, uint64_t *sink)
{
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t acc = 0;
    const char *base = reinterpret_cast<const char *>(t);
    for (uint32_t r = 0; r < rounds; r++) {
        uint64_t idx[RR_ILP];
#pragma unroll
        for (int k = 0; k < RR_ILP; k++)
            idx[k] = mod_by(mix64(tid * 977u + (uint64_t)r * RR_ILP + k) & ((1ull << 35) - 1), n, magic);
        uint64_t kv[RR_ILP];
        uint4 pv[RR_ILP], pw[RR_ILP], px[RR_ILP];
#pragma unroll
        for (int k = 0; k < RR_ILP; k++) {
            if (MODE == 0) {
                kv[k] = t[idx[k]].which_kmer;
                pv[k] = *reinterpret_cast<const uint4 *>(base + idx[k] * 24 + 8);
            } else if (MODE == 1) {
                kv[k] = t[idx[k]].which_kmer;
            } else {
                const uint4 *s = reinterpret_cast<const uint4 *>(base + ((idx[k] * 24) & ~63ull));
                pv[k] = s[0];
                pw[k] = s[1];
                px[k] = s[2];
                kv[k] = *reinterpret_cast<const uint64_t *>(s + 3);
            }
        }
#pragma unroll
        for (int k = 0; k < RR_ILP; k++) {
            acc ^= kv[k];
            if (MODE == 0)
                acc += pv[k].x ^ pv[k].w;
            if (MODE == 2)
                acc += pv[k].x ^ pw[k].y ^ px[k].z;
        }
    }
    sink[tid] = acc;
}

hipError_t launch_random_read(const kgx_sig_kmer *table, uint64_t num_sigs, uint64_t threads,
                              uint32_t rounds, int mode, uint64_t *sink, hipStream_t stream)
{
    const dim3 grid((uint32_t)(threads / 256)), block(256);
    const uint64_t m = mod_magic(num_sigs);
    if (mode == 0)
        hipLaunchKernelGGL(random_read_kernel<0>, grid, block, 0, stream, table, num_sigs, m, rounds, sink);
    else if (mode == 1)
        hipLaunchKernelGGL(random_read_kernel<1>, grid, block, 0, stream, table, num_sigs, m, rounds, sink);
    else
        hipLaunchKernelGGL(random_read_kernel<2>, grid, block, 0, stream, table, num_sigs, m, rounds, sink);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* synthetic image / queries (synth.py restated on the device)               */
/* ------------------------------------------------------------------------ */

constexpr uint64_t SEED_SRC = 0x5EED0001, SEED_KEY = 0x5EED0002, SEED_FI = 0x5EED0012,
                   SEED_AVG = 0x5EED0022, SEED_WT = 0x5EED0032, SEED_Q_SRC = 0x5EED0003,
                   SEED_Q_SUB = 0x5EED0013, SEED_Q_RES = 0x5EED0023, SEED_Q_X = 0x5EED0033;
constexpr uint32_t SRC_LEN = 300, SRC_WIN = 292;

__device__ __forceinline__ uint32_t src_code(uint64_t s, uint32_t i)
{
    return (uint32_t)(rnd(SEED_SRC, s * SRC_LEN + i) % 20u);
}

__device__ __forceinline__ uint64_t synth_key(uint64_t e, uint64_t n_src)
{
    if (e < n_src * SRC_WIN) {
        const uint64_t s = e / SRC_WIN;
        const uint32_t pos = (uint32_t)(e % SRC_WIN);
        uint64_t v = 0;
        for (int j = 0; j < KMER; j++)
            v = v * 20 + src_code(s, pos + j);
        return v;
    }
    return rnd(SEED_KEY, e) % MAX_ENCODED;
}

__global__ void synth_init_kernel(kgx_sig_kmer *t, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t *w = reinterpret_cast<uint64_t *>(t + i);
        w[0] = EMPTY_KEY;
        w[1] = 0;
        w[2] = ~0ULL; /* owner (lowest entry id) lives in function_index|function_wt */
    }
}

__global__ void synth_insert_kernel(kgx_sig_kmer *t, uint64_t n, uint64_t magic, uint64_t n_keys,
                                    uint64_t n_src, unsigned long long *n_stored)
{
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n_keys;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t key = synth_key(e, n_src);
        uint64_t h = mod_by(key, n, magic);
        for (uint64_t probes = 0; probes < n; probes++) {
            unsigned long long *kp = reinterpret_cast<unsigned long long *>(t + h);
            const unsigned long long old = atomicCAS(kp, (unsigned long long)EMPTY_KEY,
                                                     (unsigned long long)key);
            if (old == EMPTY_KEY) {
                atomicAdd(n_stored, 1ULL);
                break;
            }
            if (old == key)
                break;
            h = (h + 1 == n) ? 0 : h + 1;
        }
        atomicMin(reinterpret_cast<unsigned long long *>(t + h) + 2, (unsigned long long)e);
    }
}

__global__ void synth_payload_kernel(kgx_sig_kmer *t, uint64_t n, uint64_t n_src)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t *w = reinterpret_cast<uint64_t *>(t + i);
        if (w[0] > MAX_ENCODED) {
            w[2] = 0;
            continue;
        }
        const uint64_t e = w[2];
        int32_t fI;
        uint32_t avg;
        if (e < n_src * SRC_WIN) {
            fI = (int32_t)((e / SRC_WIN) % 100000u);
            avg = SRC_LEN - (uint32_t)(e % SRC_WIN);
        } else {
            fI = (int32_t)(rnd(SEED_FI, e) % 100000u);
            avg = (uint32_t)(rnd(SEED_AVG, e) % SRC_LEN);
        }
        const float wt = (float)(rnd(SEED_WT, e) % 49000u + 1000u) * 1e-4f;
        kgx_sig_kmer *k = t + i;
        k->otu_index = -1;
        k->avg_from_end = (uint16_t)avg;
        k->pad = 0;
        k->function_index = fI;
        k->function_wt = wt;
    }
}

hipError_t launch_synth_image(kgx_sig_kmer *table, uint64_t num_sigs, uint64_t n_keys,
                              unsigned long long *n_stored, hipStream_t stream)
{
    const uint64_t n_src = (n_keys / 4) / SRC_WIN;
    const dim3 grid(256 * 32), block(256);
    (void)hipMemsetAsync(n_stored, 0, sizeof(unsigned long long), stream);
    hipLaunchKernelGGL(synth_init_kernel, grid, block, 0, stream, table, num_sigs);
    hipLaunchKernelGGL(synth_insert_kernel, grid, block, 0, stream, table, num_sigs,
                       mod_magic(num_sigs), n_keys, n_src, n_stored);
    hipLaunchKernelGGL(synth_payload_kernel, grid, block, 0, stream, table, num_sigs, n_src);
    return hipGetLastError();
}

__global__ void synth_queries_kernel(uint64_t n_src, uint32_t n_seq, uint32_t L,
                                     uint32_t x_permille, uint64_t q0, uint8_t *res,
                                     uint64_t *seq_off)
{
    const uint64_t total = (uint64_t)n_seq * L;
    const char *alpha = "ACDEFGHIKLMNPQRSTVWY";
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t ql = t / L;
        const uint32_t i = (uint32_t)(t % L);
        const uint64_t q = q0 + ql;
        const uint64_t idx = q * L + i;
        uint32_t code = (uint32_t)(rnd(SEED_Q_RES, idx) % 20u);
        if (n_src > 0 && L <= SRC_LEN && (q % 2) == 0) {
            const uint64_t src = rnd(SEED_Q_SRC, q) % n_src;
            if (rnd(SEED_Q_SUB, idx) % 10u != 0)
                code = src_code(src, i);
        }
        uint8_t b = (uint8_t)alpha[code];
        if (x_permille && rnd(SEED_Q_X, idx) % 1000u < x_permille)
            b = 'X';
        res[t] = b;
    }
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t j = g; j <= n_seq; j += (uint64_t)gridDim.x * blockDim.x)
        seq_off[j] = j * L;
}

hipError_t launch_synth_queries(uint64_t image_n_keys, uint32_t n_seq, uint32_t length,
                                uint32_t x_permille, uint64_t q0, uint8_t *residues,
                                uint64_t *seq_off, hipStream_t stream)
{
    const uint64_t n_src = (image_n_keys / 4) / SRC_WIN;
    hipLaunchKernelGGL(synth_queries_kernel, dim3(2048), dim3(256), 0, stream, n_src, n_seq, length,
                       x_permille, q0, residues, seq_off);
    return hipGetLastError();
}

}  // namespace kgx
