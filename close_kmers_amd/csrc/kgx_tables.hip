/*
 * kgx_tables.hip -- k-mer -> id tables and /matrix pair counting in HBM.
 *
 *   kgx_kmap   : KmerPegMapping::kmer_to_id_ / kmer_to_family_id_
 *                (kmer.h:84-127; add_mapping kmer.cc:173-210, add_fam_mapping
 *                kmer.cc:212-256) as a CSR over sorted unique k-mers (ids in
 *                insertion order) plus an open-addressing index k-mer -> row
 *   kgx_matrix : MatrixRequest's matrix_proteins_ / distance_ state and its
 *                per-hit rule (matrix_request.cc:83-95,130-163) -- a device
 *                hash of seen ids (first request ordinal) and a device hash
 *                of (id1, id2) -> count, read out ordered as std::map would
 *
 * Building a table is a stable radix sort of (k-mer, id) pairs in insertion
 * order (hipCUB), so per-k-mer lists keep insertion order; the set flavour
 * drops repeats of an id within a list, keeping the first.  Hits are read
 * straight from a context's tiled device result.
 */
#include <hipcub/hipcub.hpp>

#include <memory>
#include <type_traits>
#include <mutex>
#include <vector>

#include "kgx_device.h"
#include "kgx_rt.h"

using namespace kgx;

namespace {

constexpr uint64_t EMPTY64 = ~0ull;
constexpr uint32_t NO_ID = 0xFFFFFFFFu; /* reserved: ids must be below it */

__device__ __forceinline__ uint64_t hslot(uint64_t key, uint64_t mask) { return mix64(key) & mask; }

/* slot of `key`, claiming an empty one if absent; *fresh set when claimed */
__device__ __forceinline__ uint64_t find_or_insert(uint64_t *keys, uint64_t mask, uint64_t key,
                                                   bool &fresh)
{
    uint64_t h = hslot(key, mask);
    for (;;) {
        const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long *>(keys + h),
                                        (unsigned long long)EMPTY64, (unsigned long long)key);
        if (prev == EMPTY64) {
            fresh = true;
            return h;
        }
        if (prev == key) {
            fresh = false;
            return h;
        }
        h = (h + 1) & mask;
    }
}

__device__ __forceinline__ int64_t find(const uint64_t *keys, uint64_t mask, uint64_t key)
{
    if (mask == 0 && keys == nullptr)
        return -1;
    uint64_t h = hslot(key, mask);
    for (;;) {
        const uint64_t k = keys[h];
        if (k == key)
            return (int64_t)h;
        if (k == EMPTY64)
            return -1;
        h = (h + 1) & mask;
    }
}

/* read-only view of a built table */
struct KmapView {
    const uint64_t *hkeys = nullptr; /* index: k-mer per slot */
    const uint32_t *hrow = nullptr;  /* index: row per slot */
    uint64_t hmask = 0;
    const uint64_t *starts = nullptr; /* rows + 1 */
    const uint32_t *vals = nullptr;
    /* the index again, one 16-B slot per bucket: {k-mer lo, hi, list start,
     * list length} -- one random read per probe step instead of three
     * dependent ones (key, row, starts); built when every start fits 32 bits */
    const uint4 *slots = nullptr;
};

__device__ __forceinline__ bool kmap_row(const KmapView &m, uint64_t kmer, uint64_t &a, uint64_t &b)
{
    if (m.slots) {
        uint64_t h = hslot(kmer, m.hmask);
        for (;;) {
            const uint4 e = m.slots[h];
            const uint64_t k = (uint64_t)e.y << 32 | e.x;
            if (k == kmer) {
                a = e.z;
                b = (uint64_t)e.z + e.w;
                return true;
            }
            if (k == EMPTY64)
                return false;
            h = (h + 1) & m.hmask;
        }
    }
    if (!m.hkeys)
        return false;
    const int64_t s = find(m.hkeys, m.hmask, kmer);
    if (s < 0)
        return false;
    const uint32_t r = m.hrow[s];
    a = m.starts[r];
    b = m.starts[r + 1];
    return true;
}

/* the tiled device result of a context (kgx_device_result) */
struct Tiled {
    const uint4 *hot;  /* the hit records (HIT_PACKED16) or plane 0 */
    const uint4 *cold; /* HIT_PLANES: {which_kmer lo, hi, otu, seq} per slot */
    const uint64_t *mask;
    const uint64_t *wbase;
    const uint32_t *tile_seq;
    uint32_t n_seq;
    uint32_t T; /* windows per tile */
    bool packed;
};

/* k-mer and sequence of hit i of `tile` */
__device__ __forceinline__ void hit_key_seq(const Tiled &t, uint64_t tile, uint32_t i, uint64_t &key, uint32_t &seq)
{
    const uint64_t slot = tile * t.T + i;
    if (t.packed) {
        key = HitFields<true>::key(t.hot[slot], t.hot[slot]);
        seq = window_seq(t.wbase, t.tile_seq, tile, hit_window(t.mask, tile, t.T / 64, i));
    } else {
        const uint4 h = t.cold[slot];
        key = (uint64_t)h.y << 32 | h.x;
        seq = h.w;
    }
}

__device__ __forceinline__ uint64_t hit_key(const Tiled &t, uint64_t tile, uint32_t i)
{
    const uint64_t slot = tile * t.T + i;
    if (t.packed)
        return HitFields<true>::key(t.hot[slot], t.hot[slot]);
    const uint4 h = t.cold[slot];
    return (uint64_t)h.y << 32 | h.x;
}

__device__ __forceinline__ uint32_t tile_count(const Tiled &t, uint64_t tile)
{
    const uint64_t W = t.wbase[t.n_seq];
    const uint32_t J = t.T / 64;
    uint32_t c = 0;
    for (uint32_t j = 0; j < J; j++) {
        const uint64_t w = tile * J + j;
        if (64 * w < W)
            c += (uint32_t)__popcll(t.mask[w]);
    }
    return c;
}

/* ---------------- kernels ---------------- */

__global__ void tile_counts_kernel(Tiled t, uint64_t n_tiles, uint32_t *counts)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_tiles)
        counts[i] = tile_count(t, i);
    else if (i == n_tiles)
        counts[i] = 0;
}

/* dense (k-mer, id) pairs of the tiled hits, in (sequence, position) order */
__global__ void hits_to_pairs_kernel(Tiled t, uint64_t n_tiles, const uint32_t *tile_base,
                                     const uint32_t *seq_ids, uint64_t *kmers, uint32_t *ids)
{
    const uint64_t slot = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t tile = slot / t.T;
    const uint32_t i = (uint32_t)(slot % t.T);
    if (tile >= n_tiles || i >= tile_base[tile + 1] - tile_base[tile])
        return;
    uint64_t key;
    uint32_t seq;
    hit_key_seq(t, tile, i, key, seq);
    const uint64_t at = tile_base[tile] + i;
    kmers[at] = key;
    ids[at] = seq_ids[seq];
}

__global__ void expand_rows_kernel(const uint64_t *keys, const uint64_t *starts, uint64_t n_rows,
                                   uint64_t *out)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows)
        return;
    for (uint64_t j = starts[r]; j < starts[r + 1]; j++)
        out[j] = keys[r];
}

__global__ void iota_kernel(uint32_t *p, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        p[i] = (uint32_t)i;
}

__global__ void gather_u64_kernel(const uint64_t *src, const uint32_t *idx, uint64_t n, uint64_t *dst)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        dst[i] = src[idx[i]];
}

/* (k-mer, id) order -> keep[original index] = first of its (k-mer, id) group */
__global__ void first_of_pair_kernel(const uint64_t *k_sorted, const uint32_t *orig, const uint64_t *k1,
                                     const uint32_t *v1, uint64_t n, uint8_t *keep)
{
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n)
        return;
    const uint32_t o = orig[p];
    bool first = true;
    if (p > 0) {
        const uint32_t q = orig[p - 1];
        first = !(k1[q] == k1[o] && v1[q] == v1[o]);
    }
    keep[o] = first;
    (void)k_sorted;
}

__global__ void row_heads_kernel(const uint64_t *k, uint64_t n, uint8_t *head)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        head[i] = (i == 0 || k[i] != k[i - 1]);
}

/* the 16-B index slots from the built index (n_vals < 2^32) */
__global__ void index_slots_kernel(const uint64_t *hkeys, const uint32_t *hrow, const uint64_t *starts, uint64_t cap,
                                   uint4 *slots)
{
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap)
        return;
    const uint64_t k = hkeys[s];
    if (k == EMPTY64) {
        slots[s] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);
        return;
    }
    const uint32_t r = hrow[s];
    const uint64_t a = starts[r], b = starts[r + 1];
    slots[s] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), (uint32_t)a, (uint32_t)(b - a));
}

__global__ void index_insert_kernel(const uint64_t *keys, uint64_t n, uint64_t *hkeys, uint32_t *hrow,
                                    uint64_t mask)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n)
        return;
    bool fresh;
    const uint64_t s = find_or_insert(hkeys, mask, keys[r], fresh);
    hrow[s] = (uint32_t)r;
}

__global__ void lookup_count_kernel(KmapView m, const uint64_t *kmers, uint64_t n, uint64_t *count)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    uint64_t a = 0, b = 0;
    count[i] = kmap_row(m, kmers[i], a, b) ? b - a : 0;
}

__global__ void lookup_ids_kernel(KmapView m, const uint64_t *kmers, uint64_t n, const uint64_t *off,
                                  uint32_t *ids)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    uint64_t a = 0, b = 0;
    if (kmap_row(m, kmers[i], a, b))
        for (uint64_t j = a; j < b; j++)
            ids[off[i] + (j - a)] = m.vals[j];
}

/* --- /lookup rollups (kgx_kmap_rollup) ---
 * Events are the (hit, list entry) pairs of LookupRequest::on_hit
 * (lookup_request.cc:446-482), numbered in hit order, then list order: event
 * e of hit h is eoff[h] + j for list entry j.  Hits are in (sequence,
 * position) order, so a sequence's events are one contiguous range; one wave
 * per sequence groups its events by id in LDS, summing each id's f32 weights
 * strictly in event order (the reference's sum, hit by hit), and emits one row
 * per id in first-touch order. */

constexpr uint32_t kNoEvent = 0xFFFFFFFFu;

/* the wave's index in the grid, wave-uniform */
__device__ __forceinline__ uint64_t wave_index()
{
    return (uint64_t)blockIdx.x * 4 + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

/* Passes 1 and 2 take kRollTiles tiles per wave and their hits densely, one
 * hit per lane: about a quarter of a batch's windows hit, so a lane per
 * window would leave three in four idle in a kernel bound by its dependent
 * reads (r5u: 106 us per 7.5M-residue shard with a wave per mask word). */
constexpr uint32_t kRollTiles = 2;
constexpr uint32_t kRollMaxT = 512; /* windows per tile (probe_j <= 8) */

/* the wave's hits in order (tile, then window): LDS entry r = the hit's slot
 * and window offsets from the wave's first tile; returns the count */
__device__ __forceinline__ uint32_t roll_list(const Tiled &t, uint64_t tile0, uint64_t n_tiles, uint64_t W,
                                              uint16_t *slot_off, uint16_t *win_off)
{
    const uint32_t J = t.T / 64, lane = lane_id();
    uint32_t n = 0;
    for (uint32_t k = 0; k < kRollTiles && tile0 + k < n_tiles; k++) {
        uint32_t in_tile = 0;
        for (uint32_t j = 0; j < J; j++) {
            const uint64_t w = (tile0 + k) * J + j;
            const uint64_t m = 64 * w < W ? t.mask[w] : 0ull;
            if ((m >> lane) & 1ull) {
                const uint32_t r = n + lanes_below(m);
                slot_off[r] = (uint16_t)(k * t.T + in_tile + lanes_below(m));
                win_off[r] = (uint16_t)(k * t.T + 64 * j + lane);
            }
            const uint32_t pc = (uint32_t)__popcll(m);
            n += pc;
            in_tile += pc;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return n;
}

/* Pass 1: for each hit of the wave's tiles its sequence, list start and
 * length (0 for an unmapped k-mer) at its slot; the wave's event total.  Wave
 * n_waves writes the scan's last element, 0; the grid also resets the
 * sequences' event ranges and row counts for the later passes. */
__global__ __launch_bounds__(256) void rollup_tiles_kernel(Tiled t, uint64_t n_tiles, uint64_t n_waves, KmapView m,
                                                           uint32_t *hseq, uint64_t *hstart, uint32_t *hlen,
                                                           uint64_t *wcount, uint32_t *sfirst, uint32_t *send,
                                                           uint32_t *rowcnt)
{
    extern __shared__ uint16_t roll_lds[]; /* 4 waves x (slot, window) x kRollTiles * T */
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= t.n_seq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        sfirst[i] = kNoEvent;
        send[i] = 0;
        rowcnt[i] = 0;
    }
    const uint64_t v = wave_index();
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    if (v >= n_waves) {
        if (v == n_waves && lane == 0)
            wcount[n_waves] = 0;
        return;
    }
    const uint64_t tile0 = v * kRollTiles, W = t.wbase[t.n_seq];
    uint16_t *so = roll_lds + wv * 2 * kRollTiles * t.T, *wo = so + kRollTiles * t.T;
    const uint32_t n = roll_list(t, tile0, n_tiles, W, so, wo);
    uint64_t ev = 0;
    for (uint32_t r = lane; r < n; r += 64) {
        const uint64_t slot = tile0 * t.T + so[r];
        uint64_t key;
        uint32_t seq;
        if (t.packed) {
            const uint64_t g = tile0 * t.T + wo[r];
            key = HitFields<true>::key(t.hot[slot], t.hot[slot]);
            seq = window_seq(t.wbase, t.tile_seq, g / t.T, g);
        } else {
            const uint4 h = t.cold[slot];
            key = (uint64_t)h.y << 32 | h.x;
            seq = h.w;
        }
        uint64_t a = 0, b = 0;
        const uint64_t len = kmap_row(m, key, a, b) ? b - a : 0;
        hseq[slot] = seq;
        hstart[slot] = a;
        hlen[slot] = (uint32_t)len;
        ev += len;
    }
    for (int o = 32; o > 0; o >>= 1)
        ev += __shfl_xor(ev, o);
    if (lane == 0)
        wcount[v] = ev;
}

/* Pass 2, the same waves: the events of their hits, numbered from the wave's
 * scanned base in hit order, then list order: the id and the hit's weight
 * 1.0f / (float)|list| (lookup_request.cc:459); each sequence's event range
 * [sfirst, send) by atomics at the first and last lane of each run of one
 * sequence in a 64-hit chunk.  Writes nothing when the batch has more than
 * cap events (the host runs the passes again at the true size). */
__global__ __launch_bounds__(256) void rollup_events_kernel(Tiled t, uint64_t n_tiles, uint64_t n_waves,
                                                            const uint32_t *hseq, const uint64_t *hstart,
                                                            const uint32_t *hlen, const uint64_t *vbase,
                                                            const uint32_t *vals, uint64_t cap, uint32_t *ev_id,
                                                            float *ev_w, uint32_t *sfirst, uint32_t *send)
{
    extern __shared__ uint16_t roll_lds[];
    const uint64_t v = wave_index();
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    if (v >= n_waves || vbase[n_waves] > cap)
        return;
    uint64_t e0 = vbase[v];
    if (vbase[v + 1] == e0)
        return;
    const uint64_t tile0 = v * kRollTiles, W = t.wbase[t.n_seq];
    uint16_t *so = roll_lds + wv * 2 * kRollTiles * t.T, *wo = so + kRollTiles * t.T;
    const uint32_t n = roll_list(t, tile0, n_tiles, W, so, wo);
    for (uint32_t r0 = 0; r0 < n; r0 += 64) {
        const uint32_t r = r0 + lane;
        uint64_t len = 0, a = 0;
        uint32_t seq = 0;
        if (r < n) {
            const uint64_t slot = tile0 * t.T + so[r];
            len = hlen[slot];
            a = hstart[slot];
            seq = hseq[slot];
        }
        uint64_t incl = len;
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t x = __shfl_up(incl, o);
            if (lane >= (uint32_t)o)
                incl += x;
        }
        const uint64_t e = e0 + incl - len;
        if (len) {
            const float wt = 1.0f / (float)len;
            for (uint64_t q = 0; q < len; q++) {
                ev_id[e + q] = vals[a + q];
                ev_w[e + q] = wt;
            }
        }
        /* the lanes with events: each one's neighbours among them */
        const uint64_t act = __ballot(len != 0);
        const uint64_t below = act & ((1ull << lane) - 1ull);
        const uint64_t above = lane == 63 ? 0ull : act & ~((2ull << lane) - 1ull);
        const uint32_t prev = below ? 63u - (uint32_t)__builtin_clzll(below) : lane;
        const uint32_t next = above ? (uint32_t)__builtin_ctzll(above) : lane;
        const uint32_t pseq = __shfl(seq, (int)prev), nseq = __shfl(seq, (int)next);
        if (len) {
            if (!below || pseq != seq)
                atomicMin(sfirst + seq, (uint32_t)e);
            if (!above || nseq != seq)
                atomicMax(send + seq, (uint32_t)(e + len));
        }
        e0 += __shfl(incl, 63);
    }
}

/* Pass 3, one wave per sequence: its events [sfirst, send) in chunks of 64.
 * Per chunk, the distinct ids one at a time, lowest lane first (ballot): the
 * id's table entry in LDS is found or added (first event = that lane's), and
 * its lanes' weights are added to the entry's f32 sum in lane order -- so
 * every sum is taken in event order, as the reference adds them hit by hit,
 * and entries are added in first-touch order.  Rows go to rows2[sfirst + q]
 * for the q-th entry.  A sequence with more distinct ids than one table pass
 * holds is taken in P id classes, each class's rows placed at their first
 * event's position (flag, rowdata) and compacted in event order after. */
constexpr uint32_t kRollH = 256;    /* LDS table slots per wave */
constexpr uint32_t kRollFill = 192; /* ids per table pass */

__device__ __forceinline__ uint32_t roll_hash(uint32_t id) { return (id * 0x9E3779B1u) >> 24; }
__device__ __forceinline__ uint32_t roll_class(uint32_t id, uint32_t P) { return ((id * 0x85EBCA6Bu) >> 13) & (P - 1); }

__global__ __launch_bounds__(256) void rollup_group_kernel(uint32_t n_seq, const uint32_t *sfirst,
                                                           const uint32_t *send, const uint32_t *ev_id,
                                                           const float *ev_w, int family, const uint64_t *n_events,
                                                           uint64_t cap, uint8_t *flag, uint4 *rowdata, uint4 *rows2,
                                                           uint32_t *rowcnt)
{
    __shared__ uint32_t hk[4][kRollH], hc[4][kRollH], hf[4][kRollH], hl[4][kRollFill];
    __shared__ float hw[4][kRollH];
    const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
    const uint32_t s = blockIdx.x * 4 + wv;
    if (s >= n_seq || *n_events > cap)
        return;
    const uint32_t f = sfirst[s], l = send[s];
    if (f == kNoEvent || l <= f) {
        if (lane == 0)
            rowcnt[s] = 0;
        return;
    }
    uint32_t *K = hk[wv], *C = hc[wv], *F = hf[wv], *L = hl[wv];
    float *Wt = hw[wv];
    auto row = [&](uint32_t h) {
        return family ? make_uint4(K[h], C[h], C[h], __float_as_uint(Wt[h])) : make_uint4(K[h], C[h], 0u, 0u);
    };
    uint32_t P = 1, nrows = 0;
    for (;;) {
        bool ok = true;
        for (uint32_t p = 0; p < P && ok; p++) {
            for (uint32_t i = lane; i < kRollH; i += 64)
                K[i] = NO_ID;
            __builtin_amdgcn_wave_barrier();
            uint32_t used = 0;
            for (uint32_t e = f; e < l && ok; e += 64) {
                const uint32_t i = e + lane;
                const bool valid = i < l;
                const uint32_t id = valid ? ev_id[i] : NO_ID;
                const float w = valid ? ev_w[i] : 0.0f;
                const bool mine = valid && roll_class(id, P) == p;
                uint64_t rem = __ballot(mine);
                while (rem) {
                    const uint32_t ld = (uint32_t)__builtin_ctzll(rem);
                    const uint32_t lid = (uint32_t)__builtin_amdgcn_readlane((int)id, (int)ld);
                    const uint64_t grp = __ballot(mine && id == lid);
                    rem &= ~grp;
                    uint32_t h = roll_hash(lid);
                    uint32_t kh;
                    while ((kh = K[h]) != NO_ID && kh != lid)
                        h = (h + 1) & (kRollH - 1);
                    const bool fresh = kh == NO_ID;
                    if (fresh && used == kRollFill) {
                        ok = false; /* too many ids for one pass: classes */
                        break;
                    }
                    float sum = fresh ? 0.0f : Wt[h];
                    const uint32_t cnt = (fresh ? 0u : C[h]) + (uint32_t)__popcll(grp);
                    for (uint64_t g = grp; g; g &= g - 1) {
                        const int b = (int)__builtin_ctzll(g);
                        sum += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), b)); /* hit by hit */
                    }
                    if (lane == 0) {
                        if (fresh) {
                            K[h] = lid;
                            F[h] = e + ld - f;
                            L[used] = h;
                        }
                        C[h] = cnt;
                        Wt[h] = sum;
                    }
                    used += fresh;
                    __builtin_amdgcn_wave_barrier();
                }
            }
            if (!ok)
                break;
            if (P == 1) {
                for (uint32_t q = lane; q < used; q += 64)
                    rows2[f + q] = row(L[q]);
                nrows = used;
            } else {
                for (uint32_t q = lane; q < used; q += 64) {
                    const uint32_t h = L[q];
                    flag[f + F[h]] = 1;
                    rowdata[f + F[h]] = row(h);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (ok)
            break;
        P *= 2;
        for (uint32_t i = f + lane; i < l; i += 64)
            flag[i] = 0;
    }
    if (P > 1) {
        /* the classes' rows in first-event order (this wave's own stores) */
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        uint32_t rank = 0;
        for (uint32_t e = f; e < l; e += 64) {
            const uint32_t i = e + lane;
            const bool fl = i < l && flag[i];
            const uint64_t bm = __ballot(fl);
            if (fl)
                rows2[f + rank + lanes_below(bm)] = rowdata[i];
            rank += (uint32_t)__popcll(bm);
        }
        nrows = rank;
    }
    if (lane == 0)
        rowcnt[s] = nrows;
}

/* Pass 4, one wave per sequence: its rows and offset into the mapped host
 * arrays (rows at off[s]); the last wave adds off[n] */
__global__ __launch_bounds__(256) void rollup_emit_kernel(uint32_t n_seq, const uint32_t *sfirst,
                                                          const uint32_t *rowcnt, const uint64_t *off,
                                                          const uint4 *rows2, const uint64_t *n_events, uint64_t cap,
                                                          uint4 *h_rows, uint64_t *h_off, uint64_t *h_nrows)
{
    const uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
    if (s > n_seq || *n_events > cap)
        return;
    const uint64_t o = off[s];
    if (lane == 0) {
        h_off[s] = o;
        if (s == n_seq)
            *h_nrows = o;
    }
    if (s == n_seq)
        return;
    const uint32_t c = rowcnt[s], f = sfirst[s];
    for (uint32_t r = lane; r < c; r += 64)
        h_rows[o + r] = rows2[f + r];
}

/* Exclusive sum of in[0..n) into out[0..n) by one workgroup, and out[n-1]
 * into *last_mapped (host-mapped) when given: the rollup's two scans for a
 * small batch (up to 8,192 values: 8 loads per thread, all in flight at
 * once) in one launch each instead of hipcub's two (look-back init + scan)
 * and the copy of the event total (r8: a 1-MiB /lookup piece ran 15
 * kernels, and at 16 concurrent pieces the chip's capacity was set by
 * launches, not by their work; for 25k values -- a C2 lookup shard -- one
 * workgroup was 0.28 ms slower per call than hipcub) */
constexpr uint32_t kScanOnePer = 8;
constexpr uint64_t kScanOneMax = 1024 * kScanOnePer; /* past it hipcub's multi-block scan is faster */

template <typename T>
__global__ __launch_bounds__(1024) void scan_one_kernel(const T *__restrict__ in, uint64_t n,
                                                        uint64_t *__restrict__ out, uint64_t *last_mapped)
{
    __shared__ uint64_t wsum[16];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint64_t per = (n + 1023) / 1024; /* <= kScanOnePer */
    const uint64_t a = min(n, (uint64_t)t * per), b = min(n, a + per);
    uint64_t v[kScanOnePer], own = 0; /* every load issued before the first is used */
#pragma unroll
    for (uint32_t k = 0; k < kScanOnePer; k++)
        v[k] = a + k < b ? (uint64_t)in[a + k] : 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanOnePer; k++)
        own += v[k];
    uint64_t x = own; /* inclusive scan over the wave */
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d);
        if (lane >= d)
            x += y;
    }
    if (lane == 63)
        wsum[wave] = x;
    __syncthreads();
    uint64_t run = x - own;
    for (uint32_t w = 0; w < wave; w++)
        run += wsum[w];
#pragma unroll
    for (uint32_t k = 0; k < kScanOnePer; k++) {
        const uint64_t i = a + k;
        if (i < b) {
            out[i] = run;
            if (i == n - 1 && last_mapped)
                *last_mapped = run;
            run += v[k];
        }
    }
}

/* --- /matrix --- */

__global__ void seen_insert_kernel(const uint32_t *ids, uint32_t n, uint64_t base, uint64_t *skeys,
                                   uint64_t *sord, uint64_t mask, unsigned long long *used)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n)
        return;
    bool fresh;
    const uint64_t h = find_or_insert(skeys, mask, ids[s], fresh);
    if (fresh)
        atomicAdd(used, 1ull);
    atomicMin(reinterpret_cast<unsigned long long *>(sord + h), (unsigned long long)(base + s));
}

__global__ void rehash_kernel(const uint64_t *okeys, const uint64_t *ovals, uint64_t ocap, uint64_t *nkeys,
                              uint64_t *nvals, uint64_t nmask)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ocap || okeys[i] == EMPTY64)
        return;
    bool fresh;
    const uint64_t h = find_or_insert(nkeys, nmask, okeys[i], fresh);
    nvals[h] = ovals[i];
}

/* Grid size of the reducing kernels below: a fixed grid of grid-stride
 * blocks, each adding its total once, so the shared counter takes a few
 * thousand atomics rather than one per wave (one per wave measured 0.39 ms
 * for a 3M-window /matrix batch: the same-address atomics serialise) */
constexpr uint32_t kReduceBlocks = 2048;

__device__ __forceinline__ uint64_t block_sum(uint64_t v)
{
    __shared__ uint64_t part[4]; /* 256 threads = 4 waves */
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o);
    if (lane_id() == 0)
        part[threadIdx.x >> 6] = v;
    __syncthreads();
    const uint64_t tot = part[0] + part[1] + part[2] + part[3];
    __syncthreads();
    return tot;
}

__global__ __launch_bounds__(256) void matrix_events_kernel(Tiled t, uint64_t n_tiles, KmapView m,
                                                            unsigned long long *events)
{
    const uint64_t n_slots = n_tiles * t.T;
    uint64_t ev = 0;
    for (uint64_t slot = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; slot < n_slots;
         slot += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t tile = slot / t.T;
        const uint32_t i = (uint32_t)(slot % t.T);
        if (i < tile_count(t, tile)) {
            uint64_t a = 0, b = 0;
            if (kmap_row(m, hit_key(t, tile, i), a, b))
                ev += b - a;
        }
    }
    ev = block_sum(ev);
    if (threadIdx.x == 0 && ev)
        atomicAdd(events, (unsigned long long)ev);
}

__global__ void matrix_pairs_kernel(Tiled t, uint64_t n_tiles, KmapView m, const uint32_t *seq_ids,
                                    uint64_t base, const uint64_t *skeys, const uint64_t *sord,
                                    uint64_t smask, uint64_t *pkeys, uint64_t *pcount, uint64_t pmask,
                                    unsigned long long *used)
{
    const uint64_t slot = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t tile = slot / t.T;
    const uint32_t i = (uint32_t)(slot % t.T);
    if (tile >= n_tiles || i >= tile_count(t, tile))
        return;
    uint64_t key;
    uint32_t seq;
    hit_key_seq(t, tile, i, key, seq);
    uint64_t a = 0, b = 0;
    if (!kmap_row(m, key, a, b))
        return; /* matrix_request.cc:159 reports "no mapping" on stderr */
    const uint32_t e = seq_ids[seq];
    const uint64_t my_ord = base + seq;
    for (uint64_t j = a; j < b; j++) {
        const uint32_t f = m.vals[j];
        if (f == e)
            continue;
        const int64_t q = find(skeys, smask, f);
        if (q < 0 || sord[q] > my_ord)
            continue; /* not in matrix_proteins_ yet */
        bool fresh;
        const uint64_t p = find_or_insert(pkeys, pmask, ((uint64_t)e << 32) | f, fresh);
        /* new pairs counted once per wave (the active lanes of this iteration) */
        const uint64_t fm = __ballot(fresh);
        if (fm && lane_id() == (uint32_t)(__ffsll((unsigned long long)fm) - 1))
            atomicAdd(used, (unsigned long long)__popcll(fm));
        atomicAdd(reinterpret_cast<unsigned long long *>(pcount + p), 1ull);
    }
}

/* the occupied buckets of the pair table, in any order (sorted afterwards):
 * each block counts its grid-stride share, takes one range of the output
 * with one atomic, and writes its pairs at block-scan offsets */
__global__ __launch_bounds__(256) void compact_pairs_kernel(const uint64_t *pkeys, const uint64_t *pcount,
                                                            uint64_t cap, uint64_t *okeys, uint64_t *ocount,
                                                            unsigned long long *n)
{
    __shared__ uint32_t wave_tot[4];
    __shared__ unsigned long long block_base;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t first = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t mine = 0;
    for (uint64_t i = first; i < cap; i += stride)
        mine += pkeys[i] != EMPTY64;
    /* exclusive scan of the threads' counts: within the wave, then over waves */
    uint32_t incl = mine;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o);
        if (lane_id() >= (uint32_t)o)
            incl += v;
    }
    if (lane_id() == 63)
        wave_tot[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint32_t before = incl - mine;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); w++)
        before += wave_tot[w];
    if (threadIdx.x == 0) {
        const uint32_t tot = wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
        block_base = tot ? atomicAdd(n, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    uint64_t at = block_base + before;
    for (uint64_t i = first; i < cap; i += stride)
        if (pkeys[i] != EMPTY64) {
            okeys[at] = pkeys[i];
            ocount[at] = pcount[i];
            at++;
        }
}

inline dim3 grid_for(uint64_t n, uint32_t block = 256) { return dim3((uint32_t)((n + block - 1) / block)); }

uint64_t pow2_at_least(uint64_t n)
{
    uint64_t c = 1024;
    while (c < n)
        c <<= 1;
    return c;
}

/* hipCUB temp storage helper */
struct CubTemp {
    DevBuf buf;
    size_t bytes = 0;
};

}  // namespace

/* ------------------------------------------------------------------------ */

/* buffers and a stream of one kgx_kmap_lookup call: a map serves concurrent
 * lookups (the router's workers hold the mapping's read lock), each on a
 * scratch of its own taken from the map's free list -- no allocation and no
 * shared stream per call (a hipFree per call serialised the workers) */
struct KmapScratch {
    hipStream_t st = nullptr;
    DevBuf k, c, ids;
    PinnedVec<uint64_t> cnt;
};

struct kgx_kmap {
    int device = 0;
    int mode = KGX_KMAP_APPEND;
    hipStream_t stream = nullptr;
    uint64_t n_rows = 0, n_vals = 0, hcap = 0;
    uint32_t max_id = 0; /* the largest id added (kgx_kmap_rollup's key width) */
    DevBuf keys, starts, vals, hkeys, hrow, slots;
    std::mutex scratch_mu;
    std::vector<std::unique_ptr<KmapScratch>> scratch_free;
    KmapView view() const
    {
        KmapView v;
        if (n_rows) {
            v.hkeys = hkeys.as<uint64_t>();
            v.hrow = hrow.as<uint32_t>();
            v.hmask = hcap - 1;
            v.slots = slots.p ? slots.as<uint4>() : nullptr;
            v.starts = starts.as<uint64_t>();
            v.vals = vals.as<uint32_t>();
        }
        return v;
    }
};

struct kgx_matrix {
    kgx_kmap *map = nullptr;
    uint64_t base = 0; /* request ordinal of the next sequence */
    uint64_t scap = 0, sused = 0, pcap = 0, pused = 0;
    DevBuf skeys, sord, pkeys, pcount, ids, counter, tmp_keys, tmp_count;
    CubTemp cub;
    std::vector<kgx_pair_count> result;
};

namespace {

/* Rebuild `m` from d_k/d_v (n pairs: the old rows expanded, then the new
 * pairs, in insertion order).  Consumes the buffers' contents. */
int kmap_rebuild(kgx_kmap *m, DevBuf &d_k, DevBuf &d_v, uint64_t n, hipStream_t st)
{
    if (n == 0)
        return KGX_OK;
    DevBuf k1, v1, tmp;
    HIP_TRY(k1.reserve(n * 8));
    HIP_TRY(v1.reserve(n * 4));
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, d_k.as<uint64_t>(), k1.as<uint64_t>(),
                                               d_v.as<uint32_t>(), v1.as<uint32_t>(), (int)n, 0, 64, st));
    HIP_TRY(tmp.reserve(tb));
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, d_k.as<uint64_t>(), k1.as<uint64_t>(),
                                               d_v.as<uint32_t>(), v1.as<uint32_t>(), (int)n, 0, 64, st));
    /* k1/v1: by k-mer, insertion order within a k-mer (LSD radix sort is stable) */
    if (m->mode == KGX_KMAP_SET) {
        /* order (k-mer, id, insertion): sort indices by id, then by k-mer */
        DevBuf idx, v2, i2, kg, k3, i3, keep;
        HIP_TRY(idx.reserve(n * 4));
        HIP_TRY(v2.reserve(n * 4));
        HIP_TRY(i2.reserve(n * 4));
        HIP_TRY(kg.reserve(n * 8));
        HIP_TRY(k3.reserve(n * 8));
        HIP_TRY(i3.reserve(n * 4));
        HIP_TRY(keep.reserve(n));
        hipLaunchKernelGGL(iota_kernel, grid_for(n), dim3(256), 0, st, idx.as<uint32_t>(), n);
        tb = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, v1.as<uint32_t>(), v2.as<uint32_t>(),
                                                   idx.as<uint32_t>(), i2.as<uint32_t>(), (int)n, 0, 32, st));
        HIP_TRY(tmp.reserve(tb));
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, v1.as<uint32_t>(), v2.as<uint32_t>(),
                                                   idx.as<uint32_t>(), i2.as<uint32_t>(), (int)n, 0, 32, st));
        hipLaunchKernelGGL(gather_u64_kernel, grid_for(n), dim3(256), 0, st, k1.as<uint64_t>(),
                           i2.as<uint32_t>(), n, kg.as<uint64_t>());
        tb = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kg.as<uint64_t>(), k3.as<uint64_t>(),
                                                   i2.as<uint32_t>(), i3.as<uint32_t>(), (int)n, 0, 64, st));
        HIP_TRY(tmp.reserve(tb));
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, kg.as<uint64_t>(), k3.as<uint64_t>(),
                                                   i2.as<uint32_t>(), i3.as<uint32_t>(), (int)n, 0, 64, st));
        hipLaunchKernelGGL(first_of_pair_kernel, grid_for(n), dim3(256), 0, st, k3.as<uint64_t>(),
                           i3.as<uint32_t>(), k1.as<uint64_t>(), v1.as<uint32_t>(), n, keep.as<uint8_t>());
        /* keep the firsts, in (k-mer, insertion) order */
        DevBuf nsel;
        HIP_TRY(nsel.reserve(8));
        tb = 0;
        HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, k1.as<uint64_t>(), keep.as<uint8_t>(),
                                              d_k.as<uint64_t>(), nsel.as<uint64_t>(), (int)n, st));
        HIP_TRY(tmp.reserve(tb));
        HIP_TRY(hipcub::DeviceSelect::Flagged(tmp.p, tb, k1.as<uint64_t>(), keep.as<uint8_t>(),
                                              d_k.as<uint64_t>(), nsel.as<uint64_t>(), (int)n, st));
        HIP_TRY(hipcub::DeviceSelect::Flagged(tmp.p, tb, v1.as<uint32_t>(), keep.as<uint8_t>(),
                                              d_v.as<uint32_t>(), nsel.as<uint64_t>(), (int)n, st));
        uint64_t kept = 0;
        HIP_TRY(hipMemcpyAsync(&kept, nsel.p, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        n = kept;
        std::swap(k1, d_k);
        std::swap(v1, d_v);
    }
    /* rows: unique k-mers and their starts */
    DevBuf head, nsel;
    HIP_TRY(head.reserve(n));
    HIP_TRY(nsel.reserve(8));
    hipLaunchKernelGGL(row_heads_kernel, grid_for(n), dim3(256), 0, st, k1.as<uint64_t>(), n,
                       head.as<uint8_t>());
    HIP_TRY(m->keys.reserve(n * 8));
    HIP_TRY(m->starts.reserve((n + 1) * 8));
    tb = 0;
    HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, k1.as<uint64_t>(), head.as<uint8_t>(),
                                          m->keys.as<uint64_t>(), nsel.as<uint64_t>(), (int)n, st));
    size_t tb2 = 0;
    hipcub::CountingInputIterator<uint64_t> cnt(0);
    HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb2, cnt, head.as<uint8_t>(), m->starts.as<uint64_t>(),
                                          nsel.as<uint64_t>(), (int)n, st));
    HIP_TRY(tmp.reserve(std::max(tb, tb2)));
    HIP_TRY(hipcub::DeviceSelect::Flagged(tmp.p, tb, k1.as<uint64_t>(), head.as<uint8_t>(),
                                          m->keys.as<uint64_t>(), nsel.as<uint64_t>(), (int)n, st));
    HIP_TRY(hipcub::DeviceSelect::Flagged(tmp.p, tb2, cnt, head.as<uint8_t>(), m->starts.as<uint64_t>(),
                                          nsel.as<uint64_t>(), (int)n, st));
    uint64_t rows = 0;
    HIP_TRY(hipMemcpyAsync(&rows, nsel.p, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipMemcpyAsync(m->starts.as<uint64_t>() + rows, &n, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(m->vals.reserve(n * 4));
    HIP_TRY(hipMemcpyAsync(m->vals.p, v1.p, n * 4, hipMemcpyDeviceToDevice, st));
    /* index k-mer -> row */
    const uint64_t cap = pow2_at_least(2 * rows);
    HIP_TRY(m->hkeys.reserve(cap * 8));
    HIP_TRY(m->hrow.reserve(cap * 4));
    HIP_TRY(hipMemsetAsync(m->hkeys.p, 0xFF, cap * 8, st));
    hipLaunchKernelGGL(index_insert_kernel, grid_for(rows), dim3(256), 0, st, m->keys.as<uint64_t>(), rows,
                       m->hkeys.as<uint64_t>(), m->hrow.as<uint32_t>(), cap - 1);
    if (n < (1ull << 32)) {
        HIP_TRY(m->slots.reserve(cap * 16));
        hipLaunchKernelGGL(index_slots_kernel, grid_for(cap), dim3(256), 0, st, m->hkeys.as<uint64_t>(),
                           m->hrow.as<uint32_t>(), m->starts.as<uint64_t>(), cap, m->slots.as<uint4>());
    } else {
        m->slots.release();
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
    m->n_rows = rows;
    m->n_vals = n;
    m->hcap = cap;
    return KGX_OK;
}

/* old rows expanded into d_k/d_v[0, n_vals); capacity for `extra` more */
int kmap_expand(kgx_kmap *m, DevBuf &d_k, DevBuf &d_v, uint64_t extra, hipStream_t st)
{
    const uint64_t n = m->n_vals + extra;
    HIP_TRY(d_k.reserve(std::max<uint64_t>(n, 1) * 8));
    HIP_TRY(d_v.reserve(std::max<uint64_t>(n, 1) * 4));
    if (m->n_rows) {
        hipLaunchKernelGGL(expand_rows_kernel, grid_for(m->n_rows), dim3(256), 0, st, m->keys.as<uint64_t>(),
                           m->starts.as<uint64_t>(), m->n_rows, d_k.as<uint64_t>());
        HIP_TRY(hipMemcpyAsync(d_v.p, m->vals.p, m->n_vals * 4, hipMemcpyDeviceToDevice, st));
    }
    return KGX_OK;
}

Tiled tiled_of(const kgx_ctx *c)
{
    Tiled t;
    t.hot = c->hits.as<uint4>();
    t.cold = c->hits.as<uint4>() + c->hit_slots;
    t.mask = c->hit_mask.as<uint64_t>();
    t.wbase = c->wbase.as<uint64_t>();
    t.tile_seq = c->tile_seq.as<uint32_t>();
    t.n_seq = c->n_seq;
    t.T = c->tile_windows;
    t.packed = c->hit_format == HIT_PACKED16;
    return t;
}

int check_ctx_hits(kgx_ctx *c)
{
    if (!c || !c->img)
        return fail(KGX_EINVAL, "null context");
    if (!c->have_hits)
        return fail(KGX_EINVAL, "the context has no batch with hits (want KGX_WANT_HITS)");
    return KGX_OK;
}

int upload_ids(DevBuf &d, const uint32_t *ids, uint64_t n, hipStream_t st)
{
    for (uint64_t i = 0; i < n; i++)
        if (ids[i] == NO_ID)
            return fail(KGX_EINVAL, "id 0xFFFFFFFF is reserved");
    HIP_TRY(d.reserve(std::max<uint64_t>(n, 1) * 4));
    HIP_TRY(hipMemcpyAsync(d.p, ids, n * 4, hipMemcpyHostToDevice, st));
    return KGX_OK;
}

}  // namespace

namespace kgx {

namespace {

/* rollup pass 1 on c's stream: per mask word its hits' sequence, list start
 * and length per slot and its event total; the words' event bases by a scan; the
 * total E into h_n[0] by a device store (a DMA copy would queue behind other
 * contexts' uploads) */
/* pass 1's buffers for c's planned batch */
int rollup_reserve(kgx_ctx *c, RollupScratch &r)
{
    const uint32_t n = c->n_seq;
    const uint64_t nt = c->max_tiles, n_slots = nt * c->tile_windows, nw = (nt + kRollTiles - 1) / kRollTiles;
    HIP_TRY(r.hseq.reserve(n_slots * 4));
    HIP_TRY(r.hstart.reserve(n_slots * 8));
    HIP_TRY(r.hlen.reserve(n_slots * 4));
    HIP_TRY(r.tcount.reserve((nw + 1) * 8));
    HIP_TRY(r.tbase.reserve((nw + 1) * 8));
    HIP_TRY(r.sfirst.reserve((n + 1) * 4));
    HIP_TRY(r.send.reserve((n + 1) * 4));
    HIP_TRY(r.rowcnt.reserve((n + 1) * 4));
    HIP_TRY(r.rowoff.reserve((n + 1) * 8));
    return KGX_OK;
}

int rollup_tiles(kgx_kmap *m, kgx_ctx *c, RollupScratch &r)
{
    hipStream_t st = c->stream;
    const Tiled t = tiled_of(c);
    if (t.T > kRollMaxT)
        return fail(KGX_EINVAL, "rollup: tiles of more than 512 windows");
    const uint32_t n = c->n_seq;
    const uint64_t nt = c->max_tiles, nw = (nt + kRollTiles - 1) / kRollTiles;
    const KmapView view = m->view();
    if (int rc = rollup_reserve(c, r))
        return rc;
    const dim3 wave_grid((uint32_t)((nw + 1 + 3) / 4));
    const uint32_t lds = 4 * 2 * kRollTiles * t.T * sizeof(uint16_t);
    hipLaunchKernelGGL(rollup_tiles_kernel, wave_grid, dim3(256), lds, st, t, nt, nw, view, r.hseq.as<uint32_t>(),
                       r.hstart.as<uint64_t>(), r.hlen.as<uint32_t>(), r.tcount.as<uint64_t>(),
                       r.sfirst.as<uint32_t>(), r.send.as<uint32_t>(), r.rowcnt.as<uint32_t>());
    void *dn = nullptr;
    HIP_TRY(r.h_n.device_ptr(0, &dn));
    if (nw + 1 <= kScanOneMax) { /* one launch: the scan and E into h_n[0] */
        hipLaunchKernelGGL(scan_one_kernel<uint64_t>, dim3(1), dim3(1024), 0, st, r.tcount.as<uint64_t>(), nw + 1,
                           r.tbase.as<uint64_t>(), static_cast<uint64_t *>(dn));
        HIP_TRY(hipGetLastError());
        return KGX_OK;
    }
    size_t tb = 0, tb2 = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, r.tcount.as<uint64_t>(), r.tbase.as<uint64_t>(),
                                             (int)(nw + 1), st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, r.rowcnt.as<uint32_t>(), r.rowoff.as<uint64_t>(),
                                             (int)(n + 1), st));
    HIP_TRY(r.tmp.reserve(std::max(tb, tb2)));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(r.tmp.p, tb, r.tcount.as<uint64_t>(), r.tbase.as<uint64_t>(),
                                             (int)(nw + 1), st));
    HIP_TRY(launch_copy_to_host(dn, r.tbase.as<uint64_t>() + nw, 8, 1, st));
    return KGX_OK;
}

/* rollup passes 2-4 on c's stream, sized for `cap` events (the device's total
 * E <= cap, else the kernels write nothing and the host runs them again at
 * E): the events in hit order with each sequence's range, one wave per
 * sequence grouping them by id in LDS, the rows' offsets by a scan, and the
 * rows and offsets stored straight into the mapped host arrays */
int rollup_rows(kgx_kmap *m, kgx_ctx *c, RollupScratch &r, int mode, uint64_t cap)
{
    hipStream_t st = c->stream;
    const uint32_t n = c->n_seq;
    const Tiled t = tiled_of(c);
    const uint64_t nt = c->max_tiles, nw = (nt + kRollTiles - 1) / kRollTiles;
    const KmapView view = m->view();
    const dim3 wave_grid((uint32_t)((nw + 1 + 3) / 4)), seq_grid((n + 1 + 3) / 4);
    const uint64_t *d_E = r.tbase.as<uint64_t>() + nw;
    HIP_TRY(r.ev_id.reserve(cap * 4));
    HIP_TRY(r.ev_w.reserve(cap * 4));
    HIP_TRY(r.flag.reserve(cap));
    HIP_TRY(r.rowdata.reserve(cap * 16));
    HIP_TRY(r.rows2.reserve(cap * 16));
    HIP_TRY(r.h_rows.resize(cap));
    const uint32_t lds = 4 * 2 * kRollTiles * t.T * sizeof(uint16_t);
    hipLaunchKernelGGL(rollup_events_kernel, wave_grid, dim3(256), lds, st, t, nt, nw, r.hseq.as<uint32_t>(),
                       r.hstart.as<uint64_t>(), r.hlen.as<uint32_t>(), r.tbase.as<uint64_t>(), view.vals, cap,
                       r.ev_id.as<uint32_t>(), r.ev_w.as<float>(), r.sfirst.as<uint32_t>(), r.send.as<uint32_t>());
    hipLaunchKernelGGL(rollup_group_kernel, seq_grid, dim3(256), 0, st, n, r.sfirst.as<uint32_t>(),
                       r.send.as<uint32_t>(), r.ev_id.as<uint32_t>(), r.ev_w.as<float>(),
                       mode == KGX_ROLLUP_FAMILY ? 1 : 0, d_E, cap, r.flag.as<uint8_t>(), r.rowdata.as<uint4>(),
                       r.rows2.as<uint4>(), r.rowcnt.as<uint32_t>());
    if (n + 1 <= kScanOneMax) {
        hipLaunchKernelGGL(scan_one_kernel<uint32_t>, dim3(1), dim3(1024), 0, st, r.rowcnt.as<uint32_t>(),
                           (uint64_t)n + 1, r.rowoff.as<uint64_t>(), nullptr);
    } else {
        size_t tb = 0;
        HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, r.rowcnt.as<uint32_t>(), r.rowoff.as<uint64_t>(),
                                                 (int)(n + 1), st));
        HIP_TRY(r.tmp.reserve(tb));
        HIP_TRY(hipcub::DeviceScan::ExclusiveSum(r.tmp.p, tb, r.rowcnt.as<uint32_t>(), r.rowoff.as<uint64_t>(),
                                                 (int)(n + 1), st));
    }
    void *d_rows = nullptr, *d_off = nullptr, *d_n = nullptr;
    HIP_TRY(r.h_rows.device_ptr(0, &d_rows));
    HIP_TRY(r.h_off.device_ptr(0, &d_off));
    HIP_TRY(r.h_n.device_ptr(1, &d_n));
    hipLaunchKernelGGL(rollup_emit_kernel, seq_grid, dim3(256), 0, st, n, r.sfirst.as<uint32_t>(),
                       r.rowcnt.as<uint32_t>(), r.rowoff.as<uint64_t>(), r.rows2.as<uint4>(), d_E, cap,
                       static_cast<uint4 *>(d_rows), static_cast<uint64_t *>(d_off), static_cast<uint64_t *>(d_n));
    HIP_TRY(hipGetLastError());
    return KGX_OK;
}

}  // namespace

/* The rollup enqueued behind the context's pass with no host wait when the
 * context's previous rollup gave an event count to size it by (that count +
 * 1/8); rollup_finish checks the size and runs passes 2-3 again when the
 * batch had more events.  A pool enqueues each shard's rollup right after its
 * pass, so no rollup waits in a hardware queue behind later shards' kernels
 * for a host round trip (r5r: rollups at the end of the call, 0.5 ms). */
int rollup_enqueue(kgx_kmap *m, kgx_ctx *c, int mode)
{
    if (!m || (mode != KGX_ROLLUP_PEG && mode != KGX_ROLLUP_FAMILY))
        return fail(KGX_EINVAL, "bad kmap_rollup arguments");
    int rc = check_ctx_hits(c);
    if (rc)
        return rc;
    if (c->img->device != m->device)
        return fail(KGX_EINVAL, "kmap and context are on different devices");
    HIP_TRY(hipSetDevice(m->device));
    if (!c->rollup)
        c->rollup.reset(new RollupScratch);
    RollupScratch &r = *c->rollup;
    const uint32_t n = c->n_seq;
    HIP_TRY(r.h_off.resize(n + 1));
    HIP_TRY(r.h_n.resize(4));
    r.cap = 0;
    r.enqueued = true;
    if (n == 0 || m->n_rows == 0)
        return KGX_OK;
    if ((rc = rollup_tiles(m, c, r)))
        return rc;
    if (r.hint) {
        const uint64_t cap = std::min<uint64_t>(r.hint + r.hint / 8 + 4096, (1ull << 31) - 1);
        if ((rc = rollup_rows(m, c, r, mode, cap)))
            return rc;
        r.cap = cap;
    }
    return KGX_OK;
}

int rollup_finish(kgx_kmap *m, kgx_ctx *c, int mode, kgx_rollup_result *out)
{
    if (!m || !c || !out || !c->rollup || !c->rollup->enqueued)
        return fail(KGX_EINVAL, "rollup_finish without rollup_enqueue");
    RollupScratch &r = *c->rollup;
    r.enqueued = false;
    const uint32_t n = c->n_seq;
    out->n_seq = n;
    out->offsets = r.h_off.data();
    out->rows = r.h_rows.data();
    out->n_events = 0;
    if (n == 0 || m->n_rows == 0) {
        std::fill(r.h_off.data(), r.h_off.data() + n + 1, 0ull);
        return KGX_OK;
    }
    HIP_TRY(hipSetDevice(m->device));
    HIP_TRY(host_wait(c->stream));
    std::atomic_thread_fence(std::memory_order_acquire);
    const uint64_t E = r.h_n[0];
    out->n_events = E;
    r.hint = E;
    if (E == 0) {
        std::fill(r.h_off.data(), r.h_off.data() + n + 1, 0ull);
        return KGX_OK;
    }
    if (E >= (1ull << 31))
        return fail(KGX_ERANGE, "rollup: more than 2^31 (hit, id) events in one batch");
    if (E > r.cap) { /* not sized, or sized too small: passes 2-3 at E */
        r.presize_misses += r.cap != 0;
        if (int rc = rollup_rows(m, c, r, mode, E))
            return rc;
        HIP_TRY(host_wait(c->stream));
        std::atomic_thread_fence(std::memory_order_acquire);
    }
    out->rows = r.h_rows.data();
    if (r.h_n[1] != r.h_off[n] || r.h_off[n] > E)
        return fail(KGX_EDEVICE, "rollup: row counts disagree");
    return KGX_OK;
}

}  // namespace kgx

extern "C" {

int kgx_kmap_create(int device, int mode, kgx_kmap **out)
{
    if (!out || (mode != KGX_KMAP_APPEND && mode != KGX_KMAP_SET))
        return fail(KGX_EINVAL, "bad kmap arguments");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return fail(KGX_EDEVICE, "no such HIP device " + std::to_string(device));
    if (!is_gfx950(device))
        return fail(KGX_EDEVICE, "device " + std::to_string(device) + " is not gfx950");
    HIP_TRY(hipSetDevice(device));
    kgx_kmap *m = new kgx_kmap;
    m->device = device;
    m->mode = mode;
    if (hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess) {
        delete m;
        return fail(KGX_EDEVICE, "stream creation failed");
    }
    *out = m;
    return KGX_OK;
}

int kgx_kmap_destroy(kgx_kmap *m)
{
    if (!m)
        return KGX_OK;
    (void)hipSetDevice(m->device);
    (void)hipStreamSynchronize(m->stream);
    for (DevBuf *b : {&m->keys, &m->starts, &m->vals, &m->hkeys, &m->hrow, &m->slots})
        b->release();
    for (auto &sc : m->scratch_free) {
        for (DevBuf *b : {&sc->k, &sc->c, &sc->ids})
            b->release();
        (void)hipStreamDestroy(sc->st);
    }
    (void)hipStreamDestroy(m->stream);
    delete m;
    return KGX_OK;
}

int kgx_kmap_device(const kgx_kmap *m) { return m ? m->device : -1; }

uint64_t kgx_kmap_num_kmers(const kgx_kmap *m) { return m ? m->n_rows : 0; }
uint64_t kgx_kmap_num_values(const kgx_kmap *m) { return m ? m->n_vals : 0; }

int kgx_kmap_add(kgx_kmap *m, const uint64_t *kmers, const uint32_t *ids, uint64_t n)
{
    if (!m || (n && (!kmers || !ids)))
        return fail(KGX_EINVAL, "bad kmap_add arguments");
    if (n == 0)
        return KGX_OK;
    HIP_TRY(hipSetDevice(m->device));
    hipStream_t st = m->stream;
    DevBuf d_k, d_v;
    int rc = kmap_expand(m, d_k, d_v, n, st);
    if (rc)
        return rc;
    uint32_t mx = m->max_id;
    for (uint64_t i = 0; i < n; i++) {
        if (ids[i] == NO_ID)
            return fail(KGX_EINVAL, "id 0xFFFFFFFF is reserved");
        mx = std::max(mx, ids[i]);
    }
    m->max_id = mx;
    HIP_TRY(hipMemcpyAsync(d_k.as<uint64_t>() + m->n_vals, kmers, n * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_v.as<uint32_t>() + m->n_vals, ids, n * 4, hipMemcpyHostToDevice, st));
    return kmap_rebuild(m, d_k, d_v, m->n_vals + n, st);
}

int kgx_kmap_add_hits(kgx_kmap *m, kgx_ctx *c, const uint32_t *seq_ids)
{
    if (!m)
        return fail(KGX_EINVAL, "null kmap");
    int rc = check_ctx_hits(c);
    if (rc)
        return rc;
    if (c->img->device != m->device)
        return fail(KGX_EINVAL, "kmap and context are on different devices");
    if (c->n_seq == 0)
        return KGX_OK;
    if (!seq_ids)
        return fail(KGX_EINVAL, "null seq_ids");
    HIP_TRY(hipSetDevice(m->device));
    hipStream_t st = c->stream;
    DevBuf d_ids, counts, base, tmp;
    rc = upload_ids(d_ids, seq_ids, c->n_seq, st);
    if (rc)
        return rc;
    const uint32_t batch_max = *std::max_element(seq_ids, seq_ids + c->n_seq);
    const Tiled t = tiled_of(c);
    const uint64_t nt = c->max_tiles;
    HIP_TRY(counts.reserve((nt + 1) * 4));
    HIP_TRY(base.reserve((nt + 1) * 4));
    hipLaunchKernelGGL(tile_counts_kernel, grid_for(nt + 1), dim3(256), 0, st, t, nt, counts.as<uint32_t>());
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, counts.as<uint32_t>(), base.as<uint32_t>(),
                                             (int)(nt + 1), st));
    HIP_TRY(tmp.reserve(tb));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, counts.as<uint32_t>(), base.as<uint32_t>(),
                                             (int)(nt + 1), st));
    uint32_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, base.as<uint32_t>() + nt, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (total == 0)
        return KGX_OK;
    DevBuf d_k, d_v;
    rc = kmap_expand(m, d_k, d_v, total, st);
    if (rc)
        return rc;
    m->max_id = std::max(m->max_id, batch_max);
    hipLaunchKernelGGL(hits_to_pairs_kernel, grid_for(nt * t.T), dim3(256), 0, st, t, nt, base.as<uint32_t>(),
                       d_ids.as<uint32_t>(), d_k.as<uint64_t>() + m->n_vals, d_v.as<uint32_t>() + m->n_vals);
    HIP_TRY(hipGetLastError());
    return kmap_rebuild(m, d_k, d_v, m->n_vals + total, st);
}

int kgx_kmap_lookup(kgx_kmap *m, const uint64_t *kmers, uint64_t n, uint64_t *offsets, uint32_t *ids,
                    uint64_t ids_cap)
{
    if (!m || !offsets || (n && !kmers))
        return fail(KGX_EINVAL, "bad kmap_lookup arguments");
    offsets[0] = 0;
    if (n == 0)
        return KGX_OK;
    HIP_TRY(hipSetDevice(m->device));
    std::unique_ptr<KmapScratch> sc;
    {
        std::lock_guard<std::mutex> lk(m->scratch_mu);
        if (!m->scratch_free.empty()) {
            sc = std::move(m->scratch_free.back());
            m->scratch_free.pop_back();
        }
    }
    if (!sc) {
        sc.reset(new KmapScratch);
        HIP_TRY(hipStreamCreateWithFlags(&sc->st, hipStreamNonBlocking));
    }
    struct Return { /* the scratch goes back to the free list, whatever happens */
        kgx_kmap *m;
        std::unique_ptr<KmapScratch> &sc;
        ~Return()
        {
            std::lock_guard<std::mutex> lk(m->scratch_mu);
            m->scratch_free.push_back(std::move(sc));
        }
    } give_back{m, sc};
    hipStream_t st = sc->st;
    HIP_TRY(sc->k.reserve(n * 8));
    HIP_TRY(sc->c.reserve((n + 1) * 8));
    HIP_TRY(sc->cnt.resize(n));
    HIP_TRY(hipMemcpyAsync(sc->k.p, kmers, n * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(lookup_count_kernel, grid_for(n), dim3(256), 0, st, m->view(), sc->k.as<uint64_t>(), n,
                       sc->c.as<uint64_t>());
    HIP_TRY(hipMemcpyAsync(sc->cnt.data(), sc->c.p, n * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t *cnt = sc->cnt.data();
    for (uint64_t i = 0; i < n; i++)
        offsets[i + 1] = offsets[i] + cnt[i];
    if (!ids)
        return KGX_OK;
    if (ids_cap < offsets[n])
        return fail(KGX_ERANGE, "ids buffer too small");
    HIP_TRY(sc->ids.reserve(std::max<uint64_t>(offsets[n], 1) * 4));
    HIP_TRY(hipMemcpyAsync(sc->c.p, offsets, (n + 1) * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(lookup_ids_kernel, grid_for(n), dim3(256), 0, st, m->view(), sc->k.as<uint64_t>(), n,
                       sc->c.as<uint64_t>(), sc->ids.as<uint32_t>());
    HIP_TRY(hipMemcpyAsync(ids, sc->ids.p, offsets[n] * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return KGX_OK;
}

int kgx_kmap_rollup(kgx_kmap *m, kgx_ctx *c, int mode, kgx_rollup_result *out)
{
    int rc = kgx::rollup_enqueue(m, c, mode);
    return rc ? rc : kgx::rollup_finish(m, c, mode, out);
}

int kgx_matrix_create(kgx_kmap *map, kgx_matrix **out)
{
    if (!map || !out)
        return fail(KGX_EINVAL, "bad matrix arguments");
    kgx_matrix *x = new kgx_matrix;
    x->map = map;
    *out = x;
    return KGX_OK;
}

int kgx_matrix_destroy(kgx_matrix *x)
{
    if (!x)
        return KGX_OK;
    (void)hipSetDevice(x->map->device);
    for (DevBuf *b : {&x->skeys, &x->sord, &x->pkeys, &x->pcount, &x->ids, &x->counter, &x->tmp_keys,
                      &x->tmp_count, &x->cub.buf})
        b->release();
    delete x;
    return KGX_OK;
}

namespace {

/* grow a (keys, vals) hash to hold `need` entries at load <= 1/2 */
int grow_hash(DevBuf &keys, DevBuf &vals, uint64_t &cap, uint64_t need, uint8_t val_fill, hipStream_t st)
{
    if (2 * need <= cap)
        return KGX_OK;
    const uint64_t ncap = pow2_at_least(2 * need);
    DevBuf nk, nv;
    HIP_TRY(nk.reserve(ncap * 8));
    HIP_TRY(nv.reserve(ncap * 8));
    HIP_TRY(hipMemsetAsync(nk.p, 0xFF, ncap * 8, st));
    HIP_TRY(hipMemsetAsync(nv.p, val_fill, ncap * 8, st));
    if (cap)
        hipLaunchKernelGGL(rehash_kernel, grid_for(cap), dim3(256), 0, st, keys.as<uint64_t>(),
                           vals.as<uint64_t>(), cap, nk.as<uint64_t>(), nv.as<uint64_t>(), ncap - 1);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
    std::swap(keys, nk);
    std::swap(vals, nv);
    nk.release();
    nv.release();
    cap = ncap;
    return KGX_OK;
}

}  // namespace

int kgx_matrix_add_hits(kgx_matrix *x, kgx_ctx *c, const uint32_t *seq_ids)
{
    if (!x)
        return fail(KGX_EINVAL, "null matrix");
    int rc = check_ctx_hits(c);
    if (rc)
        return rc;
    kgx_kmap *m = x->map;
    if (c->img->device != m->device)
        return fail(KGX_EINVAL, "kmap and context are on different devices");
    const uint32_t n = c->n_seq;
    if (n == 0)
        return KGX_OK;
    if (!seq_ids)
        return fail(KGX_EINVAL, "null seq_ids");
    HIP_TRY(hipSetDevice(m->device));
    hipStream_t st = c->stream;
    rc = upload_ids(x->ids, seq_ids, n, st);
    if (rc)
        return rc;
    HIP_TRY(x->counter.reserve(16));
    unsigned long long *used = x->counter.as<unsigned long long>();
    /* matrix_proteins_: every id of the batch joins the seen set at its ordinal */
    rc = grow_hash(x->skeys, x->sord, x->scap, x->sused + n, 0xFF, st);
    if (rc)
        return rc;
    HIP_TRY(hipMemsetAsync(used, 0, 16, st));
    hipLaunchKernelGGL(seen_insert_kernel, grid_for(n), dim3(256), 0, st, x->ids.as<uint32_t>(), n, x->base,
                       x->skeys.as<uint64_t>(), x->sord.as<uint64_t>(), x->scap - 1, used);
    const Tiled t = tiled_of(c);
    const uint64_t nt = c->max_tiles;
    const KmapView view = m->view();
    hipLaunchKernelGGL(matrix_events_kernel, dim3(std::min<uint64_t>(grid_for(nt * t.T).x, kReduceBlocks)),
                       dim3(256), 0, st, t, nt, view, used + 1);
    unsigned long long h[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(h, used, 16, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    x->sused += h[0];
    /* distance_: at most one new pair per event */
    rc = grow_hash(x->pkeys, x->pcount, x->pcap, x->pused + h[1], 0, st);
    if (rc)
        return rc;
    if (h[1]) {
        HIP_TRY(hipMemsetAsync(used, 0, 8, st));
        hipLaunchKernelGGL(matrix_pairs_kernel, grid_for(nt * t.T), dim3(256), 0, st, t, nt, view,
                           x->ids.as<uint32_t>(), x->base, x->skeys.as<uint64_t>(), x->sord.as<uint64_t>(),
                           x->scap - 1, x->pkeys.as<uint64_t>(), x->pcount.as<uint64_t>(), x->pcap - 1, used);
        unsigned long long fresh = 0;
        HIP_TRY(hipMemcpyAsync(&fresh, used, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        x->pused += fresh;
    }
    x->base += n;
    return KGX_OK;
}

int kgx_matrix_pairs(kgx_matrix *x, const kgx_pair_count **pairs, uint64_t *n_pairs)
{
    if (!x || !pairs || !n_pairs)
        return fail(KGX_EINVAL, "bad matrix_pairs arguments");
    x->result.clear();
    *pairs = nullptr;
    *n_pairs = 0;
    if (x->pused == 0)
        return KGX_OK;
    HIP_TRY(hipSetDevice(x->map->device));
    hipStream_t st = x->map->stream;
    const uint64_t n = x->pused;
    DevBuf k1, c1, k2, c2;
    HIP_TRY(k1.reserve(n * 8));
    HIP_TRY(c1.reserve(n * 8));
    HIP_TRY(k2.reserve(n * 8));
    HIP_TRY(c2.reserve(n * 8));
    HIP_TRY(x->counter.reserve(16));
    HIP_TRY(hipMemsetAsync(x->counter.p, 0, 8, st));
    hipLaunchKernelGGL(compact_pairs_kernel, dim3(std::min<uint64_t>(grid_for(x->pcap).x, kReduceBlocks)),
                       dim3(256), 0, st, x->pkeys.as<uint64_t>(),
                       x->pcount.as<uint64_t>(), x->pcap, k1.as<uint64_t>(), c1.as<uint64_t>(),
                       x->counter.as<unsigned long long>());
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k1.as<uint64_t>(), k2.as<uint64_t>(),
                                               c1.as<uint64_t>(), c2.as<uint64_t>(), (int)n, 0, 64, st));
    HIP_TRY(x->cub.buf.reserve(tb));
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(x->cub.buf.p, tb, k1.as<uint64_t>(), k2.as<uint64_t>(),
                                               c1.as<uint64_t>(), c2.as<uint64_t>(), (int)n, 0, 64, st));
    std::vector<uint64_t> hk(n), hc(n);
    HIP_TRY(hipMemcpyAsync(hk.data(), k2.p, n * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(hc.data(), c2.p, n * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    x->result.resize(n);
    for (uint64_t i = 0; i < n; i++)
        x->result[i] = kgx_pair_count{(uint32_t)(hk[i] >> 32), (uint32_t)hk[i], hc[i]};
    *pairs = x->result.data();
    *n_pairs = n;
    return KGX_OK;
}

}  // extern "C"
