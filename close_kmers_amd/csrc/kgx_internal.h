/*
 * kgx_internal.h -- shared definitions between the HIP kernels
 * (kgx_lookup.hip, kgx_synth.hip) and the host runtime (kgx_runtime.cpp).
 */
#ifndef KGX_INTERNAL_H
#define KGX_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kgx.h"

namespace kgx {

/* kmer_params.h:5-20 */
constexpr int KMER = 8;
constexpr uint64_t CORE = 1280000000ULL;         /* 20^7 */
constexpr uint64_t MAX_ENCODED = 25600000000ULL; /* 20^8 */
constexpr uint64_t EMPTY_KEY = MAX_ENCODED + 1;  /* kguts.cc:106-107 */
constexpr int RUN_CAP = 40000 - 2;               /* MAX_HITS_PER_SEQ - 2, kguts.cc:850 */

/*
 * Window space.  The windows of a batch are numbered globally: sequence s
 * owns windows [wbase[s], wbase[s+1]) (position p = global - wbase[s],
 * wbase = exclusive scan of max(0, len-8)).  The probe cuts this space into
 * tiles of probe_j * 64 windows -- across sequence boundaries, so short
 * sequences pack densely -- one tile per wave.  A tile's hits are stored
 * compacted, in window order, from slot tile * tile_windows; bit i of
 * hit_mask[g] says whether window 64 g + i hit.  A slot is two 16-B records
 * in two planes of one buffer: hot = {avg | flags << 16, fI, wt bits, pos}
 * (everything the run scorer reads) and cold = {which_kmer lo, hi, otu, seq}.
 */
constexpr int PROBE_WAVES = 4; /* waves per 256-thread workgroup */
/* Hit record formats (kgx_device_result.hit_format):
 *   HIT_PLANES   (AOS24 images) the two planes above;
 *   HIT_PACKED16 (PACKED16 images) one plane: the matching table record
 *     itself (layout below), flags in bits [60,63) of hi (dword 3 bits
 *     28-30), which the packed layout leaves 0.  Position and sequence are
 *     not stored: they follow from the hit's window (hit_mask bit) -- half
 *     the probe's hit-store traffic.
 * Either way the consumers (scorer, gather, k-mer tables) take a hit's
 * position from its mask bit. */
constexpr uint32_t HIT_PLANES = KGX_HIT_PLANES, HIT_PACKED16 = KGX_HIT_PACKED16;
/* probe variants (kgx_ctx_set_option "probe_variant") */
constexpr int PROBE_BUCKET = 0;    /* key + payload per bucket examined */
constexpr int PROBE_KEY_FIRST = 1; /* keys only; payload for the matching bucket */
/* default: cooperative 64-B lines (PROBE_LINE) for PACKED16 without a
 * presence filter, whole 16-B records with one; key first for AOS24 (the
 * fastest on MI355X for each case, interleaved A/B in bench.py,
 * profiles/r1_probe_ab.json) */
constexpr int PROBE_AUTO = -1;
/* PACKED16 only, no presence filter: groups of 4 (8) lanes read one aligned
 * 64-B (128-B) table line per instruction (probe_line_kernel) */
constexpr int PROBE_LINE = 2;
constexpr int PROBE_LINE8 = 3;
constexpr int PROBE_J_DEFAULT = 2;

/*
 * HBM-resident bucket layouts.  The file's 24-byte bucket (kmer_image.h:11-23)
 * straddles 64-byte sectors and needs a second dependent load for its payload;
 * when the payload ranges allow, the image is kept as one 16-byte record per
 * bucket at the SAME slot (so probe sequences and results are unchanged):
 *   lo = key[0,35) | (fI+1)[35,55) | (otu+1)[0,9) at [55,64)
 *   hi = function_wt bits[0,32) | avg_from_end[32,48) | (otu+1)[9,21) at [48,60)
 * Keys above 20^8 (empty / stop buckets) are stored as EMPTY_KEY, which stops
 * a probe exactly as the original does (kguts.cc:592); their payload is 0.
 */
struct packed_bucket {
    uint64_t lo, hi;
};
constexpr uint64_t PACK_KEY_MASK = (1ull << 35) - 1;
constexpr int64_t PACK_FI_MAX = (1ll << 20) - 2;  /* fI in [-1, PACK_FI_MAX] */
constexpr int64_t PACK_OTU_MAX = (1ll << 21) - 2; /* otu in [-1, PACK_OTU_MAX] */

__host__ __device__ inline bool packable(const kgx_sig_kmer &e)
{
    return e.which_kmer > MAX_ENCODED ||
           (e.function_index >= -1 && e.function_index <= PACK_FI_MAX && e.otu_index >= -1 &&
            e.otu_index <= PACK_OTU_MAX);
}

__host__ __device__ inline packed_bucket pack_bucket(const kgx_sig_kmer &e)
{
    packed_bucket b;
    if (e.which_kmer > MAX_ENCODED) {
        b.lo = EMPTY_KEY;
        b.hi = 0;
        return b;
    }
    uint32_t wt;
    __builtin_memcpy(&wt, &e.function_wt, 4);
    const uint64_t fi = (uint64_t)(e.function_index + 1), otu = (uint64_t)(e.otu_index + 1);
    b.lo = e.which_kmer | (fi << 35) | ((otu & 0x1FFu) << 55);
    b.hi = (uint64_t)wt | ((uint64_t)e.avg_from_end << 32) | ((otu >> 9) << 48);
    return b;
}

__host__ __device__ inline kgx_sig_kmer unpack_bucket(const packed_bucket &b)
{
    kgx_sig_kmer e;
    e.which_kmer = b.lo & PACK_KEY_MASK;
    e.otu_index = (int32_t)(((b.lo >> 55) & 0x1FFu) | (((b.hi >> 48) & 0xFFFu) << 9)) - 1;
    e.avg_from_end = (uint16_t)(b.hi >> 32);
    e.pad = 0;
    e.function_index = (int32_t)((b.lo >> 35) & 0xFFFFFu) - 1;
    const uint32_t wt = (uint32_t)b.hi;
    __builtin_memcpy(&e.function_wt, &wt, 4);
    if (e.which_kmer > MAX_ENCODED) {
        e.otu_index = 0;
        e.avg_from_end = 0;
        e.function_index = 0;
        e.function_wt = 0.0f;
    }
    return e;
}

/*
 * Optional presence filter of an image: 2^log2_bits bits in 64-bit words;
 * each stored key (<= 20^8) sets two bits of one word (a blocked Bloom
 * filter, hash independent of the slot hash).  A key whose two bits are not
 * both set is stored nowhere, so its probe would end at a stop bucket: the
 * probe skips the table for it.  No false negatives, so results never change.
 */
__host__ __device__ inline uint64_t filter_hash(uint64_t key)
{
    uint64_t h = key * 0x9E3779B97F4A7C15ull;
    return h ^ (h >> 29);
}
__host__ __device__ inline uint64_t filter_word(uint64_t h, uint32_t log2_words)
{
    return log2_words ? h >> (64 - log2_words) : 0;
}
__host__ __device__ inline uint64_t filter_bits(uint64_t h)
{
    return (1ull << (h & 63)) | (1ull << ((h >> 6) & 63));
}

/* floor((2^64-1)/n): x % n = x - umulhi(x, m)*n, corrected once (x < 2^35). */
inline uint64_t mod_magic(uint64_t n) { return n ? (~0ULL) / n : 0; }

inline bool probe_j_supported(int j) { return (j >= 1 && j <= 5) || j == 8; }

/* launchers; all asynchronous on `stream` */
size_t plan_workspace_bytes(uint32_t n_seq);
/* status[0] = 1 when the offsets are not monotone or span more than
 * n_residues bytes (the batch is then planned as empty), else 0 */
hipError_t launch_plan(const uint64_t *seq_off, uint32_t n_seq, uint64_t n_residues, uint64_t *wbase,
                       uint32_t *tile_seq, uint32_t tile_windows, void *workspace, uint32_t *status,
                       hipStream_t stream);
/* the same plan in one launch (a decoupled look-back over workgroups); look:
 * plan_look_bytes(n_seq) bytes, zero-filled when allocated and left zero by
 * every launch; tile owners past max_tiles are never written */
size_t plan_look_bytes(uint32_t n_seq);
/* the plan by one workgroup, for batches of at most 2^18 sequences */
hipError_t launch_plan_one(const uint64_t *seq_off, uint32_t n_seq, uint64_t n_residues, uint64_t *wbase,
                           uint32_t *tile_seq, uint32_t tile_windows, uint64_t max_tiles, uint32_t *status,
                           hipStream_t stream);
hipError_t launch_plan_fused(const uint64_t *seq_off, uint32_t n_seq, uint64_t n_residues, uint64_t *wbase,
                             uint32_t *tile_seq, uint32_t tile_windows, uint64_t max_tiles, void *look,
                             uint32_t *status, hipStream_t stream);
/* Probes of PACKED16 records take home_shift: a key's home bucket is
 * (key mod (num_sigs >> home_shift)) << home_shift and num_sigs counts the
 * table's buckets.  0: the reference's slot (key mod num_sigs); 2: the line
 * index of kgx_image_set_line_index (4-bucket lines, homes at line starts). */
hipError_t launch_probe(const uint8_t *residues, uint64_t n_residues, const uint64_t *seq_off,
                        const uint64_t *wbase, const uint32_t *tile_seq, uint32_t n_seq,
                        uint64_t max_tiles, const void *table, int layout, uint64_t num_sigs,
                        const uint64_t *filter, uint32_t filter_log2_words,
                        uint4 *hot, uint4 *cold, uint64_t *hit_mask, int probe_j, int variant,
                        uint32_t lds_kb, uint32_t max_blocks, hipStream_t stream, uint32_t home_shift = 0,
                        uint32_t nt_stores = 0);
/* nt_stores 1: the line probe writes its hit records and mask words with
 * non-temporal stores (context option "probe_nt", an A/B knob).
 * max_blocks > 0 caps the line probe's grid (its waves then stride over the
 * tiles; option probe_persist); 0 = one workgroup per 4 tiles.
 * The line probe over fq fragments left as DNA (PACKED16 images, probe_j
 * 1-4): anchor[s] = (first base of fragment s) << 1 | reverse strand; keys as
 * launch_probe over the translated residues (HIT_PACKED16 records) */
hipError_t launch_probe_dna(const uint8_t *bases, uint64_t n_bases, const uint64_t *anchor, const uint64_t *wbase,
                            const uint32_t *tile_seq, uint32_t n_seq, uint64_t max_tiles, const void *table,
                            uint64_t num_sigs, uint4 *hot, uint64_t *hit_mask, int probe_j, uint32_t max_blocks,
                            hipStream_t stream, uint32_t home_shift = 0);
/* set the filter bits of every stored key of the resident table */
hipError_t launch_filter_build(const void *table, int layout, uint64_t num_sigs, uint64_t *filter,
                               uint32_t log2_words, hipStream_t stream);
/* *count += the PACKED16 table's stored keys */
hipError_t launch_count_keys(const packed_bucket *t, uint64_t n, unsigned long long *count, hipStream_t stream);
/* the line index of a PACKED16 table (lines_build_kernel): 4 * n_lines
 * buckets; *overflow |= 1 when some record found no bucket */
hipError_t launch_lines_build(const packed_bucket *src, uint64_t num_sigs, packed_bucket *lines, uint64_t n_lines,
                              uint32_t *overflow, hipStream_t stream);
/* AoS -> packed; *not_packable |= 1 when some stored bucket does not fit */
hipError_t launch_pack(const kgx_sig_kmer *table, packed_bucket *packed, uint64_t n,
                       uint32_t *not_packable, hipStream_t stream);
hipError_t launch_unpack(const packed_bucket *packed, kgx_sig_kmer *out, uint64_t n,
                         hipStream_t stream);
/* the run scorer.  variant SCORE_HYBRID (0, the default): the lane machine
 * (one lane per sequence), except sequences of (LONG_SEQ, RUN_CAP] windows,
 * which the wave-parallel scorer takes; SCORE_WAVE (1): the wave scorer for
 * every sequence up to RUN_CAP windows; SCORE_LANE (2): the lane machine
 * only.  The wave scorer needs order_constraint 0 (else: the lane machine).
 * plan_status[1] = the batch's longest sequence in windows (launch_plan). */
enum { SCORE_HYBRID = 0, SCORE_WAVE = 1, SCORE_LANE = 2, SCORE_WAVE_ONLY = 3 /* internal: no sequence > RUN_CAP */ };
constexpr uint32_t LONG_SEQ = 2048;
hipError_t launch_score(uint32_t n_seq, uint64_t n_residues, const uint64_t *wbase, const uint32_t *tile_seq,
                        uint64_t max_tiles, const uint64_t *hit_mask, uint32_t tile_windows, uint4 *hot,
                        kgx_call *calls, void *ranges, uint32_t *hit_count, uint32_t *call_count,
                        kgx_params params, uint32_t want, uint32_t hit_format, int variant, uint32_t wave_tiles,
                        const uint32_t *plan_status, hipStream_t stream);
hipError_t launch_gather(uint32_t n_seq, const uint64_t *wbase, const uint64_t *hit_mask,
                         uint32_t tile_windows, const uint32_t *call_count, const uint4 *hot, const uint4 *cold,
                         const kgx_call *calls, const uint64_t *hit_dense_off,
                         const uint64_t *call_dense_off, kgx_hit *hits_out, kgx_call *calls_out,
                         uint32_t seq_base, uint32_t hit_format, const uint32_t *otu_count, const kgx_otu *otus,
                         const uint64_t *otu_dense_off, kgx_otu *otus_out, hipStream_t stream,
                         uint4 *hits16_out = nullptr, /* PACKED16: the 16-B records, dense, instead of kgx_hit */
                         uint32_t *hits12_out = nullptr); /* PACKED16: 12-B records without the key */
/* per-sequence OTU tallies in otus_by_count order at otus[window_base[s]] */
hipError_t launch_otus(uint32_t n_seq, const uint64_t *wbase, const uint64_t *hit_mask, uint32_t tile_windows,
                       const uint4 *hot, const uint4 *cold, int32_t *ws, kgx_otu *otus, uint32_t *otu_count,
                       uint32_t hit_format, hipStream_t stream);
/* find_best_call per sequence: calls[start[s] ..+ count[s]), ws same extent */
hipError_t launch_best_calls(uint32_t n_seq, const kgx_call *calls, const uint64_t *start, const uint32_t *count,
                             kgx_call *ws, kgx_best_call *out, hipStream_t stream);
/* dense CSR offsets (n + 1 each) of up to three per-sequence count arrays
 * (NULL count array: all-zero offsets) */
size_t count_scan_workspace_bytes(uint32_t n);
hipError_t launch_count_scan(uint32_t n, const uint32_t *c0, const uint32_t *c1, const uint32_t *c2, uint64_t *o0,
                             uint64_t *o1, uint64_t *o2, void *workspace, hipStream_t stream);
/* small batches: up to SMALL_PIECES arrays of 16-B words copied from mapped
 * pinned host memory to HBM in one launch (piece p covers words
 * [end16[p-1], end16[p]) of the concatenation) */
constexpr int SMALL_PIECES = 5;
struct SmallPieces {
    uint4 *dst[SMALL_PIECES];
    const uint4 *src[SMALL_PIECES];
    uint64_t end16[SMALL_PIECES];
};
hipError_t launch_small_upload(const SmallPieces &pc, hipStream_t stream);
/* small_collect + gather in one workgroup, for batches of up to
 * SMALL_GATHER_SEQ sequences (offsets into mapped h0..h2, records into the
 * mapped outputs; a NULL output is not gathered); last, token is stored to
 * mapped *done_host (when not NULL) after a system-scope fence, by the last
 * workgroup to finish (blocks_done: a zeroed device word the kernel leaves
 * zeroed; NULL = one workgroup) */
/* one launch per small batch (kgx_fused.hip, context option "small_fused"):
 * one workgroup per sequence of at most FUSED_MAX_WINDOWS windows, results
 * stored straight into mapped host memory */
constexpr uint32_t FUSED_MAX_WINDOWS = 2048;
constexpr uint32_t FUSED_MAX_SEQ = 4096;
/* a batch of at most FUSED_INLINE_SEQ sequences and FUSED_INLINE_RES residues
 * travels in the kernel arguments (host pointers h_off / h_wbase / h_res,
 * inline_res = its residue bytes; 0 = read res / off / wbase from mapped
 * memory) */
constexpr uint32_t FUSED_INLINE_SEQ = 32;
constexpr uint32_t FUSED_INLINE_RES = 2048;
hipError_t launch_fused_small(const uint8_t *res, const uint64_t *off, const uint64_t *wbase, uint32_t n,
                              uint32_t want, const void *packed_table, uint64_t num_sigs, kgx_params prm,
                              kgx_hit *hits, kgx_call *calls, uint32_t *counts, uint32_t *done, uint32_t token,
                              uint32_t max_windows, uint64_t *dbg, const uint64_t *h_off, const uint64_t *h_wbase,
                              const uint8_t *h_res, uint32_t inline_res, hipStream_t stream, uint32_t home_shift = 0);
/* resident call service (kgx_svc.cpp, svc_kernel in kgx_fused.hip): one
 * persistent workgroup per slot polls its slot's request word in mapped host
 * memory and runs fused_small_body on the slot's sequence; no launch per call.
 * A slot takes one sequence of at most SVC_MAX_RES residues. */
constexpr uint32_t SVC_MAX_RES = FUSED_MAX_WINDOWS + 8;
constexpr uint32_t SVC_RES_STRIDE = 4096;  /* bytes of residue chunks per slot */
/* a slot's residues travel in 16-B chunks: 12 residues, then the request
 * number they belong to (one 16-B store on the host, one 16-B load on the
 * device: a chunk is read whole or not at all); the service's polling wave
 * reads the first SVC_POLL_CHUNKS with the header line */
constexpr uint32_t SVC_RES_CHUNKS = (SVC_MAX_RES + 11) / 12;
constexpr uint32_t SVC_POLL_CHUNKS = 60;
static_assert(SVC_RES_CHUNKS * 16 <= SVC_RES_STRIDE, "residue chunks per slot");
constexpr uint32_t SVC_MAX_SLOTS = 64;
struct SvcSlotHdr { /* host-written, one 64-B line per slot, read whole by the polling wave */
    uint32_t req;   /* request number: the device serves it when it differs from SvcSlotOut.done */
    uint32_t stop;  /* nonzero: the service's workgroups leave */
    uint32_t len;   /* residues */
    uint32_t want;  /* KGX_WANT_HITS | KGX_WANT_CALLS | KGX_WANT_OTU */
    kgx_params prm;
    uint32_t debug; /* nonzero: phase stamps into the slot's SvcSlotDbg */
    uint32_t pad[6];
    uint32_t copy; /* = req, written before it: a line read with copy != req is incomplete */
};
struct SvcSlotDbg { /* device wall clock (100 MHz) at the phases of the last request */
    uint64_t stamp[32]; /* 0 seen, 1 residues, 2 probed, 3 compacted, 4 stored + scored, 5 fenced, 6 thread
                           0's record stores issued, 7 OTU tally entered, 8 OTU pairs in key order, 9 the
                           scorer's first chunk done, 10 probe rounds (a count), 11 the
                           probe's first round examined, 12 keys and homes computed, 13
                           thread 0's first-round loads back, 14 / 15 the scorer's first
                           chunk's runs and members / sums, 16 / 17 the shader clock (s_memtime) at the OTU sort's start / end */
};
struct SvcSlotOut { /* device-written, one 64-B line per slot */
    uint32_t nh, nc, no; /* hit / call records and OTU pairs stored */
    uint32_t done;       /* = req once the records and counts are visible */
    uint32_t left;       /* workgroups of this slot that have left (one per instance launched) */
    uint32_t pad[11];
};
static_assert(sizeof(SvcSlotHdr) == 64 && sizeof(SvcSlotOut) == 64 && sizeof(SvcSlotDbg) == 256,
              "service slot lines");
/* slots workgroups on stream; each leaves life_ticks after its start (device
 * wall clock, 100 MHz) or on stop */
hipError_t launch_svc(const SvcSlotHdr *hdr, SvcSlotOut *out, SvcSlotDbg *dbg, const uint8_t *res, kgx_hit *hits,
                      kgx_call *calls, kgx_otu *otus, uint32_t slots, const void *packed_table, uint64_t num_sigs,
                      uint64_t life_ticks, int quad_probe, hipStream_t stream, uint32_t home_shift = 0,
                      uint32_t poll_chunks = SVC_POLL_CHUNKS);
constexpr uint32_t SMALL_GATHER_SEQ = 256;
constexpr uint32_t SMALL_COLLECT_BEST_SEQ = 8192;
constexpr uint32_t SMALL_GATHER_BLOCKS = 64; /* workgroups of the small gather (one wave per sequence) */
hipError_t launch_small_gather(uint32_t n, const uint64_t *wbase, const uint64_t *hit_mask, uint32_t tile_windows,
                               const uint32_t *hit_count, const uint32_t *call_count, const uint4 *hot,
                               const uint4 *cold, const kgx_call *calls, const uint32_t *otu_count,
                               const kgx_otu *otus, kgx_hit *hits_out, kgx_call *calls_out, kgx_otu *otus_out,
                               uint64_t *h0, uint64_t *h1, uint64_t *h2, const uint32_t *status,
                               const kgx_best_call *best, kgx_best_call *best_host, uint32_t *status_host,
                               uint64_t *nwin_host, uint32_t *done_host, uint32_t token, uint32_t *blocks_done,
                               uint32_t hit_format, hipStream_t stream);
/* one workgroup: launch_count_scan's offsets into o* (HBM) and h* (mapped
 * host), plus status[0], wbase[n] and (best_host non-NULL) best[0, n) */
hipError_t launch_small_collect_best(uint32_t n, const uint32_t *c0, const uint32_t *c1, const uint32_t *c2,
                                     uint64_t *o0, uint64_t *o1, uint64_t *o2, uint64_t *h0, uint64_t *h1,
                                     uint64_t *h2, const uint32_t *status, const uint64_t *wbase,
                                     const kgx_call *calls, const uint32_t *call_count, kgx_call *ws,
                                     kgx_best_call *best, kgx_best_call *best_host, uint32_t *status_host,
                                     uint64_t *nwin_host, hipStream_t stream);
hipError_t launch_small_collect(uint32_t n, const uint32_t *c0, const uint32_t *c1, const uint32_t *c2, uint64_t *o0,
                                uint64_t *o1, uint64_t *o2, uint64_t *h0, uint64_t *h1, uint64_t *h2,
                                const uint32_t *status, const uint64_t *wbase, const kgx_best_call *best,
                                kgx_best_call *best_host, uint32_t *status_host, uint64_t *nwin_host,
                                hipStream_t stream);
/* min(*count, cap) elements of elem_bytes (a multiple of 4) from src to dst,
 * both 16-byte aligned */
hipError_t launch_copy_counted(void *dst, const void *src, const uint64_t *count, uint64_t cap,
                               uint32_t elem_bytes, int blocks, hipStream_t stream);
/* *flag_mapped = 1 when a byte of d[skip, n) is 0 (d 16-byte aligned) */
hipError_t launch_nul_scan(const uint8_t *d, uint64_t skip, uint64_t n, uint32_t *flag_mapped, hipStream_t stream);

/* device stores of bytes (4-aligned) from HBM into mapped pinned host memory */
/* up to kMax copies device -> mapped host memory in one launch; add() takes
 * byte counts (4-B aligned; 16-B aligned spans copy by 16 B) */
struct CopySpans {
    static constexpr int kMax = 8;
    void *dst[kMax];
    const void *src[kMax];
    uint64_t n[kMax];
    bool v16[kMax];
    int count = 0;
    void add(void *d, const void *s, uint64_t bytes)
    {
        if (bytes == 0)
            return;
        if (count == kMax) {
            count = kMax + 1; /* refused by launch_copy_spans */
            return;
        }
        dst[count] = d;
        src[count] = s;
        n[count] = bytes;
        count++;
    }
};
hipError_t launch_copy_spans(CopySpans spans, int copy_blocks, hipStream_t stream);
hipError_t launch_copy_to_host(void *dst_mapped, const void *src, uint64_t bytes, int blocks, hipStream_t stream);
hipError_t launch_random_read(const void *buffer, uint64_t bytes, uint64_t threads,
                              uint32_t rounds, int mode, int ilp, uint64_t *sink, hipStream_t stream);
/* the synthetic spec of n_keys entries (its source proteins), the first
 * n_entries of its entry stream inserted (entries past n_keys are random
 * keys); payload = false leaves every stored bucket's owner id in word 2 */
hipError_t launch_synth_image(kgx_sig_kmer *table, uint64_t num_sigs, uint64_t n_keys, uint64_t n_entries,
                              bool payload, unsigned long long *n_stored, hipStream_t stream);
/* hist[256] = histogram of owner byte (shift/8) over stored buckets whose
 * owner matches prefix under prefix_mask (after a payload-less insert) */
hipError_t launch_owner_hist(const kgx_sig_kmer *table, uint64_t num_sigs, uint32_t prefix, uint32_t prefix_mask,
                             uint32_t shift, unsigned long long *hist, hipStream_t stream);
hipError_t launch_entries_image(kgx_sig_kmer *table, uint64_t num_sigs, const uint64_t *keys,
                                const int32_t *fi, const int32_t *otu, const uint16_t *avg, const float *wt,
                                uint64_t n_entries, unsigned long long *n_stored, hipStream_t stream);
hipError_t launch_synth_queries(uint64_t image_n_keys, uint32_t n_seq, uint32_t length,
                                uint32_t x_permille, uint64_t q0, uint8_t *residues,
                                uint64_t *seq_off, hipStream_t stream);

}  // namespace kgx

#endif
