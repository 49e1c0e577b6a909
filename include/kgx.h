/*
 * kgx.h -- C ABI of the MI355X-native close_kmers hot path:
 *          k-mer encode -> signature-hash probe -> hit-run scoring.
 *
 * The reference runs this path as KmerGuts::process_aa_seq over a memory-mapped
 * KmerImage, one KmerGuts per CPU pool thread (threadpool.cc:18-44).  This ABI
 * replaces that per-sequence C++ call with batched entry points over plain
 * pointers and sizes (no C++ or torch types), implemented by hand-written
 * gfx950 HIP kernels (close_kmers_amd/csrc/).  The C++ facade in
 * close_kmers_amd/csrc/kguts_hip.h re-exposes the KmerGuts surface on top of
 * it; INTEGRATION.md shows the bindings.
 *
 * Error behaviour: every entry point returns KGX_OK (0) or a negative KGX_E*
 * code and never exits (the reference exit()s on bad files,
 * kmer_image.cc:88-147, kguts.cc:550-552).  kgx_last_error() returns a
 * thread-local message for the last failure.
 *
 * Threading: a kgx_image is read-only after creation and may be shared by any
 * number of contexts; a kgx_ctx is NOT thread-safe, exactly like KmerGuts
 * (kguts.h:263-266) -- create one per host worker thread (threadpool.h:42).
 */
#ifndef KGX_H
#define KGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ----------------------------------------------------- */
#define KGX_OK 0
#define KGX_EINVAL (-1)   /* bad argument */
#define KGX_EIO (-2)      /* cannot open / read a file */
#define KGX_EFORMAT (-3)  /* image size / version / entry size mismatch */
#define KGX_ENOMEM (-4)   /* host or device allocation failed */
#define KGX_EDEVICE (-5)  /* HIP runtime error or no gfx950 device */
#define KGX_ERANGE (-6)   /* image or batch larger than supported */
#define KGX_EFULL (-7)    /* image builder: table would reach half full */
#define KGX_EBUSY (-8)    /* call service: no free slot, or not a call it serves (use a batch path) */

/* ---- what kgx_process_* computes --------------------------------------- */
#define KGX_WANT_HITS 1u  /* hit list (what hit_cb receives, kguts.cc:814-815) */
#define KGX_WANT_CALLS 2u /* KmerCall runs (process_set_of_hits, kguts.cc:734-781) */
#define KGX_WANT_OTU 4u   /* OTU tallies (KmerOtuStats, kguts.h:185-219), on the device */
#define KGX_WANT_BEST 8u  /* find_best_call per sequence, on the device (kgx_best_call) */

/* ---- on-disk / in-HBM record layouts (kmer_image.h:11-23) -------------- */
typedef struct kgx_image_header { /* kmer_memory_image_t */
    uint64_t num_sigs;            /* buckets */
    uint64_t entry_size;          /* 24 */
    int64_t version;              /* 1 (KMER_VERSION, kmer_image.h:6) */
} kgx_image_header;

typedef struct kgx_sig_kmer { /* sig_kmer_t: one 24-byte bucket */
    uint64_t which_kmer;      /* > 20^8 means empty (kguts.cc:106-107) */
    int32_t otu_index;
    uint16_t avg_from_end;
    uint16_t pad;
    int32_t function_index;
    float function_wt;
} kgx_sig_kmer;

/* One hit: KmerGuts::hit_in_sequence_t (kguts.h:228-233) = the bucket copy +
 * the window offset, plus the sequence index within the batch.  32 bytes. */
typedef struct kgx_hit {
    uint64_t which_kmer;
    int32_t otu_index;
    uint16_t avg_from_end;
    uint16_t flags; /* KGX_HIT_* (the bucket's pad bytes in the reference) */
    int32_t function_index;
    float function_wt;
    uint32_t pos; /* offset of the 8-mer in the protein (pLoc, kguts.cc:803) */
    uint32_t seq; /* index of the sequence in the batch */
} kgx_hit;
/* hit flags are set only when KGX_WANT_OTU is requested (they feed the OTU
 * tally); otherwise they are 0 */
#define KGX_HIT_IN_RUN 1u /* appended to the run buffer (kguts.cc:845-851) */
#define KGX_HIT_OTU 2u    /* tallied into otu_map by an emitted call (kguts.cc:760-768) */
#define KGX_HIT_COUNTED 4u /* buffered while its function was the run's current_fI */

/* KmerCall (kguts.h:166-183), 20 bytes */
typedef struct kgx_call {
    uint32_t start;
    uint32_t end;
    int32_t count;
    uint32_t function_index;
    float weighted_hits;
} kgx_call;

/* What find_best_call (kguts.cc:1008-1199) decides for one sequence's calls,
 * computed on the device.  The function names stay on the host:
 *   kind 0  no calls: function_index -1, function "", score 0, weighted 0,
 *           score_offset left as the caller had it (kguts.cc:1015-1018)
 *   kind 1  called: function_index fi0, function = name(fi0)
 *   kind 2  ambiguous pair: function_index -1, function = the lexically
 *           larger of name(fi0), name(fi1) + " ?? " + the other
 *   kind 3  no call: function_index -1, function "", score_offset written
 * score / weighted_score / score_offset are the reference's values in every
 * kind (fi0 / fi1 are the top two functions whenever there are two). */
typedef struct kgx_best_call {
    int32_t kind;
    int32_t fi0;
    int32_t fi1;
    float score;
    float weighted_score;
    float score_offset;
} kgx_best_call;

/* one (otu_index, count) pair of KmerOtuStats::otus_by_count (kguts.h:214-218) */
typedef struct kgx_otu {
    int32_t otu_index;
    int32_t count;
} kgx_otu;

/* KmerGuts parameters (kguts.cc:236-268); kgx_params_default() gives
 * min_hits=5, max_gap=200, order_constraint=0, min_weighted_hits=0.
 * min_hits <= 0 makes the reference read hits[-2] at the final flush (UB);
 * here such a flush emits nothing. */
typedef struct kgx_params {
    int32_t min_hits;
    int32_t max_gap;
    int32_t order_constraint;
    int32_t min_weighted_hits;
} kgx_params;

/* Host views of a batch's results (CSR by sequence).  Owned by the context
 * and valid until the next call on it.  otus are in otus_by_count order. */
typedef struct kgx_result {
    uint32_t n_seq;
    const uint64_t *hit_offsets; /* n_seq + 1 */
    const kgx_hit *hits;
    const uint64_t *call_offsets; /* n_seq + 1 */
    const kgx_call *calls;
    const uint64_t *otu_offsets; /* n_seq + 1 */
    const kgx_otu *otus;
    uint64_t n_windows; /* window positions, sum of max(0, len-8); those holding a
                           non-standard residue are skipped, not probed */
    const kgx_best_call *best; /* n_seq entries with KGX_WANT_BEST, else NULL */
} kgx_result;

/* Device-resident results of kgx_run_device (pointers into HBM).
 * Windows are numbered across the batch: sequence s owns global windows
 * [window_base[s], window_base[s+1]) (position = global - window_base[s]).
 * The probe works in tiles of tile_windows consecutive windows; tile t's hits
 * are stored compacted in window order from slot t * tile_windows, and bit i
 * of hit_mask[g] is set when global window 64*g + i hit.  So the hits of a
 * sequence are, word by word of its mask range, contiguous stretches of its
 * tiles' hit lists, and a hit's window (hence its sequence and position)
 * is its mask bit.  Hit records, by hit_format:
 *   KGX_HIT_PACKED16 (PACKED16 images): one 16-byte record per slot in
 *     hits_hot, the matching table record itself (kgx_image_set_layout's
 *     packed layout), flags (KGX_HIT_*) in bits 28-30 of its 4th word;
 *     hits_cold is NULL;
 *   KGX_HIT_PLANES (AOS24 images): two 16-byte records at the same slot:
 *     hits_hot[i]  = {avg_from_end | flags << 16, function_index, function_wt, pos}
 *     hits_cold[i] = {which_kmer (low, high 32 bits), otu_index, seq}
 * Calls of s are contiguous from calls[window_base[s]]; counts are
 * hit_count[s] / call_count[s]. */
typedef struct kgx_device_result {
    uint32_t n_seq;
    uint32_t tile_windows;
    const uint64_t *window_base; /* n_seq + 1: exclusive scan of max(0, len-8) */
    const uint64_t *hit_mask;    /* ceil(window_base[n_seq] / 64) words */
    const uint32_t *hit_count;   /* n_seq */
    const uint32_t *call_count;  /* n_seq */
    const uint32_t *hits_hot;    /* 4 words per slot, capacity window_base[n_seq] slots */
    const uint32_t *hits_cold;   /* 4 words per slot */
    const kgx_call *calls;       /* capacity window_base[n_seq] */
    const kgx_best_call *best;   /* n_seq, after a score stage with KGX_WANT_BEST, else NULL */
    uint32_t hit_format;         /* KGX_HIT_PACKED16 or KGX_HIT_PLANES */
    /* with KGX_WANT_OTU (else NULL): sequence s's KmerOtuStats::otus_by_count
     * pairs at otus[window_base[s] ..+ otu_count[s]) */
    const uint32_t *otu_count;   /* n_seq */
    const kgx_otu *otus;
} kgx_device_result;
#define KGX_HIT_PLANES 0u
#define KGX_HIT_PACKED16 1u

typedef struct kgx_image kgx_image;
typedef struct kgx_ctx kgx_ctx;

/* ---- library ------------------------------------------------------------ */
const char *kgx_version(void);
const char *kgx_last_error(void);
const char *kgx_strerror(int code);
/* number of visible gfx950 devices (0 in a GPU-less container) */
int kgx_device_count(void);
int kgx_params_default(kgx_params *p);
/* How the library's host threads wait for their own device work (the small-
 * batch path, rollups, collects): KGX_WAIT_SPIN (the default: the HIP
 * runtime's own wait, which polls), KGX_WAIT_SLEEP (poll every poll_us, the
 * thread asleep in between; poll_us 0 = 20) or KGX_WAIT_BLOCK (blocking-sync
 * events).  Process-wide; the environment variable KGX_HOST_WAIT
 * (spin|sleep[:us]|block) sets the starting mode.  A server whose workers
 * share a CPU quota gives the spinning time back to its other threads. */
#define KGX_WAIT_SPIN 0
#define KGX_WAIT_SLEEP 1
#define KGX_WAIT_BLOCK 2
int kgx_set_host_wait(int mode, uint32_t poll_us);
int kgx_get_host_wait(uint32_t *poll_us);
/* set_parameters (kguts.cc:244-268) over parallel name/value string arrays:
 * resets to the defaults, then applies std::stoi to the four known names;
 * an unparsable value leaves the default (the reference only warns). */
int kgx_params_parse(kgx_params *p, const char *const *names, const char *const *values, size_t n);

/* ---- images: replaces KmerImage (kmer_image.h:25-39, kmer_image.cc) ----- */
/* Load <dir>/kmer.table.mem_map into HBM of `device`, validating size,
 * version and entry size exactly as kmer_image.cc:128-147. */
int kgx_image_open(const char *dir, int device, kgx_image **out);
/* One replica per entry of devices[0..n) (north_star: the read-only image
 * replicated per GPU): the file is read ONCE -- each chunk is pread into
 * pinned host memory and copied up to every device on that device's own
 * link -- then every replica is packed on its device.  A device may be
 * listed more than once (independent replicas on one GPU).  out[i] receives
 * the replica on devices[i]; on failure every out[i] is NULL.  Replaces one
 * KmerImage per process (threadpool.cc:18-20) when a process drives several
 * GPUs. */
int kgx_image_open_replicas(const char *dir, const int *devices, uint32_t n, kgx_image **out);
/* A replica of src on `device`, copied device to device (hipMemcpyPeer: over
 * xGMI between two GPUs, a local copy on the same GPU): same resident layout
 * and presence filter, identical lookups. */
int kgx_image_replicate(const kgx_image *src, int device, kgx_image **out);
/* Same, from an in-memory file image (header followed by the table). */
int kgx_image_from_memory(const void *file_bytes, uint64_t nbytes, int device, kgx_image **out);
/* Synthetic image built in HBM (close_kmers_amd/synth.py documents the
 * generator): n_keys entries in num_sigs buckets, duplicates dropped (lowest
 * entry id wins), linear probing as kguts.cc:166-171.  *n_stored receives the
 * number of distinct keys stored. */
int kgx_image_build_synthetic(uint64_t n_keys, uint64_t num_sigs, int device, kgx_image **out,
                              uint64_t *n_stored);
/* The same generator (source proteins of the n_keys spec), its entry stream
 * extended past n_keys with random keys, cut after the first *n_entries
 * entries that hold exactly n_distinct distinct keys (the smallest such
 * count): SURVEY §8(d)'s "1B-entry image" = 1e9 distinct keys stored. */
int kgx_image_build_synthetic_distinct(uint64_t n_keys, uint64_t n_distinct, uint64_t num_sigs, int device,
                                       kgx_image **out, uint64_t *n_entries);
/* An image from caller entries (host arrays, n each), in num_sigs buckets:
 * KmerGuts::insert_kmer semantics (kguts.cc:166-228) -- keys above 20^8
 * are skipped, KGX_EFULL when the valid entries (duplicates included) reach
 * num_sigs / 2; of duplicated keys the lowest index is the one lookups find,
 * as with the sequential builder.  Bucket placement may differ from a
 * sequential build (parallel insertion); lookups are identical. */
int kgx_image_build(const uint64_t *keys, const int32_t *function_index, const int32_t *otu_index,
                    const uint16_t *avg_from_end, const float *function_wt, uint64_t n, uint64_t num_sigs,
                    int device, kgx_image **out, uint64_t *n_stored);
/* write <dir>/kmer.table.mem_map in the file format (save_kmer_hash_table,
 * kguts.cc:194-234 with the header of kmer_image.h:25-30), loadable by
 * KmerImage and kgx_image_open */
int kgx_image_save(const kgx_image *img, const char *dir);
int kgx_image_close(kgx_image *img);
uint64_t kgx_image_num_sigs(const kgx_image *img);
int kgx_image_device(const kgx_image *img);
/* HBM-resident layouts.  The file format is never changed; in HBM an image
 * is kept either as the file's 24-byte buckets (AOS24) or, when every stored
 * bucket has function_index in [-1, 2^20-2] and otu_index in [-1, 2^21-2],
 * as one 16-byte record per bucket at the same slot (PACKED16: one aligned
 * load per bucket examined; 2/3 of the memory).  Lookups give identical
 * results in both.  Images are packed at load when they fit. */
enum { KGX_LAYOUT_AOS24 = 0, KGX_LAYOUT_PACKED16 = 1 };
int kgx_image_layout(const kgx_image *img);
/* convert the resident table in place; KGX_ERANGE if PACKED16 is asked for
 * an image whose payloads do not fit (the image is left unchanged) */
int kgx_image_set_layout(kgx_image *img, int layout);
/* Line index of a PACKED16 image: the same records again in 64-B lines of 4
 * buckets, each key's home at the start of line (key mod n_lines), n_lines =
 * stored keys * 64 / keys_per_64_lines (0 drops the index).  Built from every
 * bucket the reference's probe (lookup_hash_entry, kguts.cc:585-602) reaches
 * first for its key -- a duplicate further on, or an entry behind a stop
 * bucket, is never found there and is left out -- so every probe (batches,
 * fq, the call service) returns exactly what it returns over the reference
 * slots, while a key's chain nearly always ends in its first line: one random
 * 64-B request per window instead of ~1.05.  Costs 64 B * n_lines of HBM
 * beside the PACKED16 table, which downloads, saves and filters keep using.
 * Like set_layout, no call may run on the image meanwhile.  Replicas
 * (kgx_image_replicate) do not inherit it: build it on each that should.
 * Loads past ~48 (75% of the buckets) are accepted for tests of full lines,
 * but linear probing there walks ~1/(1-a)^2 buckets per miss: the build's
 * insert walks and the probes' chains grow steeply (results stay exact);
 * 36 is the measured load. */
int kgx_image_set_line_index(kgx_image *img, uint32_t keys_per_64_lines);
/* lines of the image's line index (0: none) */
uint64_t kgx_image_line_count(const kgx_image *img);
/* Presence filter: 2^log2_bits bits (0 removes it), two bits per stored key
 * in one 64-bit word (blocked Bloom filter).  A probe whose key misses the
 * filter skips the table -- exactly the miss it would have found -- so
 * results never change; a filter small enough to stay in the 256 MiB
 * Infinity Cache turns most misses' DRAM reads into cache reads.  It
 * depends on the key set only (layout changes keep it); contexts use it
 * unless "probe_filter" is 0. */
int kgx_image_set_filter(kgx_image *img, int log2_bits);
/* device pointer to the num_sigs * 24-byte table; NULL while PACKED16 */
const void *kgx_image_table(const kgx_image *img);
/* copy the table as the file's num_sigs * 24-byte buckets to host memory
 * (from PACKED16: pad fields read 0; buckets with a key above 20^8 read as
 * {20^8+1, 0, 0, 0, 0, 0.0}) */
int kgx_image_download(const kgx_image *img, void *dst, uint64_t nbytes);

/* ---- contexts: one per host thread, like one KmerGuts per pool thread --- */
int kgx_ctx_create(kgx_image *img, kgx_ctx **out);
int kgx_ctx_destroy(kgx_ctx *ctx);
/* the HIP stream the context launches on (hipStream_t) */
void *kgx_ctx_stream(kgx_ctx *ctx);
/* tuning knobs (results never change): "probe_variant" 0 = load key and
 * payload of every bucket examined, 1 = keys first (the 8-byte key, or the
 * packed record's low word), payload of the matching bucket only; -1 =
 * the fastest for the image (default: 2 for PACKED16, 0 for PACKED16 with a
 * presence filter, 1 for AOS24);
 * 2 / 3 = PACKED16 without a presence filter: groups of 4 / 8 lanes read one
 * aligned 64-B / 128-B table line per instruction (probe_j 1-4 / 1-2; other
 * combinations run variant 0);
 * "probe_filter" 1 (default) / 0 = use / ignore the image's presence filter;
 * "line_index" 1 (default) / 0 = this context's probes read the image's line
 * index when it has one / the reference slots (in-process A/Bs);
 * "probe_nt" 0 (default) / 1 = the line probe writes its hit records and mask
 * with non-temporal stores;
 * "plan_fused" 0 (default) = the plan (window bases, tile owners) in three
 * launches (reduce, scan, fill); 1 = one launch, a decoupled look-back over
 * workgroups (measured slower beside a probe: its waiting workgroups);
 * 2 = one workgroup of 1,024 threads (batches of up to 2^18 sequences);
 * "probe_serialize" 1 (default) / 0: this context's probes wait for the
 * image's previous probe (any context), so that probes run back to back and
 * the other kernels of the contexts overlap them;
 * "microbench_span" = bytes of the table kgx_microbench_random_read covers
 * (0 = all), "microbench_ilp" (1, 2, 4, 8, 16) reads in flight per lane and
 * "microbench_wgs" (1..32) 256-thread workgroups per CU;
 * "probe_j" = windows per lane (1, 2, 3, 4, 5 or 8, default 2; a tile
 * is 64 * probe_j windows), read at the next plan;
 * "fq_probe_j" (0..4, default 1) = windows per lane of kgx_fq_run_device's
 * DNA probe (fragments as anchors), 0 = probe_j;
 * "fq_fused" 1 (default) = the anchor fragment pass (fq_residues 0) counts,
 * scans and writes in one launch (decoupled look-back over tiles of 64
 * reads), 0 = count, scan, tail and anchor kernels;
 * "fq_plan" 1 (default) = kgx_fq_run_device plans the fragments of the
 * context's own fragment pass with one elementwise kernel (each has >= 11
 * residues, so a window base is its residue offset - 8 per earlier fragment),
 * 0 = the general plan (reduce, scan, scan);
 * "probe_stream" 1 = the image's chained probes all on one image-wide stream
 * (default 0: each on its context's stream, chained by events; same speed);
 * "probe_persist" (0..32, default 0) caps the line probe's grid at that many
 * workgroups per CU, its waves then striding over the tiles (measured slower,
 * DESIGN.md §5);
 * "score_variant" 0 (default) = hybrid run scorer: one lane per sequence,
 * except sequences of 2,049..39,998 windows, which the wave-parallel scorer
 * takes (a lane walking a 30k-aa protein would hold the stage for ms);
 * 1 = the wave-parallel scorer for every sequence (ballots over 64 queued
 * hits, serial f32 sums only); 2 = lanes only.  The wave scorer needs
 * order_constraint 0 (else lanes).  Results are identical;
 * "score_wave_tiles" (1..256, default 16) = probe tiles of windows per wave;
 * "fq_count" 1 (default) = the fq count pass scans stop codons one lane per
 * read, 0 = it translates like the emit pass (one wave per read);
 * "fq_residues" 1 (default) = kgx_fq_fragments writes the fragments'
 * residues; 0 = fragment anchors only (see kgx_fragments), for
 * kgx_fq_run_device;
 * "host_chunks" (1..64, default 6): kgx_process_batch splits a batch into up
 * to this many residue-balanced chunks of whole sequences (at least 2M
 * residues each; with "host_taper" 1, the default, the first and last are
 * half the others), alternating between the context and a twin context it
 * creates on first use, so that one chunk's D2H overlaps later chunks' H2D and
 * kernels; "host_copy" 1 (default) / 0: a chunk's results reach the host by
 * device stores into mapped pinned memory ("host_copy_blocks" workgroups,
 * default 64) / by DMA (hipMemcpyAsync).  PACKED16 images with hits wanted
 * ("host_hits16" 1, the default): hits cross PCIe as table records without
 * position or sequence (12 bytes with "host_rec12" 1, the default, the key
 * re-encoded on the host from the residues; else the 16-B records) plus the
 * batch's hit mask, and "host_threads" (default 12) host threads expand them
 * into kgx_hit records while later chunks stream ("host_nt" 1: with streaming
 * stores).  "host_h2d_first" 1 (default): a chunk's D2H starts once the next
 * chunk's residues are up (an H2D beside the D2H's stores is slowed 3-4x).
 * "host_stage_all" 1: every chunk is staged into pinned memory of its own, so
 * staging never waits for an earlier chunk's H2D (0, the default: the two
 * contexts' staging buffers, each reused once its last H2D is done; the same
 * batch time).
 * "pinned_input" 1 (default): a streamed batch whose residues already lie in
 * pinned, device-mapped host memory (kgx_host_alloc, hipHostMalloc,
 * hipHostRegister) is read by DMA straight from the caller's buffer -- no
 * staging copy on the host; a device scan looks for NUL bytes, and a batch
 * with one reruns staged, cut at the NUL as always (kgx_ctx_stat
 * "pinned_batches", "nul_reruns").
 * "host_stream_dma" 1: the streamed chunks' copies by DMA, each host region
 * copied whole at its room (0, the default: device stores of the counted
 * records into mapped memory).
 * "host_upload_stream" 1: chunks go up on a stream of their own into
 * per-batch device regions as soon as they are staged (0, the default: on
 * the context's stream, behind the chunk before).  "host_score_variant" (default 1,
 * the wave scorer; -1: the context's "score_variant"): the streamed chunks'
 * scorer.
 * "host_stream" 1 (default): chunks need no host round trip -- CSR offsets
 * are scanned on the device and the bulk copies (on a separate copy stream)
 * are sized on the device into host regions sized from the hit / call / OTU
 * rates of earlier batches; a batch that overflows them reruns on the exact
 * schedule (host_stream 0: counts to the host, then gather and copy, with
 * "counts_first" 1 holding chunk k's bulk copy until chunk k+1's counts are
 * out).  "stage_threads" (default 8): threads copying the caller's residues
 * into pinned staging.  "small_batch" (0..2^24 residues, default 2^21; 0 =
 * off): a one-chunk batch of at most this many residues is planned on the
 * host, read by the device from mapped pinned staging and its results stored
 * into mapped memory -- one host wait, no DMA copy (process_aa_seq's
 * latency), scored by the wave scorer unless "small_wave" is 0, with "small_wave_tiles"
 * (default 1) probe tiles per scorer wave.
 * "small_fused" 1 (default 0): such a batch runs as ONE launch when the image
 * is PACKED16, want is within HITS | CALLS, order_constraint is 0, min_hits
 * >= 1 and no sequence has more than 2,048 windows -- one workgroup per
 * sequence encodes, probes, scores and stores its records into mapped memory
 * (kgx_fused.hip); nothing of the batch stays on the device, so it is for
 * per-sequence callers (the facade's process_aa_seq), not for a batch that
 * kgx_kmap_add_hits / kgx_matrix_add_hits reads.  Results are
 * identical under every setting.  After a
 * chunked batch the device results are split over the two contexts:
 * kgx_kmap_add_hits / kgx_matrix_add_hits need a one-pass batch (host_chunks
 * 1, or want 0, which never chunks) */
int kgx_ctx_set_option(kgx_ctx *ctx, const char *name, int64_t value);
/* counters of the context since its creation: "fused_batches" / "small_batches"
 * (small host batches that took the one-launch path / the one-wait path),
 * "stream_fallbacks" (streamed batches rerun exact after a region overflow or
 * a NUL in pinned input), "pinned_batches" (streamed batches read straight from
 * the caller's pinned residues), "nul_reruns" */
int kgx_ctx_stat(kgx_ctx *ctx, const char *name, int64_t *value);
/* launch on a caller-owned stream instead (hipStream_t; NULL = own stream) */
int kgx_ctx_set_stream(kgx_ctx *ctx, void *stream);

/* Host-buffer batch: process_aa_seq (kguts.cc:888-908) for every sequence of
 * the batch.  residues: concatenated sequence bytes; seq_offsets[n_seq+1]
 * delimits them.  Each sequence is cut at its first NUL byte, as
 * gather_hits' strlen() bound does (kguts.cc:792).  Synchronous; the result
 * views stay valid until the next call on ctx.  Large batches run in chunks
 * (option "host_chunks"); the results are the same. */
int kgx_process_batch(kgx_ctx *ctx, const kgx_params *params, const char *residues,
                      const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want,
                      kgx_result *out);

/* ---- compact host results ----------------------------------------------
 * What crosses PCIe, handed over without building 32-byte kgx_hit records
 * (239 MB per 30M-residue C2 batch): per hit a record of the matched table
 * bucket without its key, plus one hit-mask bit per window.  A hit's window
 * -- hence its sequence and position -- is its mask bit, and its key is the
 * window's 8-mer, re-encoded from the caller's residues.  The hits come in
 * chunks of consecutive sequences:
 *   records        record_words (3 or 4) 32-bit words per hit, CSR order:
 *                  hit j of the batch (hit_offsets numbering) is at
 *                  records + record_words * (j - hit_begin); the words are
 *                  the PACKED16 bucket minus the key bits and
 *                  are opaque: kgx_compact_expand decodes them
 *   mask           chunk window w hit <=> bit w % 64 of mask[w / 64]
 *   window_start   sequence s's first chunk window is window_start[s -
 *                  seq_begin]; it owns max(0, len - 8) windows
 * hit_in_sequence_t (kguts.h:228-233) for any hit is thus built on the fly,
 * which is how the KmerGuts facade replays hit_cb (kguts.cc:814-815). */
typedef struct kgx_hit_chunk {
    uint32_t seq_begin, seq_end; /* the chunk's sequences [seq_begin, seq_end) */
    uint32_t record_words;
    uint32_t reserved;
    uint64_t hit_begin;
    const uint32_t *records;
    const uint64_t *mask;
    const uint64_t *window_start;
} kgx_hit_chunk;
typedef struct kgx_compact_result {
    /* offsets, calls, OTUs, best calls and n_windows as kgx_result; r.hits is
     * NULL when the hits are compact (n_chunks > 0), else (a batch that took
     * a path without compact records: small, one-pass or AOS24) the kgx_hit
     * records themselves, with n_chunks 0 */
    kgx_result r;
    uint32_t n_chunks;
    const kgx_hit_chunk *chunks;
} kgx_compact_result;
/* kgx_process_batch with compact hits: the same offsets, calls, OTUs and best
 * calls; the hits stay as the compact records (no kgx_hit expansion on the
 * host).  Views owned by ctx, valid until its next call. */
int kgx_process_batch_compact(kgx_ctx *ctx, const kgx_params *params, const char *residues,
                              const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want,
                              kgx_compact_result *out);
/* kgx_hit records of sequences [s_begin, s_end) of a compact result into out
 * (out[0] = the first hit of s_begin; hit_offsets[s_end] - hit_offsets[s_begin]
 * records), kgx_hit.seq = batch index + seq_base.  residues / seq_offsets are
 * the batch's, as passed to the call that produced r.  Thread-safe (reads r
 * only): ranges may be expanded on several threads at once. */
int kgx_compact_expand(const kgx_compact_result *r, const char *residues, const uint64_t *seq_offsets,
                       uint32_t s_begin, uint32_t s_end, uint32_t seq_base, kgx_hit *out);

/* Resident call service: KmerGuts::process_aa_seq for ONE sequence
 * (kguts.cc:888-908) without a kernel launch per call -- for worker pools
 * that call per sequence (threadpool.cc:18-44, lookup_request.cc:153-172).
 * Persistent workgroups on the image's device, one per slot, poll slots in
 * mapped host memory; the call writes its sequence into a free slot and spins
 * until the device has stored its records.  Thread-safe; started on the first
 * call; instances of the workgroups last life_us each and the host keeps one
 * queued behind the running one while calls arrive, so the service leaves the
 * GPU within 2 x life_us of the last call (restarted on demand).  Serves
 * PACKED16 images, want within KGX_WANT_HITS | KGX_WANT_CALLS | KGX_WANT_OTU,
 * order_constraint 0, min_hits >= 1, sequences of at most 2,056 residues;
 * anything else, or every slot busy, returns KGX_EBUSY and the caller takes a
 * batch path (kgx_process_batch*).  Results as kgx_process_batch gives them
 * for a batch of this one sequence (kgx_hit.seq = 0, hits in position order;
 * OTU pairs in otus_by_count order); hits_cap / calls_cap / otus_cap must be
 * at least the sequence's window count (len - 8) for what want asks. */
int kgx_svc_call(kgx_image *img, const kgx_params *params, const char *seq, uint64_t len, uint32_t want,
                 kgx_hit *hits, uint64_t hits_cap, uint64_t *n_hits, kgx_call *calls, uint64_t calls_cap,
                 uint64_t *n_calls, kgx_otu *otus, uint64_t otus_cap, uint64_t *n_otus);
/* slots (1..64, default 32) and life_us (default 1000: an instance's stay
 * before the next one, already enqueued, takes over; bounds how long the
 * service holds its hardware queue); stops a running service (as
 * kgx_svc_stop) and applies the settings in one step, so the next call starts
 * the service with them.  idle_us is checked (>= 10, <= life_us) and ignored:
 * a per-workgroup idle exit could strand a quiet slot's next request
 * (DESIGN.md §8.8).  The KGX_SVC_LIFE_US environment default applies only to
 * images this was never called for. */
int kgx_svc_config(kgx_image *img, uint32_t slots, uint32_t idle_us, uint32_t life_us);
/* Stops the service: its workgroups leave and its memory is freed (so do
 * kgx_svc_config, kgx_image_set_layout / set_filter and kgx_image_close).
 * Safe while other threads are inside kgx_svc_call: it waits until they have
 * returned (their calls are served); a call that starts afterwards starts a
 * new service.  A call that gets no answer within 10 s (KGX_SVC_TIMEOUT_MS)
 * returns KGX_EDEVICE and leaves its slot for good (a late answer may still
 * land in it) and the service "broken": every later call, and every call
 * still waiting, returns KGX_EBUSY (take a batch path) until kgx_svc_stop or
 * kgx_svc_config replaces the service.  Stopping never waits on the runtime
 * without a bound: it waits at most 2 s for the workgroups to leave, and a
 * service whose workgroups did not is left allocated ("leaked") rather than
 * freed under them.  A request whose residues never reached the device
 * returns KGX_EBUSY. */
int kgx_svc_stop(kgx_image *img);
/* "slots", "calls" (served), "launches" (instances enqueued), "busy" (calls
 * turned away for want of a slot), "abandoned" (slots given up after a 10-s
 * wait), "broken" (1: calls are turned away until the service is replaced),
 * "leaked" (process-wide: stopped services whose workgroups did not leave
 * within 2 s, their memory kept),
 * "devmem" (1: requests are written into fine-grained device memory through a
 * large BAR, else mapped host memory; KGX_SVC_DEVMEM=0 forces the latter),
 * "priority" (100 + the service stream's priority; the stream is created at
 * the device's highest priority, so it has a hardware queue of its own and
 * batch streams never queue behind the persistent instances;
 * KGX_SVC_PRIORITY=normal gives it a normal stream),
 * "phase_n0".."phase_n15" (with KGX_SVC_DEBUG=1: summed ns of the host wall per
 * call, the device phases, the OTU tally of calls that want it and the
 * tally's final sort by count; n8 the probe rounds x 1000, n9 the probe's
 * first round, n10 its keys and homes, n11 thread 0's first-round loads,
 * n12 / n13 the scorer's first chunk's runs / sums, n14 the final system
 * fence: what is left of the results' stores to host memory, n15 the OTU
 * sort's shader clock cycles: n15 / n7 its clock) */
int kgx_svc_stat(kgx_image *img, const char *name, uint64_t *value);

/* Host-side profile of the context's last kgx_process_batch* call with option
 * "host_profile" 1 (HIP events per chunk; otherwise zeros).  Device stages are
 * sums over the batch's chunks of HIP-event intervals; host stages are wall
 * times on the host (expand_ms summed over the expansion threads). */
typedef struct kgx_host_profile {
    uint32_t chunks;
    uint32_t streamed;   /* 1: the streamed schedule (no host round trip per chunk) */
    double wall_ms;      /* the whole call */
    double stage_ms;     /* caller residues -> pinned staging (host copy) */
    double h2d_ms;       /* staged residues -> HBM */
    double device_ms;    /* plan + probe + score */
    double gather_ms;    /* count scan + gather into dense buffers */
    double d2h_ms;       /* the bulk copy to pinned host memory (from gather end, incl. queueing) */
    double expand_ms;    /* kgx_hit records built on host threads (0 in compact mode) */
    uint64_t h2d_bytes;
    uint64_t d2h_bytes;
} kgx_host_profile;
int kgx_ctx_host_profile(kgx_ctx *ctx, kgx_host_profile *out);

/* Device-buffer batch: same computation on residues / offsets already in HBM
 * (NUL-free sequences), enqueued on the context's stream without host
 * synchronisation.  The results stay in HBM (kgx_device_result).
 * Preconditions (checked on the device): d_seq_offsets[0..n_seq] are
 * monotone, absolute indices into d_residues, and d_seq_offsets[n_seq] -
 * d_seq_offsets[0] <= n_residues (the buffers are sized from n_residues).  A
 * batch that breaks them is processed as empty (no out-of-bounds access);
 * kgx_ctx_check and kgx_device_batch_collect then return KGX_EINVAL. */
int kgx_run_device(kgx_ctx *ctx, const kgx_params *params, const uint8_t *d_residues,
                   const uint64_t *d_seq_offsets, uint32_t n_seq, uint64_t n_residues,
                   uint32_t want, kgx_device_result *out);

/* The stages kgx_run_device enqueues, for per-kernel timing:
 *   kgx_stage_plan   window/chunk bookkeeping (2 small kernels)
 *   kgx_stage_probe  encode + probe: the HBM random-access kernel
 *   kgx_stage_score  hit-run scorer (calls, OTU flags; find_best_call with KGX_WANT_BEST) */
int kgx_stage_plan(kgx_ctx *ctx, const uint64_t *d_seq_offsets, uint32_t n_seq, uint64_t n_residues);
/* waits for the context's stream; KGX_EINVAL when its last plan found bad
 * offsets (see kgx_run_device), else KGX_OK */
int kgx_ctx_check(kgx_ctx *ctx);
int kgx_stage_probe(kgx_ctx *ctx, const uint8_t *d_residues, const uint64_t *d_seq_offsets);
int kgx_stage_score(kgx_ctx *ctx, const kgx_params *params, uint32_t want);
int kgx_device_result_get(kgx_ctx *ctx, kgx_device_result *out);

/* Synthetic query batch generated in HBM (synth.py make_queries). */
int kgx_synth_queries(kgx_ctx *ctx, uint64_t image_n_keys, uint32_t n_seq, uint32_t length,
                      uint32_t x_permille, uint64_t q0, uint8_t *d_residues,
                      uint64_t *d_seq_offsets);

/* ---- pools: one batch split across GPUs --------------------------------
 * north_star: query batches are split across the GPUs of one node with no
 * collective (sequences are independent, lookup_request.cc:153; KmerGuts
 * state is per sequence, kguts.h:263-266).  A pool holds n_ctx contexts,
 * context i on images[i % n_images] (typically one replica per GPU), each
 * driven by its own host thread -- the reference's thread pool of KmerGuts
 * over one image (threadpool.cc:18-44), spread over the node's GPUs. */
typedef struct kgx_pool kgx_pool;
int kgx_pool_create(kgx_image *const *images, uint32_t n_images, uint32_t n_ctx, kgx_pool **out);
int kgx_pool_destroy(kgx_pool *pool);
uint32_t kgx_pool_size(const kgx_pool *pool);
/* context i of the pool (owned by the pool; options may be set on it) */
kgx_ctx *kgx_pool_ctx(kgx_pool *pool, uint32_t i);
/* kgx_process_batch over the pool: the batch is cut into contiguous,
 * residue-balanced shards of whole sequences (kgx_shard_cuts), one per
 * running context -- the first two contexts of each device (environment
 * KGX_POOL_PER_DEVICE; a host batch on more contexts of one device only
 * queues behind the others' waits in the process's few hardware queues) --
 * all at once, on every GPU, and the results are concatenated in input order:
 * the same CSR, the same bytes (kgx_hit.seq included) as one context
 * processing the whole batch.  The views are owned by the pool and valid
 * until its next call. */
int kgx_pool_process_batch(kgx_pool *pool, const kgx_params *params, const char *residues,
                           const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want, kgx_result *out);
/* The same with compact hits (kgx_process_batch_compact): every shard's
 * chunks, renumbered into the whole batch (seq_begin / seq_end / hit_begin),
 * pointing into the shard contexts' pinned buffers -- no host copy of any
 * hit.  When some shard's hits did not come back compact, every shard's hits
 * are expanded into one kgx_hit array instead (r.hits, n_chunks 0). */
int kgx_pool_process_batch_compact(kgx_pool *pool, const kgx_params *params, const char *residues,
                                   const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want,
                                   kgx_compact_result *out);
/* kgx_pool_lookup's map for each running context: the first of the maps
 * whose device (kgx_kmap_device; -1 for a missing map) is the context's --
 * pick[i] indexes map_device; KGX_EINVAL when a context's device has none.
 * Host only (no device needed). */
int kgx_pool_map_select(const int32_t *ctx_device, uint32_t n_ctx, const int32_t *map_device, uint32_t n_maps,
                        int32_t *pick);
/* NUMA placement (the reference binds each worker's thread and memory to a
 * node, numa.cc:13-42): every pool context's host thread is bound at creation
 * to the CPUs of its device's NUMA node that the process may use (its affinity
 * mask), so that the pinned staging it grows and the copies into it stay on
 * the device's socket (pinned host memory is placed by first touch of the
 * allocating thread's node).  KGX_POOL_NUMA=0 leaves the threads unbound.
 * kgx_pool_numa_node: the node context i's thread is bound to, -1 when it is
 * not (unknown node, no usable CPU of it, or binding off). */
int kgx_pool_numa_node(const kgx_pool *pool, uint32_t i);
/* the NUMA node of a device: /sys/bus/pci/devices/<bus id>/numa_node of its
 * PCI function (-1: unknown or no NUMA information) */
int kgx_device_numa_node(int device);
/* the CPUs of NUMA node `node` that this process may run on (its affinity
 * mask and the node's cpulist, /sys/devices/system/node/node<N>/cpulist):
 * their count, and the first cap of them in cpus (may be NULL).  Needs no
 * device. */
int kgx_numa_node_cpus(int node, uint32_t *cpus, uint32_t cap);
/* free and total HBM of a device (hipMemGetInfo) */
int kgx_device_memory(int device, uint64_t *free_bytes, uint64_t *total_bytes);
/* cut points of n_shards contiguous residue-balanced shards: shard i is
 * sequences [cuts[i], cuts[i+1]), cuts[0] = 0, cuts[n_shards] = n_seq; cut i
 * is the first sequence starting at or after residue (total * i / n_shards)
 * (close_kmers_amd/shard.py balanced_shards).  Shards may be empty. */
int kgx_shard_cuts(const uint64_t *seq_offsets, uint32_t n_seq, uint32_t n_shards, uint32_t *cuts);

/* ---- host-side rules on results (run on the CPU, no device needed) ------ */
/* find_best_call (kguts.cc:1008-1199) over one sequence's calls.  names /
 * n_names is the function.index table (function_at_index, kguts.h:361-366).
 * *function receives the called function (NUL-terminated, truncated to
 * function_cap).  *score_offset_set is 0 when the reference leaves
 * score_offset untouched (no calls). */
int kgx_find_best_call(const kgx_call *calls, size_t n_calls, const char *const *names,
                       int n_names, int32_t *function_index, char *function, size_t function_cap,
                       float *score, float *weighted_score, float *score_offset,
                       int *score_offset_set);

/* a float as the reference's iostreams print it (operator<< at the default
 * precision: printf's %.6g of the value widened to double), NUL-terminated
 * into out (cap bytes); returns the full length.  Host only. */
size_t kgx_format_g6(float v, char *out, size_t cap);

/* find_best_call for many sequences at once, on the context's device:
 * sequence s owns calls[call_offsets[s] .. call_offsets[s+1]) (host arrays);
 * out[n_seq] receives each decision (kgx_best_call).  Synchronous. */
int kgx_find_best_calls(kgx_ctx *ctx, const kgx_call *calls, const uint64_t *call_offsets, uint32_t n_seq,
                        kgx_best_call *out);

/* Random-access ceiling of the context's image buffer: about n_reads
 * uniformly random records of the resident table read with many loads in
 * flight.  mode 0: a whole 24-byte bucket (key + payload, the AOS24 probe's
 * access), 1: the 8-byte key of a 24-byte bucket, 2: one aligned 64-byte
 * sector, 3: one aligned 16-byte record (the PACKED16 probe's access),
 * 4 / 5: one aligned 64-byte / 128-byte line read cooperatively by 4 / 8
 * lanes, 16 B each, in one instruction.  *ms = kernel time (HIP events),
 * *reads = records (modes 0-3) or lines (modes 4-5) actually read. */
int kgx_microbench_random_read(kgx_ctx *ctx, uint64_t n_reads, int mode, float *ms,
                               uint64_t *reads);

/* The current device batch's results (after kgx_run_device or the three
 * stages) as the host CSR kgx_process_batch returns; buffers as there. */
int kgx_device_batch_collect(kgx_ctx *ctx, uint32_t want, kgx_result *out);

/* ---- fq reads -> protein fragments (the fq handler's input side) --------
 * For every read and frame 1, 2, 3, -1, -2, -3 (DNASequence::
 * get_possible_proteins, dna_seq.cc:9-47): genetic code 11 translation
 * (trans_table.cc:36-84; codons with a base outside ACGTU/acgtu give 'X'),
 * split at '*', fragments longer than 10 residues kept
 * (fq_process_request.cc:329-343).  The fragments form a protein batch in
 * (read, frame, position) order, on the device, owned by ctx and valid until
 * the next fq call: feed it to kgx_fq_run_device (or, when residues is set,
 * kgx_run_device).
 *
 * With the context option "fq_residues" 0 (and a PACKED16 image probed by the
 * line probe, probe_j 1-4) the residues are not written: residues is NULL and
 * each fragment carries an anchor into the reads' bases instead, from which
 * kgx_fq_run_device's probe translates each window's 8 codons itself; read
 * and frame are NULL too (frame_counts gives both: read r's fragments are
 * frame_counts[6r..6r+5] of frames 1, 2, 3, -1, -2, -3 in turn). */
typedef struct kgx_fragments {
    uint32_t n_reads;
    uint32_t n_fragments;
    uint64_t n_residues;
    const uint8_t *residues;  /* device: fragment residues, concatenated (NULL: anchors) */
    const uint64_t *offsets;  /* device: [n_fragments + 1] */
    const uint32_t *read;     /* device: read index of each fragment (NULL with anchors) */
    const int8_t *frame;      /* device: frame of each fragment (NULL with anchors) */
    const uint32_t *frame_counts; /* device: fragments per (read, frame), [n_reads * 6] */
    const uint64_t *anchors;  /* device, when residues is NULL: per fragment (byte index in bases of its
                                 first codon's first base) << 1 | 1 on the reverse strand */
    const uint8_t *bases;     /* device: the reads' bases the anchors index */
    uint64_t n_bases;         /* bytes readable from bases */
} kgx_fragments;
/* reads from host memory (bases concatenated, read_offsets[n_reads + 1]) */
int kgx_fq_fragments(kgx_ctx *ctx, const char *bases, const uint64_t *read_offsets, uint32_t n_reads,
                     kgx_fragments *out);
/* kgx_fq_fragments in two steps, so that one block's upload overlaps earlier
 * blocks' work: _upload enqueues the H2D of the reads' bases and offsets on
 * ctx's stream and returns at once (bases in pinned memory go by DMA straight
 * from there and must stay unchanged until _uploaded returns; others are
 * staged first); _uploaded runs the fragment pass over them, as
 * kgx_fq_fragments does.  Nothing else may run on ctx between the two. */
int kgx_fq_upload(kgx_ctx *ctx, const char *bases, const uint64_t *read_offsets, uint32_t n_reads);
int kgx_fq_fragments_uploaded(kgx_ctx *ctx, kgx_fragments *out);
/* kgx_fq_fragments_uploaded in two halves: _start enqueues the fragment pass
 * over the uploaded reads behind their upload and returns at once;
 * kgx_fq_fragments_finish waits for it and fills out.  The fq handler starts
 * a part's pass as soon as its upload is enqueued, a part ahead of its
 * lookup, so the pass runs in the previous probe's tail and sizing the part
 * never holds the GPU idle between two probes.  The bases stay in use until
 * _finish returns; nothing else may run on ctx between the two calls. */
int kgx_fq_fragments_uploaded_start(kgx_ctx *ctx);
/* reads already in device memory */
int kgx_fq_fragments_device(kgx_ctx *ctx, const uint8_t *d_bases, const uint64_t *d_read_offsets,
                            uint32_t n_reads, kgx_fragments *out);
/* kgx_fq_fragments_device in two halves, for chunked streams of reads: _start
 * enqueues the fragment pass on ctx's stream and returns at once; _finish
 * waits for it and fills out (the same fragments).  Between the two the host
 * can enqueue other contexts' work -- the previous chunk's lookup -- so that
 * sizing one chunk never holds the GPU between two probes.  n_bases: the
 * caller's bound on the bytes the reads span and may read (d_read_offsets[0]
 * >= 0, d_read_offsets[n_reads] <= n_bases); a span past it is an error from
 * _finish, with nothing written past the buffers.  Nothing else may run on
 * ctx between the two calls. */
int kgx_fq_fragments_device_start(kgx_ctx *ctx, const uint8_t *d_bases, const uint64_t *d_read_offsets,
                                  uint32_t n_reads, uint64_t n_bases);
int kgx_fq_fragments_finish(kgx_ctx *ctx, kgx_fragments *out);
/* lookup + run scoring of a fragment batch: kgx_run_device over
 * (residues, offsets) when the residues were written, else plan, the probe
 * over the anchors (windows translated from the bases), score.  Same results. */
int kgx_fq_run_device(kgx_ctx *ctx, const kgx_params *params, const kgx_fragments *fragments, uint32_t want,
                      kgx_device_result *out);

/* After kgx_run_device over a kgx_fragments batch (with KGX_WANT_CALLS): only
 * the reads that have a call in some fragment, in read order, with what the
 * fq handler's frame choice reads of them (fq_process_request.cc:298-365):
 * per read its fragments per frame, per fragment its length and its calls.
 * Host views owned by the context, valid until its next call:
 *   reads[n]                       read indices
 *   frame_counts[6 n]              fragments per (read, frame)
 *   frag_offsets[n + 1]            read i's fragments [frag_offsets[i], frag_offsets[i+1])
 *   frag_len[...], call_offsets[...+1], calls[...]   per fragment */
typedef struct kgx_fq_called {
    uint32_t n;
    const uint32_t *reads;
    const uint32_t *frame_counts;
    const uint64_t *frag_offsets;
    const uint32_t *frag_len;
    const uint64_t *call_offsets;
    const kgx_call *calls;
} kgx_fq_called;
int kgx_fq_called_reads(kgx_ctx *ctx, const kgx_fragments *fragments, kgx_fq_called *out);

/* ---- the fq request handler (FqProcessRequest, fq_process_request.cc) ---
 * FASTQ text in, the handler's output lines out (per read: best frame,
 * score and the frame's family matches, fq_process_request.cc:298-365, over
 * FamilyMapper family_mapper.cc:46-205).  data_dir holds function.index and
 * otu.index; genus_file / families_file / nr_fasta (NULL or "" to skip) load
 * the family DB (KmerPegMapping::load_genus_map / load_families kmer.cc:
 * 341-493; NRLoader family mode nr_loader.cc:130-176, proteins in file
 * order).  Blocks are processed as the reference processes request blocks
 * (one FamilyMapper per block); `finished` marks the last block. */
typedef struct kgx_fq kgx_fq;
int kgx_fq_create(kgx_image *img, const char *data_dir, const char *genus_file, const char *families_file,
                  const char *nr_fasta, kgx_fq **out);
int kgx_fq_destroy(kgx_fq *fq);
/* *text: output lines of the block, owned by fq, valid until the next call */
int kgx_fq_process(kgx_fq *fq, const char *fastq, uint64_t n, int finished, const char **text,
                   uint64_t *text_len);

/* ---- k-mer -> id tables in HBM ------------------------------------------
 * KmerPegMapping's kmer_to_id_ (kmer.h:84-127, filled by /add through
 * add_mapping, kmer.cc:173-210: every (k-mer, id) appended, duplicates kept)
 * and kmer_to_family_id_ (add_fam_mapping, kmer.cc:212-256: an id is added to
 * a k-mer's list once, lists in first-insertion order).  Ids are the
 * mapping's encoded ids (KmerPegMapping::encode_id); the id <-> name
 * dictionaries stay with the caller. */
typedef struct kgx_kmap kgx_kmap;
enum { KGX_KMAP_APPEND = 0, KGX_KMAP_SET = 1 };
int kgx_kmap_create(int device, int mode, kgx_kmap **out);
int kgx_kmap_destroy(kgx_kmap *map);
/* add (kmers[i], ids[i]) in order i = 0..n-1 (host arrays) */
int kgx_kmap_add(kgx_kmap *map, const uint64_t *kmers, const uint32_t *ids, uint64_t n);
/* add the hits of the context's last batch (want must have included HITS):
 * for each sequence s in order, each of its hits in position order adds
 * (hit.which_kmer, seq_ids[s]) -- the /add mapping step, add_request.cc:
 * 164-170 / 196-206.  seq_ids: host array of the batch's n_seq ids. */
int kgx_kmap_add_hits(kgx_kmap *map, kgx_ctx *ctx, const uint32_t *seq_ids);
uint64_t kgx_kmap_num_kmers(const kgx_kmap *map);
uint64_t kgx_kmap_num_values(const kgx_kmap *map);
/* host query: offsets[n+1] (CSR over the n k-mers) and, when ids != NULL,
 * the ids (ids_cap >= offsets[n]); unmapped k-mers have empty lists */
int kgx_kmap_lookup(kgx_kmap *map, const uint64_t *kmers, uint64_t n, uint64_t *offsets,
                    uint32_t *ids, uint64_t ids_cap);

/* ---- /lookup per-sequence rollups (LookupRequest::on_hit, lookup_request.cc:
 * 446-482; FamilyMapper::on_hit, family_mapper.cc:287-312) on the device ----
 * For each sequence s of the context's last batch (its hits still on the
 * device: kgx_process_batch / kgx_run_device / kgx_fq_run_device; any want),
 * each hit in position order, with L = map[hit.which_kmer] (no row: skipped):
 *   KGX_ROLLUP_FAMILY (kmer_to_family_id_): w = 1.0f / (float)|L|; for each
 *     id in L: row[id].hit_count++, .hit_total++, .weighted_total += w
 *   KGX_ROLLUP_PEG (kmer_to_id_): for each id in L: row[id].hit_count++
 * weighted_total is the f32 sum in that (hit) order.  A sequence's rows come
 * in the order its ids were first touched (hit order, then list order): a
 * caller that inserts them in that order into the request's one
 * std::unordered_map seq_score_ (cleared per sequence, as the reference does)
 * gets the map the reference's operator[] calls build, bucket by bucket, so
 * its iteration order too.  Buffers are owned by ctx and valid until its next
 * rollup. */
enum { KGX_ROLLUP_PEG = 0, KGX_ROLLUP_FAMILY = 1 };
typedef struct kgx_rollup_row { /* sequence_accumulated_score_t (lookup_request.h:26-42) + its key */
    uint32_t id;
    uint32_t hit_count;
    uint32_t hit_total;
    float weighted_total;
} kgx_rollup_row;
typedef struct kgx_rollup_result {
    uint32_t n_seq;
    const uint64_t *offsets;    /* [n_seq + 1]: sequence s's rows are [offsets[s], offsets[s+1]) */
    const kgx_rollup_row *rows; /* host */
    uint64_t n_events;          /* (hit, list entry) pairs folded */
} kgx_rollup_result;
int kgx_kmap_rollup(kgx_kmap *map, kgx_ctx *ctx, int mode, kgx_rollup_result *out);
/* the device the map lives on */
int kgx_kmap_device(const kgx_kmap *map);

/* /lookup's GPU side for a host batch on ONE context (a server worker's
 * request piece, lookup_request.cc:153-210,446-482): the pass and the rollup
 * over `map` (on the context's device) enqueued together -- upload, plan,
 * probe, score, the counts (and best calls) into mapped memory, the rollup
 * sized by the context's previous one -- and one host wait for both, instead
 * of kgx_process_batch's wait and then kgx_kmap_rollup's.  A batch
 * kgx_process_batch would run down its small-batch path (up to the context's
 * small_batch residues, 65,536 sequences, one chunk) runs down that path with
 * the rollup queued behind it; others take the one-pass path.  want within
 * KGX_WANT_CALLS | KGX_WANT_BEST; results as those two calls give them (out:
 * no hits; the views valid until the context's next call). */
int kgx_lookup(kgx_ctx *ctx, kgx_kmap *map, int mode, const kgx_params *params, const char *residues,
               const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want, kgx_result *out,
               kgx_rollup_result *rollup);
/* /lookup's GPU side for a whole host batch over a pool
 * (LookupRequest::process_work + on_hit, lookup_request.cc:153-210,446-482):
 * the batch is cut into shards of whole sequences (up to twice as many per
 * device as kgx_pool_process_batch: a shard here is one pass, no twin; a
 * device's first and last shards half the others' residues), enqueued in
 * order on the pool's per-device pass, score and rollup streams with no host
 * wait; each runs on its context's buffers as ONE pass (its hits stay on the
 * device),
 * with want within KGX_WANT_CALLS | KGX_WANT_BEST (KGX_WANT_BEST: the
 * find_best_match decision), and then kgx_kmap_rollup over maps[j], the map on
 * that context's device (one map per device the pool spans).  Nothing per hit
 * crosses PCIe.  out: hit and call offsets, calls and best calls over the whole
 * batch (out->hits NULL); rollup: every sequence's rows in input order
 * (offsets over the batch), each sequence's rows in first-touch order as
 * kgx_kmap_rollup gives them.  Views owned by the pool, valid until its next
 * call. */
int kgx_pool_lookup(kgx_pool *pool, kgx_kmap *const *maps, uint32_t n_maps, int mode, const kgx_params *params,
                    const char *residues, const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want,
                    kgx_result *out, kgx_rollup_result *rollup);

/* ---- /matrix pair counting (matrix_request.cc:83-190) --------------------
 * One kgx_matrix per /matrix request (the request's matrix_proteins_ and
 * distance_ state, matrix_request.h:25-26).  For each sequence s of a batch,
 * in order, with id e = seq_ids[s] (e joins the request's seen set first):
 * for every hit of s, for every id f in the hit k-mer's kmap list, if f != e
 * and f was seen in this request, distance_[(e, f)] += 1. */
typedef struct kgx_matrix kgx_matrix;
typedef struct kgx_pair_count { /* one distance_ entry */
    uint32_t id1, id2;
    uint64_t count;
} kgx_pair_count;
int kgx_matrix_create(kgx_kmap *map, kgx_matrix **out);
int kgx_matrix_destroy(kgx_matrix *mx);
/* add the context's last batch (want must have included HITS) */
int kgx_matrix_add_hits(kgx_matrix *mx, kgx_ctx *ctx, const uint32_t *seq_ids);
/* all pair counts so far, ordered by (id1, id2) as std::map iterates
 * distance_; the buffer is owned by mx and valid until the next call */
int kgx_matrix_pairs(kgx_matrix *mx, const kgx_pair_count **pairs, uint64_t *n_pairs);

/* ---- HIP-event timing on a context's stream ----------------------------- */
int kgx_event_create(void **event);
int kgx_event_destroy(void *event);
/* record on the stream `ctx` launches on */
int kgx_event_record(void *event, kgx_ctx *ctx);
/* milliseconds between two recorded events (waits for `end`) */
int kgx_event_elapsed_ms(void *start, void *end, float *ms);

/* Device memory helpers for callers without their own allocator. */
int kgx_device_alloc(int device, uint64_t nbytes, void **out);
int kgx_device_free(void *p);
/* Pinned (page-locked, portable) host memory.  Batch inputs that live in it
 * reach the device by DMA straight from there (kgx_fq_fragments skips its
 * staging copy for such bases). */
int kgx_host_alloc(uint64_t nbytes, void **out);
int kgx_host_free(void *p);
int kgx_memcpy_h2d(void *dst, const void *src, uint64_t nbytes);
int kgx_memcpy_d2h(void *dst, const void *src, uint64_t nbytes);
int kgx_ctx_synchronize(kgx_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* KGX_H */
