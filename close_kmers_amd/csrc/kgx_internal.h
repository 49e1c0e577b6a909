/*
 * kgx_internal.h -- shared definitions between the HIP kernels
 * (kgx_kernels.hip) and the host runtime (kgx_runtime.cpp).
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

/* Probe kernel geometry: one wave owns one chunk of PROBE_J*64 consecutive
 * windows of one sequence (a 300-aa protein is one chunk). */
constexpr int PROBE_J = 5;
constexpr int CHUNK = PROBE_J * 64;
constexpr int PROBE_WAVES = 4; /* waves per 256-thread workgroup */
/* probe variants (kgx_ctx_set_option "probe_variant") */
constexpr int PROBE_BUCKET = 0;    /* key + payload per bucket examined */
constexpr int PROBE_KEY_FIRST = 1; /* keys only; payload for the matching bucket */

/* floor((2^64-1)/n): x % n = x - umulhi(x, m)*n, corrected once (x < 2^35). */
inline uint64_t mod_magic(uint64_t n) { return n ? (~0ULL) / n : 0; }

struct Plan {
    /* device arrays, n_seq + 1 entries each */
    uint64_t *wbase;  /* exclusive scan of windows per sequence */
    uint64_t *cbase;  /* exclusive scan of chunks per sequence */
    uint32_t *chunk_seq; /* chunk -> sequence */
};

/* launchers (kgx_kernels.hip); all asynchronous on `stream` */
size_t plan_workspace_bytes(uint32_t n_seq);
hipError_t launch_plan(const uint64_t *seq_off, uint32_t n_seq, uint64_t *wbase, uint64_t *cbase,
                       uint32_t *chunk_seq, void *workspace, hipStream_t stream);
hipError_t launch_probe(const uint8_t *residues, uint64_t n_residues, const uint64_t *seq_off,
                        const uint64_t *wbase, const uint64_t *cbase, const uint32_t *chunk_seq,
                        uint32_t n_seq, uint64_t max_chunks, const kgx_sig_kmer *table,
                        uint64_t num_sigs, kgx_hit *hits, uint32_t *chunk_hits, int variant,
                        hipStream_t stream);
hipError_t launch_score(uint32_t n_seq, const uint64_t *wbase, const uint64_t *cbase,
                        const uint32_t *chunk_hits, kgx_hit *hits, kgx_call *calls, void *ranges,
                        uint32_t *hit_count, uint32_t *call_count, kgx_params params,
                        uint32_t want, hipStream_t stream);
hipError_t launch_gather(uint32_t n_seq, const uint64_t *wbase, const uint32_t *hit_count,
                         const uint32_t *call_count, const kgx_hit *hits, const kgx_call *calls,
                         const uint64_t *hit_dense_off, const uint64_t *call_dense_off,
                         kgx_hit *hits_out, kgx_call *calls_out, hipStream_t stream);
hipError_t launch_random_read(const kgx_sig_kmer *table, uint64_t num_sigs, uint64_t threads,
                              uint32_t rounds, int mode, uint64_t *sink, hipStream_t stream);
hipError_t launch_synth_image(kgx_sig_kmer *table, uint64_t num_sigs, uint64_t n_keys,
                              unsigned long long *n_stored, hipStream_t stream);
hipError_t launch_synth_queries(uint64_t image_n_keys, uint32_t n_seq, uint32_t length,
                                uint32_t x_permille, uint64_t q0, uint8_t *residues,
                                uint64_t *seq_off, hipStream_t stream);

}  // namespace kgx

#endif
