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
 * compacted, in window order, from hits[tile * tile_windows]; bit i of
 * hit_mask[g] says whether window 64 g + i hit.
 */
constexpr int PROBE_WAVES = 4; /* waves per 256-thread workgroup */
/* probe variants (kgx_ctx_set_option "probe_variant") */
constexpr int PROBE_BUCKET = 0;    /* key + payload per bucket examined */
constexpr int PROBE_KEY_FIRST = 1; /* keys only; payload for the matching bucket */
constexpr int PROBE_J_DEFAULT = 4;

/* floor((2^64-1)/n): x % n = x - umulhi(x, m)*n, corrected once (x < 2^35). */
inline uint64_t mod_magic(uint64_t n) { return n ? (~0ULL) / n : 0; }

inline bool probe_j_supported(int j) { return j == 2 || j == 4 || j == 5 || j == 8; }

/* launchers; all asynchronous on `stream` */
size_t plan_workspace_bytes(uint32_t n_seq);
hipError_t launch_plan(const uint64_t *seq_off, uint32_t n_seq, uint64_t *wbase, uint32_t *tile_seq,
                       uint32_t tile_windows, void *workspace, hipStream_t stream);
hipError_t launch_probe(const uint8_t *residues, uint64_t n_residues, const uint64_t *seq_off,
                        const uint64_t *wbase, const uint32_t *tile_seq, uint32_t n_seq,
                        uint64_t max_tiles, const kgx_sig_kmer *table, uint64_t num_sigs,
                        kgx_hit *hits, uint64_t *hit_mask, int probe_j, int variant,
                        hipStream_t stream);
hipError_t launch_score(uint32_t n_seq, const uint64_t *wbase, const uint64_t *hit_mask,
                        uint32_t tile_windows, kgx_hit *hits, kgx_call *calls, void *ranges,
                        uint32_t *hit_count, uint32_t *call_count, kgx_params params,
                        uint32_t want, hipStream_t stream);
hipError_t launch_gather(uint32_t n_seq, const uint64_t *wbase, const uint64_t *hit_mask,
                         uint32_t tile_windows, const uint32_t *call_count, const kgx_hit *hits,
                         const kgx_call *calls, const uint64_t *hit_dense_off,
                         const uint64_t *call_dense_off, kgx_hit *hits_out, kgx_call *calls_out,
                         hipStream_t stream);
hipError_t launch_random_read(const kgx_sig_kmer *table, uint64_t num_sigs, uint64_t threads,
                              uint32_t rounds, int mode, uint64_t *sink, hipStream_t stream);
hipError_t launch_synth_image(kgx_sig_kmer *table, uint64_t num_sigs, uint64_t n_keys,
                              unsigned long long *n_stored, hipStream_t stream);
hipError_t launch_synth_queries(uint64_t image_n_keys, uint32_t n_seq, uint32_t length,
                                uint32_t x_permille, uint64_t q0, uint8_t *residues,
                                uint64_t *seq_off, hipStream_t stream);

}  // namespace kgx

#endif
