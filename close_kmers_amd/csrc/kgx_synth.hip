/*
 * kgx_synth.hip -- device-side generators and the random-read ceiling.
 *
 *   synth_image   : synthetic signature image built straight into HBM in the
 *                   reference's bucket format (parallel linear-probe insert,
 *                   64-bit CAS on the key, lowest entry id wins duplicates)
 *   synth_queries : synthetic query batch; both bit-identical to synth.py
 *   random_read   : uniformly random reads of the image buffer -- the
 *                   measured denominator of the probe's roofline
 */
#include "kgx_device.h"

namespace kgx {

/* ------------------------------------------------------------------------ */
/* random-read ceiling of the image buffer (roofline denominator)            */
/* ------------------------------------------------------------------------ */

/* Every lane reads RR_ILP independent uniformly random records of the
 * resident image buffer per round: mode 0 a whole 24-byte bucket (8-byte key
 * + 16-byte payload, as the AOS24 probe does), mode 1 the 8-byte key of a
 * 24-byte bucket, mode 2 one aligned 64-byte sector, mode 3 one aligned
 * 16-byte record (as the PACKED16 probe does).  Modes 4 and 5 read one
 * random aligned 64-B (128-B) line per group of 4 (8) lanes, 16 B per lane in
 * one instruction -- the cooperative line reads of the quad probe. */

__host__ __device__ constexpr uint64_t rr_stride(int mode)
{
    return mode == 2 || mode == 4 ? 64 : mode == 5 ? 128 : mode == 3 ? 16 : 24;
}
__host__ __device__ constexpr uint32_t rr_group(int mode) { return mode == 4 ? 4 : mode == 5 ? 8 : 1; }

template <int MODE, int RR_ILP>
__global__ __launch_bounds__(256) void random_read_kernel(const char *__restrict__ base, uint64_t n,
                                                          uint64_t magic, uint32_t rounds,
                                                          uint64_t *sink)
{
    constexpr uint64_t S = rr_stride(MODE);
    constexpr uint32_t G = rr_group(MODE);
    const uint64_t tid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    const uint32_t part = threadIdx.x % G;
    uint64_t acc = 0;
    for (uint32_t r = 0; r < rounds; r++) {
        uint64_t idx[RR_ILP];
#pragma unroll
        for (int k = 0; k < RR_ILP; k++)
            idx[k] = mod_by(mix64(tid * 977u + (uint64_t)r * RR_ILP + k) & ((1ull << 35) - 1), n, magic);
        uint64_t kv[RR_ILP];
        uint4 pv[RR_ILP], pw[RR_ILP], px[RR_ILP];
#pragma unroll
        for (int k = 0; k < RR_ILP; k++) {
            const char *rec = base + idx[k] * S;
            if (MODE == 0) {
                kv[k] = *reinterpret_cast<const uint64_t *>(rec);
                pv[k] = *reinterpret_cast<const uint4 *>(rec + 8);
            } else if (MODE == 1) {
                kv[k] = *reinterpret_cast<const uint64_t *>(rec);
            } else if (MODE == 2) {
                const uint4 *q = reinterpret_cast<const uint4 *>(rec);
                pv[k] = q[0];
                pw[k] = q[1];
                px[k] = q[2];
                kv[k] = *reinterpret_cast<const uint64_t *>(q + 3);
            } else if (MODE == 3) {
                pv[k] = *reinterpret_cast<const uint4 *>(rec);
                kv[k] = pv[k].y;
            } else {
                pv[k] = *reinterpret_cast<const uint4 *>(rec + 16 * part);
                kv[k] = pv[k].y;
            }
        }
#pragma unroll
        for (int k = 0; k < RR_ILP; k++) {
            acc ^= kv[k];
            if (MODE == 0 || MODE >= 3)
                acc += pv[k].x ^ pv[k].w;
            if (MODE == 2)
                acc += pv[k].x ^ pw[k].y ^ px[k].z;
        }
    }
    sink[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
static void launch_rr_mode(dim3 grid, dim3 block, hipStream_t stream, const char *b, uint64_t n, uint64_t m,
                           uint32_t rounds, int ilp, uint64_t *sink)
{
    switch (ilp) {
    case 1: hipLaunchKernelGGL((random_read_kernel<MODE, 1>), grid, block, 0, stream, b, n, m, rounds, sink); break;
    case 2: hipLaunchKernelGGL((random_read_kernel<MODE, 2>), grid, block, 0, stream, b, n, m, rounds, sink); break;
    case 4: hipLaunchKernelGGL((random_read_kernel<MODE, 4>), grid, block, 0, stream, b, n, m, rounds, sink); break;
    case 16: hipLaunchKernelGGL((random_read_kernel<MODE, 16>), grid, block, 0, stream, b, n, m, rounds, sink); break;
    default: hipLaunchKernelGGL((random_read_kernel<MODE, 8>), grid, block, 0, stream, b, n, m, rounds, sink); break;
    }
}

hipError_t launch_random_read(const void *buffer, uint64_t bytes, uint64_t threads, uint32_t rounds, int mode,
                              int ilp, uint64_t *sink, hipStream_t stream)
{
    const dim3 grid((uint32_t)(threads / 256)), block(256);
    const char *b = static_cast<const char *>(buffer);
    const uint64_t n = bytes / rr_stride(mode), m = mod_magic(n);
    switch (mode) {
    case 0: launch_rr_mode<0>(grid, block, stream, b, n, m, rounds, ilp, sink); break;
    case 1: launch_rr_mode<1>(grid, block, stream, b, n, m, rounds, ilp, sink); break;
    case 2: launch_rr_mode<2>(grid, block, stream, b, n, m, rounds, ilp, sink); break;
    case 3: launch_rr_mode<3>(grid, block, stream, b, n, m, rounds, ilp, sink); break;
    case 4: launch_rr_mode<4>(grid, block, stream, b, n, m, rounds, ilp, sink); break;
    case 5: launch_rr_mode<5>(grid, block, stream, b, n, m, rounds, ilp, sink); break;
    default: return hipErrorInvalidValue;
    }
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

/* entries given by the caller: the same CAS insert (lowest entry index owns
 * a duplicated key, as the sequential KmerGuts::insert_kmer's earliest copy
 * is the one a probe finds), keys above 20^8 skipped (kguts.cc:203-207) */
__global__ void entries_insert_kernel(kgx_sig_kmer *t, uint64_t n, uint64_t magic, const uint64_t *keys,
                                      uint64_t n_entries, unsigned long long *n_stored)
{
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n_entries;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t key = keys[e];
        if (key > MAX_ENCODED)
            continue;
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

__global__ void entries_payload_kernel(kgx_sig_kmer *t, uint64_t n, const int32_t *fi, const int32_t *otu,
                                       const uint16_t *avg, const float *wt)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t *w = reinterpret_cast<uint64_t *>(t + i);
        if (w[0] > MAX_ENCODED) {
            w[2] = 0;
            continue;
        }
        const uint64_t e = w[2];
        kgx_sig_kmer *k = t + i;
        k->otu_index = otu[e];
        k->avg_from_end = avg[e];
        k->pad = 0;
        k->function_index = fi[e];
        k->function_wt = wt[e];
    }
}

hipError_t launch_entries_image(kgx_sig_kmer *table, uint64_t num_sigs, const uint64_t *keys,
                                const int32_t *fi, const int32_t *otu, const uint16_t *avg, const float *wt,
                                uint64_t n_entries, unsigned long long *n_stored, hipStream_t stream)
{
    const dim3 grid(8192), block(256);
    hipLaunchKernelGGL(synth_init_kernel, grid, block, 0, stream, table, num_sigs);
    (void)hipMemsetAsync(n_stored, 0, sizeof(*n_stored), stream);
    hipLaunchKernelGGL(entries_insert_kernel, grid, block, 0, stream, table, num_sigs, mod_magic(num_sigs), keys,
                       n_entries, n_stored);
    hipLaunchKernelGGL(entries_payload_kernel, grid, block, 0, stream, table, num_sigs, fi, otu, avg, wt);
    return hipGetLastError();
}

hipError_t launch_synth_image(kgx_sig_kmer *table, uint64_t num_sigs, uint64_t n_keys, uint64_t n_entries,
                              bool payload, unsigned long long *n_stored, hipStream_t stream)
{
    const uint64_t n_src = (n_keys / 4) / SRC_WIN; /* the spec's source proteins */
    const dim3 grid(256 * 32), block(256);
    (void)hipMemsetAsync(n_stored, 0, sizeof(unsigned long long), stream);
    hipLaunchKernelGGL(synth_init_kernel, grid, block, 0, stream, table, num_sigs);
    hipLaunchKernelGGL(synth_insert_kernel, grid, block, 0, stream, table, num_sigs,
                       mod_magic(num_sigs), n_entries, n_src, n_stored);
    if (payload)
        hipLaunchKernelGGL(synth_payload_kernel, grid, block, 0, stream, table, num_sigs, n_src);
    return hipGetLastError();
}

/* After an insert without payload every stored bucket holds its owner (the
 * lowest entry id with its key) in word 2.  One radix-select pass: a
 * histogram of owner byte (shift / 8) over the stored buckets whose owner
 * matches `prefix` under `prefix_mask` -- four passes find the k-th smallest
 * owner, hence how many entries of the stream hold k distinct keys. */
__global__ __launch_bounds__(256) void owner_hist_kernel(const kgx_sig_kmer *t, uint64_t n, uint32_t prefix,
                                                         uint32_t prefix_mask, uint32_t shift,
                                                         unsigned long long *hist)
{
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t *w = reinterpret_cast<const uint64_t *>(t + i);
        if (w[0] > MAX_ENCODED)
            continue;
        const uint32_t o = (uint32_t)w[2];
        if ((o & prefix_mask) == prefix)
            atomicAdd(&h[(o >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x])
        atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

hipError_t launch_owner_hist(const kgx_sig_kmer *table, uint64_t num_sigs, uint32_t prefix, uint32_t prefix_mask,
                             uint32_t shift, unsigned long long *hist, hipStream_t stream)
{
    (void)hipMemsetAsync(hist, 0, 256 * sizeof(unsigned long long), stream);
    hipLaunchKernelGGL(owner_hist_kernel, dim3(256 * 16), dim3(256), 0, stream, table, num_sigs, prefix,
                       prefix_mask, shift, hist);
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
