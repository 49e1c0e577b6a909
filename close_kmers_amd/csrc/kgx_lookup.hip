/*
 * kgx_lookup.hip -- gfx950 kernels of the lookup path.
 *
 *   plan   : wbase = exclusive scan of windows per sequence; tile -> first
 *            sequence map (two launches, 1,024 sequences per workgroup)
 *   probe  : 8-mer encode + linear-probe lookup in the HBM-resident image;
 *            one wave per tile of J*64 consecutive windows of the batch
 *            (across sequence boundaries); J probe chains in flight per lane;
 *            hits compacted per tile in window order with wave ballots
 *   score  : the gather_hits / process_set_of_hits run state machine, one
 *            lane per sequence, O(1) state (no 40,000-entry buffer)
 *   gather : tiled hits -> dense per-sequence CSR (host-buffer path)
 *
 * Reference behaviour restated (kguts.cc line numbers): residue map 273-339,
 * window set / rolling code 682-732 and 783-871, probe 585-602, run rules
 * 734-781 and 808-876.
 */
#include "kgx_device.h"
#include "kgx_lstd.h"

namespace kgx {

/* ------------------------------------------------------------------------ */
/* plan                                                                      */
/* ------------------------------------------------------------------------ */

constexpr uint32_t PLAN_PER = 4;               /* sequences per thread */
constexpr uint32_t PLAN_TILE = 256 * PLAN_PER; /* sequences per workgroup */

__device__ __forceinline__ uint64_t thread_windows(const uint64_t *seq_off, uint32_t n, uint32_t s0)
{
    uint64_t w = 0;
    for (uint32_t k = 0; k < PLAN_PER; k++)
        if (s0 + k < n)
            w += windows_of(seq_off[s0 + k + 1] - seq_off[s0 + k]);
    return w;
}

/* the batch's offsets are usable iff they are monotone and span at most
 * n_residues bytes (kgx.h, kgx_run_device); then every window count is
 * bounded by its length and the plan's buffers (sized from n_residues) hold
 * the batch.  Checked per thread over its PLAN_PER sequences. */
__device__ __forceinline__ bool thread_offsets_bad(const uint64_t *seq_off, uint32_t n, uint32_t s0,
                                                   uint64_t n_residues)
{
    const uint64_t first = seq_off[0];
    bool bad = seq_off[n] < first || seq_off[n] - first > n_residues;
    for (uint32_t k = 0; k < PLAN_PER; k++)
        if (s0 + k < n)
            bad |= seq_off[s0 + k + 1] < seq_off[s0 + k];
    return bad;
}

constexpr uint64_t PLAN_BAD = 1ull << 63; /* marks a workgroup sum whose offsets are bad */

/* inclusive scan over a 256-thread workgroup; `total` = sum of all */
__device__ __forceinline__ uint64_t block_scan(uint64_t v, uint64_t *lds4, uint64_t &total)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint64_t x = __shfl_up(v, off);
        if (lane >= off)
            v += x;
    }
    if (lane == 63)
        lds4[wave] = v;
    __syncthreads();
    uint64_t pre = 0;
    total = 0;
    for (uint32_t i = 0; i < 4; i++) {
        if (i < wave)
            pre += lds4[i];
        total += lds4[i];
    }
    return v + pre;
}

/* the longest sequence's windows (capped at 2^32 - 1) of this thread's PLAN_PER */
__device__ __forceinline__ uint32_t thread_max_windows(const uint64_t *seq_off, uint32_t n, uint32_t s0)
{
    uint64_t m = 0;
    for (uint32_t k = 0; k < PLAN_PER; k++)
        if (s0 + k < n)
            m = max(m, windows_of(seq_off[s0 + k + 1] - seq_off[s0 + k]));
    return (uint32_t)min<uint64_t>(m, 0xFFFFFFFFull);
}

__global__ __launch_bounds__(256) void plan_reduce_kernel(const uint64_t *__restrict__ seq_off,
                                                          uint32_t n, uint64_t n_residues,
                                                          uint64_t *__restrict__ sums, uint32_t *__restrict__ maxw)
{
    __shared__ uint64_t lds4[4];
    __shared__ uint32_t lmax[4];
    uint64_t total;
    const uint32_t s0 = blockIdx.x * PLAN_TILE + threadIdx.x * PLAN_PER;
    const bool bad = __syncthreads_or(thread_offsets_bad(seq_off, n, s0, n_residues));
    block_scan(bad ? 0 : thread_windows(seq_off, n, s0), lds4, total);
    /* the workgroup's longest sequence (scorer dispatch, plan_sums_scan) */
    uint32_t m = bad ? 0u : thread_max_windows(seq_off, n, s0);
    for (uint32_t off = 32; off; off >>= 1)
        m = max(m, (uint32_t)__shfl_xor((int)m, (int)off));
    if ((threadIdx.x & 63u) == 0)
        lmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        sums[blockIdx.x] = bad ? PLAN_BAD : total;
        maxw[blockIdx.x] = max(max(lmax[0], lmax[1]), max(lmax[2], lmax[3]));
    }
}

/* exclusive scan of the workgroup sums in place, one workgroup of 1,024
 * threads, each scanning 16 consecutive sums per round (a 9.9M-fragment fq
 * chunk's 9.7k sums: one round).  (Each plan_scan workgroup used to add up
 * all earlier sums itself: quadratic in the number of workgroups, 0.5 ms for
 * the 9.9M fragments of a 1M-read fq chunk; then 256 threads in rounds of
 * 256: 31 us.) */
constexpr uint32_t SUMS_PER = 16;

/* SUMS_THREADS 256 for up to 4,096 sums (C2: 98): a 4-wave workgroup finds a
 * slot beside the other context's probe at once, where a 16-wave one waited
 * for that probe to drain (550 us stretched, kernel trace r2zr; 9 us, r2zs).
 * The 12-14 us between consecutive probes did not change: that is the
 * cross-queue event wait, not the plan. */
template <uint32_t SUMS_THREADS>
__global__ __launch_bounds__(SUMS_THREADS) void plan_sums_scan_kernel(uint64_t *__restrict__ sums, uint32_t groups,
                                                                      const uint32_t *__restrict__ maxw,
                                                                      uint32_t *__restrict__ status)
{
    __shared__ uint64_t wsum[SUMS_THREADS / 64];
    __shared__ uint32_t wmax[SUMS_THREADS / 64];
    /* any workgroup that saw bad offsets empties the whole batch (sums[groups]
     * = 1 tells plan_scan) and raises the context's status word; status[1] =
     * the batch's longest sequence in windows (the scorer's dispatch) */
    bool bad = false;
    uint32_t m = 0;
    for (uint32_t i = threadIdx.x; i < groups; i += SUMS_THREADS) {
        bad |= (sums[i] & PLAN_BAD) != 0;
        m = max(m, maxw[i]);
    }
    for (uint32_t off = 32; off; off >>= 1)
        m = max(m, (uint32_t)__shfl_xor((int)m, (int)off));
    if ((threadIdx.x & 63u) == 0)
        wmax[threadIdx.x >> 6] = m;
    bad = __syncthreads_or(bad);
    if (threadIdx.x == 0) {
        uint32_t mm = 0;
        for (uint32_t w = 0; w < SUMS_THREADS / 64; w++)
            mm = max(mm, wmax[w]);
        status[1] = bad ? 0u : mm;
    }
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint64_t carry = 0;
    for (uint32_t base = 0; base < groups; base += SUMS_THREADS * SUMS_PER) {
        const uint32_t i0 = base + threadIdx.x * SUMS_PER;
        uint64_t v[SUMS_PER], t = 0;
#pragma unroll
        for (uint32_t k = 0; k < SUMS_PER; k++) {
            v[k] = i0 + k < groups && !bad ? sums[i0 + k] : 0;
            t += v[k];
        }
        /* exclusive prefix of the threads' totals: wave scan, then the waves' sums */
        uint64_t x = t;
        for (uint32_t off = 1; off < 64; off <<= 1) {
            const uint64_t y = __shfl_up(x, off);
            if (lane >= off)
                x += y;
        }
        if (lane == 63)
            wsum[wave] = x;
        __syncthreads();
        uint64_t pre = carry, tot = 0;
        for (uint32_t w = 0; w < SUMS_THREADS / 64; w++) {
            if (w < wave)
                pre += wsum[w];
            tot += wsum[w];
        }
        pre += x - t;
#pragma unroll
        for (uint32_t k = 0; k < SUMS_PER; k++) {
            if (i0 + k < groups)
                sums[i0 + k] = pre;
            pre += v[k];
        }
        carry += tot;
        __syncthreads(); /* wsum is rewritten by the next round */
    }
    if (threadIdx.x == 0) {
        sums[groups] = bad ? 1 : 0;
        status[0] = bad ? 1u : 0u;
    }
}

__global__ __launch_bounds__(256) void plan_scan_kernel(const uint64_t *__restrict__ seq_off,
                                                        uint32_t n, const uint64_t *__restrict__ sums,
                                                        uint64_t *__restrict__ wbase,
                                                        uint32_t *__restrict__ tile_seq,
                                                        uint32_t tile_windows)
{
    __shared__ uint64_t lds_b[4];
    const uint64_t before = sums[blockIdx.x]; /* windows of all earlier workgroups */
    const bool bad = sums[gridDim.x] != 0;    /* bad offsets: an empty batch */

    const uint32_t s0 = blockIdx.x * PLAN_TILE + threadIdx.x * PLAN_PER;
    const uint64_t mine = bad ? 0 : thread_windows(seq_off, n, s0);
    uint64_t tot;
    const uint64_t incl = block_scan(mine, lds_b, tot);
    uint64_t wb = before + incl - mine;
    for (uint32_t k = 0; k < PLAN_PER; k++) {
        const uint32_t s = s0 + k;
        if (s >= n)
            break;
        const uint64_t we = wb + (bad ? 0 : windows_of(seq_off[s + 1] - seq_off[s]));
        wbase[s] = wb;
        /* tiles whose first window lies in [wb, we) start inside sequence s */
        for (uint64_t t = (wb + tile_windows - 1) / tile_windows; t * tile_windows < we; t++)
            tile_seq[t] = s;
        wb = we;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 255)
        wbase[n] = before + tot;
}

/*
 * The plan in ONE launch (the default; KGX_PLAN_FUSED=0: the three kernels
 * above): plan_reduce, plan_sums_scan and plan_scan fused by a decoupled
 * look-back over the workgroups of PLAN_TILE sequences, as fq_anchor_fused
 * does for fragments.  Workgroup g publishes its windows (state 1) and, once
 * it has summed the states of the workgroups before it -- 64 at a time, one
 * per lane of wave 0, until one holds an inclusive prefix (state 2) -- its own
 * inclusive prefix; then it writes its sequences' window bases and tile
 * owners exactly as plan_scan.  Workgroups start in index order, so every
 * state waited on belongs to a workgroup already running.  State words are
 * state << 62 | value, relaxed device-scope atomics; after them in `look`: the
 * finished-workgroup ticket, the bad-offsets flag and the longest sequence.
 * The workgroup that finishes last writes the status words, empties the
 * batch when any workgroup saw bad offsets (every window base 0: what the
 * three kernels give), and zeroes `look` for the next launch (zero-filled
 * when allocated).  Tile owners are written only below max_tiles: with bad
 * offsets a workgroup's prefix may pass the buffer before the batch is
 * emptied.
 */
constexpr uint64_t LOOK_MASK = (1ull << 62) - 1;

__global__ __launch_bounds__(256) void plan_fused_kernel(const uint64_t *__restrict__ seq_off, uint32_t n,
                                                         uint64_t n_residues, uint64_t *__restrict__ wbase,
                                                         uint32_t *__restrict__ tile_seq, uint32_t tile_windows,
                                                         uint64_t max_tiles, uint64_t *__restrict__ look,
                                                         uint32_t groups, uint32_t *__restrict__ status)
{
    __shared__ uint64_t lds4[4];
    __shared__ uint32_t lmax[4];
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_last;
    uint32_t *ctl = reinterpret_cast<uint32_t *>(look + groups); /* ticket, bad, longest */
    const uint32_t g = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t s0 = g * PLAN_TILE + threadIdx.x * PLAN_PER;
    const bool bad = __syncthreads_or(thread_offsets_bad(seq_off, n, s0, n_residues));
    const uint64_t mine = bad ? 0 : thread_windows(seq_off, n, s0);
    uint64_t tot;
    const uint64_t incl = block_scan(mine, lds4, tot);
    uint32_t m = bad ? 0u : thread_max_windows(seq_off, n, s0);
    for (uint32_t off = 32; off; off >>= 1)
        m = max(m, (uint32_t)__shfl_xor((int)m, (int)off));
    if (lane == 0)
        lmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x < 64) {
        if (threadIdx.x == 0) {
            if (bad)
                __hip_atomic_fetch_or(&ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_max(&ctl[2], max(max(lmax[0], lmax[1]), max(lmax[2], lmax[3])), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&look[g], (g == 0 ? 2ull : 1ull) << 62 | tot, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        /* look back: lane l examines workgroup j - l */
        uint64_t x = 0;
        for (int64_t j = (int64_t)g - 1; j >= 0; j -= 64) {
            const int64_t idx = j - (int64_t)lane;
            uint64_t v = 2ull << 62; /* before workgroup 0: a zero prefix */
            if (idx >= 0)
                do {
                    v = __hip_atomic_load(&look[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } while ((v >> 62) == 0);
            const uint64_t pm = __ballot((v >> 62) == 2);
            const uint32_t upto = pm ? (uint32_t)__builtin_ctzll(pm) : 63u; /* lanes 0..upto count */
            uint64_t y = lane <= upto ? v & LOOK_MASK : 0;
            for (uint32_t o = 32; o; o >>= 1)
                y += __shfl_xor(y, (int)o);
            x += y;
            if (pm)
                break;
        }
        if (threadIdx.x == 0) {
            if (g)
                __hip_atomic_store(&look[g], 2ull << 62 | ((x + tot) & LOOK_MASK), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            s_prefix = x;
        }
    }
    __syncthreads();
    const uint64_t before = s_prefix;
    uint64_t wb = before + incl - mine;
    for (uint32_t k = 0; k < PLAN_PER; k++) {
        const uint32_t s = s0 + k;
        if (s >= n)
            break;
        const uint64_t we = wb + (bad ? 0 : windows_of(seq_off[s + 1] - seq_off[s]));
        wbase[s] = wb;
        /* tiles whose first window lies in [wb, we) start inside sequence s */
        for (uint64_t t = (wb + tile_windows - 1) / tile_windows; t * tile_windows < we && t < max_tiles; t++)
            tile_seq[t] = s;
        wb = we;
    }
    if (g == groups - 1 && threadIdx.x == 255)
        wbase[n] = before + tot;
    /* the last workgroup to finish: status, the bad-offsets fix-up, the reset */
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(&ctl[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == groups - 1;
    __syncthreads();
    if (!s_last)
        return;
    __threadfence();
    const uint32_t any_bad = __hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (any_bad)
        for (uint64_t s = threadIdx.x; s <= n; s += 256)
            wbase[s] = 0;
    if (threadIdx.x == 0) {
        status[0] = any_bad ? 1u : 0u;
        status[1] = any_bad ? 0u : __hip_atomic_load(&ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (uint32_t j = threadIdx.x; j < groups; j += 256)
        __hip_atomic_store(&look[j], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 3)
        __hip_atomic_store(&ctl[threadIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* The plan of a batch of up to PLAN_ONE_MAX sequences in ONE workgroup of
 * 1,024 threads (option plan_fused 2): thread t takes a contiguous run of
 * sequences, the runs' window counts are scanned across the workgroup, and
 * each thread writes its sequences' window bases and tile owners -- one
 * launch, nothing to wait on, one CU beside the probe.  Bad offsets empty the
 * batch as the three kernels do. */
constexpr uint32_t PLAN_ONE_MAX = 1u << 18;

__global__ __launch_bounds__(1024) void plan_one_kernel(const uint64_t *__restrict__ seq_off, uint32_t n,
                                                        uint64_t n_residues, uint64_t *__restrict__ wbase,
                                                        uint32_t *__restrict__ tile_seq, uint32_t tile_windows,
                                                        uint64_t max_tiles, uint32_t *__restrict__ status)
{
    __shared__ uint64_t wsum[16];
    __shared__ uint32_t wmax[16];
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const uint32_t per = (n + 1023) / 1024;
    const uint32_t s0 = min(n, t * per), s1 = min(n, s0 + per);
    const uint64_t first = seq_off[0], last = seq_off[n];
    bool bad = last < first || last - first > n_residues;
    uint64_t w = 0;
    uint32_t m = 0;
    for (uint32_t s = s0; s < s1; s++) {
        const uint64_t a = seq_off[s], b = seq_off[s + 1];
        bad |= b < a;
        const uint64_t ww = b >= a ? windows_of(b - a) : 0;
        w += ww;
        m = max(m, (uint32_t)min<uint64_t>(ww, 0xFFFFFFFFull));
    }
    bad = __syncthreads_or(bad);
    /* exclusive scan of the threads' windows: waves, then the 16 wave sums */
    uint64_t x = w;
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint64_t y = __shfl_up(x, off);
        if (lane >= off)
            x += y;
    }
    for (uint32_t off = 32; off; off >>= 1)
        m = max(m, (uint32_t)__shfl_xor((int)m, (int)off));
    if (lane == 63)
        wsum[wave] = x;
    if (lane == 0)
        wmax[wave] = m;
    __syncthreads();
    uint64_t before = 0, total = 0;
    uint32_t mm = 0;
    for (uint32_t i = 0; i < 16; i++) {
        before += i < wave ? wsum[i] : 0;
        total += wsum[i];
        mm = max(mm, wmax[i]);
    }
    uint64_t wb = bad ? 0 : before + x - w;
    for (uint32_t s = s0; s < s1; s++) {
        const uint64_t we = wb + (bad ? 0 : windows_of(seq_off[s + 1] - seq_off[s]));
        wbase[s] = wb;
        for (uint64_t k = (wb + tile_windows - 1) / tile_windows; k * tile_windows < we && k < max_tiles; k++)
            tile_seq[k] = s;
        wb = we;
    }
    if (t == 0) {
        wbase[n] = bad ? 0 : total;
        status[0] = bad ? 1u : 0u;
        status[1] = bad ? 0u : mm;
    }
}

hipError_t launch_plan_one(const uint64_t *seq_off, uint32_t n_seq, uint64_t n_residues, uint64_t *wbase,
                           uint32_t *tile_seq, uint32_t tile_windows, uint64_t max_tiles, uint32_t *status,
                           hipStream_t stream)
{
    if (n_seq > PLAN_ONE_MAX)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(plan_one_kernel, dim3(1), dim3(1024), 0, stream, seq_off, n_seq, n_residues, wbase, tile_seq,
                       tile_windows, max_tiles, status);
    return hipGetLastError();
}

size_t plan_look_bytes(uint32_t n_seq) { return ((size_t)n_seq / PLAN_TILE + 1) * sizeof(uint64_t) + 16; }

hipError_t launch_plan_fused(const uint64_t *seq_off, uint32_t n_seq, uint64_t n_residues, uint64_t *wbase,
                             uint32_t *tile_seq, uint32_t tile_windows, uint64_t max_tiles, void *look,
                             uint32_t *status, hipStream_t stream)
{
    const uint32_t groups = n_seq / PLAN_TILE + 1; /* >= 1 so wbase[n] is written */
    hipLaunchKernelGGL(plan_fused_kernel, dim3(groups), dim3(256), 0, stream, seq_off, n_seq, n_residues, wbase,
                       tile_seq, tile_windows, max_tiles, static_cast<uint64_t *>(look), groups, status);
    return hipGetLastError();
}

/* the workgroup sums + the bad-offsets word, then the workgroups' longest sequences */
size_t plan_workspace_bytes(uint32_t n_seq)
{
    return ((size_t)n_seq / PLAN_TILE + 2) * (sizeof(uint64_t) + sizeof(uint32_t));
}

hipError_t launch_plan(const uint64_t *seq_off, uint32_t n_seq, uint64_t n_residues, uint64_t *wbase,
                       uint32_t *tile_seq, uint32_t tile_windows, void *workspace, uint32_t *status,
                       hipStream_t stream)
{
    const uint32_t groups = n_seq / PLAN_TILE + 1; /* >= 1 so wbase[n] is written */
    uint32_t *maxw = reinterpret_cast<uint32_t *>(static_cast<uint64_t *>(workspace) + groups + 2);
    hipLaunchKernelGGL(plan_reduce_kernel, dim3(groups), dim3(256), 0, stream, seq_off, n_seq, n_residues,
                       static_cast<uint64_t *>(workspace), maxw);
    if (groups <= 256 * SUMS_PER)
        hipLaunchKernelGGL(plan_sums_scan_kernel<256>, dim3(1), dim3(256), 0, stream,
                           static_cast<uint64_t *>(workspace), groups, maxw, status);
    else
        hipLaunchKernelGGL(plan_sums_scan_kernel<1024>, dim3(1), dim3(1024), 0, stream,
                           static_cast<uint64_t *>(workspace), groups, maxw, status);
    hipLaunchKernelGGL(plan_scan_kernel, dim3(groups), dim3(256), 0, stream, seq_off, n_seq,
                       static_cast<const uint64_t *>(workspace), wbase, tile_seq, tile_windows);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* probe                                                                     */
/* ------------------------------------------------------------------------ */

/* 12 residue bytes at offset `abo` (a multiple of 4) of the 4-aligned base
 * residues - bm; bytes outside the batch [bm, bm + n) read as 0 (code 20).
 * Offsets and pointer arithmetic, not integer addresses, so the loads stay
 * global loads (a flat load also counts against the LDS wait counter). */
__device__ __forceinline__ uint3 load_residues(const uint8_t *residues, uint64_t bm, uint64_t n, uint64_t abo)
{
    uint32_t d[3] = {0, 0, 0};
    for (int b = 0; b < 12; b++)
        if (abo + b >= bm && abo + b < bm + n)
            d[b >> 2] |= (uint32_t)residues[abo + b - bm] << (8 * (b & 3));
    return make_uint3(d[0], d[1], d[2]);
}

/*
 * One wave = one tile of J*64 windows [g0, g0 + J*64) of the batch.  Lane l
 * owns windows g0 + 64 j + l, so slice j is 64 consecutive windows and its
 * ballot is in window order (= (sequence, position) order).  Every lane
 * finds its window's sequence by walking forward from the tile's first
 * sequence, reads the 8 residues straight from the batch (one 16-byte load),
 * maps them to codes through a 256-byte LDS table, and issues all J first
 * probes before resolving any.
 *   MODE_BUCKET: each probe round loads key and payload of its 24-B bucket;
 *   MODE_KEY_FIRST: rounds load keys only; the matching bucket's payload is
 *     loaded in the round that finds it (mostly the key's sector, in L2);
 *   MODE_PACKED: PACKED16 images -- one aligned 16-B load per bucket gives
 *     key and payload (never straddles a sector; 4 buckets per sector);
 *   MODE_PACKED_KEY_FIRST: the record's low word (key, fI, otu bits) per
 *     bucket, its high word only for the match (same sector).
 */
constexpr int MODE_BUCKET = 0, MODE_KEY_FIRST = 1, MODE_PACKED = 2, MODE_PACKED_KEY_FIRST = 3;

/* a table record; NT = non-temporal (streaming) load, so the random
 * table traffic need not displace a cache-resident presence filter */
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
template <bool NT> __device__ __forceinline__ uint4 load_record(const uint4 *p)
{
    if (NT) {
        const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *p;
}

/* the J windows g0 + 64 j + lane of a tile: their keys (big-endian base-20
 * codes, encoded_kmer kguts.cc:438-455), whether they are valid (inside the
 * batch, no code-20 residue: advance_past_ambig), and their (seq, pos) */
template <int J>
__device__ __forceinline__ void encode_tile(const uint8_t *__restrict__ residues, uint64_t n_residues,
                                            const uint64_t *__restrict__ seq_off,
                                            const uint64_t *__restrict__ wbase, uint32_t s,
                                            uint64_t W, uint64_t g0, uint32_t lane,
                                            const uint8_t *code_tab, uint64_t *key, bool *ok,
                                            uint32_t *pos, uint32_t *sq)
{
    /* byte offsets from residues - bm, which is 4-aligned */
    const uint64_t bm = reinterpret_cast<uintptr_t>(residues) & 3;
    uint64_t wb_lo = wbase[s], wb_hi = wbase[s + 1], soff = seq_off[s];
    uint64_t ab[J];
    uint32_t sh[J];
    uint4 v[J];
    bool fast[J];
    /* pass 1: each window's sequence, and one 16-byte load of its residues,
     * issued for all J windows before any is used (a window whose 16 bytes
     * would leave the batch is read bytewise in pass 2).  Loads under a
     * divergent branch stay in flight past the join only when the loaded
     * variable holds nothing older to merge with -- here and in the probes,
     * such variables are written once per round. */
#pragma unroll
    for (int j = 0; j < J; j++) {
        const uint64_t gw = g0 + 64 * j + lane;
        const bool act = gw < W;
        while (act && gw >= wb_hi) { /* next sequence (skips window-less ones) */
            s++;
            wb_lo = wb_hi;
            wb_hi = wbase[s + 1];
            soff = seq_off[s];
        }
        pos[j] = (uint32_t)(gw - wb_lo);
        sq[j] = s;
        const uint64_t a = bm + soff + (gw - wb_lo);
        ab[j] = a & ~3ull;
        sh[j] = (uint32_t)(a - ab[j]);
        ok[j] = act;
        fast[j] = ab[j] >= bm && ab[j] + 16 <= bm + n_residues;
        if (fast[j])
            v[j] = *reinterpret_cast<const uint4 *>(residues + (ab[j] - bm));
    }
    /* pass 2: codes and keys */
#pragma unroll
    for (int j = 0; j < J; j++) {
        uint3 d = make_uint3(v[j].x, v[j].y, v[j].z);
        if (!fast[j])
            d = load_residues(residues, bm, n_residues, ab[j]);
        const uint32_t lo = __builtin_amdgcn_alignbyte(d.y, d.x, sh[j]);
        const uint32_t hi = __builtin_amdgcn_alignbyte(d.z, d.y, sh[j]);
        const uint32_t c0 = code_tab[lo & 0xFF], c1 = code_tab[(lo >> 8) & 0xFF],
                       c2 = code_tab[(lo >> 16) & 0xFF], c3 = code_tab[lo >> 24];
        const uint32_t c4 = code_tab[hi & 0xFF], c5 = code_tab[(hi >> 8) & 0xFF],
                       c6 = code_tab[(hi >> 16) & 0xFF], c7 = code_tab[hi >> 24];
        /* a code-20 residue anywhere kills the window (advance_past_ambig) */
        const uint32_t cmax = max(max(max(c0, c1), max(c2, c3)), max(max(c4, c5), max(c6, c7)));
        ok[j] = ok[j] && cmax < 20u;
        /* big-endian base-20 Horner (encoded_kmer, kguts.cc:438-455) */
        const uint32_t ka = ((c0 * 20 + c1) * 20 + c2) * 20 + c3;
        const uint32_t kb = ((c4 * 20 + c5) * 20 + c6) * 20 + c7;
        key[j] = (uint64_t)ka * 160000u + kb;
    }
}

/*
 * The same J windows when the batch is the fq path's fragments left as DNA
 * (kgx_fq_run_device): fragment s is a run of codons of one frame of a read,
 * described by anchor[s] = (byte index of its first codon's first base) << 1
 * | reverse.  Forward, codon i is bases A+3i..A+3i+2; on the reverse strand it
 * is the complement of bases A-3i, A-3i-1, A-3i-2 (frame -k read backwards,
 * dna_seq.cc:9-47).  A window's 8 codons are the 24 bytes from A+3p (forward)
 * or ending at A-3p (reverse), loaded as two 16-B reads; each base becomes
 * its class through cls_tab (A0 C1 G2 T/U3, anything else 0x40, so a codon
 * with a non-base indexes past 63) and each codon its residue code through
 * cod_tab.  A reverse window's 24 bytes are reversed first (byte swaps), so
 * codon i is bytes 3i..3i+2 either way and its index is complemented by xor
 * 63.  The keys equal encode_tile's over the translated residues
 * (kgx_fq_fragments with residues).
 */
template <int J>
__device__ __forceinline__ void encode_tile_dna(const uint8_t *__restrict__ bases, uint64_t n_bases,
                                                const uint64_t *__restrict__ anchor,
                                                const uint64_t *__restrict__ wbase, uint32_t s, uint64_t W,
                                                uint64_t g0, uint32_t lane, const uint8_t *cls_tab,
                                                const uint8_t *cod_tab, uint64_t *key, bool *ok, uint32_t *pos,
                                                uint32_t *sq)
{
    const uint64_t bm = reinterpret_cast<uintptr_t>(bases) & 3;
    uint64_t wb_lo = wbase[s], wb_hi = wbase[s + 1], an = anchor[s];
    uint64_t ab[J], lo[J];
    uint32_t sh[J];
    uint4 v0[J], v1[J];
    bool fast[J], rev[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        const uint64_t gw = g0 + 64 * j + lane;
        const bool act = gw < W;
        while (act && gw >= wb_hi) {
            s++;
            wb_lo = wb_hi;
            wb_hi = wbase[s + 1];
            an = anchor[s];
        }
        const uint64_t p = gw - wb_lo;
        pos[j] = (uint32_t)p;
        sq[j] = s;
        rev[j] = an & 1u;
        const uint64_t A = an >> 1;
        lo[j] = act ? (rev[j] ? A - 3 * p - 23 : A + 3 * p) : 0; /* the window's first byte */
        const uint64_t a = bm + lo[j];
        ab[j] = a & ~3ull;
        sh[j] = (uint32_t)(a - ab[j]);
        ok[j] = act;
        fast[j] = act && ab[j] >= bm && ab[j] + 32 <= bm + n_bases;
        if (fast[j]) {
            const uint4 *q = reinterpret_cast<const uint4 *>(bases + (ab[j] - bm));
            v0[j] = q[0];
            v1[j] = q[1];
        }
    }
#pragma unroll
    for (int j = 0; j < J; j++) {
        uint32_t d[6];
        if (fast[j]) {
            const uint32_t w[7] = {v0[j].x, v0[j].y, v0[j].z, v0[j].w, v1[j].x, v1[j].y, v1[j].z};
#pragma unroll
            for (int k = 0; k < 6; k++)
                d[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh[j]);
        } else { /* near the buffer's end (or inactive): byte by byte */
#pragma unroll
            for (int k = 0; k < 6; k++)
                d[k] = 0;
            if (ok[j])
                for (int i = 0; i < 24; i++)
                    d[i >> 2] |= (uint32_t)bases[lo[j] + i] << (8 * (i & 3));
        }
        /* reverse strand: the span's bytes reversed, so that codon i is bytes
         * 3i..3i+2 either way (its index then complemented: xor 63) */
        uint32_t rd[6];
#pragma unroll
        for (int k = 0; k < 6; k++)
            rd[k] = __builtin_bswap32(d[5 - k]);
#pragma unroll
        for (int k = 0; k < 6; k++)
            d[k] = rev[j] ? rd[k] : d[k];
        const uint32_t flip = rev[j] ? 63u : 0u;
        uint32_t c[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int b0 = 3 * i, b1 = 3 * i + 1, b2 = 3 * i + 2;
            const uint32_t e1 = cls_tab[(d[b0 >> 2] >> (8 * (b0 & 3))) & 0xFFu];
            const uint32_t e2 = cls_tab[(d[b1 >> 2] >> (8 * (b1 & 3))) & 0xFFu];
            const uint32_t e3 = cls_tab[(d[b2 >> 2] >> (8 * (b2 & 3))) & 0xFFu];
            const uint32_t e = ((e1 << 4) | (e2 << 2) | e3) ^ flip; /* >= 64: a non-base */
            c[i] = cod_tab[min(e, 64u)]; /* unconditional read: entry 64 = 20 */
        }
        const uint32_t cmax = max(max(max(c[0], c[1]), max(c[2], c[3])), max(max(c[4], c[5]), max(c[6], c[7])));
        ok[j] = ok[j] && cmax < 20u;
        const uint32_t ka = ((c[0] * 20 + c[1]) * 20 + c[2]) * 20 + c[3];
        const uint32_t kb = ((c[4] * 20 + c[5]) * 20 + c[6]) * 20 + c[7];
        key[j] = (uint64_t)ka * 160000u + kb;
    }
}

/* ordered compaction of a tile's hits; one mask word per slice.  PACKED:
 * pv = the matching PACKED16 record, stored as is (HIT_PACKED16); else pv =
 * the 16 B after the key of the matching AOS24 bucket, stored as the two
 * planes (HIT_PLANES) */
template <int J, bool PACKED>
__device__ __forceinline__ void store_tile_hits(const bool *hit, const uint64_t *kv, const uint4 *pv,
                                                const uint32_t *pos, const uint32_t *sq, uint64_t g0,
                                                uint64_t W, uint32_t lane, uint4 *__restrict__ hot,
                                                uint4 *__restrict__ cold,
                                                uint64_t *__restrict__ hit_mask, bool nt = false)
{
    uint32_t count = 0;
#pragma unroll
    for (int j = 0; j < J; j++) {
        const uint64_t m = __ballot(hit[j]);
        if (hit[j]) {
            const uint64_t at = g0 + count + lanes_below(m);
            if (PACKED && nt) {
                typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
                const u32x4_t v = {pv[j].x, pv[j].y, pv[j].z, pv[j].w};
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t *>(hot + at));
            } else if (PACKED) {
                hot[at] = pv[j]; /* HIT_PACKED16: the table record itself */
            } else {
                hot[at] = make_uint4(pv[j].y & 0xFFFFu, pv[j].z, pv[j].w, pos[j]);
                cold[at] = make_uint4((uint32_t)kv[j], (uint32_t)(kv[j] >> 32), pv[j].x, sq[j]);
            }
        }
        if (lane == 0 && g0 + 64 * j < W) {
            if (nt)
                __builtin_nontemporal_store(m, hit_mask + (g0 >> 6) + j);
            else
                hit_mask[(g0 >> 6) + j] = m;
        }
        count += (uint32_t)__popcll(m);
    }
}

template <int J, int MODE, bool FILTER, bool NT = FILTER>
__global__ __launch_bounds__(256) void probe_kernel(
    const uint8_t *__restrict__ residues, uint64_t n_residues, const uint64_t *__restrict__ seq_off,
    const uint64_t *__restrict__ wbase, const uint32_t *__restrict__ tile_seq, uint32_t n_seq,
    const void *__restrict__ table_v, uint64_t num_sigs, uint64_t magic, uint32_t hs,
    const uint64_t *__restrict__ filter, uint32_t filter_log2,
    uint4 *__restrict__ hot, uint4 *__restrict__ cold, uint64_t *__restrict__ hit_mask)
{
    constexpr bool KEY_FIRST = MODE == MODE_KEY_FIRST;
    constexpr bool PACKED = MODE == MODE_PACKED || MODE == MODE_PACKED_KEY_FIRST;
    const uint64_t *__restrict__ packed_w = static_cast<const uint64_t *>(table_v);
    const kgx_sig_kmer *__restrict__ table = static_cast<const kgx_sig_kmer *>(table_v);
    const uint4 *__restrict__ packed = static_cast<const uint4 *>(table_v);
    constexpr uint32_t T = 64 * J;
    __shared__ uint8_t code_tab[256];
    code_tab[threadIdx.x] = (uint8_t)residue_code(threadIdx.x);
    __syncthreads();

    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    const uint64_t W = wbase[n_seq];
    const uint64_t tile = (uint64_t)blockIdx.x * PROBE_WAVES + wave;
    const uint64_t g0 = tile * T;
    if (g0 >= W)
        return;

    uint64_t key[J], slot[J], fw[J];
    uint32_t pos[J], sq[J];
    bool pend[J], hit[J];
    encode_tile<J>(residues, n_residues, seq_off, wbase, tile_seq[tile], W, g0, lane, code_tab, key,
                   pend, pos, sq);
#pragma unroll
    for (int j = 0; j < J; j++) {
        hit[j] = false;
        fw[j] = 0;
        if (FILTER && pend[j]) /* presence filter word (MALL-resident): issue now, test below */
            fw[j] = filter[filter_word(filter_hash(key[j]), filter_log2)];
    }
#pragma unroll
    for (int j = 0; j < J; j++) {
        if (FILTER && pend[j]) {
            const uint64_t m = filter_bits(filter_hash(key[j]));
            pend[j] = (fw[j] & m) == m; /* else stored nowhere: a miss */
        }
        slot[j] = pend[j] ? mod_by(key[j], num_sigs >> hs, magic) << hs : 0; /* hs: kgx_image_set_line_index */
    }

    uint4 rec[J]; /* the matching bucket's payload */
#pragma unroll
    for (int j = 0; j < J; j++)
        rec[j] = make_uint4(0, 0, 0, 0);

    /* linear probe rounds (lookup_hash_entry, kguts.cc:585-602); bounded by
     * num_sigs buckets where the reference would spin forever */
    for (uint64_t round = 0;; round++) {
        /* bucket slot[j] of every pending window, all J in flight at once */
        uint4 pv[J];
        uint64_t kv[J];
#pragma unroll
        for (int j = 0; j < J; j++) {
            if (pend[j]) {
                if (MODE == MODE_PACKED) {
                    pv[j] = load_record<NT>(packed + slot[j]);
                } else if (MODE == MODE_PACKED_KEY_FIRST) {
                    const uint64_t lo = packed_w[2 * slot[j]];
                    pv[j].x = (uint32_t)lo;
                    pv[j].y = (uint32_t)(lo >> 32);
                } else {
                    const kgx_sig_kmer *e = table + slot[j];
                    kv[j] = e->which_kmer;
                    if (!KEY_FIRST)
                        pv[j] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(e) + 8);
                }
            }
        }
        bool more = false;
#pragma unroll
        for (int j = 0; j < J; j++) {
            if (PACKED)
                kv[j] = ((uint64_t)pv[j].y << 32 | pv[j].x) & PACK_KEY_MASK;
            /* straight-line selects: a branch here would let the compiler
             * split the record load and re-read its payload half on a match */
            const bool m = pend[j] && kv[j] == key[j];
            const bool stop = kv[j] > MAX_ENCODED || round + 1 >= num_sigs;
            if (!KEY_FIRST && MODE != MODE_PACKED_KEY_FIRST) { /* per component: a select of */
                rec[j].x = m ? pv[j].x : rec[j].x;               /* whole uint4s goes through */
                rec[j].y = m ? pv[j].y : rec[j].y;               /* scratch memory */
                rec[j].z = m ? pv[j].z : rec[j].z;
                rec[j].w = m ? pv[j].w : rec[j].w;
            }
            if ((KEY_FIRST || MODE == MODE_PACKED_KEY_FIRST) && m) {
                if (KEY_FIRST)
                    rec[j] = *reinterpret_cast<const uint4 *>(
                        reinterpret_cast<const char *>(table + slot[j]) + 8);
                if (MODE == MODE_PACKED_KEY_FIRST) {
                    const uint64_t hi = packed_w[2 * slot[j] + 1];
                    rec[j] = make_uint4(pv[j].x, pv[j].y, (uint32_t)hi, (uint32_t)(hi >> 32));
                }
            }
            hit[j] = hit[j] || m;
            pend[j] = pend[j] && !m && !stop;
            slot[j] = pend[j] ? (slot[j] + 1 == num_sigs ? 0 : slot[j] + 1) : slot[j];
            more = more || pend[j];
        }
        if (!__any(more))
            break;
    }

    store_tile_hits<J, PACKED>(hit, key, rec, pos, sq, g0, W, lane, hot, cold, hit_mask);
}

/*
 * Cooperative-line probe of a PACKED16 image.  The encode and the ordered
 * compaction are probe_kernel's; the lookups are done by groups of G lanes
 * that read one aligned G*16-byte line of the table in one instruction (lane
 * c of the group holds bucket line + c).  A wave instruction serves 64 / G
 * windows, and a linear-probe chain costs one line request per line it
 * touches instead of one request per bucket: about 1.07 requests per window
 * instead of P-bar = 1.33 (the chip's ceiling is random line requests, and
 * 64-B lines read this way run at 45 G/s, tools/line_probe.py).
 *
 * Window w of the tile (w = 64 j + l, owned by lane l in slice j) is looked
 * up by group q = w % (64 / G) in instruction i = w / (64 / G).  The group
 * examines buckets in probe order: from the home slot to the end of its line,
 * then whole lines, wrapping at num_sigs; the first bucket whose key matches
 * (hit) or exceeds MAX_ENCODED (miss) ends the chain -- lookup_hash_entry,
 * kguts.cc:585-602.  A chain that has covered the whole table without either
 * is a miss (the reference spins forever there; probe_kernel stops after
 * num_sigs buckets -- same answer, since every bucket has been seen).
 * The matching lane writes the record to LDS for the window's owner.
 */
template <int J, int G, bool DNA>
__global__ __launch_bounds__(256) void probe_line_kernel(
    const uint8_t *__restrict__ residues, uint64_t n_residues, const uint64_t *__restrict__ seq_off,
    const uint64_t *__restrict__ wbase, const uint32_t *__restrict__ tile_seq, uint32_t n_seq,
    const uint4 *__restrict__ packed, uint64_t num_sigs, uint64_t magic, uint32_t hs, uint4 *__restrict__ hot,
    uint4 *__restrict__ cold, uint64_t *__restrict__ hit_mask, uint32_t nt)
{
    constexpr uint32_t T = 64 * J;
    constexpr uint32_t NQ = 64 / G; /* windows per instruction */
    constexpr int NI = J * G;       /* instructions per tile */
    __shared__ uint8_t code_tab[256]; /* residue -> code; DNA: base -> class */
    __shared__ uint8_t cod_tab[DNA ? 68 : 1];
    __shared__ uint4 lds_rec[PROBE_WAVES][T];
    __shared__ uint8_t lds_hit[PROBE_WAVES][T];
    if (DNA) {
        const uint32_t b = threadIdx.x | 0x20u; /* ACGTU either case (trans_table.h:45-68) */
        const bool base = b == 'a' || b == 'c' || b == 'g' || b == 't' || b == 'u';
        code_tab[threadIdx.x] = base ? (uint8_t)(((b >> 1) ^ (b >> 2)) & 3u) : (uint8_t)0x40;
        if (threadIdx.x < 65)
            cod_tab[threadIdx.x] = threadIdx.x < 64 ? (uint8_t)residue_code((uint8_t)code11_aa(threadIdx.x)) : 20;
    } else {
        code_tab[threadIdx.x] = (uint8_t)residue_code(threadIdx.x);
    }
    __syncthreads();

    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    const uint64_t W = wbase[n_seq];
    /* one tile per wave, or (a grid smaller than the tiles, option
     * probe_persist) the wave strides over tiles: every wave leaves once its
     * next tile lies past the batch's last window */
    for (uint64_t tile = (uint64_t)blockIdx.x * PROBE_WAVES + wave; tile * T < W;
         tile += (uint64_t)gridDim.x * PROBE_WAVES) {
    const uint64_t g0 = tile * T;

    uint64_t key[J];
    uint32_t pos[J], sq[J];
    bool ok[J];
    if (DNA)
        encode_tile_dna<J>(residues, n_residues, seq_off, wbase, tile_seq[tile], W, g0, lane, code_tab, cod_tab,
                           key, ok, pos, sq);
    else
        encode_tile<J>(residues, n_residues, seq_off, wbase, tile_seq[tile], W, g0, lane, code_tab, key, ok,
                       pos, sq);
    uint64_t home[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        home[j] = ok[j] ? mod_by(key[j], num_sigs >> hs, magic) << hs : 0; /* hs 2: line-aligned homes */
        lds_hit[wave][64 * j + lane] = 0;
    }

    const uint32_t q = lane / G, c = lane % G;
    uint64_t K[NI], cur[NI];
    uint32_t live = 0; /* bit i: instruction i's chain is still open */
#pragma unroll
    for (int i = 0; i < NI; i++) {
        const uint32_t owner = NQ * (i % G) + q; /* slice i / G */
        K[i] = __shfl(key[i / G], (int)owner);
        cur[i] = __shfl(home[i / G], (int)owner);
        live |= (uint32_t)__shfl((int)ok[i / G], (int)owner) << i;
    }
    /* lines a chain may visit before it has covered the whole table */
    const uint64_t max_lines = num_sigs / G + 2;
    for (uint64_t round = 0;; round++) {
        /* only open chains load; d is fresh each round (no merge with an
         * older value at the branch join, so no wait for the load there) */
        uint4 d[NI];
#pragma unroll
        for (int i = 0; i < NI; i++) {
            const uint64_t line = cur[i] - cur[i] % G;
            if ((live >> i & 1u) && line + c < num_sigs)
                d[i] = packed[line + c];
        }
        bool more = false;
#pragma unroll
        for (int i = 0; i < NI; i++) {
            const bool act = live >> i & 1u;
            const uint64_t line = cur[i] - cur[i] % G;
            const uint64_t b = line + c;
            const uint64_t kb = ((uint64_t)d[i].y << 32 | d[i].x) & PACK_KEY_MASK;
            const bool valid = act && b < num_sigs && b >= cur[i];
            const uint64_t mm = __ballot(valid && kb == K[i]);
            const uint64_t me = __ballot(valid && kb > MAX_ENCODED);
            const uint32_t gm = (uint32_t)(mm >> (G * q)) & ((1u << G) - 1);
            const uint32_t ge = (uint32_t)(me >> (G * q)) & ((1u << G) - 1);
            if (act) {
                const uint32_t ev = gm | ge;
                if (ev) {
                    const uint32_t first = __builtin_ctz(ev);
                    if (c == first && (gm >> first & 1u)) {
                        const uint32_t w = NQ * i + q;
                        lds_rec[wave][w] = d[i];
                        lds_hit[wave][w] = 1;
                    }
                    live &= ~(1u << i);
                } else if (round + 1 >= max_lines) {
                    live &= ~(1u << i);
                } else {
                    cur[i] = line + G >= num_sigs ? 0 : line + G;
                    more = true;
                }
            }
        }
        if (!__any(more))
            break;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    bool hit[J];
    uint4 pv[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        hit[j] = lds_hit[wave][64 * j + lane] != 0;
        pv[j] = hit[j] ? lds_rec[wave][64 * j + lane] : make_uint4(0, 0, 0, 0);
    }
    store_tile_hits<J, true>(hit, key, pv, pos, sq, g0, W, lane, hot, cold, hit_mask, nt != 0);
    } /* tiles */
}

template <int J, int G, bool DNA = false>
static void launch_probe_line(dim3 grid, hipStream_t stream, const uint8_t *residues, uint64_t n_residues,
                              const uint64_t *seq_off, const uint64_t *wbase, const uint32_t *tile_seq,
                              uint32_t n_seq, const void *table, uint64_t num_sigs, uint32_t hs, uint4 *hot,
                              uint4 *cold, uint64_t *hit_mask, uint32_t dyn_lds, uint32_t nt = 0)
{
    hipLaunchKernelGGL((probe_line_kernel<J, G, DNA>), grid, dim3(64 * PROBE_WAVES), dyn_lds, stream, residues,
                       n_residues, seq_off, wbase, tile_seq, n_seq, static_cast<const uint4 *>(table),
                       num_sigs, mod_magic(num_sigs >> hs), hs, hot, cold, hit_mask, nt);
}

template <int J, int MODE>
static void launch_probe_m(dim3 grid, hipStream_t stream, const uint8_t *residues, uint64_t n_residues,
                           const uint64_t *seq_off, const uint64_t *wbase, const uint32_t *tile_seq,
                           uint32_t n_seq, const void *table, uint64_t num_sigs, uint32_t hs,
                           const uint64_t *filter, uint32_t filter_log2, uint4 *hot, uint4 *cold,
                           uint64_t *hit_mask)
{
    const uint64_t magic = mod_magic(num_sigs >> hs);
    if (filter)
        hipLaunchKernelGGL((probe_kernel<J, MODE, true>), grid, dim3(64 * PROBE_WAVES), 0, stream, residues,
                           n_residues, seq_off, wbase, tile_seq, n_seq, table, num_sigs, magic, hs, filter,
                           filter_log2, hot, cold, hit_mask);
    else
        hipLaunchKernelGGL((probe_kernel<J, MODE, false>), grid, dim3(64 * PROBE_WAVES), 0, stream, residues,
                           n_residues, seq_off, wbase, tile_seq, n_seq, table, num_sigs, magic, hs, filter,
                           filter_log2, hot, cold, hit_mask);
}

template <int J>
static void launch_probe_j(dim3 grid, hipStream_t stream, int mode, const uint8_t *residues,
                           uint64_t n_residues, const uint64_t *seq_off, const uint64_t *wbase,
                           const uint32_t *tile_seq, uint32_t n_seq, const void *table,
                           uint64_t num_sigs, uint32_t hs, const uint64_t *filter, uint32_t filter_log2,
                           uint4 *hot, uint4 *cold, uint64_t *hit_mask)
{
#define KGX_PROBE_M(M)                                                                               \
    launch_probe_m<J, M>(grid, stream, residues, n_residues, seq_off, wbase, tile_seq, n_seq, table,  \
                         num_sigs, hs, filter, filter_log2, hot, cold, hit_mask)
    if (mode == MODE_PACKED_KEY_FIRST)
        KGX_PROBE_M(MODE_PACKED_KEY_FIRST);
    else if (mode == MODE_PACKED)
        KGX_PROBE_M(MODE_PACKED);
    else if (mode == MODE_KEY_FIRST)
        KGX_PROBE_M(MODE_KEY_FIRST);
    else
        KGX_PROBE_M(MODE_BUCKET);
#undef KGX_PROBE_M
}

hipError_t launch_probe(const uint8_t *residues, uint64_t n_residues, const uint64_t *seq_off,
                        const uint64_t *wbase, const uint32_t *tile_seq, uint32_t n_seq,
                        uint64_t max_tiles, const void *table, int layout, uint64_t num_sigs,
                        const uint64_t *filter, uint32_t filter_log2,
                        uint4 *hot, uint4 *cold, uint64_t *hit_mask, int probe_j, int variant,
                        uint32_t lds_kb, uint32_t max_blocks, hipStream_t stream, uint32_t hs, uint32_t nt)
{
    if (max_tiles == 0)
        return hipSuccess;
    if (hs && layout != KGX_LAYOUT_PACKED16)
        return hipErrorInvalidValue; /* line-aligned homes exist for PACKED16 records only */
    /* lds_kb > 0: each probe workgroup reserves that much LDS (unused beyond
     * its own ~9 KB), capping the probe at 160 / lds_kb workgroups per CU so
     * that other contexts' kernels find room beside it */
    const uint32_t dyn_lds = lds_kb * 1024u > 9216u ? lds_kb * 1024u - 9216u : 0u;
    const dim3 grid((uint32_t)((max_tiles + PROBE_WAVES - 1) / PROBE_WAVES));
    /* the line probe strides over tiles when its grid is capped */
    const dim3 lgrid(max_blocks ? std::min<uint32_t>(grid.x, max_blocks) : grid.x);
    if (variant == PROBE_AUTO && layout == KGX_LAYOUT_PACKED16 && !filter)
        variant = PROBE_LINE;
    if ((variant == PROBE_LINE || variant == PROBE_LINE8) && layout == KGX_LAYOUT_PACKED16 && !filter) {
#define KGX_LINE(JJ, GG)                                                                             \
    launch_probe_line<JJ, GG>(lgrid, stream, residues, n_residues, seq_off, wbase, tile_seq, n_seq, table, \
                              num_sigs, hs, hot, cold, hit_mask, dyn_lds, nt);                       \
    return hipGetLastError()
        const int key = probe_j * 10 + (variant == PROBE_LINE8 ? 8 : 4);
        switch (key) {
        case 14: KGX_LINE(1, 4);
        case 24: KGX_LINE(2, 4);
        case 34: KGX_LINE(3, 4);
        case 44: KGX_LINE(4, 4);
        case 18: KGX_LINE(1, 8);
        case 28: KGX_LINE(2, 8);
        default: break; /* other tile sizes: the per-bucket kernel below */
        }
#undef KGX_LINE
    }
    const bool kf = variant == PROBE_AUTO ? layout != KGX_LAYOUT_PACKED16 : variant == PROBE_KEY_FIRST;
    const int mode = layout == KGX_LAYOUT_PACKED16 ? (kf ? MODE_PACKED_KEY_FIRST : MODE_PACKED)
                                                   : (kf ? MODE_KEY_FIRST : MODE_BUCKET);
#define KGX_PROBE_J(JJ)                                                                              \
    launch_probe_j<JJ>(grid, stream, mode, residues, n_residues, seq_off, wbase, tile_seq, n_seq,   \
                       table, num_sigs, hs, filter, filter_log2, hot, cold, hit_mask)
    switch (probe_j) {
    case 1: KGX_PROBE_J(1); break;
    case 2: KGX_PROBE_J(2); break;
    case 3: KGX_PROBE_J(3); break;
    case 4: KGX_PROBE_J(4); break;
    case 5: KGX_PROBE_J(5); break;
    case 8: KGX_PROBE_J(8); break;
    default: return hipErrorInvalidValue;
    }
#undef KGX_PROBE_J
    return hipGetLastError();
}

hipError_t launch_probe_dna(const uint8_t *bases, uint64_t n_bases, const uint64_t *anchor, const uint64_t *wbase,
                            const uint32_t *tile_seq, uint32_t n_seq, uint64_t max_tiles, const void *table,
                            uint64_t num_sigs, uint4 *hot, uint64_t *hit_mask, int probe_j, uint32_t max_blocks,
                            hipStream_t stream, uint32_t hs)
{
    if (max_tiles == 0)
        return hipSuccess;
    const uint32_t tiles_grid = (uint32_t)((max_tiles + PROBE_WAVES - 1) / PROBE_WAVES);
    const dim3 grid(max_blocks ? std::min<uint32_t>(tiles_grid, max_blocks) : tiles_grid);
#define KGX_DNA(JJ)                                                                                  \
    launch_probe_line<JJ, 4, true>(grid, stream, bases, n_bases, anchor, wbase, tile_seq, n_seq, table,  \
                                   num_sigs, hs, hot, nullptr, hit_mask, 0);                        \
    return hipGetLastError()
    switch (probe_j) {
    case 1: KGX_DNA(1);
    case 2: KGX_DNA(2);
    case 3: KGX_DNA(3);
    case 4: KGX_DNA(4);
    default: return hipErrorInvalidValue;
    }
#undef KGX_DNA
}

/* ------------------------------------------------------------------------ */
/* resident layout conversion                                                */
/* ------------------------------------------------------------------------ */

__global__ __launch_bounds__(256) void pack_kernel(const kgx_sig_kmer *__restrict__ table,
                                                   packed_bucket *__restrict__ packed, uint64_t n,
                                                   uint32_t *not_packable)
{
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const kgx_sig_kmer e = table[i];
        bad |= !packable(e);
        packed[i] = pack_bucket(e);
    }
    if (__any(bad) && lane_id() == 0)
        atomicOr(not_packable, 1u);
}

__global__ __launch_bounds__(256) void unpack_kernel(const packed_bucket *__restrict__ packed,
                                                     kgx_sig_kmer *__restrict__ out, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = unpack_bucket(packed[i]);
}

__global__ __launch_bounds__(256) void filter_build_kernel(const void *__restrict__ table, int layout, uint64_t n,
                                                           uint64_t *__restrict__ filter, uint32_t log2_words)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t key = layout == KGX_LAYOUT_PACKED16
                                 ? static_cast<const packed_bucket *>(table)[i].lo & PACK_KEY_MASK
                                 : static_cast<const kgx_sig_kmer *>(table)[i].which_kmer;
        if (key > MAX_ENCODED)
            continue;
        const uint64_t h = filter_hash(key);
        atomicOr(reinterpret_cast<unsigned long long *>(filter + filter_word(h, log2_words)),
                 (unsigned long long)filter_bits(h));
    }
}

hipError_t launch_filter_build(const void *table, int layout, uint64_t num_sigs, uint64_t *filter,
                               uint32_t log2_words, hipStream_t stream)
{
    hipLaunchKernelGGL(filter_build_kernel, dim3(8192), dim3(256), 0, stream, table, layout, num_sigs, filter,
                       log2_words);
    return hipGetLastError();
}

/* stored keys of a PACKED16 table (grid-stride blocks, one atomic each) */
__global__ __launch_bounds__(256) void count_keys_kernel(const packed_bucket *__restrict__ t, uint64_t n,
                                                         unsigned long long *count)
{
    uint64_t c = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        c += (t[i].lo & PACK_KEY_MASK) <= MAX_ENCODED;
    for (int o = 32; o > 0; o >>= 1)
        c += __shfl_xor(c, o);
    if (lane_id() == 0 && c)
        atomicAdd(count, (unsigned long long)c);
}

/* The line index (kgx_image_set_line_index): every bucket b of the reference
 * table whose key the reference's probe of that key reaches first --
 * lookup_hash_entry (kguts.cc:585-602) walks from key mod num_sigs and stops at
 * the key or at a stop bucket, so a duplicate further on or an entry behind a
 * stop is never found -- is inserted into the line table by linear probing
 * from the start of line (key mod n_lines), 4 buckets a line, by a 64-bit CAS
 * on the record's first word.  A probe of the line table from that home finds
 * exactly the records the reference finds, so results are unchanged while
 * almost every chain ends in its first 64-B line. */
__global__ __launch_bounds__(256) void lines_build_kernel(const packed_bucket *__restrict__ src, uint64_t num_sigs,
                                                          uint64_t src_magic, packed_bucket *lines, uint64_t n_lines,
                                                          uint64_t line_magic, uint32_t *overflow)
{
    const uint64_t NB = 4 * n_lines;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < num_sigs;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const packed_bucket e = src[b];
        const uint64_t key = e.lo & PACK_KEY_MASK;
        if (key > MAX_ENCODED)
            continue;
        bool first = true;
        for (uint64_t x = mod_by(key, num_sigs, src_magic); x != b; x = x + 1 == num_sigs ? 0 : x + 1) {
            const uint64_t k2 = src[x].lo & PACK_KEY_MASK;
            if (k2 == key || k2 > MAX_ENCODED) {
                first = false;
                break;
            }
        }
        if (!first)
            continue;
        uint64_t x = mod_by(key, n_lines, line_magic) * 4;
        bool placed = false;
        for (uint64_t n = 0; n < NB && !placed; n++) {
            const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long *>(&lines[x].lo),
                                                      (unsigned long long)EMPTY_KEY, (unsigned long long)e.lo);
            if (prev == (unsigned long long)EMPTY_KEY) {
                lines[x].hi = e.hi;
                placed = true;
            }
            x = x + 1 == NB ? 0 : x + 1;
        }
        if (!placed)
            atomicOr(overflow, 1u);
    }
}

__global__ __launch_bounds__(256) void fill_empty_kernel(packed_bucket *t, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        t[i].lo = EMPTY_KEY;
        t[i].hi = 0;
    }
}

hipError_t launch_count_keys(const packed_bucket *t, uint64_t n, unsigned long long *count, hipStream_t stream)
{
    hipLaunchKernelGGL(count_keys_kernel, dim3(4096), dim3(256), 0, stream, t, n, count);
    return hipGetLastError();
}

hipError_t launch_lines_build(const packed_bucket *src, uint64_t num_sigs, packed_bucket *lines, uint64_t n_lines,
                              uint32_t *overflow, hipStream_t stream)
{
    hipLaunchKernelGGL(fill_empty_kernel, dim3(8192), dim3(256), 0, stream, lines, 4 * n_lines);
    hipLaunchKernelGGL(lines_build_kernel, dim3(8192), dim3(256), 0, stream, src, num_sigs, mod_magic(num_sigs), lines,
                       n_lines, mod_magic(n_lines), overflow);
    return hipGetLastError();
}

hipError_t launch_pack(const kgx_sig_kmer *table, packed_bucket *packed, uint64_t n,
                       uint32_t *not_packable, hipStream_t stream)
{
    hipLaunchKernelGGL(pack_kernel, dim3(8192), dim3(256), 0, stream, table, packed, n, not_packable);
    return hipGetLastError();
}

hipError_t launch_unpack(const packed_bucket *packed, kgx_sig_kmer *out, uint64_t n,
                         hipStream_t stream)
{
    hipLaunchKernelGGL(unpack_kernel, dim3(8192), dim3(256), 0, stream, packed, out, n);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* hits of one sequence in the tiled layout                                  */
/* ------------------------------------------------------------------------ */

/*
 * Calls f(storage_start, count, ordinal0) for each run of the sequence's hits
 * (windows [gw0, gw1)): within one mask word, the sequence's hits are a
 * contiguous stretch of its tile's compacted hits.  Returns the hit count.
 */
template <class F>
__device__ __forceinline__ uint32_t for_each_run(const uint64_t *__restrict__ hit_mask,
                                                 uint32_t tile_windows, uint64_t gw0, uint64_t gw1,
                                                 F &&f)
{
    if (gw0 >= gw1)
        return 0;
    const uint32_t J = tile_windows / 64;
    const uint64_t gfirst = gw0 >> 6, glast = (gw1 - 1) >> 6;
    uint64_t tile = gfirst / J;
    uint32_t pre = 0; /* tile's hits before word g */
    for (uint64_t g = tile * J; g < gfirst; g++)
        pre += (uint32_t)__popcll(hit_mask[g]);
    uint32_t ordinal = 0;
    uint64_t next = hit_mask[gfirst];
    for (uint64_t g = gfirst; g <= glast; g++) {
        if (g != gfirst && g % J == 0) {
            tile = g / J;
            pre = 0;
        }
        const uint64_t full = next;
        if (g < glast)
            next = hit_mask[g + 1]; /* in flight while f works on word g */
        const uint32_t lo = g == gfirst ? (uint32_t)(gw0 & 63) : 0u;
        const uint32_t hi = g == glast ? (uint32_t)((gw1 - 1) & 63) + 1 : 64u;
        const uint64_t bits = full & bit_range(lo, hi);
        const uint32_t cnt = (uint32_t)__popcll(bits);
        if (cnt) /* the hits' positions: bit b of `bits` is position 64 g + b - gw0 */
            f(tile * tile_windows + pre + (uint32_t)__popcll(full & bit_range(0, lo)), cnt, ordinal, bits,
              (uint32_t)(64 * g - gw0));
        ordinal += cnt;
        pre += (uint32_t)__popcll(full);
    }
    return ordinal;
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
 * With OTU output requested, buffered hits are flagged KGX_HIT_IN_RUN (and
 * KGX_HIT_COUNTED when their function is their run's current_fI); each
 * emitted call records its run's ordinal hit range, and a second walk flags
 * the COUNTED hits inside emitted ranges KGX_HIT_OTU -- the hits the
 * reference tallies into otu_map (kguts.cc:760-768).
 */
struct RunTail {
    uint32_t pos, fI, idx;
    float wt;
    uint32_t avg;
    uint32_t fb; /* the record's flag dword without flags */
    uint64_t at; /* storage index */
};

constexpr int SCORE_BATCH = 8; /* records per load batch (double-buffered); 2 for short sequences */

template <bool PK, int SB = SCORE_BATCH>
__device__ __forceinline__ void score_sequence(
    uint32_t s, const uint64_t *__restrict__ wbase, const uint64_t *__restrict__ hit_mask,
    uint32_t tile_windows, uint4 *__restrict__ hot, kgx_call *__restrict__ calls,
    uint2 *__restrict__ ranges, uint32_t *__restrict__ hit_count, uint32_t *__restrict__ call_count,
    const kgx_params &prm, uint32_t want)
{
    const uint64_t gw0 = wbase[s], gw1 = wbase[s + 1];
    const bool want_calls = (want & KGX_WANT_CALLS) != 0;
    const bool want_otu = (want & KGX_WANT_OTU) != 0;
    if (!want_calls && !want_otu) {
        /* process_set_of_hits returns before doing anything (kguts.cc:737) */
        hit_count[s] = for_each_run(hit_mask, tile_windows, gw0, gw1,
                                    [](uint64_t, uint32_t, uint32_t, uint64_t, uint32_t) {});
        call_count[s] = 0;
        return;
    }
    if (!want_otu && prm.min_hits > 0 && gw1 > gw0) {
        /* fewer hits than min_hits: no run can reach a call (a call counts
         * at most the sequence's hits, kguts.cc:757-770), and without OTU
         * output the run flags are not kept -- count and leave without
         * reading a record (fq fragments: ~16 windows, < 1 hit each) */
        uint32_t nh = 0;
        for (uint64_t g = gw0 >> 6; g <= (gw1 - 1) >> 6; g++) {
            const uint32_t lo = g == (gw0 >> 6) ? (uint32_t)(gw0 & 63) : 0u;
            const uint32_t hi = g == ((gw1 - 1) >> 6) ? (uint32_t)((gw1 - 1) & 63) + 1 : 64u;
            nh += (uint32_t)__popcll(hit_mask[g] & bit_range(lo, hi));
        }
        if ((int)nh < prm.min_hits) {
            hit_count[s] = nh;
            call_count[s] = 0;
            return;
        }
    }

    typedef HitFields<PK> HF;
    constexpr uint32_t F_RUN = KGX_HIT_IN_RUN << HF::FLAG_SHIFT, F_CNT = KGX_HIT_COUNTED << HF::FLAG_SHIFT,
                       F_OTU = KGX_HIT_OTU << HF::FLAG_SHIFT;
    constexpr int FD = HF::FLAG_DWORD;
    uint32_t *hw = reinterpret_cast<uint32_t *>(hot); /* 4 dwords per hit, flags in dword FD */
    const uint64_t cbase = gw0; /* calls / ranges of s live at [gw0, ...) */
    const uint32_t gap = (uint32_t)prm.max_gap;
    int n = 0;
    uint32_t cur = 0, first_pos = 0, last_pos = 0, last_idx = 0, run_start = 0;
    int cnt = 0;
    float wsum = 0.0f;
    RunTail p1 = {0, 0, 0, 0.0f, 0, 0, 0}, p2 = {0, 0, 0, 0.0f, 0, 0, 0};
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
                calls[cbase + ncalls] = cl;
            }
            if (want_otu)
                ranges[cbase + ncalls] = make_uint2(run_start, last_idx);
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
                hw[4 * p2.at + FD] = p2.fb | F_RUN | F_CNT;
                hw[4 * p1.at + FD] = p1.fb | F_RUN | F_CNT;
            }
        } else {
            n = 0;
        }
    };

    auto step = [&](const uint4 &r, uint32_t i, uint64_t at, uint32_t pos) {
        const uint32_t avg = HF::avg(r);
        const uint32_t fI = HF::fi(r);
        const float wt = __uint_as_float(HF::wt(r));
        const uint32_t fb = HF::flag_base(r);
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
                    hw[4 * at + FD] = fb | F_RUN | (counted ? F_CNT : 0u);
                if (counted) {
                    cnt++;
                    wsum += wt;
                    last_pos = pos;
                    last_idx = i;
                }
                p2 = p1;
                p1 = RunTail{pos, fI, i, wt, avg, fb, at};
            }
            /* pair switch (kguts.cc:852-856) */
            if (n > 1 && cur != fI && p2.fI == p1.fI)
                flush();
        }
    };

    /* hits are read SB at a time and double-buffered: batch b+1's
     * loads are in flight while batch b runs through the state machine (the
     * machine is serial, its inputs are not) */
    auto load_batch = [&](uint4 *rb, uint64_t at0, uint32_t b, uint32_t c) {
#pragma unroll
        for (int k = 0; k < SB; k++)
            if (b + k < c)
                rb[k] = hot[at0 + b + k];
    };
    const uint32_t nh = for_each_run(hit_mask, tile_windows, gw0, gw1,
                                     [&](uint64_t at0, uint32_t c, uint32_t ord0, uint64_t bits, uint32_t pbase) {
        uint4 ra[SB], rb[SB];
        load_batch(ra, at0, 0, c);
        for (uint32_t b = 0; b < c; b += 2 * SB) {
            if (b + SB < c)
                load_batch(rb, at0, b + SB, c);
#pragma unroll
            for (int k = 0; k < SB; k++)
                if (b + k < c) {
                    step(ra[k], ord0 + b + k, at0 + b + k, pbase + (uint32_t)__builtin_ctzll(bits));
                    bits &= bits - 1;
                }
            if (b + SB >= c)
                break;
            if (b + 2 * SB < c)
                load_batch(ra, at0, b + 2 * SB, c);
#pragma unroll
            for (int k = 0; k < SB; k++)
                if (b + SB + k < c) {
                    step(rb[k], ord0 + b + SB + k, at0 + b + SB + k,
                         pbase + (uint32_t)__builtin_ctzll(bits));
                    bits &= bits - 1;
                }
        }
    });
    if (n >= prm.min_hits) /* kguts.cc:873-876 */
        flush();
    hit_count[s] = nh;
    call_count[s] = want_calls ? ncalls : 0;

    /* OTU flags: COUNTED hits inside an emitted call's ordinal range (ranges
     * are disjoint and in order) */
    if (want_otu && ncalls > 0) {
        uint32_t ci = 0;
        uint2 rg = ranges[cbase];
        const uint32_t end = ranges[cbase + ncalls - 1].y;
        for_each_run(hit_mask, tile_windows, gw0, gw1,
                     [&](uint64_t at0, uint32_t c, uint32_t ord0, uint64_t, uint32_t) {
            for (uint32_t k = 0; k < c; k++) {
                const uint32_t i = ord0 + k;
                if (i > end)
                    return;
                while (i > rg.y) /* i <= end keeps ci < ncalls */
                    rg = ranges[cbase + ++ci];
                if (i >= rg.x) {
                    const uint32_t f = hw[4 * (at0 + k) + FD];
                    if (f & F_CNT)
                        hw[4 * (at0 + k) + FD] = f | F_OTU;
                }
            }
        });
    }
}

/* skip_above: sequences with windows in (skip_above, RUN_CAP] are the wave
 * scorer's (hybrid dispatch); ~0u = none */
template <bool PK, int SB>
__global__ __launch_bounds__(256) void score_kernel(
    uint32_t n_seq, const uint64_t *__restrict__ wbase, const uint64_t *__restrict__ hit_mask,
    uint32_t tile_windows, uint4 *__restrict__ hot, kgx_call *__restrict__ calls,
    uint2 *__restrict__ ranges, uint32_t *__restrict__ hit_count, uint32_t *__restrict__ call_count,
    kgx_params prm, uint32_t want, uint32_t skip_above)
{
    /* grid-stride: a capped grid (KGX_SCORE_GRID_CAP) walks several
     * sequences per lane */
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n_seq; s += gridDim.x * blockDim.x) {
        const uint64_t w = wbase[s + 1] - wbase[s];
        if (w > skip_above && w <= (uint64_t)RUN_CAP)
            continue;
        score_sequence<PK, SB>(s, wbase, hit_mask, tile_windows, hot, calls, ranges, hit_count, call_count, prm,
                               want);
    }
}

/* ------------------------------------------------------------------------ */
/* score, wave-parallel                                                      */
/* ------------------------------------------------------------------------ */

/*
 * The same run rules (gather_hits kguts.cc:808-876, process_set_of_hits
 * kguts.cc:734-781) evaluated 64 hits at a time by one wave, for
 * order_constraint == 0 and sequences of at most RUN_CAP windows (every hit is
 * then buffered: the 40,000-entry cap never binds).  Under those conditions
 * the state machine reduces to per-hit predicates over a hit and its
 * predecessor in the same sequence:
 *   brk[i]  = first hit of its sequence, or prev.pos + max_gap < pos
 *             (unsigned, kguts.cc:821-831): a new run starts at i;
 *   mark[i] = brk[i] or fI[i] == fI[i-1]: after hit i, current_fI = fI[i];
 *   cur[i]  = fI of the last marked hit at or before i (a segmented scan:
 *             one ballot and a highest-set-bit per lane);
 *   switch  = fI[i] == fI[i-1] != cur[i-1] (kguts.cc:852-856): the run so far
 *             is flushed and the carried pair i-1, i starts a new sub-run
 *             (kguts.cc:771-779; a gap flush never carries: its last two hits
 *             would have switched already).
 * Sub-runs start at brk hits and one hit before switch hits; a sub-run's call
 * counts its hits with fI == its current_fI (its first hit always does), from
 * its first hit to the last such hit, and is emitted when count >= min_hits
 * and the f32 sum of their weights, added in hit order from 0.0f, is >=
 * min_weighted_hits -- the same condition at a gap, a switch and the final
 * flush.  Everything but that sum is ballots, bit counts and shuffles; the
 * sums run serially (v_readlane + v_add_f32 in hit order) only over sub-runs
 * that reach min_hits.
 *
 * Work: wave w takes the sequences whose first window lies in windows
 * [w R, (w+1) R) (R = SCORE_WAVE_TILES tiles; found from tile_seq), walks
 * their hit-mask words (64 at a time in a register) and queues each hit's
 * (position, sequence, first window, storage slot) in LDS; every 64 queued
 * hits -- of one long sequence or of many short fragments -- are one chunk.
 * The open sub-run, the last hit and the open sequence's call count carry
 * from chunk to chunk.  A sub-run that spans chunks and is emitted gets its
 * OTU flags by a walk over its windows.  Sequences longer than RUN_CAP
 * windows run the serial machine (score_sequence) on one lane.
 */
constexpr uint32_t SQ = 256; /* queue entries per wave: a chunk in flight, the next, a word's overflow */

struct ScoreQueue {
    uint32_t pos[SQ];
    uint32_t seq[SQ];
    uint32_t at[SQ];
    uint64_t mw[64]; /* hit-mask words gb .. gb + 63 */
    uint64_t wb[65]; /* window bases of sequences sb .. sb + 64 */
};


/* first sequence whose first window is >= x (x a tile boundary below the
 * batch's window count); tile_seq[x / T] owns window x */
__device__ __forceinline__ uint32_t seq_lower_bound(const uint64_t *__restrict__ wbase,
                                                    const uint32_t *__restrict__ tile_seq, uint32_t T, uint64_t x)
{
    uint32_t s = tile_seq[x / T];
    if (wbase[s] < x)
        return s + 1;
    while (s > 0 && wbase[s - 1] == x) /* empty sequences right before it */
        s--;
    return s;
}

template <bool PK>
__global__ __launch_bounds__(256) void score_wave_kernel(
    uint32_t n_seq, const uint64_t *__restrict__ wbase, const uint32_t *__restrict__ tile_seq,
    const uint64_t *__restrict__ hit_mask, uint32_t tile_windows, uint32_t wave_tiles, uint4 *__restrict__ hot,
    kgx_call *__restrict__ calls, uint32_t *__restrict__ hit_count, uint32_t *__restrict__ call_count,
    kgx_params prm, uint32_t want, uint32_t only_above, const uint32_t *__restrict__ plan_status)
{
    /* hybrid dispatch: only sequences over only_above windows are this
     * kernel's; the plan's longest-sequence word says whether there are any */
    if (only_above && plan_status[1] <= only_above)
        return;
    __shared__ ScoreQueue queues[4];
    typedef HitFields<PK> HF;
    constexpr uint32_t F_RUN = KGX_HIT_IN_RUN << HF::FLAG_SHIFT, F_CNT = KGX_HIT_COUNTED << HF::FLAG_SHIFT,
                       F_OTU = KGX_HIT_OTU << HF::FLAG_SHIFT;
    constexpr int FD = HF::FLAG_DWORD;
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    ScoreQueue &Q = queues[threadIdx.x >> 6];
    uint32_t *hw = reinterpret_cast<uint32_t *>(hot);
    const uint32_t lane = lane_id();
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t R = (uint64_t)tile_windows * wave_tiles;
    const uint64_t W = wbase[n_seq];
    const uint64_t x0 = (uint64_t)w * R;
    if (w > 0 && x0 >= W)
        return;
    const uint32_t s_lo = w == 0 ? 0u : seq_lower_bound(wbase, tile_seq, tile_windows, x0);
    const uint32_t s_hi = x0 + R >= W ? n_seq : seq_lower_bound(wbase, tile_seq, tile_windows, x0 + R);
    const bool want_calls = (want & KGX_WANT_CALLS) != 0;
    const bool want_otu = (want & KGX_WANT_OTU) != 0;
    const bool scoring = want_calls || want_otu;
    const uint32_t J = tile_windows / 64;
    const uint32_t gap = (uint32_t)prm.max_gap;
    const float min_wh = (float)prm.min_weighted_hits;

    /* ---- the open sub-run (O) and the last hit, carried across chunks ---- */
    bool o_valid = false, o_span = false;
    uint32_t o_seq = NONE, o_cur = 0, o_cnt = 0, o_first = 0, o_last = 0, o_ncalls = 0;
    float o_wsum = 0.0f;
    uint32_t p_pos = 0, p_fi = 0, p_fb = 0, p_at = 0;
    float p_wt = 0.0f;

    /* OTU flags of an emitted sub-run that spans chunks: its hits are the
     * sequence's hits in windows [first, last]; the ones with fI == cur count */
    auto otu_fixup = [&](uint64_t gw0, uint32_t first, uint32_t last, uint32_t cur) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); /* earlier flag stores are done */
        const uint64_t a = gw0 + first, b = gw0 + last;
        for (uint64_t g = a >> 6; g <= (b >> 6); g++) {
            const uint64_t full = hit_mask[g];
            const uint32_t lo = g == (a >> 6) ? (uint32_t)(a & 63) : 0u;
            const uint32_t hi = g == (b >> 6) ? (uint32_t)(b & 63) + 1 : 64u;
            const uint64_t bits = full & bit_range(lo, hi);
            const uint64_t tile = g / J;
            uint32_t pre = 0;
            for (uint64_t q = tile * J; q < g; q++)
                pre += (uint32_t)__popcll(hit_mask[q]);
            if ((bits >> lane) & 1) {
                const uint64_t at = tile * tile_windows + pre + lanes_below(full);
                const uint4 r = hot[at];
                if (HF::fi(r) == cur)
                    hw[4 * at + FD] = HF::flag_base(r) | F_RUN | F_CNT | F_OTU;
            }
        }
    };
    /* flush of O: the call (kguts.cc:757-770) when count and weight reach the minimums */
    auto close_open = [&]() -> bool {
        const bool em = (int)o_cnt >= prm.min_hits && o_wsum >= min_wh;
        if (em) {
            const uint64_t gw0 = wbase[o_seq];
            if (want_calls && lane == 0) {
                kgx_call cl;
                cl.start = o_first;
                cl.end = o_last + (KMER - 1);
                cl.count = (int32_t)o_cnt;
                cl.function_index = o_cur;
                cl.weighted_hits = o_wsum;
                calls[gw0 + o_ncalls] = cl;
            }
            o_ncalls++;
            if (want_otu && o_span)
                otu_fixup(gw0, o_first, o_last, o_cur);
        }
        return em;
    };

    uint32_t qhead = 0, qissue = 0, qtail = 0;

    /* one chunk: queue entries [qhead, qhead + n), n <= 64, records in r */
    auto process_chunk = [&](uint32_t n, const uint4 &r) {
        const uint32_t k = lane;
        const bool act = k < n;
        const uint64_t ACT = n >= 64 ? ~0ull : ((1ull << n) - 1);
        const uint32_t e = (qhead + k) & (SQ - 1);
        const uint32_t pos = act ? Q.pos[e] : 0u;
        const uint32_t seq = act ? Q.seq[e] : NONE;
        const uint32_t at = act ? Q.at[e] : 0u;
        const uint32_t fi = HF::fi(r);
        const float wt = __uint_as_float(HF::wt(r));
        const uint32_t fb = HF::flag_base(r);

        /* the predecessor of each hit (lane 0: the carried last hit) */
        uint32_t ppos = __shfl_up(pos, 1), pfi = __shfl_up(fi, 1), pseq = __shfl_up(seq, 1);
        if (k == 0) {
            ppos = p_pos;
            pfi = p_fi;
            pseq = o_valid ? o_seq : NONE;
        }
        const bool newseq = seq != pseq;
        const bool brk = newseq || (ppos + gap < pos);
        const bool eqp = !brk && fi == pfi;
        const uint64_t M = __ballot(act && (brk || eqp));
        const int jm = hibit(M & lanes_le(k));
        uint32_t cur = __shfl(fi, jm < 0 ? 0 : jm);
        if (jm < 0)
            cur = o_cur;
        uint32_t pcur = __shfl_up(cur, 1);
        if (k == 0)
            pcur = o_cur;
        const bool sw = act && eqp && fi != pcur;
        const uint64_t SW = __ballot(sw), NS = __ballot(act && newseq);
        const uint64_t S = (__ballot(act && brk) | (SW >> 1)) & ACT; /* sub-run starts */
        const bool memb = act && (fi == cur || ((S >> k) & 1));
        const uint64_t MEMB = __ballot(memb);

        /* a switch at lane 0: O is flushed before this chunk and the pair
         * (last hit, lane 0) starts the new O */
        if (SW & 1) {
            close_open();
            if (want_otu && lane == 0)
                hw[4 * (uint64_t)p_at + FD] = p_fb | F_RUN | F_CNT;
            o_cur = rl32(fi, 0);
            o_cnt = 1;
            o_wsum = 0.0f + p_wt;
            o_first = p_pos;
            o_last = p_pos;
            o_span = true;
        }
        /* lanes before the first start continue O */
        const uint32_t fs = S ? lowbit(S) : n;
        if (fs > 0) {
            uint64_t mm = MEMB & bit_range(0, fs);
            o_cnt += (uint32_t)__popcll(mm);
            if (mm)
                o_last = rl32(pos, (uint32_t)hibit(mm));
            while (mm) {
                o_wsum = o_wsum + rlf(wt, lowbit(mm));
                mm &= mm - 1;
            }
        }
        bool o_emitted = false;
        if (fs < n && o_valid) {
            o_emitted = close_open();
            if (fs == 0 && (NS & 1)) /* O's sequence ended in the previous chunk */
                if (lane == 0)
                    call_count[o_seq] = want_calls ? o_ncalls : 0u;
        }

        /* sub-runs that start in this chunk, one per start lane */
        const bool is_start = (S >> k) & 1;
        const uint64_t above = S & ~lanes_le(k);
        const uint32_t e_k = above ? lowbit(above) : n;
        const uint64_t msg = MEMB & bit_range(k, e_k);
        const uint32_t c_seg = (uint32_t)__popcll(msg);
        const int lm = hibit(msg);
        const uint32_t last_pos = __shfl(pos, lm < 0 ? 0 : lm);
        const bool closed = e_k < n;
        const int b_open = hibit(S); /* the sub-run left open at the chunk's end */
        /* the f32 sums, serially, for the sub-runs that can be emitted and the open one */
        uint64_t SUM = __ballot(is_start && closed && (int)c_seg >= prm.min_hits);
        if (b_open >= 0)
            SUM |= 1ull << b_open;
        float ws = 0.0f;
        while (SUM) {
            const uint32_t b = lowbit(SUM);
            SUM &= SUM - 1;
            const uint64_t ab = S & ~lanes_le(b);
            uint64_t mm = MEMB & bit_range(b, ab ? lowbit(ab) : n);
            float acc = 0.0f;
            while (mm) {
                acc = acc + rlf(wt, lowbit(mm));
                mm &= mm - 1;
            }
            if (lane == b)
                ws = acc;
        }
        const uint64_t EMIT = __ballot(is_start && closed && (int)c_seg >= prm.min_hits && ws >= min_wh);
        /* call index: the calls of the lane's sequence before it (O's sequence
         * continues through the lanes before the chunk's first new sequence) */
        const int fsq = hibit(NS & lanes_le(k));
        const uint32_t from = fsq < 0 ? 0u : (uint32_t)fsq;
        const uint32_t idx = (fsq < 0 ? o_ncalls : 0u) + (uint32_t)__popcll(EMIT & bit_range(from, k));
        if (want_calls && ((EMIT >> k) & 1)) {
            kgx_call cl;
            cl.start = pos;
            cl.end = last_pos + (KMER - 1);
            cl.count = (int32_t)c_seg;
            cl.function_index = fi;
            cl.weighted_hits = ws;
            calls[wbase[seq] + idx] = cl;
        }
        /* sequences whose last hit is in this chunk (not its last lane) */
        if (act && k + 1 < n && ((NS >> (k + 1)) & 1))
            call_count[seq] = want_calls ? idx + (uint32_t)((EMIT >> k) & 1) : 0u;
        if (want_otu && act) {
            const int bk = hibit(S & lanes_le(k));
            const bool em = bk >= 0 ? ((EMIT >> bk) & 1) != 0 : o_emitted;
            hw[4 * (uint64_t)at + FD] = fb | F_RUN | (memb ? F_CNT : 0u) | (memb && em ? F_OTU : 0u);
        }

        /* carry */
        if (b_open >= 0) {
            const uint32_t b = (uint32_t)b_open;
            o_valid = true;
            o_seq = rl32(seq, b);
            o_cur = rl32(fi, b);
            o_cnt = rl32(c_seg, b);
            o_wsum = rlf(ws, b);
            o_first = rl32(pos, b);
            o_last = rl32(last_pos, b);
            o_ncalls = rl32(idx, b);
        }
        o_span = true;
        const uint32_t l = n - 1;
        p_pos = rl32(pos, l);
        p_fi = rl32(fi, l);
        p_wt = rlf(wt, l);
        p_fb = rl32(fb, l);
        p_at = rl32(at, l);
        qhead += n;
    };

    /* records of the queued chunk in flight while the previous one is scored */
    uint4 rpend = make_uint4(0, 0, 0, 0);
    uint32_t npend = 0;
    auto issue = [&](uint32_t n_new) { /* entries [qissue, qissue + n_new) */
        wave_lds_sync();
        uint4 r = make_uint4(0, 0, 0, 0);
        if (lane < n_new)
            r = hot[Q.at[(qissue + lane) & (SQ - 1)]];
        if (npend)
            process_chunk(npend, rpend);
        rpend = r;
        npend = n_new;
        qissue += n_new;
        wave_lds_sync();
    };

    /* ---- walk the wave's sequences and their hit-mask words ---- */
    uint32_t sb = NONE; /* Q.wb[j] = wbase[sb + j] */
    uint32_t hb = s_lo; /* lane j: hit count of sequence hb + j */
    uint32_t vhc = 0;
    uint64_t gb = ~0ull; /* Q.mw[j] = hit_mask[gb + j] */
    uint64_t pg = ~0ull, pfull = 0;
    uint32_t ppre = 0;
    auto flush_counts = [&](uint32_t upto) { /* sequences [hb, upto) */
        if (lane < upto - hb && vhc != NONE) {
            hit_count[hb + lane] = vhc;
            if (vhc == 0 || !scoring)
                call_count[hb + lane] = 0;
        }
    };
    for (uint32_t s = s_lo; s < s_hi; s++) {
        if (s - hb > 63) {
            flush_counts(s);
            hb = s;
            vhc = 0;
        }
        if (sb == NONE || s + 1 - sb > 64) {
            wave_lds_sync();
            sb = s;
            Q.wb[lane] = wbase[min(sb + lane, n_seq)];
            if (lane == 0)
                Q.wb[64] = wbase[min(sb + 64, n_seq)];
            wave_lds_sync();
        }
        const uint64_t gw0 = uni64(Q.wb[s - sb]), gw1 = uni64(Q.wb[s + 1 - sb]);
        if (gw1 - gw0 > (uint64_t)RUN_CAP || (only_above && gw1 - gw0 <= only_above)) {
            /* score_long_kernel's / (hybrid) the lane scorer's */
            if (lane == s - hb)
                vhc = NONE;
            continue;
        }
        uint32_t nh = 0;
        if (gw0 < gw1) {
            const uint64_t g0 = gw0 >> 6, g1 = (gw1 - 1) >> 6;
            for (uint64_t g = g0; g <= g1; g++) {
                if (gb == ~0ull || g - gb > 63) {
                    wave_lds_sync();
                    gb = g;
                    Q.mw[lane] = (gb + lane) * 64 < W ? hit_mask[gb + lane] : 0ull;
                    wave_lds_sync();
                }
                const uint64_t full = uni64(Q.mw[g - gb]);
                if (g != pg) { /* hits of g's tile before word g */
                    if (pg != ~0ull && g == pg + 1)
                        ppre = g % J == 0 ? 0u : ppre + (uint32_t)__popcll(pfull);
                    else {
                        ppre = 0;
                        for (uint64_t q = (g / J) * J; q < g; q++)
                            ppre += (uint32_t)__popcll(hit_mask[q]);
                    }
                    pg = g;
                    pfull = full;
                }
                const uint32_t lo = g == g0 ? (uint32_t)(gw0 & 63) : 0u;
                const uint32_t hi = g == g1 ? (uint32_t)((gw1 - 1) & 63) + 1 : 64u;
                const uint64_t bits = full & bit_range(lo, hi);
                if (!bits)
                    continue;
                const uint32_t c = (uint32_t)__popcll(bits);
                nh += c;
                if (!scoring)
                    continue;
                if ((bits >> lane) & 1) {
                    const uint32_t slot = (qtail + lanes_below(bits)) & (SQ - 1);
                    Q.pos[slot] = (uint32_t)(64 * g + lane - gw0);
                    Q.seq[slot] = s;
                    Q.at[slot] = (uint32_t)((g / J) * tile_windows + ppre + lanes_below(full));
                }
                qtail += c;
                if (qtail - qissue >= 64)
                    issue(64);
            }
        }
        if (lane == s - hb)
            vhc = nh;
    }
    flush_counts(s_hi);
    if (!scoring)
        return;
    if (qtail != qissue)
        issue(qtail - qissue);
    if (npend) {
        wave_lds_sync();
        process_chunk(npend, rpend);
    }
    if (o_valid) {
        close_open();
        if (lane == 0)
            call_count[o_seq] = want_calls ? o_ncalls : 0u;
    }
}

/* the sequences past RUN_CAP windows (the wave kernel leaves them): the
 * lane machine, which keeps the reference's 40,000-hit cap */
template <bool PK>
__global__ __launch_bounds__(256) void score_long_kernel(
    uint32_t n_seq, const uint64_t *__restrict__ wbase, const uint64_t *__restrict__ hit_mask,
    uint32_t tile_windows, uint4 *__restrict__ hot, kgx_call *__restrict__ calls,
    uint2 *__restrict__ ranges, uint32_t *__restrict__ hit_count, uint32_t *__restrict__ call_count,
    kgx_params prm, uint32_t want)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n_seq && wbase[s + 1] - wbase[s] > (uint64_t)RUN_CAP)
        score_sequence<PK>(s, wbase, hit_mask, tile_windows, hot, calls, ranges, hit_count, call_count, prm, want);
}

hipError_t launch_score(uint32_t n_seq, uint64_t n_residues, const uint64_t *wbase, const uint32_t *tile_seq,
                        uint64_t max_tiles, const uint64_t *hit_mask, uint32_t tile_windows, uint4 *hot,
                        kgx_call *calls, void *ranges, uint32_t *hit_count, uint32_t *call_count,
                        kgx_params params, uint32_t want, uint32_t hit_format, int variant, uint32_t wave_tiles,
                        const uint32_t *plan_status, hipStream_t stream)
{
    if (n_seq == 0)
        return hipSuccess;
    const bool pk = hit_format == HIT_PACKED16;
    const dim3 lanes((n_seq + 255) / 256);
    /* the wave scorer: order_constraint 0, hit slots in 32 bits */
    const bool wave_ok = !params.order_constraint && max_tiles * tile_windows < (1ull << 32);
    wave_tiles = std::max<uint32_t>(1, wave_tiles);
    const uint64_t waves = std::max<uint64_t>(1, (max_tiles + wave_tiles - 1) / wave_tiles);
    const dim3 wgrid((uint32_t)((waves + 3) / 4));
#define KGX_WAVE(P, ABOVE)                                                                                      \
    hipLaunchKernelGGL(score_wave_kernel<P>, wgrid, dim3(256), 0, stream, n_seq, wbase, tile_seq, hit_mask,     \
                       tile_windows, wave_tiles, hot, calls, hit_count, call_count, params, want, (ABOVE), plan_status)
    if (variant == SCORE_WAVE_ONLY && wave_ok) { /* the caller knows no sequence exceeds RUN_CAP windows */
        if (pk)
            KGX_WAVE(true, 0u);
        else
            KGX_WAVE(false, 0u);
        return hipGetLastError();
    }
    if ((variant == SCORE_WAVE || variant == SCORE_WAVE_ONLY) && wave_ok) { /* every sequence up to RUN_CAP windows */
        if (pk) {
            KGX_WAVE(true, 0u);
            hipLaunchKernelGGL(score_long_kernel<true>, lanes, dim3(256), 0, stream, n_seq, wbase, hit_mask,
                               tile_windows, hot, calls, static_cast<uint2 *>(ranges), hit_count, call_count, params,
                               want);
        } else {
            KGX_WAVE(false, 0u);
            hipLaunchKernelGGL(score_long_kernel<false>, lanes, dim3(256), 0, stream, n_seq, wbase, hit_mask,
                               tile_windows, hot, calls, static_cast<uint2 *>(ranges), hit_count, call_count, params,
                               want);
        }
        return hipGetLastError();
    }
    /* the lane machine; in the hybrid (the default) sequences of (LONG_SEQ,
     * RUN_CAP] windows go to the wave scorer instead: one lane walking a
     * 30k-aa protein's hits would hold the whole stage for milliseconds */
    const bool hybrid = variant == SCORE_HYBRID && wave_ok;
    const uint32_t skip = hybrid ? LONG_SEQ : ~0u;
    /* short sequences (fq fragments: ~16 windows, <1 hit each) take the
     * 2-record batches: fewer registers, more waves to hide the loads of
     * sequences that mostly have no hits */
    const bool small = n_residues < 64ull * n_seq;
    /* KGX_SCORE_GRID_CAP (experiments): at most this many workgroups, each
     * lane walking several sequences, so the scorer holds fewer wave slots
     * beside the next batch's probe */
    static const uint32_t grid_cap = [] {
        const char *e = std::getenv("KGX_SCORE_GRID_CAP");
        return e ? (uint32_t)std::max(0L, std::strtol(e, nullptr, 10)) : 0u;
    }();
    const dim3 sgrid(grid_cap ? std::min<uint32_t>(lanes.x, grid_cap) : lanes.x);
#define KGX_SCORE(P, B)                                                                                          \
    hipLaunchKernelGGL((score_kernel<P, B>), sgrid, dim3(256), 0, stream, n_seq, wbase, hit_mask, tile_windows, hot, \
                       calls, static_cast<uint2 *>(ranges), hit_count, call_count, params, want, skip)
    if (pk && small)
        KGX_SCORE(true, 2);
    else if (pk)
        KGX_SCORE(true, SCORE_BATCH);
    else if (small)
        KGX_SCORE(false, 2);
    else
        KGX_SCORE(false, SCORE_BATCH);
#undef KGX_SCORE
    if (hybrid) {
        if (pk)
            KGX_WAVE(true, LONG_SEQ);
        else
            KGX_WAVE(false, LONG_SEQ);
    }
#undef KGX_WAVE
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* best call: find_best_call (kguts.cc:1008-1199), one lane per sequence     */
/* (best_call_decide, kgx_lstd.h; the sequence's calls are rewritten in its */
/* own stretch of the workspace)                                            */
/* ------------------------------------------------------------------------ */
__global__ __launch_bounds__(256) void best_call_kernel(uint32_t n_seq, const kgx_call *__restrict__ calls,
                                                        const uint64_t *__restrict__ start,
                                                        const uint32_t *__restrict__ count, kgx_call *__restrict__ ws,
                                                        kgx_best_call *__restrict__ out)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n_seq)
        out[s] = best_call_decide(calls + start[s], count[s], ws + start[s]);
}

hipError_t launch_best_calls(uint32_t n_seq, const kgx_call *calls, const uint64_t *start, const uint32_t *count,
                             kgx_call *ws, kgx_best_call *out, hipStream_t stream)
{
    if (n_seq == 0)
        return hipSuccess;
    hipLaunchKernelGGL(best_call_kernel, dim3((n_seq + 255) / 256), dim3(256), 0, stream, n_seq, calls, start,
                       count, ws, out);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* OTU tallies: KmerOtuStats (kguts.h:185-219), one lane per sequence         */
/* ------------------------------------------------------------------------ */

/* otu_map[oI]++ over the hits the scorer flagged KGX_HIT_OTU (the hits
 * process_set_of_hits tallies, kguts.cc:760-768), then finalize(): the map's
 * pairs in key order, std::sort by count, larger first (kguts.h:214-218).
 * Scratch: ws / otus of sequence s start at window_base[s] (a sequence has
 * no more flagged hits than windows). */
constexpr int64_t OTU_LDS = 24; /* flagged hits per lane sorted in LDS (24 x 256 x 4 B = 24 KiB) */

template <bool PK>
__global__ __launch_bounds__(256) void otu_kernel(uint32_t n_seq, const uint64_t *__restrict__ wbase,
                                                  const uint64_t *__restrict__ hit_mask, uint32_t tile_windows,
                                                  const uint4 *__restrict__ hot, const uint4 *__restrict__ cold,
                                                  int32_t *__restrict__ ws, kgx_otu *__restrict__ otus,
                                                  uint32_t *__restrict__ otu_count)
{
    typedef HitFields<PK> HF;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_seq)
        return;
    const uint64_t gw0 = wbase[s], gw1 = wbase[s + 1];
    int32_t *v = ws + gw0;
    int64_t n = 0;
    int32_t vmin = INT32_MAX, vmax = INT32_MIN;
    /* the lane's first OTU_LDS values also in LDS: sorting them there avoids
     * a chain of dependent global loads and stores per compare */
    __shared__ int32_t lv[OTU_LDS][256];
    int32_t *mine = &lv[0][threadIdx.x];
    for_each_run(hit_mask, tile_windows, gw0, gw1, [&](uint64_t at0, uint32_t c, uint32_t, uint64_t, uint32_t) {
        for (uint32_t k = 0; k < c; k++) {
            const uint4 h = hot[at0 + k];
            if (HF::flags(h) & KGX_HIT_OTU) {
                const int32_t x = (int32_t)HF::otu(h, PK ? h : cold[at0 + k]);
                if (n < OTU_LDS)
                    mine[256 * n] = x;
                v[n++] = x;
                vmin = min(vmin, x);
                vmax = max(vmax, x);
            }
        }
    });
    int64_t m;
    kgx_otu *o = otus + gw0;
    if (n == 0) {
        m = 0;
    } else if (vmin == vmax) { /* one OTU: otu_map holds one pair, nothing to sort */
        o[0] = kgx_otu{vmin, (int32_t)n};
        m = 1;
    } else if (n <= OTU_LDS) {
        /* the map's keys in order: any sort of plain ints gives the same
         * array (equal values are indistinguishable); insertion sort in LDS */
        for (int64_t i = 1; i < n; i++) {
            const int32_t x = mine[256 * i];
            int64_t j = i - 1;
            while (j >= 0 && mine[256 * j] > x) {
                mine[256 * (j + 1)] = mine[256 * j];
                j--;
            }
            mine[256 * (j + 1)] = x;
        }
        m = 0;
        for (int64_t i = 0; i < n;) {
            int64_t j = i + 1;
            while (j < n && mine[256 * j] == mine[256 * i])
                j++;
            o[m++] = kgx_otu{mine[256 * i], (int32_t)(j - i)};
            i = j;
        }
        /* finalize()'s std::sort of the pairs, replayed (tie order matters) */
        lstd_sort(o, m, [](const kgx_otu &lhs, const kgx_otu &rhs) { return rhs.count < lhs.count; });
    } else {
        m = otu_finalize(v, n, o);
    }
    otu_count[s] = (uint32_t)m;
}

hipError_t launch_otus(uint32_t n_seq, const uint64_t *wbase, const uint64_t *hit_mask, uint32_t tile_windows,
                       const uint4 *hot, const uint4 *cold, int32_t *ws, kgx_otu *otus, uint32_t *otu_count,
                       uint32_t hit_format, hipStream_t stream)
{
    if (n_seq == 0)
        return hipSuccess;
    if (hit_format == HIT_PACKED16)
        hipLaunchKernelGGL(otu_kernel<true>, dim3((n_seq + 255) / 256), dim3(256), 0, stream, n_seq, wbase, hit_mask,
                           tile_windows, hot, cold, ws, otus, otu_count);
    else
        hipLaunchKernelGGL(otu_kernel<false>, dim3((n_seq + 255) / 256), dim3(256), 0, stream, n_seq, wbase,
                           hit_mask, tile_windows, hot, cold, ws, otus, otu_count);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* gather: tiled hits / sparse calls -> dense CSR, one wave per sequence     */
/* ------------------------------------------------------------------------ */

constexpr uint32_t CS_PER = 4, CS_TILE = 256 * CS_PER;

struct Counts3 {
    const uint32_t *c[3]; /* NULL: an all-zero array */
};
struct Offsets3 {
    uint64_t *o[3];
};

/* sequence s's records, by one wave, to its dense CSR slots (hits from hoff_s,
 * calls from coff_s, OTUs from ooff_s; each read only for the outputs asked) */
template <bool PK>
__device__ __forceinline__ void gather_one(
    uint32_t s, const uint64_t *__restrict__ wbase, const uint64_t *__restrict__ hit_mask,
    uint32_t tile_windows, const uint32_t *__restrict__ call_count, const uint4 *__restrict__ hot,
    const uint4 *__restrict__ cold, const kgx_call *__restrict__ calls, uint64_t hoff_s, uint64_t coff_s,
    kgx_hit *__restrict__ hits_out, kgx_call *__restrict__ calls_out, uint32_t seq_base,
    const uint32_t *__restrict__ otu_count, const kgx_otu *__restrict__ otus, uint64_t ooff_s,
    kgx_otu *__restrict__ otus_out, uint4 *__restrict__ hits16_out, uint32_t *__restrict__ hits12_out)
{
    const uint32_t lane = lane_id();
    const uint64_t gw0 = wbase[s], gw1 = wbase[s + 1];
    if ((hits_out || (PK && (hits16_out || hits12_out))) && gw0 < gw1) {
        const uint32_t J = tile_windows / 64;
        const uint64_t gfirst = gw0 >> 6, glast = (gw1 - 1) >> 6;
        uint64_t done = 0; /* hits of s written so far */
        for (uint64_t gb = gfirst; gb <= glast; gb += 64) {
            /* lane l takes mask word gb + l: its run inside the tile */
            const uint64_t g = gb + lane;
            uint64_t at = 0, bits = 0;
            uint32_t cnt = 0;
            if (g <= glast) {
                const uint64_t tile = g / J;
                uint32_t pre = 0;
                for (uint64_t x = tile * J; x < g; x++)
                    pre += (uint32_t)__popcll(hit_mask[x]);
                const uint64_t full = hit_mask[g];
                const uint32_t lo = g == gfirst ? (uint32_t)(gw0 & 63) : 0u;
                const uint32_t hi = g == glast ? (uint32_t)((gw1 - 1) & 63) + 1 : 64u;
                bits = full & bit_range(lo, hi);
                cnt = (uint32_t)__popcll(bits);
                at = tile * tile_windows + pre + (uint32_t)__popcll(full & bit_range(0, lo));
            }
            /* exclusive prefix of cnt over the wave */
            uint32_t incl = cnt;
            for (uint32_t off = 1; off < 64; off <<= 1) {
                const uint32_t x = __shfl_up(incl, off);
                if (lane >= off)
                    incl += x;
            }
            const uint64_t dst0 = hoff_s + done + (incl - cnt);
            /* a lane's run is read GB records at a time, all in flight before
             * any is stored (a load-store loop would wait on every record) */
            constexpr uint32_t GB = 4;
            if (PK && hits16_out) { /* the records as stored: position = mask bit */
                for (uint32_t i0 = 0; i0 < cnt; i0 += GB) {
                    uint4 h[GB];
#pragma unroll
                    for (uint32_t k = 0; k < GB; k++)
                        if (i0 + k < cnt)
                            h[k] = hot[at + i0 + k];
#pragma unroll
                    for (uint32_t k = 0; k < GB; k++)
                        if (i0 + k < cnt)
                            hits16_out[dst0 + i0 + k] = h[k];
                }
                done += __shfl(incl, 63);
                continue;
            }
            if (PK && hits12_out) { /* the records less the key (the host re-encodes it) */
                for (uint32_t i0 = 0; i0 < cnt; i0 += GB) {
                    uint4 h[GB];
#pragma unroll
                    for (uint32_t k = 0; k < GB; k++)
                        if (i0 + k < cnt)
                            h[k] = hot[at + i0 + k];
#pragma unroll
                    for (uint32_t k = 0; k < GB; k++)
                        if (i0 + k < cnt) {
                            uint32_t *d = hits12_out + 3 * (dst0 + i0 + k);
                            d[0] = h[k].z;      /* function_wt bits */
                            d[1] = h[k].w;      /* avg_from_end | (otu+1) high 12 << 16 | flags << 28 */
                            d[2] = h[k].y >> 3; /* (fI+1) | (otu+1) low 9 << 20: packed lo >> 35 */
                        }
                }
                done += __shfl(incl, 63);
                continue;
            }
            uint4 *dst = reinterpret_cast<uint4 *>(hits_out + dst0);
            const uint32_t pbase = (uint32_t)(64 * g - gw0);
            for (uint32_t i0 = 0; i0 < cnt; i0 += GB) { /* kgx_hit from its record(s) */
                uint4 h[GB], c[GB];
#pragma unroll
                for (uint32_t k = 0; k < GB; k++)
                    if (i0 + k < cnt) {
                        h[k] = hot[at + i0 + k];
                        if (!PK)
                            c[k] = cold[at + i0 + k];
                    }
#pragma unroll
                for (uint32_t k = 0; k < GB; k++) {
                    if (i0 + k >= cnt)
                        break;
                    const uint32_t i = i0 + k;
                    const uint32_t pos = pbase + (uint32_t)__builtin_ctzll(bits);
                    bits &= bits - 1;
                    if (PK) {
                        typedef HitFields<true> HF;
                        const uint64_t key = HF::key(h[k], h[k]);
                        dst[2 * i] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), HF::otu(h[k], h[k]),
                                                HF::avg(h[k]) | HF::flags(h[k]) << 16);
                        dst[2 * i + 1] = make_uint4(HF::fi(h[k]), HF::wt(h[k]), pos, s + seq_base);
                    } else {
                        dst[2 * i] = make_uint4(c[k].x, c[k].y, c[k].z, h[k].x);
                        dst[2 * i + 1] = make_uint4(h[k].y, h[k].z, pos, s + seq_base);
                    }
                }
            }
            done += __shfl(incl, 63);
        }
    }
    if (calls_out) {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(calls + gw0);
        uint32_t *dst = reinterpret_cast<uint32_t *>(calls_out + coff_s);
        const uint32_t n = 5 * call_count[s];
        for (uint32_t i = lane; i < n; i += 64)
            dst[i] = src[i];
    }
    if (otus_out) {
        const kgx_otu *src = otus + gw0;
        kgx_otu *dst = otus_out + ooff_s;
        for (uint32_t i = lane; i < otu_count[s]; i += 64)
            dst[i] = src[i];
    }
}

template <bool PK>
__global__ __launch_bounds__(256) void gather_kernel(
    uint32_t n_seq, const uint64_t *__restrict__ wbase, const uint64_t *__restrict__ hit_mask,
    uint32_t tile_windows, const uint32_t *__restrict__ call_count, const uint4 *__restrict__ hot,
    const uint4 *__restrict__ cold, const kgx_call *__restrict__ calls, const uint64_t *__restrict__ hoff,
    const uint64_t *__restrict__ coff, kgx_hit *__restrict__ hits_out, kgx_call *__restrict__ calls_out,
    uint32_t seq_base, const uint32_t *__restrict__ otu_count, const kgx_otu *__restrict__ otus,
    const uint64_t *__restrict__ ooff, kgx_otu *__restrict__ otus_out, uint4 *__restrict__ hits16_out,
    uint32_t *__restrict__ hits12_out)
{
    const uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= n_seq)
        return;
    const bool want_hits = hits_out || (PK && (hits16_out || hits12_out));
    gather_one<PK>(s, wbase, hit_mask, tile_windows, call_count, hot, cold, calls, want_hits ? hoff[s] : 0,
                   calls_out ? coff[s] : 0, hits_out, calls_out, seq_base, otu_count, otus,
                   otus_out ? ooff[s] : 0, otus_out, hits16_out, hits12_out);
}

/* small batches (<= SMALL_GATHER_SEQ sequences): small_collect and gather in
 * one launch -- every workgroup scans the counts into LDS (workgroup 0 also
 * into the caller's mapped offsets), then its four waves gather sequences
 * 4 b .. 4 b + 3 from those offsets (SMALL_GATHER_BLOCKS workgroups at most,
 * striding); the workgroup that finishes last (a device counter, reset by
 * it) stores the token */
template <bool PK>
__global__ __launch_bounds__(256) void small_gather_kernel(
    uint32_t n, const uint64_t *__restrict__ wbase, const uint64_t *__restrict__ hit_mask, uint32_t tile_windows,
    const uint32_t *__restrict__ hit_count, const uint32_t *__restrict__ call_count, const uint4 *__restrict__ hot,
    const uint4 *__restrict__ cold, const kgx_call *__restrict__ calls, const uint32_t *__restrict__ otu_count,
    const kgx_otu *__restrict__ otus, kgx_hit *__restrict__ hits_out, kgx_call *__restrict__ calls_out,
    kgx_otu *__restrict__ otus_out, Offsets3 off_host, const uint32_t *__restrict__ status,
    const kgx_best_call *__restrict__ best, kgx_best_call *__restrict__ best_host, uint32_t *__restrict__ status_host,
    uint64_t *__restrict__ nwin_host, uint32_t *done_host, uint32_t token, uint32_t *blocks_done)
{
    __shared__ uint64_t lds4[3][4];
    __shared__ uint64_t lo[3][SMALL_GATHER_SEQ + 1];
    __shared__ uint32_t last;
    const uint32_t t = threadIdx.x;
    const bool first = blockIdx.x == 0;
    const uint32_t *cnt[3] = {hit_count, calls_out ? call_count : nullptr, otus_out ? otu_count : nullptr};
    for (int a = 0; a < 3; a++) {
        const uint64_t v = t < n && cnt[a] ? cnt[a][t] : 0;
        uint64_t tot;
        const uint64_t ex = block_scan(v, lds4[a], tot) - v;
        if (t < n) {
            lo[a][t] = ex;
            if (first)
                off_host.o[a][t] = ex;
        }
        if (t == 0) {
            lo[a][n] = tot;
            if (first)
                off_host.o[a][n] = tot;
        }
    }
    if (first && best_host && t < n)
        best_host[t] = best[t];
    if (first && t == 0) {
        status_host[0] = status[0];
        nwin_host[0] = wbase[n];
    }
    __syncthreads();
    for (uint32_t s = blockIdx.x * 4 + (t >> 6); s < n; s += 4 * gridDim.x)
        gather_one<PK>(s, wbase, hit_mask, tile_windows, call_count, hot, cold, calls, lo[0][s], lo[1][s], hits_out,
                       calls_out, 0u, otu_count, otus, lo[2][s], otus_out, nullptr, nullptr);
    /* the batch's last word: every store above, of every workgroup, is
     * visible to the host before the host sees done_host == token (it polls
     * instead of a stream sync) */
    if (done_host) {
        __threadfence_system();
        __syncthreads();
        if (t == 0) {
            last = gridDim.x == 1 || atomicAdd(blocks_done, 1u) == gridDim.x - 1;
            if (last && gridDim.x > 1)
                *blocks_done = 0; /* for the next launch on this stream */
        }
        __syncthreads();
        if (t == 0 && last) {
            __threadfence_system();
            *reinterpret_cast<volatile uint32_t *>(done_host) = token;
        }
    }
}

hipError_t launch_small_gather(uint32_t n, const uint64_t *wbase, const uint64_t *hit_mask, uint32_t tile_windows,
                               const uint32_t *hit_count, const uint32_t *call_count, const uint4 *hot,
                               const uint4 *cold, const kgx_call *calls, const uint32_t *otu_count,
                               const kgx_otu *otus, kgx_hit *hits_out, kgx_call *calls_out, kgx_otu *otus_out,
                               uint64_t *h0, uint64_t *h1, uint64_t *h2, const uint32_t *status,
                               const kgx_best_call *best, kgx_best_call *best_host, uint32_t *status_host,
                               uint64_t *nwin_host, uint32_t *done_host, uint32_t token, uint32_t *blocks_done,
                               uint32_t hit_format, hipStream_t stream)
{
    if (n == 0 || n > SMALL_GATHER_SEQ)
        return hipErrorInvalidValue;
    const Offsets3 off_host = {{h0, h1, h2}};
    /* one wave per sequence (blocks_done NULL: one workgroup) */
    const uint32_t blocks = blocks_done ? std::min<uint32_t>((n + 3) / 4, SMALL_GATHER_BLOCKS) : 1u;
    if (hit_format == HIT_PACKED16)
        hipLaunchKernelGGL(small_gather_kernel<true>, dim3(blocks), dim3(256), 0, stream, n, wbase, hit_mask,
                           tile_windows, hit_count, call_count, hot, cold, calls, otu_count, otus, hits_out, calls_out,
                           otus_out, off_host, status, best, best_host, status_host, nwin_host, done_host, token,
                           blocks_done);
    else
        hipLaunchKernelGGL(small_gather_kernel<false>, dim3(blocks), dim3(256), 0, stream, n, wbase, hit_mask,
                           tile_windows, hit_count, call_count, hot, cold, calls, otu_count, otus, hits_out,
                           calls_out, otus_out, off_host, status, best, best_host, status_host, nwin_host,
                           done_host, token, blocks_done);
    return hipGetLastError();
}

hipError_t launch_gather(uint32_t n_seq, const uint64_t *wbase, const uint64_t *hit_mask,
                         uint32_t tile_windows, const uint32_t *call_count, const uint4 *hot, const uint4 *cold,
                         const kgx_call *calls, const uint64_t *hoff, const uint64_t *coff,
                         kgx_hit *hits_out, kgx_call *calls_out, uint32_t seq_base, uint32_t hit_format,
                         const uint32_t *otu_count, const kgx_otu *otus, const uint64_t *ooff, kgx_otu *otus_out,
                         hipStream_t stream, uint4 *hits16_out, uint32_t *hits12_out)
{
    if (n_seq == 0)
        return hipSuccess;
    if (hit_format == HIT_PACKED16)
        hipLaunchKernelGGL(gather_kernel<true>, dim3((n_seq + 3) / 4), dim3(256), 0, stream, n_seq, wbase,
                           hit_mask, tile_windows, call_count, hot, cold, calls, hoff, coff, hits_out,
                           calls_out, seq_base, otu_count, otus, ooff, otus_out, hits16_out, hits12_out);
    else
        hipLaunchKernelGGL(gather_kernel<false>, dim3((n_seq + 3) / 4), dim3(256), 0, stream, n_seq, wbase,
                           hit_mask, tile_windows, call_count, hot, cold, calls, hoff, coff, hits_out,
                           calls_out, seq_base, otu_count, otus, ooff, otus_out, hits16_out, hits12_out);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* count scan: a chunk's dense CSR offsets from its per-sequence counts, on  */
/* the device (the streamed host path needs no host round trip between the  */
/* scorer and the gather): off[a][i] = sum_{j<i} count[a][j], i in [0, n]   */
/* ------------------------------------------------------------------------ */


__device__ __forceinline__ uint64_t thread_count(const uint32_t *c, uint32_t n, uint32_t i0)
{
    uint64_t v = 0;
    if (c)
        for (uint32_t k = 0; k < CS_PER; k++)
            if (i0 + k < n)
                v += c[i0 + k];
    return v;
}

__global__ __launch_bounds__(256) void count_reduce_kernel(Counts3 cnt, uint32_t n, uint64_t *__restrict__ sums)
{
    __shared__ uint64_t lds4[3][4];
    const uint32_t i0 = blockIdx.x * CS_TILE + threadIdx.x * CS_PER;
    for (int a = 0; a < 3; a++) {
        uint64_t total;
        block_scan(thread_count(cnt.c[a], n, i0), lds4[a], total);
        if (threadIdx.x == 0)
            sums[3 * (uint64_t)blockIdx.x + a] = total;
    }
}

/* exclusive scan of the 3 x groups workgroup sums in place, one workgroup */
__global__ __launch_bounds__(256) void count_sums_scan_kernel(uint64_t *__restrict__ sums, uint32_t groups)
{
    __shared__ uint64_t lds4[3][4];
    uint64_t carry[3] = {0, 0, 0};
    for (uint32_t base = 0; base < groups; base += 256) {
        const uint32_t i = base + threadIdx.x;
        for (int a = 0; a < 3; a++) {
            const uint64_t v = i < groups ? sums[3 * (uint64_t)i + a] : 0;
            uint64_t tot;
            const uint64_t incl = block_scan(v, lds4[a], tot);
            if (i < groups)
                sums[3 * (uint64_t)i + a] = carry[a] + incl - v;
            carry[a] += tot;
        }
        __syncthreads(); /* lds4 is rewritten by the next round */
    }
}

__global__ __launch_bounds__(256) void count_scan_kernel(Counts3 cnt, uint32_t n, const uint64_t *__restrict__ sums,
                                                         Offsets3 off)
{
    __shared__ uint64_t lds4[3][4];
    const uint32_t i0 = blockIdx.x * CS_TILE + threadIdx.x * CS_PER;
    for (int a = 0; a < 3; a++) {
        uint64_t tot;
        const uint64_t mine = thread_count(cnt.c[a], n, i0);
        uint64_t at = sums[3 * (uint64_t)blockIdx.x + a] + block_scan(mine, lds4[a], tot) - mine;
        /* entries [i0, i0 + CS_PER) of the n + 1 offsets */
        for (uint32_t k = 0; k < CS_PER && i0 + k <= n; k++) {
            off.o[a][i0 + k] = at;
            if (cnt.c[a] && i0 + k < n)
                at += cnt.c[a][i0 + k];
        }
    }
}

size_t count_scan_workspace_bytes(uint32_t n)
{
    return (size_t)3 * ((n + 1 + CS_TILE - 1) / CS_TILE) * sizeof(uint64_t);
}

hipError_t launch_count_scan(uint32_t n, const uint32_t *c0, const uint32_t *c1, const uint32_t *c2, uint64_t *o0,
                             uint64_t *o1, uint64_t *o2, void *workspace, hipStream_t stream)
{
    const uint32_t groups = (n + 1 + CS_TILE - 1) / CS_TILE; /* n + 1 offsets */
    Counts3 cnt = {{c0, c1, c2}};
    Offsets3 off = {{o0, o1, o2}};
    uint64_t *sums = static_cast<uint64_t *>(workspace);
    hipLaunchKernelGGL(count_reduce_kernel, dim3(groups), dim3(256), 0, stream, cnt, n, sums);
    hipLaunchKernelGGL(count_sums_scan_kernel, dim3(1), dim3(256), 0, stream, sums, groups);
    hipLaunchKernelGGL(count_scan_kernel, dim3(groups), dim3(256), 0, stream, cnt, n,
                       static_cast<const uint64_t *>(sums), off);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* small batches (one or a few sequences, e.g. the facade's process_aa_seq): */
/* the host plans the batch itself and the device reads it from mapped      */
/* pinned memory, and the counts are scanned and the results land in mapped */
/* memory too, so a batch costs one host wait and no DMA copies             */
/* ------------------------------------------------------------------------ */

/* pieces of mapped pinned host memory -> HBM: one 16-B load per thread over
 * the pieces' concatenation (one PCIe round trip for a small batch) */
__global__ __launch_bounds__(256) void small_upload_kernel(SmallPieces pc)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pc.end16[SMALL_PIECES - 1];
         i += stride) {
        int p = 0;
#pragma unroll
        for (int k = 0; k < SMALL_PIECES - 1; k++)
            p += i >= pc.end16[k];
        const uint64_t j = i - (p ? pc.end16[p - 1] : 0);
        pc.dst[p][j] = pc.src[p][j];
    }
}

hipError_t launch_small_upload(const SmallPieces &pc, hipStream_t stream)
{
    const uint64_t n16 = pc.end16[SMALL_PIECES - 1];
    if (n16 == 0)
        return hipSuccess;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((n16 + 255) / 256, 256);
    hipLaunchKernelGGL(small_upload_kernel, dim3(blocks), dim3(256), 0, stream, pc);
    return hipGetLastError();
}

/* one workgroup: the dense CSR offsets of up to three count arrays, stored in
 * HBM (the gather's) and in mapped host memory (the caller's), plus the plan
 * status word, the window total and the best calls */
__global__ __launch_bounds__(256) void small_collect_kernel(Counts3 cnt, uint32_t n, Offsets3 off, Offsets3 off_host,
                                                            const uint32_t *__restrict__ status,
                                                            const uint64_t *__restrict__ wbase,
                                                            const kgx_best_call *__restrict__ best,
                                                            kgx_best_call *__restrict__ best_host,
                                                            uint32_t *__restrict__ status_host,
                                                            uint64_t *__restrict__ nwin_host)
{
    __shared__ uint64_t lds4[3][4];
    uint64_t carry[3] = {0, 0, 0};
    for (uint32_t base = 0; base <= n; base += CS_TILE) {
        const uint32_t i0 = base + threadIdx.x * CS_PER;
        for (int a = 0; a < 3; a++) {
            uint64_t tot;
            const uint64_t mine = thread_count(cnt.c[a], n, i0);
            uint64_t at = carry[a] + block_scan(mine, lds4[a], tot) - mine;
            for (uint32_t k = 0; k < CS_PER && i0 + k <= n; k++) {
                off.o[a][i0 + k] = at;
                off_host.o[a][i0 + k] = at;
                if (cnt.c[a] && i0 + k < n)
                    at += cnt.c[a][i0 + k];
            }
            carry[a] += tot;
        }
        __syncthreads(); /* lds4 is rewritten by the next round */
    }
    if (best_host)
        for (uint32_t s = threadIdx.x; s < n; s += blockDim.x)
            best_host[s] = best[s];
    if (threadIdx.x == 0) {
        status_host[0] = status[0];
        nwin_host[0] = wbase[n];
    }
}

hipError_t launch_small_collect(uint32_t n, const uint32_t *c0, const uint32_t *c1, const uint32_t *c2, uint64_t *o0,
                                uint64_t *o1, uint64_t *o2, uint64_t *h0, uint64_t *h1, uint64_t *h2,
                                const uint32_t *status, const uint64_t *wbase, const kgx_best_call *best,
                                kgx_best_call *best_host, uint32_t *status_host, uint64_t *nwin_host,
                                hipStream_t stream)
{
    Counts3 cnt = {{c0, c1, c2}};
    Offsets3 off = {{o0, o1, o2}};
    Offsets3 off_host = {{h0, h1, h2}};
    hipLaunchKernelGGL(small_collect_kernel, dim3(1), dim3(256), 0, stream, cnt, n, off, off_host, status, wbase,
                       best, best_host, status_host, nwin_host);
    return hipGetLastError();
}

/* small_collect + best_call_kernel in one launch for batches of up to
 * SMALL_COLLECT_BEST_SEQ sequences: block b owns offsets [256 b, 256 b + 256)
 * (the last one offset n too), sums the counts before its range itself (at
 * most 3 x 8,192 values from L2), scans its own, and decides its sequences'
 * best calls (best_call_decide, into the device array and the mapped host
 * one).  One launch instead of two, and no one-workgroup serial scan. */
__global__ __launch_bounds__(256) void small_collect_best_kernel(
    Counts3 cnt, uint32_t n, Offsets3 off, Offsets3 off_host, const uint32_t *__restrict__ status,
    const uint64_t *__restrict__ wbase, const kgx_call *__restrict__ calls, const uint32_t *__restrict__ call_count,
    kgx_call *__restrict__ ws, kgx_best_call *__restrict__ best, kgx_best_call *__restrict__ best_host,
    uint32_t *__restrict__ status_host, uint64_t *__restrict__ nwin_host)
{
    __shared__ uint64_t lds_pre[3][4], lds_own[3][4];
    const uint32_t t = threadIdx.x, s0 = blockIdx.x * 256u, i = s0 + t;
    for (int a = 0; a < 3; a++) {
        uint64_t v = 0, before = 0, tot = 0;
        if (cnt.c[a]) {
#pragma unroll 8
            for (uint32_t j = t; j < s0; j += 256)
                v += cnt.c[a][j];
        }
        (void)block_scan(v, lds_pre[a], before);
        const uint64_t mine = cnt.c[a] && i < n ? cnt.c[a][i] : 0;
        const uint64_t at = before + block_scan(mine, lds_own[a], tot) - mine;
        if (i <= n) {
            off.o[a][i] = at;
            off_host.o[a][i] = at;
        }
    }
    if (i < n) {
        const uint64_t w = wbase[i];
        const kgx_best_call b = best_call_decide(calls + w, call_count[i], ws + w);
        best[i] = b;
        if (best_host)
            best_host[i] = b;
    }
    if (blockIdx.x == 0 && t == 0) {
        status_host[0] = status[0];
        nwin_host[0] = wbase[n];
    }
}

hipError_t launch_small_collect_best(uint32_t n, const uint32_t *c0, const uint32_t *c1, const uint32_t *c2,
                                     uint64_t *o0, uint64_t *o1, uint64_t *o2, uint64_t *h0, uint64_t *h1,
                                     uint64_t *h2, const uint32_t *status, const uint64_t *wbase,
                                     const kgx_call *calls, const uint32_t *call_count, kgx_call *ws,
                                     kgx_best_call *best, kgx_best_call *best_host, uint32_t *status_host,
                                     uint64_t *nwin_host, hipStream_t stream)
{
    if (n > SMALL_COLLECT_BEST_SEQ)
        return hipErrorInvalidValue;
    Counts3 cnt = {{c0, c1, c2}};
    Offsets3 off = {{o0, o1, o2}};
    Offsets3 off_host = {{h0, h1, h2}};
    hipLaunchKernelGGL(small_collect_best_kernel, dim3(n / 256 + 1), dim3(256), 0, stream, cnt, n, off, off_host,
                       status, wbase, calls, call_count, ws, best, best_host, status_host, nwin_host);
    return hipGetLastError();
}

/* min(*count, cap) elements of elem_bytes each, src -> dst: the size comes
 * from the device (a chunk's scanned total), the room from the host.  The
 * bytes move as 16-B stores (one 1-KB run per wave instruction over PCIe),
 * the last < 16 as 4-B stores; both ends 16-B aligned. */
__global__ __launch_bounds__(256) void copy_counted_kernel(uint4 *__restrict__ dst, const uint4 *__restrict__ src,
                                                           const uint64_t *__restrict__ count, uint64_t cap,
                                                           uint32_t elem_bytes)
{
    const uint64_t bytes = (*count < cap ? *count : cap) * elem_bytes;
    const uint64_t n16 = bytes / 16;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t i = tid; i < n16; i += stride)
        dst[i] = src[i];
    const uint32_t tail = (uint32_t)(bytes - 16 * n16) / 4; /* elem_bytes is a multiple of 4 */
    if (tid < tail)
        reinterpret_cast<uint32_t *>(dst + n16)[tid] = reinterpret_cast<const uint32_t *>(src + n16)[tid];
}

hipError_t launch_copy_counted(void *dst, const void *src, const uint64_t *count, uint64_t cap,
                               uint32_t elem_bytes, int blocks, hipStream_t stream)
{
    if (cap == 0)
        return hipSuccess;
    if (elem_bytes % 4 != 0 || (uintptr_t)dst % 16 != 0 || (uintptr_t)src % 16 != 0)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(copy_counted_kernel, dim3(blocks), dim3(256), 0, stream, static_cast<uint4 *>(dst),
                       static_cast<const uint4 *>(src), count, cap, elem_bytes);
    return hipGetLastError();
}

/* any NUL among bytes [skip, n) of d -> *flag = 1 (a store into mapped host
 * memory).  Residues the device reads straight from the caller's pinned
 * buffer are not NUL-cut on the host (gather_hits' strlen bound, kguts.cc:792),
 * so the host path checks them here and reruns a batch that has one. */
__global__ __launch_bounds__(256) void nul_scan_kernel(const uint4 *__restrict__ d, uint64_t skip, uint64_t n,
                                                       uint32_t *flag)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n16 = n / 16;
    bool nul = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const uint4 v = d[i];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        if (16 * i >= skip) {
            for (int j = 0; j < 4; j++)
                nul |= ((w[j] - 0x01010101u) & ~w[j] & 0x80808080u) != 0;
        } else { /* the first word: bytes before skip are not the batch's */
            for (int b = 0; b < 16; b++)
                nul |= 16 * i + b >= skip && ((w[b / 4] >> (8 * (b % 4))) & 0xFFu) == 0;
        }
    }
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid < n - 16 * n16 && 16 * n16 + tid >= skip)
        nul |= reinterpret_cast<const uint8_t *>(d)[16 * n16 + tid] == 0;
    if (__ballot(nul) && lane_id() == 0)
        __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_nul_scan(const uint8_t *d, uint64_t skip, uint64_t n, uint32_t *flag_mapped, hipStream_t stream)
{
    if (n <= skip)
        return hipSuccess;
    if ((uintptr_t)d % 16 != 0)
        return hipErrorInvalidValue;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((n / 16 + 255) / 256 + 1, 1024);
    hipLaunchKernelGGL(nul_scan_kernel, dim3(blocks), dim3(256), 0, stream, reinterpret_cast<const uint4 *>(d), skip,
                       n, flag_mapped);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* copy to mapped pinned host memory: the device's own stores stream the     */
/* results over PCIe (one contiguous 1-KB run per wave instruction), so the */
/* D2H needs no DMA-engine slot and overlaps other streams' H2D copies      */
/* ------------------------------------------------------------------------ */

__global__ __launch_bounds__(256) void copy16_kernel(uint4 *__restrict__ dst, const uint4 *__restrict__ src,
                                                     uint64_t n)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        dst[i] = src[i];
}

__global__ __launch_bounds__(256) void copy4_kernel(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src,
                                                    uint64_t n)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        dst[i] = src[i];
}

hipError_t launch_copy_to_host(void *dst, const void *src, uint64_t bytes, int copy_blocks, hipStream_t stream)
{
    if (bytes == 0)
        return hipSuccess;
    const bool v16 = ((uintptr_t)dst % 16 == 0) && ((uintptr_t)src % 16 == 0) && bytes % 16 == 0;
    if (!v16 && (((uintptr_t)dst | (uintptr_t)src | bytes) % 4 != 0))
        return hipErrorInvalidValue;
    const uint64_t n = v16 ? bytes / 16 : bytes / 4;
    /* PCIe writes are posted: a few waves keep the link busy, and a full
     * grid would starve the kernels of the other stream (latency-bound
     * scorer, plan) that this copy is meant to run beside */
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, (uint64_t)copy_blocks);
    if (v16)
        hipLaunchKernelGGL(copy16_kernel, dim3(blocks), dim3(256), 0, stream, static_cast<uint4 *>(dst),
                           static_cast<const uint4 *>(src), n);
    else
        hipLaunchKernelGGL(copy4_kernel, dim3(blocks), dim3(256), 0, stream, static_cast<uint32_t *>(dst),
                           static_cast<const uint32_t *>(src), n);
    return hipGetLastError();
}

/* several spans in one launch (blockIdx.y = span): a collect's counts, totals
 * and best calls cost one kernel instead of five back-to-back ones */
__global__ __launch_bounds__(256) void copy_spans_kernel(CopySpans sp)
{
    const uint32_t k = blockIdx.y;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sp.v16[k]) {
        uint4 *d = static_cast<uint4 *>(sp.dst[k]);
        const uint4 *s = static_cast<const uint4 *>(sp.src[k]);
        for (uint64_t i = i0; i < sp.n[k]; i += stride)
            d[i] = s[i];
    } else {
        uint32_t *d = static_cast<uint32_t *>(sp.dst[k]);
        const uint32_t *s = static_cast<const uint32_t *>(sp.src[k]);
        for (uint64_t i = i0; i < sp.n[k]; i += stride)
            d[i] = s[i];
    }
}

hipError_t launch_copy_spans(CopySpans sp, int copy_blocks, hipStream_t stream)
{
    if (sp.count == 0)
        return hipSuccess;
    if (sp.count > CopySpans::kMax)
        return hipErrorInvalidValue;
    uint64_t most = 1;
    for (int k = 0; k < sp.count; k++) {
        const uintptr_t d = reinterpret_cast<uintptr_t>(sp.dst[k]), s = reinterpret_cast<uintptr_t>(sp.src[k]);
        const uint64_t bytes = sp.n[k];
        sp.v16[k] = d % 16 == 0 && s % 16 == 0 && bytes % 16 == 0;
        if (!sp.v16[k] && ((d | s | bytes) % 4 != 0))
            return hipErrorInvalidValue;
        sp.n[k] = sp.v16[k] ? bytes / 16 : bytes / 4;
        most = std::max(most, sp.n[k]);
    }
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((most + 255) / 256, (uint64_t)copy_blocks);
    hipLaunchKernelGGL(copy_spans_kernel, dim3(blocks, (uint32_t)sp.count), dim3(256), 0, stream, sp);
    return hipGetLastError();
}

}  // namespace kgx
