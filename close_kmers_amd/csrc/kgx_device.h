/*
 * kgx_device.h -- device helpers shared by the gfx950 kernels.
 */
#ifndef KGX_DEVICE_H
#define KGX_DEVICE_H

#include "kgx_internal.h"

namespace kgx {

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

/* x % n for x < 2^35, n >= 1, m = floor((2^64-1)/n): the quotient estimate
 * is exact or one short, so one conditional subtraction finishes it */
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

/* number of set bits of `mask` below this lane */
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint64_t windows_of(uint64_t len) { return len >= 9 ? len - 8 : 0; }

/* bits [lo, hi) of a 64-bit word, 0 <= lo <= hi <= 64 */
__device__ __forceinline__ uint64_t bit_range(uint32_t lo, uint32_t hi)
{
    const uint64_t upto_hi = hi >= 64 ? ~0ull : ((1ull << hi) - 1);
    const uint64_t below_lo = lo >= 64 ? ~0ull : ((1ull << lo) - 1);
    return upto_hi & ~below_lo;
}

}  // namespace kgx

#endif
