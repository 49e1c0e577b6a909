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

/* NCBI genetic code 11 (trans_table.cc:8-15) indexed e1*16 + e2*4 + e3 with
 * A=0 C=1 G=2 T/U=3 (trans_table.h:45-83); tests/test_fq_host.py re-derives
 * it from the table text */
__device__ __forceinline__ char code11_aa(uint32_t e)
{
    const char *t = "KNKNTTTTRSRSIIMIQHQHPPPPRRRRLLLLEDEDAAAAGGGGVVVV*Y*YSSSS*CWCLFLF";
    return t[e & 63u];
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

/* wave-level helpers of the wave-parallel scorers */
__device__ __forceinline__ uint64_t lanes_le(uint32_t k) { return k >= 63 ? ~0ull : ((2ull << k) - 1); }
__device__ __forceinline__ int hibit(uint64_t m) { return m ? 63 - (int)__clzll((long long)m) : -1; }
__device__ __forceinline__ uint32_t lowbit(uint64_t m) { return (uint32_t)__builtin_ctzll(m); }
__device__ __forceinline__ uint32_t rl32(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float rlf(float v, uint32_t l)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
/* acc + w of each lane in mm, lane order (an f32 sum taken hit by hit).  Past
 * a few lanes, every lane is added with non-members as -0.0f (x + -0.0f == x
 * bit for bit), so the 64 lane reads do not wait on the chain of adds */
__device__ __forceinline__ float sum_lanes_in_order(float acc, float w, uint64_t mm)
{
    if (__popcll(mm) < 12) {
        while (mm) {
            acc = acc + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), (int)__builtin_ctzll(mm)));
            mm &= mm - 1;
        }
        return acc;
    }
    /* each lane masks its own weight first, so a step is one lane read and
     * one add (no scalar select between them) */
    const float wm = ((mm >> lane_id()) & 1ull) ? w : -0.0f;
#pragma unroll
    for (int l = 0; l < 64; l++)
        acc = acc + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wm), l));
    return acc;
}
/* (the builtins return int: widen through uint32_t, or a low half >= 2^31
 * sign-extends into the high half) */
__device__ __forceinline__ uint64_t uni64(uint64_t v)
{
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32;
}
/* v of lane (lane ^ j), j < 64, every lane active: one DPP move where one
 * does it -- j 1 and 2 quad permutes, j 8 a rotation by 8 within the 16-lane
 * row -- and ds_bpermute (an LDS round trip) otherwise */
__device__ __forceinline__ int32_t xor_lane(int32_t v, uint32_t j)
{
    switch (j) {
    case 1:
        return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false); /* quad_perm [1,0,3,2] */
    case 2:
        return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false); /* quad_perm [2,3,0,1] */
    case 8:
        return __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false); /* row_ror:8 */
    default:
        return __shfl_xor(v, (int)j);
    }
}
/* v of lane s (0-3) of this lane's quad: one DPP quad_perm move (s a
 * constant once unrolled) */
__device__ __forceinline__ uint32_t quad_bcast32(uint32_t v, uint32_t s)
{
    switch (s & 3u) {
    case 0:
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x00, 0xF, 0xF, false); /* [0,0,0,0] */
    case 1:
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x55, 0xF, 0xF, false); /* [1,1,1,1] */
    case 2:
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xAA, 0xF, 0xF, false); /* [2,2,2,2] */
    default:
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xFF, 0xF, 0xF, false); /* [3,3,3,3] */
    }
}
__device__ __forceinline__ uint64_t quad_bcast64(uint64_t v, uint32_t s)
{
    return (uint64_t)quad_bcast32((uint32_t)(v >> 32), s) << 32 | quad_bcast32((uint32_t)v, s);
}
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* ---- hit records (kgx_internal.h: HIT_PLANES / HIT_PACKED16) ---- */

/* the fields of one hit record (hot = plane 0 / the packed record,
 * cold = plane 1, unused for PACKED16) */
template <bool PK> struct HitFields {
    __device__ __forceinline__ static uint32_t avg(const uint4 &h) { return PK ? (h.w & 0xFFFFu) : (h.x & 0xFFFFu); }
    __device__ __forceinline__ static uint32_t fi(const uint4 &h) { return PK ? ((h.y >> 3) & 0xFFFFFu) - 1u : h.y; }
    __device__ __forceinline__ static uint32_t wt(const uint4 &h) { return h.z; }
    /* the dword that carries the flags, its flag-free value, the flag shift */
    static constexpr int FLAG_DWORD = PK ? 3 : 0;
    static constexpr int FLAG_SHIFT = PK ? 28 : 16;
    __device__ __forceinline__ static uint32_t flag_base(const uint4 &h) { return PK ? (h.w & 0x0FFFFFFFu) : (h.x & 0xFFFFu); }
    __device__ __forceinline__ static uint32_t flags(const uint4 &h) { return PK ? (h.w >> 28) & 7u : (h.x >> 16) & 0xFFFFu; }
    __device__ __forceinline__ static uint64_t key(const uint4 &h, const uint4 &c)
    {
        return PK ? (((uint64_t)h.y << 32 | h.x) & PACK_KEY_MASK) : ((uint64_t)c.y << 32 | c.x);
    }
    __device__ __forceinline__ static uint32_t otu(const uint4 &h, const uint4 &c)
    {
        return PK ? (((h.y >> 23) & 0x1FFu) | (((h.w >> 16) & 0xFFFu) << 9)) - 1u : c.z;
    }
};

/* the window (global index) of hit i of `tile`: the i-th set bit of the
 * tile's J mask words */
__device__ __forceinline__ uint64_t hit_window(const uint64_t *__restrict__ mask, uint64_t tile, uint32_t J,
                                               uint32_t i)
{
    for (uint32_t j = 0; j < J; j++) {
        uint64_t m = mask[tile * J + j];
        const uint32_t pc = (uint32_t)__popcll(m);
        if (i < pc) {
            for (; i; i--)
                m &= m - 1;
            return 64 * (tile * J + j) + (uint64_t)__builtin_ctzll(m);
        }
        i -= pc;
    }
    return ~0ull; /* not reached for i < the tile's hit count */
}

/* the sequence owning global window g, walking on from the tile's first */
__device__ __forceinline__ uint32_t window_seq(const uint64_t *__restrict__ wbase, const uint32_t *__restrict__ tile_seq,
                                               uint64_t tile, uint64_t g)
{
    uint32_t s = tile_seq[tile];
    while (wbase[s + 1] <= g)
        s++;
    return s;
}

}  // namespace kgx

#endif
