/*
 * kgx_fq.hip -- the fq path's read -> protein fragments step on the device.
 *
 * For every read and frame 1, 2, 3, -1, -2, -3 (DNASequence::
 * get_possible_proteins, dna_seq.cc:9-47): translate with genetic code 11
 * (TranslationTable::translate, trans_table.cc:65-84; any base outside
 * ACGTU/acgtu makes its codon 'X'; the reverse strand is the complement of
 * dna_seq.h:28-111 read backwards, frame -k starting at offset k-1), split at
 * '*' (boost::split, token_compress_on) and keep the fragments longer than
 * 10 residues (fq_process_request.cc:333).  Output: the fragments as a
 * batch of protein sequences, in (read, frame, position) order -- the order
 * the handler visits them -- with their read index and frame.
 *
 * With fq_residues 0 the emit is fq_desc_lane_kernel instead: per fragment
 * an anchor into the bases and no residues; the probe then translates each
 * window's codons itself (launch_probe_dna), so the residues never go
 * through HBM.
 *
 * Launches: count (one wave per read: fragments and residues of the six
 * frames; per workgroup of 64 reads their sums), a scan of the sums
 * (hipcub), emit (the same waves translate again and write each fragment's
 * offset, read, frame and first codon, and the residues, at the scanned
 * bases).  The output buffers are sized by the bound of 2 residues per base,
 * so nothing waits for the host in between.  A single pass -- translate once,
 * keep the residues in LDS, place each tile by a decoupled look-back over
 * the earlier tiles' totals -- measured slower (2.8-3.4 ms per 1M reads vs
 * 1.2 ms): the tiles of a launch finish translating at about the same time
 * and each then waits on a look-back chain of device-scope flag reads.
 */
#include <hipcub/hipcub.hpp>

#include "kgx_device.h"
#include "kgx_rt.h"

using namespace kgx;

namespace {

constexpr uint32_t MIN_FRAGMENT = 11; /* prot.length() > 10 */

/* NCBI table 11 (trans_table.cc:8-15) re-indexed e1*16 + e2*4 + e3 with
 * A=0 C=1 G=2 T=3 (trans_table.h:45-83); [64] = 'X' for any codon with a base
 * outside ACGTU.  tests/test_fq_host.py re-derives it from the table text. */
__constant__ char kCode11[66] = "KNKNTTTTRSRSIIMIQHQHPPPPRRRRLLLLEDEDAAAAGGGGVVVV*Y*YSSSS*CWCLFLFX";

/* TranslationTable::encode_char (trans_table.h:45-68) */
__device__ __forceinline__ uint32_t base_class(uint8_t c)
{
    switch (c | 0x20) {
    case 'a': return 0;
    case 'c': return 1;
    case 'g': return 2;
    case 't':
    case 'u': return 3;
    default: return 4;
    }
}

/* frame f's k-th residue of the read [b, b+len), from global memory: the
 * serial path of reads whose frames exceed 64 codons */
struct FrameReader {
    const uint8_t *b;
    uint64_t len;
    int frame;
    __device__ uint64_t n_codons() const
    {
        const uint64_t off = (uint64_t)(frame < 0 ? -frame : frame) - 1;
        return len >= off ? (len - off) / 3 : 0;
    }
    __device__ uint32_t cls(uint64_t i) const /* class of base i of the frame's strand */
    {
        if (frame > 0)
            return base_class(b[i]);
        const uint32_t c = base_class(b[len - 1 - i]);
        return c < 4 ? 3 - c : 4; /* complement: a<->t, c<->g; others stay outside ACGTU */
    }
    __device__ char aa(uint64_t k) const
    {
        const uint64_t i = (uint64_t)(frame < 0 ? -frame : frame) - 1 + 3 * k;
        const uint32_t e1 = cls(i), e2 = cls(i + 1), e3 = cls(i + 2);
        return (e1 < 4 && e2 < 4 && e3 < 4) ? kCode11[e1 * 16 + e2 * 4 + e3] : kCode11[64];
    }
};

__device__ __forceinline__ int frame_of(uint32_t f) { return f < 3 ? (int)f + 1 : -(int)(f - 2); }

/* serial walk of one frame: (fragments, residues); emit when out_res != null */
__device__ void frame_serial(const FrameReader &fr, uint32_t r, uint64_t fi, uint64_t ri, uint32_t &frags,
                             uint64_t &res, uint8_t *out_res, uint64_t *out_off, uint32_t *out_read,
                             int8_t *out_frame, uint32_t *out_start)
{
    const uint64_t nc = fr.n_codons();
    uint64_t run = 0, start = 0;
    frags = 0;
    res = 0;
    for (uint64_t k = 0; k <= nc; k++) {
        if (k == nc || fr.aa(k) == '*') {
            if (run >= MIN_FRAGMENT) {
                if (out_res) {
                    out_off[fi + frags] = ri + res;
                    out_read[fi + frags] = r;
                    out_frame[fi + frags] = (int8_t)fr.frame;
                    out_start[fi + frags] = (uint32_t)start;
                    for (uint64_t j = 0; j < run; j++)
                        out_res[ri + res + j] = (uint8_t)fr.aa(start + j);
                }
                frags++;
                res += run;
            }
            run = 0;
            start = k + 1;
        } else {
            run++;
        }
    }
}

/*
 * Short reads (every frame <= 64 codons: up to 194 bases) take the wave path:
 * one wave per read, lane k = codon k of a frame.
 *
 *  - staging: each lane loads one aligned dword of the read (4 bases) and
 *    turns it into 4 nibbles, bits 0-1 = base class (A0 C1 G2 T/U3, by
 *    arithmetic on the ASCII code), bit 2 = not in ACGTU; the wave's nibble
 *    string sits in LDS (16 bits per lane, 8 bases per dword);
 *  - a codon is 12 bits of that string (one funnel shift of two dwords);
 *    its table index is a few shifts (the reverse strand complements with
 *    xor 3 and reverses the three fields), the residue one LDS byte read;
 *  - a frame's stops are one ballot; the residues kept (runs of >= 11 codons
 *    between stops, fq_process_request.cc:333) and the fragment starts are
 *    computed on that wave-uniform mask with scalar shifts and ands; each
 *    lane places its residue with a masked bit count.
 */
constexpr uint32_t WAVES_PER_WG = 4;
constexpr uint64_t SHORT_READ = 3 * 64 + 2;
constexpr uint32_t FQ_READS_PER_WAVE = 16;
constexpr uint32_t FQ_TILE = WAVES_PER_WG * FQ_READS_PER_WAVE; /* reads per workgroup */
constexpr uint32_t NIB_WORDS = 34; /* 64 lanes x 4 nibbles + a funnel-shift pad (a short read needs <= 26) */

/* 4 bases (the bytes of w) -> 4 nibbles, base j at bits 4j */
__device__ __forceinline__ uint32_t nibbles4(uint32_t w)
{
    uint32_t out = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t b = ((w >> (8 * j)) & 0xFFu) | 0x20u;
        const uint32_t cls = ((b >> 1) ^ (b >> 2)) & 3u;     /* a 0, c 1, g 2, t/u 3 */
        const uint32_t d = b - 0x60u;                        /* a=1 c=3 g=7 t=20 u=21 */
        const uint32_t ok = d < 32u ? (0x30008Au >> d) & 1u : 0u;
        out |= (cls | ((ok ^ 1u) << 2)) << (4 * j);
    }
    return out;
}

/* the read's bytes as the dword this lane stages (0 past the read), and the
 * nibble position of base 0 (the read's offset in its first dword) */
__device__ __forceinline__ uint32_t load_read_dword(const uint8_t *b, uint64_t len, uint32_t lane, uint32_t &mis)
{
    mis = (uint32_t)(reinterpret_cast<uintptr_t>(b) & 3);
    const uint32_t words = (uint32_t)((mis + len + 3) / 4);
    /* pointer arithmetic, not an integer round trip: the compiler keeps the
     * global address space (a flat load would also count against the LDS
     * wait counter and serialise the staging loads behind LDS operations) */
    return lane < words && len ? reinterpret_cast<const uint32_t *>(b - mis)[lane] : 0u;
}

/* a wave-uniform value the compiler cannot prove uniform (a shuffle
 * result), moved to scalar registers: what depends on it -- frame lengths,
 * stop masks, run masks -- then runs on the scalar unit */
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v)
{
    /* the builtin returns int: widen through uint32_t (a low half >= 2^31
     * would otherwise sign-extend into the high half) */
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32;
}

/* the wave's short reads -> their nibble strings in LDS (slot j = read j).
 * my_off: lane i <= n holds read i's start offset.  Every read's dword load
 * is issued before the first is converted: a wave keeps 16 loads in flight
 * instead of waiting out one memory latency per read. */
__device__ __forceinline__ void stage_wave_reads(uint32_t (*slots)[NIB_WORDS], const uint8_t *bases, uint64_t my_off,
                                                 uint32_t n, uint32_t lane)
{
    uint32_t v[FQ_READS_PER_WAVE];
#pragma unroll
    for (uint32_t j = 0; j < FQ_READS_PER_WAVE; j++) {
        const uint64_t ob = uniform_u64(__shfl(my_off, (int)j)), oe = uniform_u64(__shfl(my_off, (int)j + 1));
        uint32_t mis;
        v[j] = j < n && oe - ob <= SHORT_READ ? load_read_dword(bases + ob, oe - ob, lane, mis) : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < FQ_READS_PER_WAVE; j++) {
        uint16_t *s16 = reinterpret_cast<uint16_t *>(slots[j]);
        s16[lane] = (uint16_t)nibbles4(v[j]);
        if (lane < 2 * (NIB_WORDS - 32)) /* pad beyond 64 lanes' halves */
            s16[64 + lane] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* nibble position of a read's base 0 in its staged string */
__device__ __forceinline__ uint32_t read_mis(const uint8_t *b) { return (uint32_t)(reinterpret_cast<uintptr_t>(b) & 3); }

/* all six frames (f 0-2: +1..+3, 3-5: -1..-3) of a staged short read: this
 * lane's residue of each ('*' past the frame) and each frame's stop mask
 * (codons past the frame count as stops).  Straight-line code: the twelve
 * LDS dword reads of the six codons go out together, then the six table
 * reads, so a read costs two LDS latencies instead of twelve. */
__device__ __forceinline__ void translate6(const uint32_t *W, const char *code, uint32_t mis, uint32_t len,
                                           uint32_t lane, char aa[6], uint64_t stops[6])
{
    uint32_t p[6], nc[6], lo[6], hi[6], at[6];
#pragma unroll
    for (uint32_t f = 0; f < 6; f++) {
        const uint32_t off = f < 3 ? f : f - 3;
        nc[f] = len >= off ? (len - off) / 3 : 0;
        /* first nibble of the codon's three bases, in ascending base order
         * (lanes past the frame read base 0: harmless, their residue is '*') */
        p[f] = mis + (lane < nc[f] ? (f < 3 ? off + 3 * lane : len - 3 - off - 3 * lane) : 0u);
    }
#pragma unroll
    for (uint32_t f = 0; f < 6; f++) {
        lo[f] = W[p[f] >> 3];
        hi[f] = W[(p[f] >> 3) + 1];
    }
#pragma unroll
    for (uint32_t f = 0; f < 6; f++) {
        const uint32_t x = __builtin_amdgcn_alignbit(hi[f], lo[f], (p[f] & 7u) * 4u);
        const uint32_t idx = f < 3 ? (((x & 3u) << 4) | ((x >> 2) & 0xCu) | ((x >> 8) & 3u))
                                   : ((((x >> 4) & 0x30u) | ((x >> 2) & 0xCu) | (x & 3u)) ^ 0x3Fu);
        at[f] = (x & 0x444u) ? 64u : idx;
    }
#pragma unroll
    for (uint32_t f = 0; f < 6; f++)
        aa[f] = code[at[f]];
    /* lanes past a frame read some codon: the beyond-frame mask covers them
     * (their residue is never stored, it is not in a kept run) */
#pragma unroll
    for (uint32_t f = 0; f < 6; f++)
        stops[f] = __ballot(aa[f] == '*') | (nc[f] >= 64 ? 0ull : ~0ull << nc[f]);
}

/* codons in runs of >= 11 between stops (S: the wave-uniform stop mask;
 * bits past 63 are stops), on the mask itself: scalar shifts and ands.
 * (Per-lane bit scans of S and a ballot moved the work to the vector units
 * and measured no faster: 511 vs 493 us per 1M reads for the count pass.) */
__device__ __forceinline__ uint64_t kept_runs(uint64_t S)
{
    const uint64_t Z = ~S;
    const uint64_t a1 = Z & (Z >> 1);                 /* bit p: p..p+1 are codons */
    const uint64_t a2 = a1 & (a1 >> 2);               /* p..p+3 */
    const uint64_t a3 = a2 & (a2 >> 4);               /* p..p+7 */
    const uint64_t w = a3 & (a1 >> 8) & (Z >> 10);    /* p..p+10: a run of 11 starts at p */
    uint64_t d = w | (w << 1);
    d |= d << 2;
    d |= d << 4;                                      /* covered by a window starting p-7..p */
    return d | (d << 3);                              /* p-10..p */
}

__device__ __forceinline__ uint32_t popc_below(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v)
{
    for (uint32_t o = 32; o; o >>= 1)
        v += __shfl_xor(v, o);
    return v;
}

/* per-workgroup LDS: the code table and the nibble strings of every read */
struct FqLds {
    char code[68];
    uint32_t nib[WAVES_PER_WG][FQ_READS_PER_WAVE][NIB_WORDS];
};

__device__ __forceinline__ void fq_lds_init(FqLds &t)
{
    if (threadIdx.x < 65)
        t.code[threadIdx.x] = kCode11[threadIdx.x];
    __syncthreads();
}

/* one read's fragments and residues (all frames), uniform over the wave */
__device__ __forceinline__ void count_short(const uint32_t *W, const char *code, uint32_t mis, uint32_t len,
                                            uint32_t lane, uint32_t &nf, uint32_t &nr)
{
    nf = nr = 0;
    char aa[6];
    uint64_t stops[6];
    translate6(W, code, mis, len, lane, aa, stops);
#pragma unroll
    for (uint32_t f = 0; f < 6; f++) {
        const uint64_t kept = kept_runs(stops[f]);
        nf += (uint32_t)__popcll(kept & ~(kept << 1));
        nr += (uint32_t)__popcll(kept);
    }
}

/* 1. per read: fragments and residues; per workgroup: their sums */
__global__ __launch_bounds__(256) void fq_count_kernel(const uint8_t *bases, const uint64_t *read_off,
                                                       uint32_t n_reads, uint2 *read_counts, ulonglong2 *tile_sum)
{
    __shared__ FqLds t;
    __shared__ uint64_t sums[2][WAVES_PER_WG];
    fq_lds_init(t);
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint64_t r0 = (uint64_t)blockIdx.x * FQ_TILE + w * FQ_READS_PER_WAVE;
    const uint32_t n = (uint32_t)(r0 < n_reads ? std::min<uint64_t>(FQ_READS_PER_WAVE, n_reads - r0) : 0);
    const uint64_t my_off = n && lane <= n ? read_off[r0 + lane] : 0;
    uint64_t wf = 0, wr = 0;
    stage_wave_reads(t.nib[w], bases, my_off, n, lane);
    for (uint32_t j = 0; j < n; j++) {
        const uint64_t ob = uniform_u64(__shfl(my_off, (int)j)), oe = uniform_u64(__shfl(my_off, (int)j + 1));
        const uint64_t len = oe - ob;
        uint32_t nf, nr;
        if (len <= SHORT_READ) {
            count_short(t.nib[w][j], t.code, read_mis(bases + ob), (uint32_t)len, lane, nf, nr);
        } else {
            uint32_t frags = 0;
            uint64_t res = 0;
            if (lane < 6)
                frame_serial(FrameReader{bases + ob, len, frame_of(lane)}, 0, 0, 0, frags, res, nullptr, nullptr,
                             nullptr, nullptr, nullptr);
            nf = (uint32_t)wave_sum(lane < 6 ? frags : 0);
            nr = (uint32_t)wave_sum(lane < 6 ? res : 0);
        }
        if (lane == 0)
            read_counts[r0 + j] = make_uint2(nf, nr);
        wf += nf;
        wr += nr;
    }
    if (lane == 0) {
        sums[0][w] = wf;
        sums[1][w] = wr;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t F = 0, R = 0;
        for (uint32_t i = 0; i < WAVES_PER_WG; i++) {
            F += sums[0][i];
            R += sums[1][i];
        }
        tile_sum[blockIdx.x] = make_ulonglong2(F, R);
        if (blockIdx.x == gridDim.x - 1)
            tile_sum[gridDim.x] = make_ulonglong2(0, 0); /* the scan's last element = the totals */
    }
}

/*
 * 1'. The same counts, one LANE per read: a read's fragments follow from its
 * stop codons alone, so the count pass does not translate.  Every base is
 * turned into its class nibble (nibbles4: A0 C1 G2 T/U3, bit 2 = outside
 * ACGTU) and the last three nibbles are compared with the stop codons:
 *   forward strand  TAA TAG TGA                         (trans_table.cc:8-15)
 *   reverse strand  their reverse complements TTA CTA TCA read forward
 * giving two masks per 64 bases, bit q = a stop codon whose last forward
 * base is q.  Frame +k's codons end at q = k+1 (mod 3), frame -k's at
 * q = len-k (mod 3); a run between consecutive stops of a frame (or the
 * frame's ends) spans (q' - q)/3 - 1 codons and is kept when >= 11
 * (fq_process_request.cc:333).  Blocks of 64 bases: the block's 17 dword
 * loads are in flight together; each frame carries its last stop across
 * blocks, so any read length takes this path.
 */
constexpr uint64_t EVERY3 = 0x9249249249249249ull; /* bits 0, 3, ..., 63 */

/* the runs of frame f ending at the stops in m (bit i = a stop ending at base
 * base + i): v(f, prev, q, L) for each kept run of L codons between the stops
 * ending at prev and q */
template <class V>
__device__ __forceinline__ void frame_runs(uint64_t m, int base, uint32_t f, int &prev, V &v)
{
    while (m) {
        const int q = base + __builtin_ctzll(m);
        m &= m - 1;
        const int L = (q - prev) / 3 - 1;
        if (L >= (int)MIN_FRAGMENT)
            v(f, prev, q, L);
        prev = q;
    }
}

/* each frame's first virtual stop (prev) and last one (hi), and the residue
 * class mod 3 of its stops' last bases (rho): frame +k (f = k-1) has codons at
 * f + 3i, so stops end at q = f + 3i + 2; frame -k (f = 3+k-1) reads the
 * complement backwards from top = len-k, so its stops end at q = top - 3i */
__device__ __forceinline__ void frame_bounds(uint32_t len, int *prev, int *hi, uint32_t *rho)
{
#pragma unroll
    for (uint32_t f = 0; f < 3; f++) {
        const uint32_t nc = len >= f ? (len - f) / 3 : 0;
        prev[f] = (int)f - 1;
        hi[f] = (int)(f + 2 + 3 * nc);
        rho[f] = (f + 2) % 3;
        const int top = (int)len - (int)f - 1;
        prev[3 + f] = top - 3 * (int)nc;
        hi[3 + f] = top + 3;
        rho[3 + f] = (uint32_t)((top % 3 + 3) % 3);
    }
}

/* counting visitor: (fragments, residues) of a read */
struct RunCount {
    uint32_t nf = 0, nr = 0;
    __device__ __forceinline__ void operator()(uint32_t, int, int, int L)
    {
        nf++;
        nr += (uint32_t)L;
    }
};

/* a read's kept runs straight from its bytes in memory, one base at a time:
 * the path of waves whose reads do not fit the LDS span (few registers, so
 * the staged path keeps its occupancy) */
template <class V>
__device__ __forceinline__ void lane_read_runs_global(const uint8_t *b, uint32_t len, V &v)
{
    int prev[6], hi[6];
    uint32_t rho[6];
    frame_bounds(len, prev, hi, rho);
    uint32_t hist = 0x444; /* nibbles of the last three bases, newest lowest; bit 2 = not a base yet */
    uint64_t ef = 0, er = 0;
    for (uint32_t q = 0; q < len; q++) {
        hist = ((hist << 4) | (nibbles4(b[q]) & 0xFu)) & 0xFFFu;
        const uint32_t fs = hist == 0x300u || hist == 0x302u || hist == 0x320u;
        const uint32_t rs = hist == 0x330u || hist == 0x130u || hist == 0x310u;
        ef |= (uint64_t)fs << (q & 63);
        er |= (uint64_t)rs << (q & 63);
        if ((q & 63) == 63 || q + 1 == len) { /* a block of 64 bases is complete */
            const uint32_t blk = q >> 6;
            for (uint32_t f = 0; f < 6; f++) {
                const uint32_t sh = (rho[f] + 3 - blk % 3) % 3;
                frame_runs((f < 3 ? ef : er) & (EVERY3 << sh), 64 * (int)blk, f, prev[f], v);
            }
            ef = er = 0;
        }
    }
    for (uint32_t f = 0; f < 6; f++) {
        const int L = (hi[f] - prev[f]) / 3 - 1;
        if (L >= (int)MIN_FRAGMENT)
            v(f, prev[f], hi[f], L);
    }
}

/* bit j of the result = bit 4j of m (m's bits outside 0x11111111 clear) */
__device__ __forceinline__ uint32_t nib_compress(uint32_t m)
{
    m = (m | (m >> 3)) & 0x03030303u;
    m = (m | (m >> 6)) & 0x000F000Fu;
    return (m | (m >> 12)) & 0xFFu;
}

/* stop codons ending at the 8 bases of x (nibble string, base j at bits
 * 4j; prev = the 8 bases before): forward TAA TAG TGA / reverse strand TTA
 * CTA TCA read forward.  Bit j of fs / rs.  SWAR over the nibbles: the
 * per-base class tests are 64-bit masks, the bases one and two back are the
 * same masks shifted by one and two nibbles. */
__device__ __forceinline__ void stops8(uint32_t x, uint32_t prev, uint32_t &fs, uint32_t &rs)
{
    constexpr uint64_t N1 = 0x1111111111111111ull;
    const uint64_t y = (uint64_t)x << 32 | prev;
    const uint64_t lo = y & N1, hi = (y >> 1) & N1, ok = ~(y >> 2) & N1;
    const uint64_t A = ~lo & ~hi & ok, C = lo & ~hi & ok, G = ~lo & hi & ok, T = lo & hi & ok;
    const uint64_t A1 = A << 4, C1 = C << 4, G1 = G << 4, T1 = T << 4, C2 = C << 8, T2 = T << 8;
    const uint64_t f = T2 & ((A1 & (A | G)) | (G1 & A));
    const uint64_t r = A & ((T1 & (T2 | C2)) | (C1 & T2));
    fs = nib_compress((uint32_t)(f >> 32));
    rs = nib_compress((uint32_t)(r >> 32));
}

/* lane_read_runs over the wave's nibble string (ns: byte o of the staged
 * span at bits 4o; the read's base p is nibble loc + p) */
template <class V>
__device__ __forceinline__ void lane_read_runs_ns(const uint32_t *ns, uint32_t loc, uint32_t len, V &v)
{
    int prev[6], hi[6];
    uint32_t rho[6];
    frame_bounds(len, prev, hi, rho);
    const uint32_t sh = (loc & 7u) * 4u;
    uint32_t px = 0x44444444u; /* no bases before base 0 */
    for (uint32_t blk = 0; 64 * blk < len; blk++) {
        const uint32_t w0 = (loc + 64 * blk) >> 3;
        uint64_t ef = 0, er = 0;
        uint32_t lo = ns[w0];
#pragma unroll 2
        for (uint32_t i = 0; i < 8; i++) {
            const uint32_t hi = ns[w0 + i + 1];
            const uint32_t x = __builtin_amdgcn_alignbit(hi, lo, sh); /* bases 64 blk + 8i .. +7 */
            lo = hi;
            uint32_t fs, rs;
            stops8(x, px, fs, rs);
            ef |= (uint64_t)fs << (8 * i);
            er |= (uint64_t)rs << (8 * i);
            px = x;
        }
        const uint32_t left = len - 64 * blk;
        const uint64_t in = left >= 64 ? ~0ull : ((1ull << left) - 1);
        ef &= in;
        er &= in;
        const int base = 64 * (int)blk;
#pragma unroll
        for (uint32_t f = 0; f < 6; f++) {
            const uint32_t shf = (rho[f] + 3 - blk % 3) % 3;
            frame_runs((f < 3 ? ef : er) & (EVERY3 << shf), base, f, prev[f], v);
        }
    }
#pragma unroll
    for (uint32_t f = 0; f < 6; f++) {
        const int L = (hi[f] - prev[f]) / 3 - 1;
        if (L >= (int)MIN_FRAGMENT)
            v(f, prev[f], hi[f], L);
    }
}

/* per read: (fragments, residues); per 64 reads (the emit kernel's tile):
 * their sums.  The wave's reads are usually back to back: their byte span is
 * copied into the wave's LDS with 16-B coalesced loads and each lane reads its
 * read from there (lanes reading their own reads straight from memory touch
 * 64 lines per load, 150 bytes apart, and the L1 thrashes).  A wave whose span
 * does not fit reads from memory. */
constexpr uint32_t COUNT_SPAN = 12288;               /* span bytes a wave stages */
constexpr uint32_t NS_WORDS = COUNT_SPAN / 8 + 16;     /* their nibble string + slack */

/* the wave's span [first, end) of bases as a nibble string in LDS, 16 bytes
 * per lane per round, coalesced (+1 round of zeros: the funnel shifts' pad);
 * false when the span does not fit (or is empty).  a = its 16-aligned start. */
__device__ __forceinline__ bool stage_span(uint32_t *ns, const uint8_t *bases, uint64_t first, uint64_t end,
                                           uint32_t lane, uintptr_t &a)
{
    a = reinterpret_cast<uintptr_t>(bases + first) & ~(uintptr_t)15;
    const uint64_t bytes = reinterpret_cast<uintptr_t>(bases + end) - a;
    if (!(end > first && bytes <= COUNT_SPAN))
        return false;
    const uint4 *src = reinterpret_cast<const uint4 *>(a);
    const uint32_t nv = (uint32_t)((bytes + 15) / 16);
    /* 4 loads in flight per lane before any is converted.  The loads are
     * unconditional (past the span they re-read its last 16 bytes) and the
     * zero pad is a select afterwards: a load under a branch whose value
     * merges at the join is waited for right there, and one wait per 16 B
     * made the staging ~10 dependent round trips per wave */
    constexpr uint32_t U = 4;
    for (uint32_t i0 = lane; i0 < nv + 1; i0 += 64 * U) {
        uint4 v[U];
#pragma unroll
        for (uint32_t k = 0; k < U; k++)
            v[k] = src[min(i0 + 64 * k, nv - 1)];
#pragma unroll
        for (uint32_t k = 0; k < U; k++) {
            const uint32_t i = i0 + 64 * k;
            const bool in = i < nv;
            const uint4 w = make_uint4(in ? v[k].x : 0u, in ? v[k].y : 0u, in ? v[k].z : 0u, in ? v[k].w : 0u);
            if (i < nv + 1) {
                ns[2 * i] = nibbles4(w.x) | nibbles4(w.y) << 16;
                ns[2 * i + 1] = nibbles4(w.z) | nibbles4(w.w) << 16;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return true;
}

/* per-frame counting visitor */
struct RunCount6 {
    uint32_t nf[6] = {0, 0, 0, 0, 0, 0}, nr[6] = {0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ void operator()(uint32_t f, int, int, int L)
    {
        nf[f]++;
        nr[f] += (uint32_t)L;
    }
};

/* FRAMES (the anchors' pass): also each frame's fragments and residues,
 * frame_nf / frame_nr[6r + f] */
template <bool FRAMES>
__global__ __launch_bounds__(256) void fq_count_lane_kernel(const uint8_t *bases, const uint64_t *read_off,
                                                            uint32_t n_reads, uint2 *read_counts, ulonglong2 *tile_sum,
                                                            uint32_t n_tiles, uint32_t *frame_nf, uint32_t *frame_nr)
{
    __shared__ uint32_t nspan[WAVES_PER_WG][NS_WORDS];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t tile = blockIdx.x * WAVES_PER_WG + wv;
    if (tile >= n_tiles)
        return;
    uint32_t *ns = nspan[wv];
    const uint64_t r0 = (uint64_t)tile * FQ_TILE;
    const uint32_t n = (uint32_t)std::min<uint64_t>(FQ_TILE, n_reads - r0);
    const uint64_t r = r0 + lane;
    const uint64_t ob = lane < n ? read_off[r] : 0, oe = lane < n ? read_off[r + 1] : 0;
    /* the wave's span [a, e): 16-aligned start */
    const uint64_t first = uniform_u64(__shfl(ob, 0)), end = uniform_u64(__shfl(oe, (int)n - 1));
    uintptr_t a = 0;
    const bool staged = stage_span(ns, bases, first, end, lane, a);
    uint32_t nf = 0, nr = 0;
    if (FRAMES) {
        if (lane < n) {
            RunCount6 rc;
            if (staged)
                lane_read_runs_ns(ns, (uint32_t)(reinterpret_cast<uintptr_t>(bases + ob) - a), (uint32_t)(oe - ob),
                                  rc);
            else
                lane_read_runs_global(bases + ob, (uint32_t)(oe - ob), rc);
#pragma unroll
            for (uint32_t f = 0; f < 6; f++) {
                frame_nf[r * 6 + f] = rc.nf[f];
                frame_nr[r * 6 + f] = rc.nr[f];
                nf += rc.nf[f];
                nr += rc.nr[f];
            }
        }
    } else if (staged) {
        if (lane < n) {
            RunCount rc;
            lane_read_runs_ns(ns, (uint32_t)(reinterpret_cast<uintptr_t>(bases + ob) - a), (uint32_t)(oe - ob), rc);
            nf = rc.nf;
            nr = rc.nr;
        }
    } else if (lane < n) {
        RunCount rc;
        lane_read_runs_global(bases + ob, (uint32_t)(oe - ob), rc);
        nf = rc.nf;
        nr = rc.nr;
    }
    if (lane < n)
        read_counts[r] = make_uint2(nf, nr);
    const uint64_t F = wave_sum(nf), R = wave_sum(nr);
    if (lane == 0) {
        tile_sum[tile] = make_ulonglong2(F, R);
        if (tile == n_tiles - 1)
            tile_sum[n_tiles] = make_ulonglong2(0, 0); /* the scan's last element = the totals */
    }
}

/* writing visitor: fragment records in (frame, position) order.  A reverse
 * frame's runs are found in ascending base order, which is descending
 * position on its strand: they are placed from the frame's end backwards. */
struct RunWrite {
    uint32_t fi[6]; /* next fragment slot (forward) / last unwritten (reverse) */
    uint64_t ri[6]; /* next residue offset (forward) / end of the unwritten (reverse) */
    uint64_t ob;    /* the read's first byte */
    uint64_t *out_off, *out_anchor;
    __device__ __forceinline__ void operator()(uint32_t f, int prev, int q, int L)
    {
        uint32_t idx;
        uint64_t ro, anchor;
        if (f < 3) { /* codons f + 3i: the run starts at base prev + 1 */
            idx = fi[f]++;
            ro = ri[f];
            ri[f] += (uint32_t)L;
            anchor = (ob + (uint64_t)(prev + 1)) << 1;
        } else { /* codon i = complement of bases top - 3i .. top - 3i - 2, the
                  * run's first codon the one after the stop ending at q */
            idx = fi[f]--;
            ri[f] -= (uint32_t)L;
            ro = ri[f];
            anchor = ((ob + (uint64_t)(q - 3)) << 1) | 1u;
        }
        out_off[idx] = ro;
        out_anchor[idx] = anchor;
    }
};

/*
 * 3'. fragment records without residues (fq_residues = 0): one lane per read,
 * as the count pass, which left each frame's fragment and residue counts
 * (frame_nf / frame_nr).  Each fragment gets its offset and anchor = (byte
 * index of its first codon's first base) << 1 | reverse strand, which the
 * DNA probe (launch_probe_dna) translates windows from; no residue is written.
 * Per-fragment read and frame are not written either (the per-(read, frame)
 * counts hold them): lanes ~10 fragments apart store scattered, and each
 * array costs ~60 us per 1M reads.
 */
__global__ __launch_bounds__(256) void fq_desc_lane_kernel(const uint8_t *bases, const uint64_t *read_off,
                                                           uint32_t n_reads, const uint2 *read_counts,
                                                           const ulonglong2 *tile_base, uint32_t n_tiles,
                                                           const uint32_t *frame_nf, const uint32_t *frame_nr,
                                                           uint32_t *frag_base, uint64_t *out_off, uint64_t *out_anchor,
                                                           const uint64_t *totals, uint64_t max_frag)
{
    __shared__ uint32_t nspan[WAVES_PER_WG][NS_WORDS];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t tile = blockIdx.x * WAVES_PER_WG + wv;
    if (tile >= n_tiles || totals[0] > max_frag) /* more fragments than the buffers hold: fq_tail flagged it */
        return;
    uint32_t *ns = nspan[wv];
    const uint64_t r0 = (uint64_t)tile * FQ_TILE;
    const uint32_t n = (uint32_t)std::min<uint64_t>(FQ_TILE, n_reads - r0);
    const uint64_t r = r0 + lane;
    const uint64_t ob = lane < n ? read_off[r] : 0, oe = lane < n ? read_off[r + 1] : 0;
    /* the read's first fragment and residue: the tile's base + the earlier reads' counts */
    const uint2 cnt = lane < n ? read_counts[r] : make_uint2(0, 0);
    uint64_t pf = cnt.x, pr = cnt.y;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint64_t xf = __shfl_up(pf, o), xr = __shfl_up(pr, o);
        if (lane >= o) {
            pf += xf;
            pr += xr;
        }
    }
    const ulonglong2 tb = tile_base[tile];
    const uint64_t first = uniform_u64(__shfl(ob, 0)), end = uniform_u64(__shfl(oe, (int)n - 1));
    uintptr_t a = 0;
    const bool staged = stage_span(ns, bases, first, end, lane, a);
    if (lane >= n)
        return;
    const uint32_t len = (uint32_t)(oe - ob);
    RunWrite w;
    uint64_t fb = tb.x + pf - cnt.x, rb = tb.y + pr - cnt.y;
#pragma unroll
    for (uint32_t f = 0; f < 6; f++) {
        const uint32_t nf = frame_nf[r * 6 + f], nr = frame_nr[r * 6 + f];
        frag_base[r * 6 + f] = (uint32_t)fb;
        w.fi[f] = (uint32_t)(f < 3 ? fb : fb + nf - 1);
        w.ri[f] = f < 3 ? rb : rb + nr;
        fb += nf;
        rb += nr;
    }
    w.ob = ob;
    w.out_off = out_off;
    w.out_anchor = out_anchor;
    if (staged)
        lane_read_runs_ns(ns, (uint32_t)(reinterpret_cast<uintptr_t>(bases + ob) - a), len, w);
    else
        lane_read_runs_global(bases + ob, len, w);
}

/*
 * 3''. count + scan + anchors in ONE pass (option fq_fused, the default with
 * anchors): the count kernel, the scan of its wave sums, the tail kernel and
 * the anchor kernel above fused by a decoupled look-back.  A wave takes the
 * next tile of 64 reads from a counter (so every tile it waits on belongs to a
 * wave already running), counts its reads' runs per frame into registers,
 * publishes the tile's sums, sums the published sums / prefixes of the tiles
 * before it (64 predecessors per step, one per lane), publishes its inclusive
 * prefix, and writes its reads' fragment offsets and anchors from the same
 * staged nibble string -- the reads are read once, and the per-(read, frame)
 * residue counts never leave the registers.  A tile's state is ONE 64-bit
 * word, state << 62 | fragments << 31 | residues (1 sums, 2 prefix; zeroed
 * before the launch), stored and loaded with relaxed device-scope atomics:
 * no release / acquire, whose cross-XCD L2 write-backs made a first version
 * with separate flag and value words 1.6x slower end to end.  Needs fewer
 * than 2^31 fragments and residues per batch (the host checks).  The wave
 * that draws the last id resets the counter.  Same outputs as count -> scan
 * -> tail -> desc, bit for bit.
 */
constexpr uint64_t LB_MASK31 = (1ull << 31) - 1;
__global__ __launch_bounds__(256) void fq_anchor_fused_kernel(
    const uint8_t *bases, const uint64_t *read_off, uint32_t n_reads, uint32_t n_tiles, uint32_t total_waves,
    uint32_t *tile_ctr, uint64_t *tile_state, uint32_t *frame_nf, uint32_t *frag_base, uint64_t *out_off,
    uint64_t *out_anchor, uint64_t *totals, uint64_t max_frag, uint64_t max_res)
{
    __shared__ uint32_t nspan[WAVES_PER_WG][NS_WORDS];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t tile = 0;
    if (lane == 0)
        tile = atomicAdd(tile_ctr, 1u);
    tile = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)tile, 0));
    if (tile == total_waves - 1 && lane == 0)
        __hip_atomic_store(tile_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); /* every id is drawn */
    if (tile >= n_tiles)
        return;
    uint32_t *ns = nspan[wv];
    const uint64_t r0 = (uint64_t)tile * FQ_TILE;
    const uint32_t n = (uint32_t)std::min<uint64_t>(FQ_TILE, n_reads - r0);
    const uint64_t r = r0 + lane;
    const uint64_t ob = lane < n ? read_off[r] : 0, oe = lane < n ? read_off[r + 1] : 0;
    const uint64_t first = uniform_u64(__shfl(ob, 0)), end = uniform_u64(__shfl(oe, (int)n - 1));
    uintptr_t a = 0;
    const bool staged = stage_span(ns, bases, first, end, lane, a);
    const uint32_t len = (uint32_t)(oe - ob);
    RunCount6 rc;
    if (lane < n) {
        if (staged)
            lane_read_runs_ns(ns, (uint32_t)(reinterpret_cast<uintptr_t>(bases + ob) - a), len, rc);
        else
            lane_read_runs_global(bases + ob, len, rc);
    }
    uint64_t nf = 0, nr = 0;
#pragma unroll
    for (uint32_t f = 0; f < 6; f++) {
        nf += rc.nf[f];
        nr += rc.nr[f];
    }
    const uint64_t F = wave_sum(nf), R = wave_sum(nr);
    /* publish the tile's sums (tile 0: its prefix) */
    if (lane == 0)
        __hip_atomic_store(&tile_state[tile], (tile == 0 ? 2ull : 1ull) << 62 | F << 31 | R, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    /* look back: lane l examines tile j - l */
    uint64_t xf = 0, xr = 0;
    for (int64_t j = (int64_t)tile - 1; j >= 0; j -= 64) {
        const int64_t idx = j - (int64_t)lane;
        uint64_t v = 2ull << 62; /* before tile 0: a zero prefix */
        if (idx >= 0)
            do {
                v = __hip_atomic_load(&tile_state[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } while ((v >> 62) == 0);
        const uint64_t pm = __ballot((v >> 62) == 2);
        const uint32_t upto = pm ? (uint32_t)__builtin_ctzll(pm) : 63u; /* lanes 0..upto count */
        const bool in = lane <= upto;
        xf += wave_sum(in ? (v >> 31) & LB_MASK31 : 0);
        xr += wave_sum(in ? v & LB_MASK31 : 0);
        if (pm)
            break;
    }
    xf = uniform_u64(xf);
    xr = uniform_u64(xr);
    const uint64_t tf = xf + F, tr = xr + R;
    if (lane == 0 && tile != 0)
        __hip_atomic_store(&tile_state[tile], 2ull << 62 | (tf & LB_MASK31) << 31 | (tr & LB_MASK31),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    /* the batch's totals and CSR tails (fq_tail_kernel's work) */
    if (tile == n_tiles - 1 && lane == 0) {
        const bool over = tf > max_frag || tr > max_res;
        totals[0] = over ? max_frag + 1 : tf;
        totals[1] = tr;
        if (!over) {
            out_off[tf] = tr;
            frag_base[(uint64_t)n_reads * 6] = (uint32_t)tf;
            frame_nf[(uint64_t)n_reads * 6] = 0;
        }
    }
    /* a batch past the buffers writes nothing beyond them (the finish
     * reports it from the totals) */
    if (tf > max_frag || tr > max_res || lane >= n)
        return;
    /* the read's first fragment and residue: the tile's prefix + the earlier reads' counts */
    uint64_t pf = nf, pr = nr;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint64_t yf = __shfl_up(pf, o), yr = __shfl_up(pr, o);
        if (lane >= o) {
            pf += yf;
            pr += yr;
        }
    }
    RunWrite w;
    uint64_t fb = xf + pf - nf, rb = xr + pr - nr;
#pragma unroll
    for (uint32_t f = 0; f < 6; f++) {
        frame_nf[r * 6 + f] = rc.nf[f];
        frag_base[r * 6 + f] = (uint32_t)fb;
        w.fi[f] = (uint32_t)(f < 3 ? fb : fb + rc.nf[f] - 1);
        w.ri[f] = f < 3 ? rb : rb + rc.nr[f];
        fb += rc.nf[f];
        rb += rc.nr[f];
    }
    w.ob = ob;
    w.out_off = out_off;
    w.out_anchor = out_anchor;
    if (staged)
        lane_read_runs_ns(ns, (uint32_t)(reinterpret_cast<uintptr_t>(bases + ob) - a), len, w);
    else
        lane_read_runs_global(bases + ob, len, w);
}

struct PairSum {
    __host__ __device__ ulonglong2 operator()(const ulonglong2 &a, const ulonglong2 &b) const
    {
        return make_ulonglong2(a.x + b.x, a.y + b.y);
    }
};

/* 2b. after the exclusive scan of the workgroup sums (hipcub): the batch
 * totals and the CSR tails */
__global__ void fq_tail_kernel(const ulonglong2 *tile_base, uint64_t n_tiles, uint32_t n_reads, uint64_t *totals,
                               uint64_t *out_off, uint32_t *frag_base, uint32_t *n_frag, uint64_t max_frag,
                               uint64_t max_res)
{
    const ulonglong2 tot = tile_base[n_tiles];
    /* a caller's span bound that is too small (kgx_fq_fragments_device_start)
     * shows as totals past the buffers: the emit passes then write nothing and
     * the finish reports it */
    const bool over = tot.x > max_frag || tot.y > max_res;
    totals[0] = over ? max_frag + 1 : tot.x;
    totals[1] = tot.y;
    if (over)
        return;
    out_off[tot.x] = tot.y;
    frag_base[(uint64_t)n_reads * 6] = (uint32_t)tot.x;
    n_frag[(uint64_t)n_reads * 6] = 0;
}

/* 3. fragment records (offset, read, frame, first codon), residues and the
 * per-(read, frame) counts / first fragments, at the scanned bases */
__global__ __launch_bounds__(256) void fq_emit_kernel(const uint8_t *bases, const uint64_t *read_off,
                                                      uint32_t n_reads, const uint2 *read_counts,
                                                      const ulonglong2 *tile_base,
                                                      uint32_t *n_frag, uint32_t *frag_base, uint8_t *out_res,
                                                      uint64_t *out_off, uint32_t *out_read, int8_t *out_frame,
                                                      uint32_t *out_start, const uint64_t *totals, uint64_t max_frag)
{
    if (totals[0] > max_frag) /* fq_tail flagged an overflow: write nothing */
        return;
    __shared__ FqLds t;
    fq_lds_init(t);
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint64_t tile0 = (uint64_t)blockIdx.x * FQ_TILE;
    /* the tile's reads' counts, lane i = read tile0 + i: exclusive prefix */
    const uint2 c = lane < FQ_TILE && tile0 + lane < n_reads ? read_counts[tile0 + lane] : make_uint2(0, 0);
    uint64_t pf = c.x, pr = c.y;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint64_t xf = __shfl_up(pf, o), xr = __shfl_up(pr, o);
        if (lane >= o) {
            pf += xf;
            pr += xr;
        }
    }
    pf -= c.x;
    pr -= c.y;
    const uint64_t r0 = tile0 + w * FQ_READS_PER_WAVE;
    const uint32_t n = (uint32_t)(r0 < n_reads ? std::min<uint64_t>(FQ_READS_PER_WAVE, n_reads - r0) : 0);
    const ulonglong2 tb = tile_base[blockIdx.x];
    uint64_t F = tb.x + __shfl(pf, (int)(w * FQ_READS_PER_WAVE));
    uint64_t R = tb.y + __shfl(pr, (int)(w * FQ_READS_PER_WAVE));
    const uint64_t my_off = n && lane <= n ? read_off[r0 + lane] : 0;
    stage_wave_reads(t.nib[w], bases, my_off, n, lane);
    for (uint32_t j = 0; j < n; j++) {
        const uint64_t r = r0 + j;
        const uint64_t ob = uniform_u64(__shfl(my_off, (int)j)), oe = uniform_u64(__shfl(my_off, (int)j + 1));
        const uint64_t len = oe - ob;
        uint32_t my_nf = 0;
        uint64_t my_fb = 0;
        if (len <= SHORT_READ) {
            char aas[6];
            uint64_t stops[6];
            translate6(t.nib[w][j], t.code, read_mis(bases + ob), (uint32_t)len, lane, aas, stops);
#pragma unroll
            for (uint32_t f = 0; f < 6; f++) {
                const char aa = aas[f];
                const uint64_t kept = kept_runs(stops[f]);
                const uint64_t starts = kept & ~(kept << 1);
                if (lane == f) {
                    my_nf = (uint32_t)__popcll(starts);
                    my_fb = F;
                }
                const uint64_t ri = R + popc_below(kept);
                if ((kept >> lane) & 1)
                    out_res[ri] = (uint8_t)aa;
                if ((starts >> lane) & 1) {
                    const uint64_t fi = F + popc_below(starts);
                    out_off[fi] = ri;
                    out_read[fi] = (uint32_t)r;
                    out_frame[fi] = (int8_t)frame_of(f);
                    out_start[fi] = lane;
                }
                F += (uint64_t)__popcll(starts);
                R += (uint64_t)__popcll(kept);
            }
        } else {
            /* lanes 0-5 = frames: count, place after the earlier frames, emit */
            uint32_t frags = 0;
            uint64_t res = 0;
            const FrameReader fr{bases + ob, len, frame_of(lane < 6 ? lane : 0)};
            if (lane < 6)
                frame_serial(fr, 0, 0, 0, frags, res, nullptr, nullptr, nullptr, nullptr, nullptr);
            uint64_t ef = lane < 6 ? frags : 0, er = lane < 6 ? res : 0;
            for (uint32_t o = 1; o < 8; o <<= 1) {
                const uint64_t xf = __shfl_up(ef, o), xr = __shfl_up(er, o);
                if (lane >= o) {
                    ef += xf;
                    er += xr;
                }
            }
            const uint64_t tf = __shfl(ef, 5), tr = __shfl(er, 5);
            ef -= lane < 6 ? frags : 0;
            er -= lane < 6 ? res : 0;
            if (lane < 6) {
                frame_serial(fr, (uint32_t)r, F + ef, R + er, frags, res, out_res, out_off, out_read, out_frame,
                             out_start);
                my_nf = frags;
                my_fb = F + ef;
            }
            F += tf;
            R += tr;
        }
        if (lane < 6) {
            n_frag[r * 6 + lane] = my_nf;
            frag_base[r * 6 + lane] = (uint32_t)my_fb;
        }
    }
}

inline dim3 grid_for(uint64_t n) { return dim3((uint32_t)((n + 255) / 256)); }

/* launch_fq_plan: fragment i's window base wbase[i] = (off[i] - off[0]) - 8 i
 * (each fragment has len - 8 windows, len >= 9), the tiles whose first
 * window lies in its windows get tile_seq = i, wbase[n] = the total;
 * block_max[workgroup] = its longest fragment in windows */
__global__ __launch_bounds__(256) void fq_plan_kernel(const uint64_t *__restrict__ off, uint32_t n,
                                                      uint64_t *__restrict__ wbase, uint32_t *__restrict__ tile_seq,
                                                      uint32_t tw, uint32_t tw_shift, uint32_t *__restrict__ block_max)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t o0 = off[0];
    uint32_t w = 0;
    if (i < n) {
        const uint64_t a = off[i], b = off[i + 1];
        const uint64_t wb = (a - o0) - 8 * i;
        w = (uint32_t)(b - a - 8);
        wbase[i] = wb;
        const uint64_t t0 = tw_shift ? (wb + tw - 1) >> tw_shift : (wb + tw - 1) / tw;
        for (uint64_t t = t0; t * tw < wb + w; t++)
            tile_seq[t] = (uint32_t)i;
    } else if (i == n) {
        wbase[n] = (off[n] - o0) - 8 * (uint64_t)n;
    }
    /* the workgroup's longest fragment into block_max (one address for the
     * whole grid would serialise its atomics: 1.5 ms per 155k waves) */
    __shared__ uint32_t wmax[4];
    for (uint32_t o = 32; o; o >>= 1) /* every lane shuffles (w = 0 past the batch) */
        w = max(w, (uint32_t)__shfl_xor((int)w, (int)o));
    if ((threadIdx.x & 63u) == 0)
        wmax[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0)
        block_max[blockIdx.x] = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
}

/* status[0] = 0 (no bad offsets), status[1] = the longest fragment */
__global__ __launch_bounds__(1024) void fq_plan_max_kernel(const uint32_t *__restrict__ block_max, uint32_t n,
                                                           uint32_t *__restrict__ status)
{
    __shared__ uint32_t wmax[16];
    uint32_t m = 0;
    for (uint32_t i = threadIdx.x; i < n; i += 1024)
        m = max(m, block_max[i]);
    for (uint32_t o = 32; o; o >>= 1)
        m = max(m, (uint32_t)__shfl_xor((int)m, (int)o));
    if ((threadIdx.x & 63u) == 0)
        wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t k = 1; k < 16; k++)
            m = max(m, wmax[k]);
        status[0] = 0;
        status[1] = m;
    }
}

}  // namespace

namespace kgx {

hipError_t launch_fq_plan(const uint64_t *off, uint32_t n, uint64_t *wbase, uint32_t *tile_seq, uint32_t tile_windows,
                          uint32_t *status, uint32_t *block_max, hipStream_t stream)
{
    const uint32_t shift = (tile_windows & (tile_windows - 1)) ? 0u : (uint32_t)__builtin_ctz(tile_windows);
    const dim3 grid = grid_for((uint64_t)n + 1);
    hipLaunchKernelGGL(fq_plan_kernel, grid, dim3(256), 0, stream, off, n, wbase, tile_seq, tile_windows, shift,
                       block_max);
    hipLaunchKernelGGL(fq_plan_max_kernel, dim3(1), dim3(1024), 0, stream, block_max, grid.x, status);
    return hipGetLastError();
}

/* fragments of the reads in [d_bases, read_off) into the ctx's fq buffers.
 * n_bases: the bytes the reads span (read_off[n] - read_off[0]), which bounds
 * the output: six frames give at most 2 residues per base, a fragment has at
 * least 11 residues.  Launches: count -> scan of the workgroup sums (hipcub)
 * -> emit, with no host round trip between them; one readback of the totals. */
/* the fragment pass up to the totals' D2H, without waiting (fq_fragments_finish
 * waits); n_bases bounds the output buffers, bound the bytes readable from d_bases */
int fq_fragments_enqueue(kgx_ctx *c, const uint8_t *d_bases, const uint64_t *d_read_off, uint32_t n_reads,
                         uint64_t n_bases, uint64_t bound)
{
    /* fragments as anchors into the bases (no residues) when asked and the probe can take them */
    const bool desc = !c->fq_residues && probe_takes_dna(c);
    hipStream_t st = c->stream;
    const uint64_t n_rf = (uint64_t)n_reads * 6;
    const uint64_t max_res = 2 * n_bases, max_frag = max_res / MIN_FRAGMENT + 1;
    const uint64_t n_tiles = ((uint64_t)n_reads + FQ_TILE - 1) / FQ_TILE;
    HIP_TRY(c->fq_nfrag.reserve((n_rf + 1) * 4));
    HIP_TRY(c->fq_fbase.reserve((n_rf + 1) * 4));
    /* per-read counts, the workgroup sums, their scan, the totals, the scan's scratch */
    const uint64_t rc_bytes = ((uint64_t)n_reads + 1) * sizeof(uint2), ts_bytes = (n_tiles + 1) * sizeof(ulonglong2);
    size_t scan_bytes = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveScan(nullptr, scan_bytes, (ulonglong2 *)nullptr, (ulonglong2 *)nullptr,
                                              PairSum(), make_ulonglong2(0, 0), (int)(n_tiles + 1), st));
    const uint64_t ws_bytes = rc_bytes + 2 * ts_bytes + 16 + 256 + scan_bytes + 16;
    HIP_TRY(c->fq_tmp.reserve(ws_bytes));
    if (desc) {
        HIP_TRY(c->fq_anchor.reserve((max_frag + 1) * 8));
        HIP_TRY(c->fq_nres.reserve((n_rf + 1) * 4));
    }
    else {
        HIP_TRY(c->fq_res.reserve(max_res + 16));
        HIP_TRY(c->fq_read.reserve((max_frag + 1) * 4));
        HIP_TRY(c->fq_frame.reserve(max_frag + 1));
        HIP_TRY(c->fq_start.reserve((max_frag + 1) * 4));
    }
    HIP_TRY(c->fq_off.reserve((max_frag + 1) * 8));

    HIP_TRY(c->h_fq_tot.resize(2));
    char *ws = static_cast<char *>(c->fq_tmp.p);
    uint2 *read_counts = reinterpret_cast<uint2 *>(ws);
    ulonglong2 *tile_sum = reinterpret_cast<ulonglong2 *>(ws + ((rc_bytes + 15) & ~15ull));
    ulonglong2 *tile_base = tile_sum + (n_tiles + 1);
    uint64_t *totals = reinterpret_cast<uint64_t *>(tile_base + (n_tiles + 1));
    void *scan_tmp = ws + ((((rc_bytes + 15) & ~15ull) + 2 * ts_bytes + 16 + 255) & ~255ull);
    if (n_reads && desc && c->fq_fused && max_res < (1ull << 31)) {
        /* one pass: count + look-back scan + anchors */
        const uint32_t grid = (uint32_t)((n_tiles + WAVES_PER_WG - 1) / WAVES_PER_WG);
        const size_t cap0 = c->fq_look.cap;
        HIP_TRY(c->fq_look.reserve(256 + n_tiles * sizeof(uint64_t)));
        char *lb = static_cast<char *>(c->fq_look.p);
        if (c->fq_look.cap != cap0) /* fresh memory: the tile counter starts at 0 */
            HIP_TRY(hipMemsetAsync(lb, 0, 4, st));
        HIP_TRY(hipMemsetAsync(lb + 256, 0, n_tiles * sizeof(uint64_t), st)); /* no tile published */
        hipLaunchKernelGGL(fq_anchor_fused_kernel, dim3(grid), dim3(256), 0, st, d_bases, d_read_off, n_reads,
                           (uint32_t)n_tiles, grid * WAVES_PER_WG, reinterpret_cast<uint32_t *>(lb),
                           reinterpret_cast<uint64_t *>(lb + 256), c->fq_nfrag.as<uint32_t>(),
                           c->fq_fbase.as<uint32_t>(), c->fq_off.as<uint64_t>(), c->fq_anchor.as<uint64_t>(), totals,
                           max_frag, max_res);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->h_fq_tot.data(), totals, 16, hipMemcpyDeviceToHost, st));
        c->fq_pend = {true, desc, n_reads, max_frag, max_res, d_bases, bound};
        return KGX_OK;
    }
    if (n_reads && desc)
        hipLaunchKernelGGL(fq_count_lane_kernel<true>, dim3((uint32_t)((n_tiles + WAVES_PER_WG - 1) / WAVES_PER_WG)),
                           dim3(256), 0, st, d_bases, d_read_off, n_reads, read_counts, tile_sum, (uint32_t)n_tiles,
                           c->fq_nfrag.as<uint32_t>(), c->fq_nres.as<uint32_t>());
    else if (n_reads && c->fq_count)
        hipLaunchKernelGGL(fq_count_lane_kernel<false>, dim3((uint32_t)((n_tiles + WAVES_PER_WG - 1) / WAVES_PER_WG)),
                           dim3(256), 0, st, d_bases, d_read_off, n_reads, read_counts, tile_sum, (uint32_t)n_tiles,
                           nullptr, nullptr);
    else if (n_reads)
        hipLaunchKernelGGL(fq_count_kernel, dim3((uint32_t)n_tiles), dim3(256), 0, st, d_bases, d_read_off, n_reads,
                           read_counts, tile_sum);
    else
        HIP_TRY(hipMemsetAsync(tile_sum, 0, sizeof(ulonglong2), st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveScan(scan_tmp, scan_bytes, tile_sum, tile_base, PairSum(),
                                              make_ulonglong2(0, 0), (int)(n_tiles + 1), st));
    hipLaunchKernelGGL(fq_tail_kernel, dim3(1), dim3(1), 0, st, tile_base, n_tiles, n_reads, totals,
                       c->fq_off.as<uint64_t>(), c->fq_fbase.as<uint32_t>(), c->fq_nfrag.as<uint32_t>(), max_frag,
                       max_res);
    if (n_reads && desc)
        hipLaunchKernelGGL(fq_desc_lane_kernel, dim3((uint32_t)((n_tiles + WAVES_PER_WG - 1) / WAVES_PER_WG)),
                           dim3(256), 0, st, d_bases, d_read_off, n_reads, read_counts, tile_base, (uint32_t)n_tiles,
                           c->fq_nfrag.as<uint32_t>(), c->fq_nres.as<uint32_t>(), c->fq_fbase.as<uint32_t>(),
                           c->fq_off.as<uint64_t>(), c->fq_anchor.as<uint64_t>(), totals, max_frag);
    else if (n_reads)
        hipLaunchKernelGGL(fq_emit_kernel, dim3((uint32_t)n_tiles), dim3(256), 0, st, d_bases, d_read_off, n_reads,
                           read_counts, tile_base, c->fq_nfrag.as<uint32_t>(), c->fq_fbase.as<uint32_t>(),
                           c->fq_res.as<uint8_t>(), c->fq_off.as<uint64_t>(), c->fq_read.as<uint32_t>(),
                           c->fq_frame.as<int8_t>(), c->fq_start.as<uint32_t>(), totals, max_frag);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(c->h_fq_tot.data(), totals, 16, hipMemcpyDeviceToHost, st));
    c->fq_pend = {true, desc, n_reads, max_frag, max_res, d_bases, bound};
    return KGX_OK;
}

/* wait for the enqueued fragment pass and describe its output */
int fq_fragments_finish(kgx_ctx *c, kgx_fragments *out)
{
    if (!c->fq_pend.active)
        return fail(KGX_EINVAL, "no fragment pass started on this context");
    const FqPending p = c->fq_pend;
    c->fq_pend.active = false;
    HIP_TRY(hipStreamSynchronize(c->stream));
    const bool desc = p.desc;
    const uint64_t nf = c->h_fq_tot[0], nr = c->h_fq_tot[1];
    if (nf > p.max_frag || nr > p.max_res)
        return fail(KGX_EINVAL, "fq fragments overflowed their bound (the reads span more than n_bases)");
    const uint32_t n_reads = p.n_reads;
    const uint8_t *d_bases = p.bases;
    const uint64_t bound = p.bound;
    out->n_reads = n_reads;
    out->n_fragments = (uint32_t)nf;
    out->n_residues = nr;
    out->residues = desc ? nullptr : c->fq_res.as<uint8_t>();
    out->anchors = desc ? c->fq_anchor.as<uint64_t>() : nullptr;
    out->bases = d_bases;
    out->n_bases = bound;
    out->offsets = c->fq_off.as<uint64_t>();
    out->read = desc ? nullptr : c->fq_read.as<uint32_t>();
    out->frame = desc ? nullptr : c->fq_frame.as<int8_t>();
    out->frame_counts = c->fq_nfrag.as<uint32_t>();
    return KGX_OK;
}

int fq_fragments(kgx_ctx *c, const uint8_t *d_bases, const uint64_t *d_read_off, uint32_t n_reads,
                 uint64_t n_bases, uint64_t bound, kgx_fragments *out)
{
    const int rc = fq_fragments_enqueue(c, d_bases, d_read_off, n_reads, n_bases, bound);
    return rc ? rc : fq_fragments_finish(c, out);
}

/* ---- reads with calls (kgx_fq_called_reads) ---- */

/* flag[r] = read r has a fragment with a call (fbase = scanned per-(read,
 * frame) fragment counts: read r's fragments are [fbase[6r], fbase[6r+6])) */
__global__ void fq_flag_called_kernel(uint32_t n_reads, const uint32_t *fbase, const uint32_t *call_count,
                                      uint32_t *flag)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_reads)
        return;
    uint32_t any = 0;
    for (uint32_t g = fbase[6 * r]; g < fbase[6 * r + 6] && !any; g++)
        any = call_count[g] != 0;
    flag[r] = any;
}

/* per selected read: its fragment and call totals */
__global__ void fq_called_sizes_kernel(uint32_t n, const uint32_t *reads, const uint32_t *fbase,
                                       const uint32_t *call_count, uint64_t *nfrag, uint64_t *ncall)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n)
        return;
    if (i == n) { /* the scans' tails */
        nfrag[n] = 0;
        ncall[n] = 0;
        return;
    }
    const uint64_t r = reads[i];
    uint64_t c = 0;
    for (uint32_t g = fbase[6 * r]; g < fbase[6 * r + 6]; g++)
        c += call_count[g];
    nfrag[i] = fbase[6 * r + 6] - fbase[6 * r];
    ncall[i] = c;
}

/* per selected read: frame counts, fragment lengths, per-fragment call CSR and the calls */
__global__ void fq_called_fill_kernel(uint32_t n, const uint32_t *reads, const uint32_t *fbase,
                                      const uint32_t *frame_counts, const uint64_t *frag_off,
                                      const uint32_t *call_count, const uint64_t *wbase, const kgx_call *calls,
                                      const uint64_t *fo, const uint64_t *co, uint32_t *out_fc, uint32_t *out_len,
                                      uint64_t *out_coff, kgx_call *out_calls)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t r = reads[i];
    for (int f = 0; f < 6; f++)
        out_fc[6 * i + f] = frame_counts[6 * r + f];
    uint64_t at = fo[i], c = co[i];
    for (uint32_t g = fbase[6 * r]; g < fbase[6 * r + 6]; g++, at++) {
        out_len[at] = (uint32_t)(frag_off[g + 1] - frag_off[g]);
        out_coff[at] = c;
        const kgx_call *src = calls + wbase[g];
        for (uint32_t k = 0; k < call_count[g]; k++)
            out_calls[c++] = src[k];
    }
    if (i == n - 1)
        out_coff[at] = c;
}

int fq_called_reads(kgx_ctx *c, const kgx_fragments *fr, kgx_fq_called *out)
{
    hipStream_t st = c->stream;
    const uint32_t n_reads = fr->n_reads;
    if (c->n_seq != fr->n_fragments || !c->have_hits)
        return fail(KGX_EINVAL, "kgx_fq_called_reads: run kgx_run_device over these fragments first");
    const uint32_t *fbase = c->fq_fbase.as<uint32_t>();
    HIP_TRY(c->fqc_flag.reserve(((uint64_t)n_reads + 1) * 4));
    HIP_TRY(c->fqc_reads.reserve(((uint64_t)n_reads + 1) * 4));
    HIP_TRY(c->fqc_nsel.reserve(8));
    if (n_reads)
        hipLaunchKernelGGL(fq_flag_called_kernel, grid_for(n_reads), dim3(256), 0, st, n_reads, fbase,
                           c->call_count.as<uint32_t>(), c->fqc_flag.as<uint32_t>());
    size_t tb = 0;
    hipcub::CountingInputIterator<uint32_t> ids(0);
    HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, ids, c->fqc_flag.as<uint32_t>(), c->fqc_reads.as<uint32_t>(),
                                          c->fqc_nsel.as<uint32_t>(), (int)n_reads, st));
    HIP_TRY(c->fq_tmp.reserve(tb));
    HIP_TRY(hipcub::DeviceSelect::Flagged(c->fq_tmp.p, tb, ids, c->fqc_flag.as<uint32_t>(),
                                          c->fqc_reads.as<uint32_t>(), c->fqc_nsel.as<uint32_t>(), (int)n_reads, st));
    HIP_TRY(c->h_fqc_n.resize(1));
    HIP_TRY(hipMemcpyAsync(c->h_fqc_n.data(), c->fqc_nsel.p, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint32_t n = n_reads ? c->h_fqc_n[0] : 0;
    HIP_TRY(c->fqc_nfrag.reserve(((uint64_t)n + 1) * 8));
    HIP_TRY(c->fqc_ncall.reserve(((uint64_t)n + 1) * 8));
    HIP_TRY(c->fqc_fo.reserve(((uint64_t)n + 1) * 8));
    HIP_TRY(c->fqc_co.reserve(((uint64_t)n + 1) * 8));
    hipLaunchKernelGGL(fq_called_sizes_kernel, grid_for(n + 1), dim3(256), 0, st, n, c->fqc_reads.as<uint32_t>(),
                       fbase, c->call_count.as<uint32_t>(), c->fqc_nfrag.as<uint64_t>(), c->fqc_ncall.as<uint64_t>());
    size_t t1 = 0, t2 = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, c->fqc_nfrag.as<uint64_t>(), c->fqc_fo.as<uint64_t>(),
                                             (int)(n + 1), st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, c->fqc_ncall.as<uint64_t>(), c->fqc_co.as<uint64_t>(),
                                             (int)(n + 1), st));
    HIP_TRY(c->fq_tmp.reserve(std::max(t1, t2)));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(c->fq_tmp.p, t1, c->fqc_nfrag.as<uint64_t>(), c->fqc_fo.as<uint64_t>(),
                                             (int)(n + 1), st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(c->fq_tmp.p, t2, c->fqc_ncall.as<uint64_t>(), c->fqc_co.as<uint64_t>(),
                                             (int)(n + 1), st));
    HIP_TRY(c->h_fqc_tot.resize(2));
    HIP_TRY(hipMemcpyAsync(c->h_fqc_tot.data(), c->fqc_fo.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(c->h_fqc_tot.data() + 1, c->fqc_co.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t nf = c->h_fqc_tot[0], nc = c->h_fqc_tot[1];
    HIP_TRY(c->fqc_fc.reserve(((uint64_t)n * 6 + 1) * 4));
    HIP_TRY(c->fqc_len.reserve((nf + 1) * 4));
    HIP_TRY(c->fqc_coff.reserve((nf + 1) * 8));
    HIP_TRY(c->fqc_calls.reserve((nc + 1) * sizeof(kgx_call)));
    if (n)
        hipLaunchKernelGGL(fq_called_fill_kernel, grid_for(n), dim3(256), 0, st, n, c->fqc_reads.as<uint32_t>(), fbase,
                           fr->frame_counts, fr->offsets, c->call_count.as<uint32_t>(), c->wbase.as<uint64_t>(),
                           c->calls.as<kgx_call>(), c->fqc_fo.as<uint64_t>(), c->fqc_co.as<uint64_t>(),
                           c->fqc_fc.as<uint32_t>(), c->fqc_len.as<uint32_t>(), c->fqc_coff.as<uint64_t>(),
                           c->fqc_calls.as<kgx_call>());
    else
        HIP_TRY(hipMemsetAsync(c->fqc_coff.p, 0, 8, st));
    HIP_TRY(hipGetLastError());
    HIP_TRY(c->h_fqc_reads.resize(n + 1));
    HIP_TRY(c->h_fqc_fc.resize((uint64_t)n * 6 + 1));
    HIP_TRY(c->h_fqc_fo.resize(n + 1));
    HIP_TRY(c->h_fqc_len.resize(nf + 1));
    HIP_TRY(c->h_fqc_coff.resize(nf + 1));
    HIP_TRY(c->h_fqc_calls.resize(nc + 1));
    if (n) {
        HIP_TRY(hipMemcpyAsync(c->h_fqc_reads.data(), c->fqc_reads.p, (uint64_t)n * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(c->h_fqc_fc.data(), c->fqc_fc.p, (uint64_t)n * 24, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipMemcpyAsync(c->h_fqc_fo.data(), c->fqc_fo.p, ((uint64_t)n + 1) * 8, hipMemcpyDeviceToHost, st));
    if (nf)
        HIP_TRY(hipMemcpyAsync(c->h_fqc_len.data(), c->fqc_len.p, nf * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(c->h_fqc_coff.data(), c->fqc_coff.p, (nf + 1) * 8, hipMemcpyDeviceToHost, st));
    if (nc)
        HIP_TRY(hipMemcpyAsync(c->h_fqc_calls.data(), c->fqc_calls.p, nc * sizeof(kgx_call), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    out->n = n;
    out->reads = c->h_fqc_reads.data();
    out->frame_counts = c->h_fqc_fc.data();
    out->frag_offsets = c->h_fqc_fo.data();
    out->frag_len = c->h_fqc_len.data();
    out->call_offsets = c->h_fqc_coff.data();
    out->calls = c->h_fqc_calls.data();
    return KGX_OK;
}

}  // namespace kgx

extern "C" {

int kgx_fq_fragments_device(kgx_ctx *c, const uint8_t *d_bases, const uint64_t *d_read_offsets, uint32_t n_reads,
                            kgx_fragments *out)
{
    if (!c || !out || (n_reads && (!d_bases || !d_read_offsets)))
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(c->img->device));
    /* the span of the reads bounds the output buffers */
    uint64_t ends[2] = {0, 0};
    if (n_reads) {
        HIP_TRY(c->h_fq_tot.resize(2));
        HIP_TRY(hipMemcpyAsync(c->h_fq_tot.data(), d_read_offsets, 8, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(c->h_fq_tot.data() + 1, d_read_offsets + n_reads, 8, hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        ends[0] = c->h_fq_tot[0];
        ends[1] = c->h_fq_tot[1];
        if (ends[1] < ends[0])
            return fail(KGX_EINVAL, "read offsets not monotone");
    }
    return fq_fragments(c, d_bases, d_read_offsets, n_reads, ends[1] - ends[0], ends[1], out);
}

int kgx_fq_fragments_device_start(kgx_ctx *c, const uint8_t *d_bases, const uint64_t *d_read_offsets,
                                  uint32_t n_reads, uint64_t n_bases)
{
    if (!c || (n_reads && (!d_bases || !d_read_offsets)))
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(c->img->device));
    return fq_fragments_enqueue(c, d_bases, d_read_offsets, n_reads, n_bases, n_bases);
}

int kgx_fq_fragments_finish(kgx_ctx *c, kgx_fragments *out)
{
    if (!c || !out)
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(c->img->device));
    return fq_fragments_finish(c, out);
}

int kgx_fq_called_reads(kgx_ctx *c, const kgx_fragments *fragments, kgx_fq_called *out)
{
    if (!c || !fragments || !out)
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(c->img->device));
    return fq_called_reads(c, fragments, out);
}

int kgx_fq_upload(kgx_ctx *c, const char *bases, const uint64_t *read_offsets, uint32_t n_reads)
{
    if (!c || (n_reads && !read_offsets))
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(c->img->device));
    const uint64_t r0 = n_reads ? read_offsets[0] : 0;
    const uint64_t nb = n_reads ? read_offsets[n_reads] - r0 : 0;
    if (nb && !bases)
        return fail(KGX_EINVAL, "null bases");
    HIP_TRY(c->h_fq_roff.resize((uint64_t)n_reads + 1));
    uint64_t *off = c->h_fq_roff.data();
    off[0] = 0;
    for (uint32_t r = 1; r <= n_reads; r++) {
        if (read_offsets[r] < read_offsets[r - 1])
            return fail(KGX_EINVAL, "read_offsets not monotone");
        off[r] = read_offsets[r] - r0;
    }
    HIP_TRY(c->fq_bases.reserve(nb + 16));
    HIP_TRY(c->fq_roff.reserve(((uint64_t)n_reads + 1) * 8));
    /* the small copy first: copies from all streams share the DMA engine in order */
    HIP_TRY(hipMemcpyAsync(c->fq_roff.p, off, ((uint64_t)n_reads + 1) * 8, hipMemcpyHostToDevice, c->stream));
    if (nb) {
        /* bases in pinned memory (kgx_host_alloc) go by DMA straight from
         * there; others through the context's pinned staging */
        const bool pinned = host_pinned_range(bases + r0, nb);
        if (!pinned) {
            HIP_TRY(c->h_res.resize(nb));
            parallel_memcpy(c->h_res.data(), bases + r0, nb);
        }
        HIP_TRY(hipMemcpyAsync(c->fq_bases.p, pinned ? static_cast<const void *>(bases + r0) : c->h_res.data(), nb,
                               hipMemcpyHostToDevice, c->stream));
    }
    c->fq_up.active = true;
    c->fq_up.n_reads = n_reads;
    c->fq_up.n_bases = nb;
    return KGX_OK;
}

int kgx_fq_fragments_uploaded(kgx_ctx *c, kgx_fragments *out)
{
    if (!c || !out)
        return fail(KGX_EINVAL, "null argument");
    if (!c->fq_up.active)
        return fail(KGX_EINVAL, "no reads uploaded on this context (kgx_fq_upload)");
    HIP_TRY(hipSetDevice(c->img->device));
    c->fq_up.active = false;
    const uint64_t nb = c->fq_up.n_bases;
    return fq_fragments(c, c->fq_bases.as<uint8_t>(), c->fq_roff.as<uint64_t>(), c->fq_up.n_reads, nb, nb, out);
}

int kgx_fq_fragments_uploaded_start(kgx_ctx *c)
{
    if (!c)
        return fail(KGX_EINVAL, "null argument");
    if (!c->fq_up.active)
        return fail(KGX_EINVAL, "no reads uploaded on this context (kgx_fq_upload)");
    HIP_TRY(hipSetDevice(c->img->device));
    c->fq_up.active = false;
    const uint64_t nb = c->fq_up.n_bases;
    return fq_fragments_enqueue(c, c->fq_bases.as<uint8_t>(), c->fq_roff.as<uint64_t>(), c->fq_up.n_reads, nb, nb);
}

int kgx_fq_fragments(kgx_ctx *c, const char *bases, const uint64_t *read_offsets, uint32_t n_reads,
                     kgx_fragments *out)
{
    if (!c || !out || (n_reads && !read_offsets))
        return fail(KGX_EINVAL, "null argument");
    const int rc = kgx_fq_upload(c, bases, read_offsets, n_reads);
    return rc ? rc : kgx_fq_fragments_uploaded(c, out);
}

}  // extern "C"
