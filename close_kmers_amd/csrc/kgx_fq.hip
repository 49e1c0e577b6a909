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
 * Launches: count (one wave per read: fragments and residues per frame),
 * scans, emit (the same waves write each fragment's offset, read, frame and
 * first codon, and the residues, at the scanned bases).
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

/* frame f's k-th residue of the read [b, b+len); b may point into LDS */
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

/* the same over a short read staged in LDS as base classes (0-3, 4 = not
 * ACGTU), with the code table in LDS: every codon is LDS reads only */
struct LdsFrameReader {
    const uint8_t *cls_b; /* LDS: class of base i */
    const char *code;     /* LDS copy of kCode11 */
    uint64_t len;
    int frame;
    __device__ uint64_t n_codons() const
    {
        const uint64_t off = (uint64_t)(frame < 0 ? -frame : frame) - 1;
        return len >= off ? (len - off) / 3 : 0;
    }
    __device__ uint32_t cls(uint64_t i) const
    {
        if (frame > 0)
            return cls_b[i];
        const uint32_t c = cls_b[len - 1 - i];
        return c < 4 ? 3 - c : 4;
    }
    __device__ char aa(uint64_t k) const
    {
        const uint64_t i = (uint64_t)(frame < 0 ? -frame : frame) - 1 + 3 * k;
        const uint32_t e1 = cls(i), e2 = cls(i + 1), e3 = cls(i + 2);
        return code[(e1 | e2 | e3) < 4 ? e1 * 16 + e2 * 4 + e3 : 64];
    }
};

/* per-workgroup LDS tables: base -> class, and the code-11 table */
struct FqTables {
    uint8_t cls[256];
    char code[68];
};
__device__ __forceinline__ void fq_tables_init(FqTables &t)
{
    t.cls[threadIdx.x] = (uint8_t)base_class((uint8_t)threadIdx.x);
    if (threadIdx.x < 65)
        t.code[threadIdx.x] = kCode11[threadIdx.x];
    __syncthreads();
}

__device__ __forceinline__ int frame_of(uint32_t f) { return f < 3 ? (int)f + 1 : -(int)(f - 2); }

/*
 * One wave per read.  When every frame of the read has at most 64 codons
 * (reads up to 194 bases), lane k holds codon k of the frame: the stop mask
 * is a ballot, each lane finds its run's ends with bit scans, and kept
 * residues / run starts are counted and placed with popcounts, so the
 * residue stores of a frame are one contiguous, coalesced stretch.  Longer
 * reads take the serial path: lanes 0..5 walk one frame each.
 */
constexpr uint32_t WAVES_PER_WG = 4;
constexpr uint64_t SHORT_READ = 3 * 64 + 2;

struct FrameFragments { /* one frame's ballot view (lane k = codon k) */
    uint64_t kept;   /* lanes whose residue is in a fragment */
    uint64_t starts; /* lanes that start a fragment */
    char aa;         /* this lane's residue */
};

template <class Reader> __device__ __forceinline__ FrameFragments frame_fragments(const Reader &fr, uint32_t lane)
{
    const uint64_t nc = fr.n_codons();
    const bool valid = lane < nc;
    const char aa = valid ? fr.aa(lane) : '*';
    const uint64_t stop = __ballot(aa == '*') | (nc >= 64 ? 0ull : ~0ull << nc);
    const uint64_t below = lane ? stop & (~0ull >> (64 - lane)) : 0ull;
    const uint32_t run_start = below ? 64u - (uint32_t)__builtin_clzll(below) : 0u; /* after the last stop below */
    const uint64_t at_or_above = stop >> lane;
    const uint32_t run_end = at_or_above ? lane + (uint32_t)__builtin_ctzll(at_or_above) : 64u; /* next stop */
    const bool in_kept_run = valid && aa != '*' && run_end - run_start >= MIN_FRAGMENT;
    FrameFragments r;
    r.kept = __ballot(in_kept_run);
    r.starts = __ballot(in_kept_run && lane == run_start);
    r.aa = aa;
    return r;
}

__device__ __forceinline__ uint32_t popc_below(uint64_t m, uint32_t lane)
{
    return lane ? (uint32_t)__popcll(m & (~0ull >> (64 - lane))) : 0u;
}

/* serial walk of one frame: (fragments, residues); emit when out_res != null */
__device__ void frame_serial(const FrameReader &fr, uint32_t r, uint32_t fi, uint64_t ri, uint32_t &frags,
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

/* a short read -> this wave's LDS slot as base classes, with one aligned
 * dword load per lane (every dword holds a byte of the read, so none reaches
 * past the read's own aligned words); returns the read's first class in LDS.
 * The frames then take their codons from LDS instead of 18 scattered global
 * byte loads and 6 constant-memory table loads per lane. */
constexpr uint32_t LDS_READ_WORDS = (SHORT_READ + 3) / 4 + 1;
__device__ __forceinline__ const uint8_t *stage_read(uint32_t *slot, const uint8_t *b, uint64_t len, uint32_t lane,
                                                     const uint8_t *cls_tab)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(b), a0 = a & ~(uintptr_t)3;
    const uint32_t mis = (uint32_t)(a - a0);
    const uint32_t words = (uint32_t)((mis + len + 3) / 4);
    __builtin_amdgcn_wave_barrier(); /* the previous read's LDS loads are done (grid-stride loop) */
    if (lane < words) { /* 4 bases -> 4 class bytes */
        const uint32_t w = reinterpret_cast<const uint32_t *>(a0)[lane];
        slot[lane] = (uint32_t)cls_tab[w & 0xFF] | (uint32_t)cls_tab[(w >> 8) & 0xFF] << 8 |
                     (uint32_t)cls_tab[(w >> 16) & 0xFF] << 16 | (uint32_t)cls_tab[w >> 24] << 24;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return reinterpret_cast<const uint8_t *>(slot) + mis;
}

__device__ __forceinline__ void count_read(const uint8_t *bases, const uint64_t *read_off, uint64_t r, uint32_t lane,
                                           uint32_t *slot, const FqTables &tabs, uint32_t *n_frag, uint64_t *n_res)
{
    const uint8_t *b = bases + read_off[r];
    const uint64_t len = read_off[r + 1] - read_off[r];
    if (len <= SHORT_READ) {
        const uint8_t *lb = len ? stage_read(slot, b, len, lane, tabs.cls) : tabs.cls;
        for (uint32_t f = 0; f < 6; f++) {
            const FrameFragments ff = frame_fragments(LdsFrameReader{lb, tabs.code, len, frame_of(f)}, lane);
            if (lane == 0) {
                n_frag[r * 6 + f] = (uint32_t)__popcll(ff.starts);
                n_res[r * 6 + f] = (uint64_t)__popcll(ff.kept);
            }
        }
    } else if (lane < 6) {
        uint32_t frags;
        uint64_t res;
        frame_serial(FrameReader{b, len, frame_of(lane)}, (uint32_t)r, 0, 0, frags, res, nullptr, nullptr, nullptr,
                     nullptr, nullptr);
        n_frag[r * 6 + lane] = frags;
        n_res[r * 6 + lane] = res;
    }
}

__global__ __launch_bounds__(256) void fq_count_kernel(const uint8_t *bases, const uint64_t *read_off,
                                                       uint32_t n_reads, uint32_t *n_frag, uint64_t *n_res)
{
    __shared__ uint32_t lds_read[WAVES_PER_WG][LDS_READ_WORDS];
    __shared__ FqTables tabs;
    fq_tables_init(tabs);
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t stride = (uint64_t)gridDim.x * WAVES_PER_WG;
    if (blockIdx.x == 0 && threadIdx.x == 0) { /* the scans' tail */
        n_frag[(uint64_t)n_reads * 6] = 0;
        n_res[(uint64_t)n_reads * 6] = 0;
    }
    for (uint64_t r = (uint64_t)blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6); r < n_reads; r += stride)
        count_read(bases, read_off, r, lane, lds_read[threadIdx.x >> 6], tabs, n_frag, n_res);
}

__device__ __forceinline__ void emit_read(const uint8_t *bases, const uint64_t *read_off, uint64_t r, uint32_t lane,
                                          uint32_t *slot, const FqTables &tabs, const uint32_t *frag_base,
                                          const uint64_t *res_base,
                                          uint8_t *out_res, uint64_t *out_off, uint32_t *out_read, int8_t *out_frame,
                                          uint32_t *out_start)
{
    const uint8_t *b = bases + read_off[r];
    const uint64_t len = read_off[r + 1] - read_off[r];
    if (len <= SHORT_READ) {
        const uint8_t *lb = len ? stage_read(slot, b, len, lane, tabs.cls) : tabs.cls;
        for (uint32_t f = 0; f < 6; f++) {
            const LdsFrameReader fr{lb, tabs.code, len, frame_of(f)};
            const FrameFragments ff = frame_fragments(fr, lane);
            const uint64_t g = r * 6 + f;
            const uint64_t ri = res_base[g] + popc_below(ff.kept, lane);
            if ((ff.kept >> lane) & 1)
                out_res[ri] = (uint8_t)ff.aa;
            if ((ff.starts >> lane) & 1) {
                const uint64_t fi = frag_base[g] + popc_below(ff.starts, lane);
                out_off[fi] = ri;
                out_read[fi] = (uint32_t)r;
                out_frame[fi] = (int8_t)fr.frame;
                out_start[fi] = lane;
            }
        }
    } else if (lane < 6) {
        const uint64_t g = r * 6 + lane;
        uint32_t frags;
        uint64_t res;
        frame_serial(FrameReader{b, len, frame_of(lane)}, (uint32_t)r, frag_base[g], res_base[g], frags, res, out_res,
                     out_off, out_read, out_frame, out_start);
    }
}

/* fragment records (offset, read, frame, first codon) and residues */
__global__ __launch_bounds__(256) void fq_emit_kernel(const uint8_t *bases, const uint64_t *read_off,
                                                      uint32_t n_reads, const uint32_t *frag_base,
                                                      const uint64_t *res_base, uint8_t *out_res, uint64_t *out_off,
                                                      uint32_t *out_read, int8_t *out_frame, uint32_t *out_start)
{
    __shared__ uint32_t lds_read[WAVES_PER_WG][LDS_READ_WORDS];
    __shared__ FqTables tabs;
    fq_tables_init(tabs);
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t stride = (uint64_t)gridDim.x * WAVES_PER_WG;
    for (uint64_t r = (uint64_t)blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6); r < n_reads; r += stride)
        emit_read(bases, read_off, r, lane, lds_read[threadIdx.x >> 6], tabs, frag_base, res_base, out_res, out_off,
                  out_read, out_frame, out_start);
}

__global__ void fq_close_kernel(const uint32_t *frag_base, const uint64_t *res_base, uint64_t n_rf,
                                uint64_t *out_off)
{
    out_off[frag_base[n_rf]] = res_base[n_rf];
}

inline dim3 grid_for(uint64_t n) { return dim3((uint32_t)((n + 255) / 256)); }

}  // namespace

namespace kgx {

/* fragments of the reads in [d_bases, read_off) into the ctx's fq buffers */
int fq_fragments(kgx_ctx *c, const uint8_t *d_bases, const uint64_t *d_read_off, uint32_t n_reads,
                 kgx_fragments *out)
{
    hipStream_t st = c->stream;
    const uint64_t n_rf = (uint64_t)n_reads * 6;
    HIP_TRY(c->fq_nfrag.reserve((n_rf + 1) * 4));
    HIP_TRY(c->fq_nres.reserve((n_rf + 1) * 8));
    HIP_TRY(c->fq_fbase.reserve((n_rf + 1) * 4));
    HIP_TRY(c->fq_rbase.reserve((n_rf + 1) * 8));
    /* one wave per read in a grid-stride loop: workgroups live for many
     * reads, so the dispatcher is not the limit (a read is ~100 cycles of
     * work; a launch per read spent longer starting waves than running them) */
    const dim3 wgs((uint32_t)std::min<uint64_t>((uint64_t)n_reads / WAVES_PER_WG + 1, 256ull * 16));
    if (n_reads)
        hipLaunchKernelGGL(fq_count_kernel, wgs, dim3(256), 0, st, d_bases, d_read_off, n_reads,
                           c->fq_nfrag.as<uint32_t>(), c->fq_nres.as<uint64_t>());
    else {
        HIP_TRY(hipMemsetAsync(c->fq_nfrag.p, 0, 4, st));
        HIP_TRY(hipMemsetAsync(c->fq_nres.p, 0, 8, st));
    }
    size_t tb1 = 0, tb2 = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb1, c->fq_nfrag.as<uint32_t>(), c->fq_fbase.as<uint32_t>(),
                                             (int)(n_rf + 1), st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, c->fq_nres.as<uint64_t>(), c->fq_rbase.as<uint64_t>(),
                                             (int)(n_rf + 1), st));
    HIP_TRY(c->fq_tmp.reserve(std::max(tb1, tb2)));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(c->fq_tmp.p, tb1, c->fq_nfrag.as<uint32_t>(),
                                             c->fq_fbase.as<uint32_t>(), (int)(n_rf + 1), st));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(c->fq_tmp.p, tb2, c->fq_nres.as<uint64_t>(),
                                             c->fq_rbase.as<uint64_t>(), (int)(n_rf + 1), st));
    uint32_t nf = 0;
    uint64_t nr = 0;
    HIP_TRY(hipMemcpyAsync(&nf, c->fq_fbase.as<uint32_t>() + n_rf, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&nr, c->fq_rbase.as<uint64_t>() + n_rf, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(c->fq_res.reserve(nr + 16));
    HIP_TRY(c->fq_off.reserve(((uint64_t)nf + 1) * 8));
    HIP_TRY(c->fq_read.reserve(((uint64_t)nf + 1) * 4));
    HIP_TRY(c->fq_frame.reserve((uint64_t)nf + 1));
    HIP_TRY(c->fq_start.reserve(((uint64_t)nf + 1) * 4));
    if (n_reads)
        hipLaunchKernelGGL(fq_emit_kernel, wgs, dim3(256), 0, st, d_bases, d_read_off, n_reads,
                           c->fq_fbase.as<uint32_t>(), c->fq_rbase.as<uint64_t>(), c->fq_res.as<uint8_t>(),
                           c->fq_off.as<uint64_t>(), c->fq_read.as<uint32_t>(), c->fq_frame.as<int8_t>(),
                           c->fq_start.as<uint32_t>());
    hipLaunchKernelGGL(fq_close_kernel, dim3(1), dim3(1), 0, st, c->fq_fbase.as<uint32_t>(),
                       c->fq_rbase.as<uint64_t>(), n_rf, c->fq_off.as<uint64_t>());
    HIP_TRY(hipGetLastError());
    out->n_reads = n_reads;
    out->n_fragments = nf;
    out->n_residues = nr;
    out->residues = c->fq_res.as<uint8_t>();
    out->offsets = c->fq_off.as<uint64_t>();
    out->read = c->fq_read.as<uint32_t>();
    out->frame = c->fq_frame.as<int8_t>();
    out->frame_counts = c->fq_nfrag.as<uint32_t>();
    return KGX_OK;
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
    return fq_fragments(c, d_bases, d_read_offsets, n_reads, out);
}

int kgx_fq_called_reads(kgx_ctx *c, const kgx_fragments *fragments, kgx_fq_called *out)
{
    if (!c || !fragments || !out)
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(c->img->device));
    return fq_called_reads(c, fragments, out);
}

int kgx_fq_fragments(kgx_ctx *c, const char *bases, const uint64_t *read_offsets, uint32_t n_reads,
                     kgx_fragments *out)
{
    if (!c || !out || (n_reads && !read_offsets))
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(c->img->device));
    const uint64_t r0 = n_reads ? read_offsets[0] : 0;
    const uint64_t nb = n_reads ? read_offsets[n_reads] - r0 : 0;
    if (nb && !bases)
        return fail(KGX_EINVAL, "null bases");
    std::vector<uint64_t> off(n_reads + 1, 0);
    for (uint32_t r = 0; r <= n_reads && n_reads; r++) {
        if (r && read_offsets[r] < read_offsets[r - 1])
            return fail(KGX_EINVAL, "read_offsets not monotone");
        off[r] = read_offsets[r] - r0;
    }
    HIP_TRY(c->fq_bases.reserve(nb + 16));
    HIP_TRY(c->fq_roff.reserve(((uint64_t)n_reads + 1) * 8));
    if (nb) { /* through the context's pinned staging: DMA at link speed */
        HIP_TRY(c->h_res.resize(nb));
        parallel_memcpy(c->h_res.data(), bases + r0, nb);
        HIP_TRY(hipMemcpyAsync(c->fq_bases.p, c->h_res.data(), nb, hipMemcpyHostToDevice, c->stream));
    }
    HIP_TRY(hipMemcpyAsync(c->fq_roff.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, c->stream));
    return fq_fragments(c, c->fq_bases.as<uint8_t>(), c->fq_roff.as<uint64_t>(), n_reads, out);
}

}  // extern "C"
