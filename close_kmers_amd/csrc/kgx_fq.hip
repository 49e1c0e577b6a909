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
 * Launches: count (one thread per (read, frame): fragments and residues),
 * scans, emit (the same threads write each fragment's offset, read, frame
 * and first codon at the scanned bases), fill (one wave per fragment writes
 * its residues, consecutive lanes on consecutive bytes).
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

/* frame f's k-th residue of the read [b, b+len) */
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

__global__ void fq_count_kernel(const uint8_t *bases, const uint64_t *read_off, uint32_t n_reads,
                                uint32_t *n_frag, uint64_t *n_res)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (uint64_t)n_reads * 6) {
        if (g == (uint64_t)n_reads * 6) {
            n_frag[g] = 0;
            n_res[g] = 0;
        }
        return;
    }
    const uint32_t r = (uint32_t)(g / 6), f = (uint32_t)(g % 6);
    const FrameReader fr{bases + read_off[r], read_off[r + 1] - read_off[r], frame_of(f)};
    const uint64_t nc = fr.n_codons();
    uint32_t frags = 0;
    uint64_t res = 0, run = 0;
    for (uint64_t k = 0; k <= nc; k++) {
        if (k == nc || fr.aa(k) == '*') {
            if (run >= MIN_FRAGMENT) {
                frags++;
                res += run;
            }
            run = 0;
        } else {
            run++;
        }
    }
    n_frag[g] = frags;
    n_res[g] = res;
}

/* fragment records (offset, read, frame, first codon); residues by fq_fill */
__global__ void fq_emit_kernel(const uint8_t *bases, const uint64_t *read_off, uint32_t n_reads,
                               const uint32_t *frag_base, const uint64_t *res_base, uint64_t *out_off,
                               uint32_t *out_read, int8_t *out_frame, uint32_t *out_start)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (uint64_t)n_reads * 6)
        return;
    const uint32_t r = (uint32_t)(g / 6), f = (uint32_t)(g % 6);
    const FrameReader fr{bases + read_off[r], read_off[r + 1] - read_off[r], frame_of(f)};
    const uint64_t nc = fr.n_codons();
    uint32_t fi = frag_base[g];
    uint64_t ri = res_base[g];
    uint64_t run = 0, start = 0;
    for (uint64_t k = 0; k <= nc; k++) {
        if (k == nc || fr.aa(k) == '*') {
            if (run >= MIN_FRAGMENT) {
                out_off[fi] = ri;
                out_read[fi] = r;
                out_frame[fi] = (int8_t)fr.frame;
                out_start[fi] = (uint32_t)start;
                fi++;
                ri += run;
            }
            run = 0;
            start = k + 1;
        } else {
            run++;
        }
    }
}

/* one wave per fragment (grid-stride): consecutive lanes write consecutive
 * residues, so the byte stores coalesce */
__global__ __launch_bounds__(256) void fq_fill_kernel(const uint8_t *bases, const uint64_t *read_off,
                                                      uint32_t n_frag, const uint64_t *off, const uint32_t *rd,
                                                      const int8_t *frm, const uint32_t *start, uint8_t *out_res)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    for (uint64_t f = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); f < n_frag; f += waves) {
        const uint32_t r = rd[f];
        const FrameReader fr{bases + read_off[r], read_off[r + 1] - read_off[r], frm[f]};
        const uint64_t o = off[f], len = off[f + 1] - o, s = start[f];
        for (uint64_t k = lane; k < len; k += 64)
            out_res[o + k] = (uint8_t)fr.aa(s + k);
    }
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
    hipLaunchKernelGGL(fq_count_kernel, grid_for(n_rf + 1), dim3(256), 0, st, d_bases, d_read_off, n_reads,
                       c->fq_nfrag.as<uint32_t>(), c->fq_nres.as<uint64_t>());
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
    hipLaunchKernelGGL(fq_emit_kernel, grid_for(n_rf), dim3(256), 0, st, d_bases, d_read_off, n_reads,
                       c->fq_fbase.as<uint32_t>(), c->fq_rbase.as<uint64_t>(), c->fq_off.as<uint64_t>(),
                       c->fq_read.as<uint32_t>(), c->fq_frame.as<int8_t>(), c->fq_start.as<uint32_t>());
    hipLaunchKernelGGL(fq_close_kernel, dim3(1), dim3(1), 0, st, c->fq_fbase.as<uint32_t>(),
                       c->fq_rbase.as<uint64_t>(), n_rf, c->fq_off.as<uint64_t>());
    if (nf)
        hipLaunchKernelGGL(fq_fill_kernel, dim3((uint32_t)std::min<uint64_t>(((uint64_t)nf + 3) / 4, 65536)),
                           dim3(256), 0, st, d_bases, d_read_off, nf, c->fq_off.as<uint64_t>(),
                           c->fq_read.as<uint32_t>(), c->fq_frame.as<int8_t>(), c->fq_start.as<uint32_t>(),
                           c->fq_res.as<uint8_t>());
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
    if (nb)
        HIP_TRY(hipMemcpyAsync(c->fq_bases.p, bases + r0, nb, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->fq_roff.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, c->stream));
    return fq_fragments(c, c->fq_bases.as<uint8_t>(), c->fq_roff.as<uint64_t>(), n_reads, out);
}

}  // extern "C"
