/* Address-translation cost of random reads over large HBM spans.
 *
 * Allocates one big buffer (hipMalloc, or hipExtMallocWithFlags with
 * hipDeviceMallocContiguous when argv[2] is "contig"), then for spans of
 * 1, 4, 16, 64 GB and the whole buffer measures
 *   - latency: one workgroup of 256 threads, each a chain of dependent random
 *     16-B reads (the next address folds in the loaded value), ns per read --
 *     the call service's probe round;
 *   - one round per launch, and one round every 10 us in a resident
 *     workgroup (the call service's cadence) as 256 single 16-B reads, as
 *     the service's thread loads (293 lines, four 16-B loads each) and by
 *     quads (the same lines, 4 lanes a line), each with the gap sleeping,
 *     spinning, or spinning with a read now and then;
 *   - rate: a grid of 64K waves, 4 lanes per aligned random 64-B line, G lines/s
 *     -- the batch probe's ceiling.
 *
 * Build: hipcc --offload-arch=gfx950 -O3 tools/tlb_probe.cpp -o tools/tlb_probe
 *        -Lclose_kmers_amd -lkgx -Wl,-rpath,'$ORIGIN/../close_kmers_amd'
 *
 * "frag" allocates the buffer after the image build's allocations instead,
 * "first" before them;
 * "kgx" reads a synthetic image's AOS24 table built by libkgx.
 *
 *     tlb_probe GB [contig|frag|first|kgx]
 */
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>

#include "../include/kgx.h"

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));          \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__global__ __launch_bounds__(256) void chain_kernel(const uint4 *buf, uint64_t n16, uint32_t rounds, uint32_t fold,
                                                    uint64_t *ns_out, uint64_t *sink)
{
    const uint32_t t = threadIdx.x;
    uint64_t s = mix(0x9e3779b97f4a7c15ull * (t + 1) + blockIdx.x + ((uint64_t)fold << 32)); /* fold: a fresh start per launch */
    uint32_t acc = 0;
    __syncthreads();
    const uint64_t t0 = wall_clock64();
    for (uint32_t r = 0; r < rounds; r++) {
        const uint4 v = buf[s % n16];
        acc += v.x;
        s = mix(s + (v.y & fold)); /* fold = 0 at run time: a real dependency */
        __syncthreads();
    }
    const uint64_t t1 = wall_clock64();
    if (t == 0)
        ns_out[0] = (t1 - t0) * 10; /* wall_clock64 ticks at 100 MHz */
    if (acc == 0xFFFFFFFFu)
        sink[0] = acc;
}

/* one resident workgroup: every gap_ticks (100 MHz) one round of random
 * reads (svc 0: 256 16-B reads; 1: the call service's thread loads, 293 lines
 * as four 16-B loads each; 2: the same lines by quads), its duration summed
 * -- the call service's cadence */
__global__ __launch_bounds__(256) void resident_kernel(const uint4 *buf, uint64_t n16, uint32_t rounds, uint32_t gap_ticks,
                                                       uint32_t svc, uint32_t idle, uint64_t *ns_out, uint64_t *sink)
{
    const uint32_t t = threadIdx.x;
    uint32_t acc = 0;
    uint64_t total = 0;
    for (uint32_t r = 0; r < rounds; r++) {
        const uint64_t w0 = wall_clock64();
        /* the gap: 0 sleeping, 1 spinning, 2 spinning with one random read
         * per wave every ~1 us */
        uint32_t k = 0;
        while (wall_clock64() - w0 < gap_ticks) {
            if (idle == 0)
                __builtin_amdgcn_s_sleep(2);
            else if (idle == 2 && (++k & 63) == 0 && (t & 63) == 0)
                acc += buf[mix(w0 + k + t) % n16].x;
        }
        __syncthreads();
        const uint64_t s = mix(0x9e3779b97f4a7c15ull * (t + 1) + ((uint64_t)r << 32) + 12345);
        const uint64_t t0 = wall_clock64();
        if (svc == 2) {
            /* by quads: lanes 4g..4g+3 read window g + 64 j's line, 16 B each,
             * in one instruction per j */
            const uint64_t n_lines = n16 / 4;
            const uint32_t g = t >> 2, sub = t & 3;
            uint4 v[5];
#pragma unroll
            for (uint32_t j = 0; j < 5; j++) {
                const uint32_t w = g + 64 * j;
                const uint64_t line = mix(0x9e3779b97f4a7c15ull * (w + 1) + ((uint64_t)r << 32) + 777) % n_lines;
                v[j] = w < 293 ? buf[4 * line + sub] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (uint32_t j = 0; j < 5; j++)
                acc += v[j].x;
        } else if (svc) {
            /* the call service's round: windows t and t + 256 of 293, each an
             * aligned 64-B line read as four 16-B loads */
            const uint64_t n_lines = n16 / 4;
            const uint64_t l0 = s % n_lines, l1 = mix(s + 1) % n_lines;
            const bool two = t + 256 < 293;
            uint4 v[8];
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) {
                v[q] = buf[4 * l0 + q];
                if (two)
                    v[4 + q] = buf[4 * l1 + q];
            }
#pragma unroll
            for (uint32_t q = 0; q < 4; q++)
                acc += v[q].x + (two ? v[4 + q].x : 0u);
        } else {
            const uint4 v = buf[s % n16];
            acc += v.x;
        }
        __syncthreads_or(acc == 0xFFFFFFFFu);
        total += wall_clock64() - t0;
    }
    if (t == 0)
        ns_out[0] = total * 10;
    if (acc == 0xFFFFFFFFu)
        sink[0] = acc;
}

__global__ __launch_bounds__(256) void line_kernel(const uint4 *buf, uint64_t n_lines, uint32_t per_quad, uint64_t *sink)
{
    const uint32_t t = blockIdx.x * 256 + threadIdx.x, q = t >> 2, l = t & 3;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < per_quad; i += 4) {
        uint4 v[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            const uint64_t line = mix(((uint64_t)q << 20) + i + j) % n_lines;
            v[j] = buf[4 * line + l];
        }
#pragma unroll
        for (uint32_t j = 0; j < 4; j++)
            acc += v[j].x ^ v[j].w;
    }
    if (acc == 0xFFFFFFFFu)
        sink[0] = acc;
}

int main(int argc, char **argv)
{
    const uint64_t gb = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 100;
    const bool contig = argc > 2 && std::strcmp(argv[2], "contig") == 0;
    const bool frag = argc > 2 && std::strcmp(argv[2], "frag") == 0;
    const bool alloc_first = argc > 2 && std::strcmp(argv[2], "first") == 0; /* the buffer before the build's */
    const uint64_t bytes = gb << 30;
    uint4 *buf = nullptr;
    void *keep = nullptr;
    if (frag) {
        /* the image build's history: an 85-GB AOS24 table, its 57-GB PACKED16
         * copy, the AOS24 table freed, then the line index */
        void *aos = nullptr;
        CHECK(hipMalloc(&aos, 85ull << 30));
        CHECK(hipMemset(aos, 0, 85ull << 30));
        CHECK(hipMalloc(&keep, 57ull << 30));
        CHECK(hipMemset(keep, 0, 57ull << 30));
        CHECK(hipFree(aos));
    }
    const bool via_kgx = argc > 2 && std::strcmp(argv[2], "kgx") == 0;
    hipError_t ae = hipSuccess;
    kgx_image *img = nullptr;
    uint64_t avail = bytes; /* the buffer's bytes: every read stays below */
    if (via_kgx) {
        /* the synthetic image's own AOS24 table (gb = its 24-B buckets in GiB) */
        const uint64_t num_sigs = bytes / 24;
        uint64_t stored = 0;
        if (kgx_image_build_synthetic(num_sigs / 4, num_sigs, 0, &img, &stored) != 0) {
            std::printf("{\"error\": \"%s\"}\n", kgx_last_error());
            return 1;
        }
        /* the build packs the table to PACKED16: back to AOS24, whose
         * device pointer kgx_image_table returns */
        if (kgx_image_set_layout(img, KGX_LAYOUT_AOS24) != 0) {
            std::printf("{\"error\": \"%s\"}\n", kgx_last_error());
            return 1;
        }
        buf = (uint4 *)kgx_image_table(img);
        avail = num_sigs * 24;
        if (!buf) {
            std::printf("{\"error\": \"no AOS24 table\"}\n");
            return 1;
        }
    } else {
        ae = contig ? hipExtMallocWithFlags((void **)&buf, bytes, hipDeviceMallocContiguous)
                    : hipMalloc((void **)&buf, bytes);
        if (ae == hipSuccess && alloc_first) {
            void *aos = nullptr;
            CHECK(hipMalloc(&aos, 85ull << 30));
            CHECK(hipMemset(aos, 0, 85ull << 30));
            CHECK(hipMalloc(&keep, 57ull << 30));
            CHECK(hipMemset(keep, 0, 57ull << 30));
            CHECK(hipFree(aos));
        }
    }
    if (ae != hipSuccess) {
        std::printf("{\"gb\": %llu, \"contig\": %d, \"alloc\": \"%s\"}\n", (unsigned long long)gb, contig,
                    hipGetErrorString(ae));
        return 0;
    }
    if (!via_kgx)
        CHECK(hipMemset(buf, 0, bytes));
    uint64_t *d_ns = nullptr, *sink = nullptr;
    CHECK(hipMalloc((void **)&d_ns, 64));
    CHECK(hipMalloc((void **)&sink, 64));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::printf("{\"gb\": %llu, \"contig\": %d, \"frag\": %d, \"spans\": [", (unsigned long long)gb, contig, frag);
    const uint64_t spans[] = {1, 4, 16, 64, gb};
    bool first = true;
    uint64_t last = 0;
    for (uint64_t sg : spans) {
        if (sg > gb || sg == last)
            continue;
        last = sg;
        const uint64_t n16 = std::min(sg << 30, avail) / 16;
        const uint32_t rounds = 200;
        uint64_t ns = 0;
        double lat = 1e30;
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(chain_kernel, dim3(1), dim3(256), 0, 0, buf, n16, rounds, 0u, d_ns, sink);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(&ns, d_ns, 8, hipMemcpyDeviceToHost));
            lat = std::min(lat, (double)ns / rounds);
        }
        double lat1 = 0;
        for (int rep = 0; rep < 200; rep++) {
            hipLaunchKernelGGL(chain_kernel, dim3(1), dim3(256), 0, 0, buf, n16, 1u, (uint32_t)rep, d_ns, sink);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(&ns, d_ns, 8, hipMemcpyDeviceToHost));
            lat1 += (double)ns / 200;
        }
        /* [pattern: single, svc threads, quads][idle: sleep, spin, spin + reads] */
        double res[3][3];
        for (uint32_t pat = 0; pat < 3; pat++)
            for (uint32_t idle = 0; idle < 3; idle++) {
                hipLaunchKernelGGL(resident_kernel, dim3(1), dim3(256), 0, 0, buf, n16, 200u, 1000u, pat, idle, d_ns,
                                   sink);
                CHECK(hipDeviceSynchronize());
                CHECK(hipMemcpy(&ns, d_ns, 8, hipMemcpyDeviceToHost));
                res[pat][idle] = (double)ns / 200;
            }
        const uint32_t blocks = 16384, per_quad = 64;
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CHECK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(line_kernel, dim3(blocks), dim3(256), 0, 0, buf, n16 / 4, per_quad, sink);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        const double lines = (double)blocks * 64 * per_quad;
        std::printf("%s{\"span_gb\": %llu, \"chain_ns_per_read\": %.1f, \"one_round_ns\": %.1f, \"resident_ns\": {\"single\": [%.0f, %.0f, %.0f], \"svc\": [%.0f, %.0f, %.0f], \"quad\": [%.0f, %.0f, %.0f]}, "
                    "\"lines_g_per_s\": %.2f}",
                    first ? "" : ", ", (unsigned long long)sg, lat, lat1, res[0][0], res[0][1], res[0][2], res[1][0],
                    res[1][1], res[1][2], res[2][0], res[2][1], res[2][2], lines / (best * 1e-3) / 1e9);
        first = false;
        std::fflush(stdout);
    }
    std::printf("]}\n");
    if (img)
        kgx_image_close(img);
    else
        CHECK(hipFree(buf));
    if (keep)
        CHECK(hipFree(keep));
    return 0;
}
