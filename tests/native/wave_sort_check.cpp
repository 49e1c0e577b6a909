/*
 * wave_sort_check -- lstd_sort_wave64 / lstd_sort_wave<4> (kgx_wave_sort.h:
 * libstdc++'s std::sort of at most 64 / 256 elements, replayed by one wave in
 * LDS, as the call service picks them) against the serial
 * replay lstd_sort (kgx_lstd.h, itself checked against libstdc++ by
 * lstd_check.cpp) on OTU pairs sorted by count (less_second, kguts.h:214-218),
 * the call service's use.  One workgroup of one wave runs the cases one after
 * another and times each sort with the device wall clock.
 *
 *   wave_sort_check CASES SEED
 *
 * Runs lstd_sort_wave64 (pairs in LDS) and lstd_sort_wave64_reg (pairs in
 * registers) in turn; prints "ok CASES <variant>" and one JSON line of mean ns
 * per sort by size band for each; exit 1 on the first mismatch.
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <random>
#include <vector>

#include "kgx_internal.h"
#include "kgx_wave_sort.h"

using namespace kgx;

struct ByCount {
    __host__ __device__ bool operator()(const kgx_otu &l, const kgx_otu &r) const { return r.count < l.count; }
};

__global__ __launch_bounds__(64) void wave_sort_kernel(const kgx_otu *in, const uint32_t *n_of, uint32_t cases,
                                                       kgx_otu *out, uint64_t *ns, int reg)
{
    __shared__ kgx_otu a[256];
    __shared__ kgx_otu bl[256], br[256]; /* bl: also lstd_sort_wave64's 192 elements of scratch */
    __shared__ uint8_t seg[256];
    __shared__ LstdPart st[64];
    const uint32_t lane = threadIdx.x;
    for (uint32_t c = 0; c < cases; c++) {
        const uint32_t n = n_of[c];
        for (uint32_t i = lane; i < n; i += 64)
            a[i] = in[256 * c + i];
        wave_lds_sync();
        const uint64_t t0 = wall_clock64();
        if (n <= 64 && reg)
            lstd_sort_wave64_reg(a, n, ByCount{}, bl, br);
        else if (n <= 64)
            lstd_sort_wave64(a, n, ByCount{}, bl, st); /* bl, br: its 192 elements of scratch */
        else
            lstd_sort_wave<4>(a, n, ByCount{}, bl, br, seg, st);
        const uint64_t t1 = wall_clock64();
        for (uint32_t i = lane; i < n; i += 64)
            out[256 * c + i] = a[i];
        if (lane == 0)
            ns[c] = (t1 - t0) * 10; /* 100 MHz */
        wave_lds_sync();
    }
}

/* the register sort as the call service runs it: wave 0 of a 256-thread
 * workgroup sorts while waves 1-3 wait at the barrier, with most of the LDS
 * allocated (`big`: 96 KiB more) */
__global__ __launch_bounds__(256) void wave_sort_wg_kernel(const kgx_otu *in, const uint32_t *n_of, uint32_t cases,
                                                           kgx_otu *out, uint64_t *ns, int big, uint64_t *clk)
{
    extern __shared__ uint8_t dyn[];
    __shared__ kgx_otu a[256], bl[256], br[256];
    const uint32_t t = threadIdx.x;
    if (big && t == 0)
        dyn[0] = 0;
    for (uint32_t c = 0; c < cases; c++) {
        const uint32_t n = n_of[c];
        for (uint32_t i = t; i < n; i += 256)
            a[i] = in[256 * c + i];
        __syncthreads();
        if (t < 64) {
            const uint64_t t0 = wall_clock64(), k0 = __builtin_amdgcn_s_memtime();
            lstd_sort_wave64_reg(a, n, ByCount{}, bl, br);
            const uint64_t t1 = wall_clock64(), k1 = __builtin_amdgcn_s_memtime();
            if (t == 0) {
                ns[c] = (t1 - t0) * 10;
                clk[c] = k1 - k0;
            }
        }
        __syncthreads();
        for (uint32_t i = t; i < n; i += 256)
            out[256 * c + i] = a[i];
        __syncthreads();
    }
}

/* ... and with the service's own layout: the pairs at the start of a
 * 32-KiB uint4 record array (hrec), the scratch 256 and 320 pairs past them,
 * the comparator a lambda */
__global__ __launch_bounds__(256) void wave_sort_svc_layout_kernel(const kgx_otu *in, const uint32_t *n_of,
                                                                   uint32_t cases, kgx_otu *out, uint64_t *ns)
{
    __shared__ uint4 hrec[256 * 8];
    kgx_otu *o = reinterpret_cast<kgx_otu *>(hrec);
    const uint32_t t = threadIdx.x;
    const auto by_count = [](const kgx_otu &lhs, const kgx_otu &rhs) { return rhs.count < lhs.count; };
    for (uint32_t c = 0; c < cases; c++) {
        const uint32_t n = n_of[c];
        for (uint32_t i = t; i < n; i += 256)
            o[i] = in[256 * c + i];
        __syncthreads();
        if (t < 64) {
            const uint64_t t0 = wall_clock64();
            lstd_sort_wave64_reg(o, n, by_count, o + 256, o + 320);
            const uint64_t t1 = wall_clock64();
            if (t == 0)
                ns[c] = (t1 - t0) * 10;
        }
        __syncthreads();
        for (uint32_t i = t; i < n; i += 256)
            out[256 * c + i] = o[i];
        __syncthreads();
    }
}

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            return 2;                                                              \
        }                                                                          \
    } while (0)

int main(int argc, char **argv)
{
    const uint32_t cases = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 2000;
    std::mt19937_64 rng(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1);
    std::vector<kgx_otu> in(256 * (size_t)cases), want(256 * (size_t)cases), got(256 * (size_t)cases);
    std::vector<uint32_t> n_of(cases);
    for (uint32_t c = 0; c < cases; c++) {
        const uint32_t n = c % 4 == 3 ? 65 + (uint32_t)(rng() % 192) : 2 + (uint32_t)(rng() % 63);
        /* counts over a narrow range (ties everywhere, as a call's OTU tallies
         * have) or a wide one; OTU ids ascending, as the map leaves them */
        const uint32_t span = c % 3 == 0 ? 3 : c % 3 == 1 ? 8 : 1000;
        n_of[c] = n;
        for (uint32_t i = 0; i < n; i++)
            in[256 * (size_t)c + i] = kgx_otu{(int32_t)i * 7 - 5, 1 + (int32_t)(rng() % span)};
        for (uint32_t i = 0; i < n; i++)
            want[256 * (size_t)c + i] = in[256 * (size_t)c + i];
        lstd_sort(want.data() + 256 * (size_t)c, (int64_t)n, ByCount{});
    }
    kgx_otu *d_in = nullptr, *d_out = nullptr;
    uint32_t *d_n = nullptr;
    uint64_t *d_ns = nullptr;
    CHECK(hipMalloc(&d_in, in.size() * sizeof(kgx_otu)));
    CHECK(hipMalloc(&d_out, in.size() * sizeof(kgx_otu)));
    CHECK(hipMalloc(&d_n, cases * sizeof(uint32_t)));
    CHECK(hipMalloc(&d_ns, cases * sizeof(uint64_t)));
    CHECK(hipMemcpy(d_in, in.data(), in.size() * sizeof(kgx_otu), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_n, n_of.data(), cases * sizeof(uint32_t), hipMemcpyHostToDevice));
    /* variant 0: lstd_sort_wave64 (elements in LDS), 1: lstd_sort_wave64_reg
     * (elements in registers); past 64 both use lstd_sort_wave<4> */
    const uint32_t bands[] = {2, 9, 17, 33, 65, 129, 257};
    for (int reg = 0; reg < 2; reg++) {
        hipLaunchKernelGGL(wave_sort_kernel, dim3(1), dim3(64), 0, 0, d_in, d_n, cases, d_out, d_ns, reg);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        std::vector<uint64_t> ns(cases);
        CHECK(hipMemcpy(got.data(), d_out, got.size() * sizeof(kgx_otu), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(ns.data(), d_ns, cases * sizeof(uint64_t), hipMemcpyDeviceToHost));
        for (uint32_t c = 0; c < cases; c++)
            for (uint32_t i = 0; i < n_of[c]; i++) {
                const kgx_otu &g = got[256 * (size_t)c + i], &w = want[256 * (size_t)c + i];
                if (g.otu_index != w.otu_index || g.count != w.count) {
                    std::printf("mismatch (variant %d) case %u (n %u) at %u: (%d,%d) vs (%d,%d)\n", reg, c,
                                n_of[c], i, g.otu_index, g.count, w.otu_index, w.count);
                    return 1;
                }
            }
        /* mean ns per sort by size band */
        std::printf("ok %u %s\n{", cases, reg ? "registers" : "lds");
        for (int b = 0; b < 6; b++) {
            double t = 0;
            uint32_t k = 0;
            for (uint32_t c = 0; c < cases; c++)
                if (n_of[c] >= bands[b] && n_of[c] < bands[b + 1]) {
                    t += (double)ns[c];
                    k++;
                }
            std::printf("%s\"n%u-%u_ns\": %.0f", b ? ", " : "", bands[b], bands[b + 1] - 1, k ? t / k : 0.0);
        }
        std::printf("}\n");
    }
    /* the same register sorts of 33-64 pairs, one launch each: the first
     * (only) sort of a dispatch, as a call of the service meets it, against
     * the loop's warm instruction cache above */
    {
        double t = 0;
        uint32_t k = 0;
        for (uint32_t c = 0; c < cases && k < 200; c++) {
            if (n_of[c] < 33 || n_of[c] > 64)
                continue;
            hipLaunchKernelGGL(wave_sort_kernel, dim3(1), dim3(64), 0, 0, d_in + 256 * (size_t)c, d_n + c, 1u,
                               d_out + 256 * (size_t)c, d_ns + c, 1);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            uint64_t v = 0;
            CHECK(hipMemcpy(&v, d_ns + c, sizeof v, hipMemcpyDeviceToHost));
            t += (double)v;
            k++;
        }
        std::printf("{\"cold_n33-64_ns\": %.0f, \"cold_sorts\": %u}\n", k ? t / k : 0.0, k);
    }
    /* lists shaped like the service's 36-OTU calls (tests/perf_svc_otu_phases.py,
     * mod 97): 36 pairs whose counts are ~150 hits dealt over them at random */
    {
        const uint32_t K = std::min<uint32_t>(cases, 500);
        std::vector<kgx_otu> in36(256 * (size_t)K), want36(256 * (size_t)K);
        std::vector<uint32_t> n36(K, 36);
        for (uint32_t c = 0; c < K; c++) {
            int cnt[36] = {0};
            for (int h = 0; h < (c & 1 ? 292 : 150); h++)
                cnt[rng() % 36]++;
            for (uint32_t i = 0; i < 36; i++)
                in36[256 * (size_t)c + i] = kgx_otu{(int32_t)i * 97 + 3, cnt[i]};
            std::copy(in36.begin() + 256 * (size_t)c, in36.begin() + 256 * (size_t)c + 36,
                      want36.begin() + 256 * (size_t)c);
            lstd_sort(want36.data() + 256 * (size_t)c, (int64_t)36, ByCount{});
        }
        CHECK(hipMemcpy(d_in, in36.data(), in36.size() * sizeof(kgx_otu), hipMemcpyHostToDevice));
        CHECK(hipMemcpy(d_n, n36.data(), K * sizeof(uint32_t), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(wave_sort_kernel, dim3(1), dim3(64), 0, 0, d_in, d_n, K, d_out, d_ns, 1);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        std::vector<uint64_t> ns(K);
        std::vector<kgx_otu> got36(in36.size());
        CHECK(hipMemcpy(got36.data(), d_out, got36.size() * sizeof(kgx_otu), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(ns.data(), d_ns, K * sizeof(uint64_t), hipMemcpyDeviceToHost));
        double t = 0;
        for (uint32_t c = 0; c < K; c++) {
            t += (double)ns[c];
            for (uint32_t i = 0; i < 36; i++) {
                const kgx_otu &g = got36[256 * (size_t)c + i], &w = want36[256 * (size_t)c + i];
                if (g.otu_index != w.otu_index || g.count != w.count) {
                    std::printf("mismatch (36-OTU lists) case %u at %u\n", c, i);
                    return 1;
                }
            }
        }
        std::printf("{\"svc36_ns\": %.0f, \"svc36_sorts\": %u}\n", t / K, K);
        for (int big = 0; big < 2; big++) {
            uint64_t *d_clk = nullptr;
            CHECK(hipMalloc(&d_clk, K * sizeof(uint64_t)));
            hipLaunchKernelGGL(wave_sort_wg_kernel, dim3(1), dim3(256), big ? 96 * 1024 : 0, 0, d_in, d_n, K, d_out,
                               d_ns, big, d_clk);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            std::vector<uint64_t> clk(K);
            CHECK(hipMemcpy(ns.data(), d_ns, K * sizeof(uint64_t), hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(clk.data(), d_clk, K * sizeof(uint64_t), hipMemcpyDeviceToHost));
            (void)hipFree(d_clk);
            double tw = 0, cw = 0;
            for (uint32_t c = 0; c < K; c++) {
                tw += (double)ns[c];
                cw += (double)clk[c];
            }
            std::printf("{\"svc36_wg256_%s_ns\": %.0f, \"clock_mhz\": %.0f}\n", big ? "lds96k" : "lds", tw / K,
                        cw / tw * 1e3);
        }
        hipLaunchKernelGGL(wave_sort_svc_layout_kernel, dim3(1), dim3(256), 0, 0, d_in, d_n, K, d_out, d_ns);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(ns.data(), d_ns, K * sizeof(uint64_t), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(got36.data(), d_out, got36.size() * sizeof(kgx_otu), hipMemcpyDeviceToHost));
        double tl = 0, to = 0;
        for (uint32_t c = 0; c < K; c++) {
            tl += (double)ns[c];
            to += (c & 1) ? (double)ns[c] : 0.0;
            for (uint32_t i = 0; i < 36; i++)
                if (got36[256 * (size_t)c + i].otu_index != want36[256 * (size_t)c + i].otu_index ||
                    got36[256 * (size_t)c + i].count != want36[256 * (size_t)c + i].count) {
                    std::printf("mismatch (service layout) case %u at %u\n", c, i);
                    return 1;
                }
        }
        std::printf("{\"svc36_svc_layout_ns\": %.0f, \"hits292_ns\": %.0f, \"hits150_ns\": %.0f}\n", tl / K,
                    to / (K / 2), (tl - to) / (K - K / 2));
    }
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    (void)hipFree(d_n);
    (void)hipFree(d_ns);
    return 0;
}
