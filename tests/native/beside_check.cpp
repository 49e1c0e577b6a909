/*
 * beside_check -- a server whose pool mixes per-sequence calls and chunk
 * batches on one image (threadpool.cc:18-60: some workers run
 * process_aa_seq per sequence, another a handler's whole chunk): T threads
 * call the resident service (kgx_svc_call) while one thread runs
 * kgx_process_batch on its own context, over and over.  Native threads, so
 * the clocks time the GPU paths, not a Python harness's GIL
 * (tests/test_gpu_svc.py::test_svc_beside_batches_on_the_same_image).
 *
 *   beside_check N_KEYS NUM_SIGS QUERIES.bin T SECONDS
 *
 * QUERIES.bin: uint64 n, uint64 offsets[n+1], residues.  The image is the
 * bench's synthetic one (N_KEYS distinct keys, bench.py C2).  Every batch run
 * beside the service must equal the batch run alone, byte for byte; every
 * service answer must equal its sequence's slice of that batch.  Prints one
 * JSON line; exit 1 on a mismatch or an ABI error.
 *
 * Evidence for the tail: per batch the batch thread's
 * involuntary / voluntary context switches (getrusage RUSAGE_THREAD) and the
 * split of its time between kgx_process_batch and copying the result; for
 * the slowest batches the service calls that overlapped them (count, the
 * longest) -- so a slow batch can be told apart as host preemption, a
 * service-side stall, or the device.
 */
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include <sys/resource.h>

#include "kgx.h"

using clk = std::chrono::steady_clock;

static double pct(std::vector<double> v, double p)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[std::min(v.size() - 1, (size_t)(p / 100.0 * (double)v.size()))];
}

struct Batch {
    std::vector<uint64_t> hoff, coff;
    std::vector<kgx_hit> hits;
    std::vector<kgx_call> calls;
    bool operator==(const Batch &o) const
    {
        return hoff == o.hoff && coff == o.coff && hits.size() == o.hits.size() && calls.size() == o.calls.size() &&
               !std::memcmp(hits.data(), o.hits.data(), hits.size() * sizeof(kgx_hit)) &&
               !std::memcmp(calls.data(), o.calls.data(), calls.size() * sizeof(kgx_call));
    }
};

int main(int argc, char **argv)
{
    if (argc < 6) {
        std::fprintf(stderr, "usage: beside_check N_KEYS NUM_SIGS QUERIES.bin T SECONDS\n");
        return 2;
    }
    const uint64_t n_keys = std::strtoull(argv[1], nullptr, 10), num_sigs = std::strtoull(argv[2], nullptr, 10);
    const int T = std::max(1, std::atoi(argv[4]));
    const double seconds = std::atof(argv[5]);
    std::ifstream in(argv[3], std::ios::binary);
    uint64_t n = 0;
    in.read(reinterpret_cast<char *>(&n), 8);
    std::vector<uint64_t> off(n + 1);
    in.read(reinterpret_cast<char *>(off.data()), (std::streamsize)(8 * (n + 1)));
    std::string res(off[n], '\0');
    in.read(&res[0], (std::streamsize)res.size());
    if (!in || n == 0) {
        std::fprintf(stderr, "beside_check: short query file\n");
        return 2;
    }
    kgx_image *img = nullptr;
    uint64_t entries = 0;
    kgx_ctx *ctx = nullptr;
    if (kgx_image_build_synthetic_distinct(n_keys, n_keys, num_sigs, 0, &img, &entries) != KGX_OK ||
        kgx_ctx_create(img, &ctx) != KGX_OK) {
        std::fprintf(stderr, "beside_check: %s\n", kgx_last_error());
        return 1;
    }
    kgx_params prm;
    kgx_params_default(&prm);
    const uint32_t want = KGX_WANT_HITS | KGX_WANT_CALLS;
    auto run_batch = [&](Batch &b) {
        kgx_result r;
        if (kgx_process_batch(ctx, &prm, res.data(), off.data(), (uint32_t)n, want, &r) != KGX_OK)
            return false;
        b.hoff.assign(r.hit_offsets, r.hit_offsets + n + 1);
        b.coff.assign(r.call_offsets, r.call_offsets + n + 1);
        b.hits.assign(r.hits, r.hits + b.hoff[n]);
        b.calls.assign(r.calls, r.calls + b.coff[n]);
        return true;
    };
    Batch ref;
    if (!run_batch(ref)) { /* warm: the context's buffers grow to the batch */
        std::fprintf(stderr, "beside_check: %s\n", kgx_last_error());
        return 1;
    }
    {   /* warm: the service starts (its slot memory, its first instances) */
        std::vector<kgx_hit> h(4096);
        std::vector<kgx_call> c(4096);
        uint64_t nh = 0, nc = 0;
        if (kgx_svc_call(img, &prm, res.data(), off[1], want, h.data(), h.size(), &nh, c.data(), c.size(), &nc,
                         nullptr, 0, nullptr) != KGX_OK) {
            std::fprintf(stderr, "beside_check: %s\n", kgx_last_error());
            return 1;
        }
    }
    std::vector<double> alone;
    for (int rep = 0; rep < 30; rep++) {
        Batch b;
        const auto t0 = clk::now();
        if (!run_batch(b)) {
            std::fprintf(stderr, "beside_check: %s\n", kgx_last_error());
            return 1;
        }
        alone.push_back(std::chrono::duration<double, std::milli>(clk::now() - t0).count());
        if (!(b == ref)) {
            std::fprintf(stderr, "beside_check: batches alone differ\n");
            return 1;
        }
    }
    std::atomic<bool> stop{false}, failed{false};
    std::atomic<uint64_t> n_calls{0}, n_busy{0}, svc_bad{0};
    std::vector<double> beside;
    struct BatchRec {
        double t0, t1, call_ms; /* ms from the run's start; kgx_process_batch alone */
        long nivcsw, nvcsw;     /* the batch thread's context switches during the batch */
    };
    std::vector<BatchRec> brec;
    uint64_t batch_bad = 0;
    const auto T0 = clk::now();
    auto since = [&](clk::time_point t) { return std::chrono::duration<double, std::milli>(t - T0).count(); };
    std::thread bt([&]() {
        while (!stop.load()) {
            Batch b;
            struct rusage ra, rb;
            getrusage(RUSAGE_THREAD, &ra);
            const auto t0 = clk::now();
            kgx_result r;
            if (kgx_process_batch(ctx, &prm, res.data(), off.data(), (uint32_t)n, want, &r) != KGX_OK) {
                failed = true;
                return;
            }
            const auto tc = clk::now();
            b.hoff.assign(r.hit_offsets, r.hit_offsets + n + 1);
            b.coff.assign(r.call_offsets, r.call_offsets + n + 1);
            b.hits.assign(r.hits, r.hits + b.hoff[n]);
            b.calls.assign(r.calls, r.calls + b.coff[n]);
            const auto t1 = clk::now();
            getrusage(RUSAGE_THREAD, &rb);
            beside.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
            brec.push_back({since(t0), since(t1), std::chrono::duration<double, std::milli>(tc - t0).count(),
                            rb.ru_nivcsw - ra.ru_nivcsw, rb.ru_nvcsw - ra.ru_nvcsw});
            batch_bad += !(b == ref);
        }
    });
    /* every service call's [start, end) in ms from T0, per thread */
    std::vector<std::vector<std::pair<double, double>>> calls_t(T);
    std::vector<std::thread> ws;
    const auto t_end = clk::now() + std::chrono::duration<double>(seconds);
    const auto t0 = clk::now();
    for (int t = 0; t < T; t++)
        ws.emplace_back([&, t]() {
            std::vector<kgx_hit> h(4096);
            std::vector<kgx_call> c(4096);
            for (uint64_t k = (uint64_t)t; clk::now() < t_end; k += (uint64_t)T) {
                const uint64_t s = k % n, len = off[s + 1] - off[s];
                uint64_t nh = 0, nc = 0;
                const auto c0 = clk::now();
                const int rc = kgx_svc_call(img, &prm, res.data() + off[s], len, want, h.data(), h.size(), &nh,
                                            c.data(), c.size(), &nc, nullptr, 0, nullptr);
                calls_t[t].emplace_back(since(c0), since(clk::now()));
                if (rc == KGX_EBUSY) {
                    n_busy++;
                    continue;
                }
                if (rc != KGX_OK) {
                    failed = true;
                    return;
                }
                n_calls++;
                bool ok = nh == ref.hoff[s + 1] - ref.hoff[s] && nc == ref.coff[s + 1] - ref.coff[s];
                for (uint64_t j = 0; ok && j < nh; j++) {
                    kgx_hit x = h[j];
                    x.seq = (uint32_t)s;
                    ok = !std::memcmp(&x, &ref.hits[ref.hoff[s] + j], sizeof x);
                }
                ok = ok && !std::memcmp(c.data(), ref.calls.data() + ref.coff[s], nc * sizeof(kgx_call));
                svc_bad += !ok;
            }
        });
    for (auto &w : ws)
        w.join();
    const double tp = std::chrono::duration<double>(clk::now() - t0).count();
    stop = true;
    bt.join();
    /* the tail's evidence: batches with / without an involuntary switch, and
     * the five slowest batches with what overlapped them */
    std::vector<double> with_sw, without_sw;
    for (const BatchRec &b : brec)
        (b.nivcsw > 0 ? with_sw : without_sw).push_back(b.t1 - b.t0);
    std::vector<size_t> order(brec.size());
    for (size_t i = 0; i < order.size(); i++)
        order[i] = i;
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return brec[a].t1 - brec[a].t0 > brec[b].t1 - brec[b].t0; });
    std::string slow = "[";
    for (size_t k = 0; k < std::min<size_t>(5, order.size()); k++) {
        const BatchRec &b = brec[order[k]];
        size_t overl = 0;
        double longest = 0.0;
        for (const auto &v : calls_t)
            for (const auto &c : v)
                if (c.second > b.t0 && c.first < b.t1) {
                    overl++;
                    longest = std::max(longest, c.second - c.first);
                }
        char buf[320];
        std::snprintf(buf, sizeof buf,
                      "%s{\"ms\": %.3f, \"in_process_batch_ms\": %.3f, \"nivcsw\": %ld, \"nvcsw\": %ld, "
                      "\"service_calls_overlapping\": %zu, \"longest_overlapping_call_ms\": %.3f}",
                      k ? ", " : "", b.t1 - b.t0, b.call_ms, b.nivcsw, b.nvcsw, overl, longest);
        slow += buf;
    }
    slow += "]";
    std::vector<double> call_ms;
    for (const auto &v : calls_t)
        for (const auto &c : v)
            call_ms.push_back(c.second - c.first);
    struct rusage self;
    getrusage(RUSAGE_SELF, &self);
    std::printf("{\"tail_evidence\": {\"batches_with_involuntary_switch\": %zu, \"p50_ms_with\": %.3f, "
                "\"max_ms_with\": %.3f, \"batches_without\": %zu, \"p50_ms_without\": %.3f, \"p99_ms_without\": %.3f, "
                "\"max_ms_without\": %.3f, \"service_call_ms\": {\"p50\": %.4f, \"p99\": %.4f, \"max\": %.3f}, "
                "\"process_nivcsw\": %ld, \"slowest\": %s}}\n",
                with_sw.size(), pct(with_sw, 50), pct(with_sw, 100), without_sw.size(), pct(without_sw, 50),
                pct(without_sw, 99), pct(without_sw, 100), pct(call_ms, 50), pct(call_ms, 99), pct(call_ms, 100),
                self.ru_nivcsw, slow.c_str());
    std::printf("{\"service_threads\": %d, \"batch_proteins\": %llu, \"batch_alone_ms\": {\"p50\": %.3f, \"max\": %.3f}, "
                "\"batch_beside_ms\": {\"n\": %zu, \"p50\": %.3f, \"p90\": %.3f, \"p99\": %.3f, \"max\": %.3f, "
                "\"over_5ms\": %zu, \"argmax\": %zu}, "
                "\"service_calls\": %llu, \"service_calls_per_s\": %.4g, \"service_busy\": %llu, "
                "\"batch_mismatches\": %llu, \"service_mismatches\": %llu, \"failed\": %d}\n",
                T, (unsigned long long)n, pct(alone, 50), pct(alone, 100), beside.size(), pct(beside, 50),
                pct(beside, 90), pct(beside, 99), pct(beside, 100),
                (size_t)std::count_if(beside.begin(), beside.end(), [](double v) { return v > 5.0; }),
                (size_t)(std::max_element(beside.begin(), beside.end()) - beside.begin()), (unsigned long long)n_calls.load(), (double)n_calls.load() / tp,
                (unsigned long long)n_busy.load(), (unsigned long long)batch_bad,
                (unsigned long long)svc_bad.load(), failed.load() ? 1 : 0);
    if (failed)
        std::fprintf(stderr, "beside_check: %s\n", kgx_last_error());
    kgx_ctx_destroy(ctx);
    kgx_image_close(img);
    return failed || batch_bad || svc_bad ? 1 : 0;
}
