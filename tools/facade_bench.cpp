/*
 * facade_bench -- what the unchanged per-sequence drop-in costs: the
 * reference's handler loop calls KmerGuts::process_aa_seq once per sequence
 * (lookup_request.cc:153-172, query_request.cc:103-151); through the facade
 * each call is one GPU round trip.  Times that call on single 300-aa C2
 * proteins (latency distribution) and the same sequences through
 * process_aa_batch (one pass), with the lookup handler's outputs (calls + a
 * hit callback, no OTU stats); then the reference's pool shape: T worker
 * threads, one KmerGuts each over the shared image (threadpool.cc:18-44),
 * each calling process_aa_seq per sequence (aggregate rate per T).
 *
 *   facade_bench KMER_DIR N_KEYS NUM_SIGS QUERIES.bin [N_CALLS]
 *
 * QUERIES.bin: uint64 n, uint64 offsets[n+1], residues.  Prints one JSON line.
 */
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <thread>
#include <atomic>
#include <vector>

#include "kguts_hip.h"

using clk = std::chrono::steady_clock;

static double pct(std::vector<double> v, double p)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[std::min(v.size() - 1, (size_t)(p / 100.0 * (double)v.size()))];
}

static double mean(const std::vector<double> &v)
{
    double t = 0;
    for (double x : v)
        t += x;
    return v.empty() ? 0.0 : t / (double)v.size();
}

int main(int argc, char **argv)
{
    if (argc < 5) {
        std::fprintf(stderr, "usage: facade_bench KMER_DIR N_KEYS NUM_SIGS QUERIES.bin [N_CALLS]\n");
        return 2;
    }
    const std::string dir = argv[1];
    const uint64_t n_keys = std::strtoull(argv[2], nullptr, 10), num_sigs = std::strtoull(argv[3], nullptr, 10);
    const size_t n_calls = argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 2000;
    std::ifstream in(argv[4], std::ios::binary);
    uint64_t n = 0;
    in.read(reinterpret_cast<char *>(&n), 8);
    std::vector<uint64_t> off(n + 1);
    in.read(reinterpret_cast<char *>(off.data()), (std::streamsize)(8 * (n + 1)));
    std::string res(off[n], '\0');
    in.read(&res[0], (std::streamsize)res.size());
    if (!in) {
        std::fprintf(stderr, "facade_bench: short query file\n");
        return 2;
    }
    /* the bench's image: n_keys distinct keys stored (bench.py C2) */
    kgx_image *img = nullptr;
    uint64_t entries = 0;
    const uint64_t stored = n_keys;
    if (kgx_image_build_synthetic_distinct(n_keys, n_keys, num_sigs, 0, &img, &entries) != KGX_OK) {
        std::fprintf(stderr, "facade_bench: %s\n", kgx_last_error());
        return 1;
    }
    auto image = std::make_shared<kgx::KmerImage>(img);
    kgx::KmerGuts kg(dir, image);
    kg.coalesce = false; /* the single-thread latencies: one pass per call */
    const size_t m = std::min<size_t>(n, n_calls);
    std::vector<std::string> seqs(m);
    for (size_t i = 0; i < m; i++)
        seqs[i] = res.substr(off[i], off[i + 1] - off[i]);

    /* unbatched: one process_aa_seq per sequence, as the reference's loop;
     * first on the ordinary batch path (small_batch 0: device plan, counts
     * round trip, gather round trip), then on the default one-wait path */
    uint64_t hits = 0, calls = 0, residues = 0, hits0 = 0, calls0 = 0;
    std::vector<double> lat, lat0;
    double t_seq = 0;
    for (int pass = 0; pass < 2; pass++) {
        if (kgx_ctx_set_option(kg.ctx(), "small_batch", pass == 0 ? 0 : 65536) != KGX_OK) {
            std::fprintf(stderr, "facade_bench: %s\n", kgx_last_error());
            return 1;
        }
        for (int warm = 0; warm < 20; warm++) {
            auto cv = std::make_shared<std::vector<kgx::KmerCall>>();
            kg.process_aa_seq("w", seqs[warm % m], cv, [](kgx::KmerGuts::hit_in_sequence_t) {}, nullptr);
        }
        hits0 = hits;
        calls0 = calls;
        hits = calls = residues = 0;
        lat0.swap(lat);
        lat.clear();
        lat.reserve(m);
        const auto t_all = clk::now();
        for (size_t i = 0; i < m; i++) {
            auto cv = std::make_shared<std::vector<kgx::KmerCall>>();
            const auto t0 = clk::now();
            kg.process_aa_seq("q", seqs[i], cv, [&](kgx::KmerGuts::hit_in_sequence_t) { hits++; }, nullptr);
            lat.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
            calls += cv->size();
            residues += seqs[i].size();
        }
        t_seq = std::chrono::duration<double>(clk::now() - t_all).count();
    }

    /* the same sequences, one process_aa_batch */
    uint64_t bhits = 0, bcalls = 0;
    std::vector<double> tb;
    for (int rep = 0; rep < 6; rep++) {
        std::vector<kgx::KmerGuts::SeqJob> jobs(m);
        for (size_t i = 0; i < m; i++) {
            jobs[i].id = "q";
            jobs[i].seq = seqs[i];
            jobs[i].calls = std::make_shared<std::vector<kgx::KmerCall>>();
            jobs[i].hit_cb = [&](kgx::KmerGuts::hit_in_sequence_t) { bhits++; };
        }
        const auto t0 = clk::now();
        kg.process_aa_batch(jobs);
        tb.push_back(std::chrono::duration<double>(clk::now() - t0).count());
        if (rep == 0)
            for (auto &j : jobs)
                bcalls += j.calls->size();
    }
    const double t_batch = pct(tb, 50);

    /* one pass's latency by batch size (process_aa_batch of k proteins, one
     * thread): what a coalesced pass of k concurrent calls costs */
    std::string bs_json;
    /* KGX_FACADE_BATCH=k: only this pass size, and no thread sweep (kernel traces) */
    const char *only = std::getenv("KGX_FACADE_BATCH");
    std::vector<size_t> sizes = {1, 2, 4, 8, 16, 32, 64};
    if (only)
        sizes = {(size_t)std::strtoull(only, nullptr, 10)};
    /* with the one-launch path the facade's per-sequence calls take (small_fused) */
    if (kgx_ctx_set_option(kg.ctx(), "small_fused", 1) != KGX_OK)
        return 1;
    for (size_t k : sizes) {
        std::vector<double> lt;
        for (int rep = 0; rep < 200; rep++) {
            std::vector<kgx::KmerGuts::SeqJob> jobs(k);
            for (size_t i = 0; i < k; i++) {
                jobs[i].id = "q";
                jobs[i].seq = seqs[(rep * k + i) % m];
                jobs[i].calls = std::make_shared<std::vector<kgx::KmerCall>>();
                jobs[i].hit_cb = [](kgx::KmerGuts::hit_in_sequence_t) {};
            }
            const auto t0 = clk::now();
            kg.process_aa_batch(jobs);
            if (rep >= 20)
                lt.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
        }
        char b[120];
        std::snprintf(b, sizeof b, "%s\"%zu\": {\"p50_us\": %.1f, \"p99_us\": %.1f}", bs_json.empty() ? "" : ", ", k,
                      pct(lt, 50), pct(lt, 99));
        bs_json += b;
        std::fprintf(stderr, "[facade] pass of %zu proteins: p50 %.1f us, p99 %.1f us\n", k, pct(lt, 50), pct(lt, 99));
    }
    (void)kgx_ctx_set_option(kg.ctx(), "small_fused", 0);

    /* the worker pool: T threads, one KmerGuts (context) each, per-sequence
     * calls; concurrent calls coalesced into shared passes (the default) or
     * one pass per call */
    std::string pool_json;
    bool pool_ok = true;
    /* KGX_FACADE_THREADS="16" or "8,16": only these pool sizes; KGX_FACADE_MODES="1" coalesced only */
    std::vector<int> threads = {1, 4, 8, 16, 32};
    if (const char *e = std::getenv("KGX_FACADE_THREADS")) {
        threads.clear();
        for (const char *q = e; *q;) {
            threads.push_back(std::atoi(q));
            while (*q && *q != ',')
                q++;
            if (*q == ',')
                q++;
        }
    }
    /* modes: 2 = the resident call service (kgx_svc_call, the default),
     * 1 = the coalescer (service off), 0 = one pass per call;
     * KGX_FACADE_MODES="2" or "2,1": only these */
    std::vector<int> modes = {2, 1, 0};
    if (const char *e = std::getenv("KGX_FACADE_MODES")) {
        modes.clear();
        for (const char *q = e; *q; q++)
            if (*q >= '0' && *q <= '2')
                modes.push_back(*q - '0');
    }
    /* each pool run makes R passes over the m sequences (enough calls to
     * time a pool of 16 threads at ~1M calls/s) */
    const size_t R = std::getenv("KGX_FACADE_REPS") ? std::strtoull(std::getenv("KGX_FACADE_REPS"), nullptr, 10) : 10;
    static const char *mode_name[3] = {"per_call_T", "coalesced_T", "service_T"};
    const bool with_otu = std::getenv("KGX_FACADE_OTU") && std::atoi(std::getenv("KGX_FACADE_OTU")) != 0;
    for (int co : modes)
        for (int T : threads) {
            if (only)
                break;
            std::vector<std::unique_ptr<kgx::KmerGuts>> kgs;
            for (int t = 0; t < T; t++) {
                kgs.emplace_back(new kgx::KmerGuts(dir, image));
                kgs.back()->coalesce = co != 0;
                kgs.back()->service = co == 2;
            }
            std::vector<uint64_t> th_hits(T, 0);
            std::vector<std::vector<double>> th_lat(T);
            /* the pool's queue: each worker takes the next sequence (threadpool.cc:33-60); a
             * fixed stride would hand even threads only the planted (hit-rich) proteins */
            std::atomic<size_t> next{0};
            auto work = [&](int t, bool count) {
                const size_t total = count ? m * R : m;
                for (size_t k; (k = next.fetch_add(1, std::memory_order_relaxed)) < total;) {
                    const size_t i = k % m;
                    auto cv = std::make_shared<std::vector<kgx::KmerCall>>();
                    uint64_t h = 0;
                    const auto q0 = clk::now();
                    /* KGX_FACADE_OTU=1: OTU stats wanted too (query_request.cc's per-sequence shape) */
                    auto os = with_otu ? std::make_shared<kgx::KmerOtuStats>() : nullptr;
                    kgs[t]->process_aa_seq("q", seqs[i], cv, [&h](kgx::KmerGuts::hit_in_sequence_t) { h++; },
                                           os);
                    if (count) {
                        th_lat[t].push_back(std::chrono::duration<double, std::micro>(clk::now() - q0).count());
                        th_hits[t] += h;
                    }
                }
            };
            next = 0;
            { /* warm: buffer growth on every context */
                std::vector<std::thread> ws;
                for (int t = 0; t < T; t++)
                    ws.emplace_back(work, t, false);
                for (auto &w : ws)
                    w.join();
            }
            const uint64_t passes0 = image->coalescer().passes, calls0 = image->coalescer().calls;
            uint64_t svc0 = 0, svc1 = 0, ph0[14] = {}, ph1[14] = {};
            (void)kgx_svc_stat(image->handle(), "calls", &svc0);
            for (int k = 0; k < 14; k++) {
                const std::string nm = "phase_n" + std::to_string(k);
                (void)kgx_svc_stat(image->handle(), nm.c_str(), &ph0[k]);
            }
            next = 0;
            const auto t0 = clk::now();
            std::vector<std::thread> ws;
            for (int t = 0; t < T; t++)
                ws.emplace_back(work, t, true);
            for (auto &w : ws)
                w.join();
            const double tp = std::chrono::duration<double>(clk::now() - t0).count();
            uint64_t ph = 0;
            std::vector<double> all;
            for (int t = 0; t < T; t++) {
                ph += th_hits[t];
                all.insert(all.end(), th_lat[t].begin(), th_lat[t].end());
            }
            pool_ok = pool_ok && ph == hits * R;
            const uint64_t np = image->coalescer().passes - passes0, nc = image->coalescer().calls - calls0;
            (void)kgx_svc_stat(image->handle(), "calls", &svc1);
            const double nm = (double)(m * R);
            /* KGX_SVC_DEBUG=1: mean per call of the host wall and the device phases (us) */
            std::string phases;
            for (int k = 0; k < 14; k++) {
                const std::string nm2 = "phase_n" + std::to_string(k);
                (void)kgx_svc_stat(image->handle(), nm2.c_str(), &ph1[k]);
                if (svc1 > svc0 && ph1[0] > ph0[0]) {
                    char q[40];
                    std::snprintf(q, sizeof q, "%s%.2f", phases.empty() ? "" : ", ",
                                  (double)(ph1[k] - ph0[k]) / 1e3 / (double)(svc1 - svc0));
                    phases += q;
                }
            }
            if (!phases.empty())
                std::fprintf(stderr, "[facade] %s%d service phases (us: wall, residues, probe, compact, store+score, "
                             "stores, first chunk, rest, probe rounds, first round, keys, own loads, chunk runs, chunk sums): %s\n", mode_name[co], T, phases.c_str());
            char b[400];
            std::snprintf(b, sizeof b,
                          "%s\"%s%d\": {\"calls_per_s\": %.4g, \"residues_per_s\": %.4g, \"p50_us\": %.1f, "
                          "\"p99_us\": %.1f, \"mean_us\": %.2f, \"calls_per_pass\": %.2f, \"service_calls\": %llu}",
                          pool_json.empty() ? "" : ", ", mode_name[co], T, nm / tp, (double)(residues * R) / tp,
                          pct(all, 50), pct(all, 99), mean(all), np ? (double)nc / (double)np : 1.0,
                          (unsigned long long)(svc1 - svc0));
            pool_json += b;
            std::fprintf(stderr, "[facade] %s%d: %.4g calls/s, %.4g residues/s, p50 %.1f us, p99 %.1f us, mean %.2f us "
                         "(a thread's call cycle %.2f us)\n", mode_name[co], T, nm / tp, (double)(residues * R) / tp,
                         pct(all, 50), pct(all, 99), mean(all), tp * 1e6 * T / nm);
        }
    /* KGX_FACADE_BESIDE=T: T service callers (one KmerGuts each) and, at the
     * same time, one batch caller (its own KmerGuts: process_aa_batch of the m
     * proteins, over and over) on the same image -- a server whose pool mixes
     * per-sequence calls and chunk batches (threadpool.cc:33-60).  Native
     * threads: a Python harness's GIL would time itself. */
    std::string beside_json;
    if (const char *e = std::getenv("KGX_FACADE_BESIDE")) {
        const int T = std::max(1, std::atoi(e));
        std::vector<std::unique_ptr<kgx::KmerGuts>> kgs;
        for (int t = 0; t <= T; t++) {
            kgs.emplace_back(new kgx::KmerGuts(dir, image));
            kgs.back()->coalesce = t < T;
            kgs.back()->service = t < T;
        }
        auto batch_once = [&](kgx::KmerGuts &g) {
            std::vector<kgx::KmerGuts::SeqJob> jobs(m);
            for (size_t i = 0; i < m; i++) {
                jobs[i].id = "q";
                jobs[i].seq = seqs[i];
                jobs[i].calls = std::make_shared<std::vector<kgx::KmerCall>>();
                jobs[i].hit_cb = [](kgx::KmerGuts::hit_in_sequence_t) {};
            }
            const auto t0 = clk::now();
            g.process_aa_batch(jobs);
            return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        };
        std::vector<double> alone;
        for (int rep = 0; rep < 30; rep++)
            alone.push_back(batch_once(*kgs[T]));
        std::atomic<bool> stop{false};
        std::atomic<uint64_t> n_calls{0};
        std::vector<double> beside;
        std::thread bt([&]() {
            while (!stop.load())
                beside.push_back(batch_once(*kgs[T]));
        });
        std::vector<std::thread> ws;
        const auto t0 = clk::now();
        for (int t = 0; t < T; t++)
            ws.emplace_back([&, t]() {
                for (size_t k = t; k < m * R; k += T) {
                    auto cv = std::make_shared<std::vector<kgx::KmerCall>>();
                    kgs[t]->process_aa_seq("q", seqs[k % m], cv, [](kgx::KmerGuts::hit_in_sequence_t) {}, nullptr);
                    n_calls++;
                }
            });
        for (auto &w : ws)
            w.join();
        const double tp = std::chrono::duration<double>(clk::now() - t0).count();
        stop = true;
        bt.join();
        char b[400];
        std::snprintf(b, sizeof b,
                      ", \"beside\": {\"service_threads\": %d, \"batch_proteins\": %zu, \"batch_alone_ms\": {\"p50\": %.3f, "
                      "\"max\": %.3f}, \"batch_beside_ms\": {\"n\": %zu, \"p50\": %.3f, \"p90\": %.3f, \"max\": %.3f}, "
                      "\"service_calls_per_s\": %.4g}",
                      T, m, pct(alone, 50), pct(alone, 100), beside.size(), pct(beside, 50), pct(beside, 90),
                      pct(beside, 100), (double)n_calls / tp);
        beside_json = b;
        std::fprintf(stderr, "[facade] beside %d service callers: batch of %zu alone p50 %.3f ms, beside p50 %.3f p90 %.3f "
                     "max %.3f ms (%zu batches); service %.4g calls/s\n", T, m, pct(alone, 50), pct(beside, 50),
                     pct(beside, 90), pct(beside, 100), beside.size(), (double)n_calls / tp);
    }
    std::printf("{\"metric\": \"KmerGuts facade per-call latency (process_aa_seq, one 300-aa C2 protein per call)\", "
                "\"calls\": %zu, \"latency_us\": {\"median\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"mean\": %.1f}, "
                "\"latency_us_ordinary_path\": {\"median\": %.1f, \"p90\": %.1f, \"p99\": %.1f}, "
                "\"unbatched_residues_per_s\": %.4g, \"batched\": {\"sequences\": %zu, \"ms\": %.3f, "
                "\"residues_per_s\": %.4g}, \"hits\": %llu, \"calls_out\": %llu, \"batch_hits_per_rep\": %llu, "
                "\"batch_calls\": %llu, \"keys_stored\": %llu, \"pass_latency_by_batch\": {%s}, "
                "\"worker_pool_by_threads\": {%s}%s}\n",
                m, pct(lat, 50), pct(lat, 90), pct(lat, 99), t_seq * 1e6 / (double)m, pct(lat0, 50), pct(lat0, 90),
                pct(lat0, 99), (double)residues / t_seq, m,
                t_batch * 1e3, (double)residues / t_batch, (unsigned long long)hits, (unsigned long long)calls,
                (unsigned long long)(bhits / 6), (unsigned long long)bcalls, (unsigned long long)stored,
                bs_json.c_str(), pool_json.c_str(), beside_json.c_str());
    return hits * 6 == bhits && calls == bcalls && hits == hits0 && calls == calls0 && pool_ok ? 0 : 3;
}
