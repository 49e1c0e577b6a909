/*
 * The reference's pool shape through the KmerGuts facade, for
 * tests/test_gpu_coalesce.py: T worker threads, one KmerGuts each over one
 * shared KmerImage (threadpool.cc:18-44), each calling process_aa_seq once per
 * sequence (lookup_request.cc:153-172) with a hit callback, a calls vector and
 * OTU stats.  Concurrent calls are coalesced into shared GPU passes
 * (SeqCoalescer); every thread must still see exactly its own sequences'
 * results, in position order.  Thread t takes sequences i = t, t + T, ... and
 * parameter set t % 3 (so passes group calls by parameters).
 *
 *   coalesce_check DATA_DIR QUERIES.bin T OUT.bin [coalesce 0|1] [otu 0|1]
 *
 * otu 0: no OTU stats asked (the lookup handler's outputs, which take the
 * one-launch path); OUT.bin then holds no OTU pairs (n_otus 0).
 *
 * QUERIES.bin: uint64 n, uint64 offsets[n+1], residues.  OUT.bin, per
 * sequence in input order: u32 n_hits, n_hits x kgx_hit (seq = 0, flags = 0),
 * u32 n_calls, n_calls x kgx_call, u32 n_otus, n_otus x (i32 otu, i32 count)
 * in otus_by_count order.
 */
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "kguts_hip.h"

struct SeqOut {
    std::vector<kgx_hit> hits;
    std::vector<kgx_call> calls;
    std::vector<std::pair<int, int>> otus;
};

int main(int argc, char **argv)
{
    if (argc < 5) {
        std::fprintf(stderr, "usage: coalesce_check DATA_DIR QUERIES.bin T OUT.bin [coalesce]\n");
        return 2;
    }
    const std::string dir = argv[1];
    const int T = std::atoi(argv[3]);
    const bool coalesce = argc > 5 ? std::atoi(argv[5]) != 0 : true;
    const bool with_otu = argc > 6 ? std::atoi(argv[6]) != 0 : true;
    const int svc_slots = argc > 7 ? std::atoi(argv[7]) : 0; /* call service slots (0: its default) */
    std::ifstream in(argv[2], std::ios::binary);
    uint64_t n = 0;
    in.read(reinterpret_cast<char *>(&n), 8);
    std::vector<uint64_t> off(n + 1);
    in.read(reinterpret_cast<char *>(off.data()), (std::streamsize)(8 * (n + 1)));
    std::string res(off[n], '\0');
    in.read(&res[0], (std::streamsize)res.size());
    if (!in) {
        std::fprintf(stderr, "coalesce_check: short query file\n");
        return 2;
    }
    std::vector<std::string> seqs(n);
    for (uint64_t i = 0; i < n; i++)
        seqs[i] = res.substr(off[i], off[i + 1] - off[i]);
    try {
        auto image = std::make_shared<kgx::KmerImage>(dir, 0);
        if (svc_slots && kgx_svc_config(image->handle(), (uint32_t)svc_slots, 1000, 4000) != KGX_OK)
            throw std::runtime_error("kgx_svc_config");
        std::vector<std::unique_ptr<kgx::KmerGuts>> kgs;
        for (int t = 0; t < T; t++) {
            kgs.emplace_back(new kgx::KmerGuts(dir, image));
            kgs.back()->coalesce = coalesce;
            /* parameter sets: defaults, min_hits 3 / max_gap 50, order constraint */
            std::map<std::string, std::string> p;
            if (t % 3 == 1) {
                p["min_hits"] = "3";
                p["max_gap"] = "50";
            } else if (t % 3 == 2) {
                p["order_constraint"] = "1";
            }
            kgs.back()->set_parameters(p);
        }
        std::vector<SeqOut> out(n);
        std::vector<std::string> errs(T);
        std::vector<std::thread> ws;
        for (int t = 0; t < T; t++)
            ws.emplace_back([&, t] {
                try {
                    for (uint64_t i = (uint64_t)t; i < n; i += (uint64_t)T) {
                        auto calls = std::make_shared<std::vector<kgx::KmerCall>>();
                        auto otu = with_otu ? std::make_shared<kgx::KmerOtuStats>() : nullptr;
                        SeqOut &o = out[i];
                        kgs[t]->process_aa_seq("q", seqs[i], calls,
                                               [&o](kgx::KmerGuts::hit_in_sequence_t h) {
                                                   kgx_hit x{};
                                                   x.which_kmer = h.hit.which_kmer;
                                                   x.otu_index = h.hit.otu_index;
                                                   x.avg_from_end = h.hit.avg_from_end;
                                                   x.function_index = h.hit.function_index;
                                                   x.function_wt = h.hit.function_wt;
                                                   x.pos = h.offset;
                                                   o.hits.push_back(x);
                                               },
                                               otu);
                        for (const auto &c : *calls)
                            o.calls.push_back(kgx_call{c.start, c.end, c.count, c.function_index, c.weighted_hits});
                        if (otu)
                            o.otus = otu->otus_by_count;
                    }
                } catch (const std::exception &e) {
                    errs[t] = e.what();
                }
            });
        for (auto &w : ws)
            w.join();
        for (int t = 0; t < T; t++)
            if (!errs[t].empty()) {
                std::fprintf(stderr, "coalesce_check: thread %d: %s\n", t, errs[t].c_str());
                return 1;
            }
        FILE *f = std::fopen(argv[4], "wb");
        if (!f)
            return 1;
        for (const SeqOut &o : out) {
            uint32_t k = (uint32_t)o.hits.size();
            std::fwrite(&k, 4, 1, f);
            std::fwrite(o.hits.data(), sizeof(kgx_hit), k, f);
            k = (uint32_t)o.calls.size();
            std::fwrite(&k, 4, 1, f);
            std::fwrite(o.calls.data(), sizeof(kgx_call), k, f);
            k = (uint32_t)o.otus.size();
            std::fwrite(&k, 4, 1, f);
            for (const auto &p : o.otus) {
                const int32_t v[2] = {p.first, p.second};
                std::fwrite(v, 4, 2, f);
            }
        }
        std::fclose(f);
        const auto &co = image->coalescer();
        uint64_t svc_calls = 0;
        (void)kgx_svc_stat(image->handle(), "calls", &svc_calls);
        std::printf("{\"passes\": %llu, \"calls\": %llu, \"svc_calls\": %llu}\n", (unsigned long long)co.passes,
                    (unsigned long long)co.calls, (unsigned long long)svc_calls);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "coalesce_check: %s\n", e.what());
        return 1;
    }
    return 0;
}
