/*
 * kgx_query.cpp -- request-handler surface over the HIP engine.
 *
 * Prints, for every sequence of a FASTA file, what the reference's handlers
 * print, computing everything through the KmerGuts facade (one batched GPU
 * pass per file, like one work list of a request chunk):
 *
 *   query          query_request.cc:103-151 (details=0, find_best_call=0)
 *   query_details  query_request.cc:103-151 with details=1 (HIT lines)
 *   query_best     query_request.cc:124-135 (find_best_call=1)
 *   add            add_request.cc:305-353 (silent=0)
 *   fq             the input is FASTQ: fq_process_request.cc:230-365 over
 *                  FamilyMapper; genus=, families=, nr= load the family DB
 *   lookup         /lookup (lookup_request.cc:153-400): family_mode=1 loads
 *                  the family DB (genus=, families=, nr=); otherwise the FASTA
 *                  is first /add-ed into kmer_to_id_
 *   matrix         /add of the FASTA into an empty mapping, then one /matrix
 *                  request over the same FASTA (matrix_request.cc:83-190)
 *
 * usage: kgx_query DATA_DIR FASTA MODE [name=value ...]   (KGX_DEVICE=n)
 */
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "kguts_hip.h"

using namespace kgx;

int main(int argc, char **argv)
{
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s DATA_DIR FASTA MODE [name=value ...]\n", argv[0]);
        return 2;
    }
    const std::string dir = argv[1], fasta = argv[2], mode = argv[3];
    if (mode != "query" && mode != "query_details" && mode != "query_best" && mode != "add" &&
        mode != "matrix" && mode != "fq" && mode != "lookup") {
        std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
        return 2;
    }
    std::map<std::string, std::string> qp;
    for (int i = 4; i < argc; i++) {
        std::string a = argv[i];
        size_t eq = a.find('=');
        if (eq != std::string::npos)
            qp[a.substr(0, eq)] = a.substr(eq + 1);
    }
    const char *dev = std::getenv("KGX_DEVICE");
    try {
        auto image = std::make_shared<KmerImage>(dir, dev ? std::atoi(dev) : 0);
        KmerGuts kguts(dir, image);
        kguts.set_parameters(qp);

        if (mode == "fq") {
            auto mapping = std::make_shared<KmerPegMapping>(kgx_image_device(image->handle()));
            if (!qp["genus"].empty())
                mapping->load_genus_map(qp["genus"]);
            if (!qp["families"].empty())
                mapping->load_families(qp["families"]);
            if (!qp["nr"].empty())
                mapping->load_nr_families(kguts, qp["nr"]);
            std::ifstream in(fasta, std::ios::binary);
            if (!in) {
                std::fprintf(stderr, "cannot open %s\n", fasta.c_str());
                return 1;
            }
            std::stringstream ss;
            ss << in.rdbuf();
            FqRequest req(kguts, mapping);
            std::ostringstream os;
            req.process(ss.str(), true, os);
            const std::string s = os.str();
            std::fwrite(s.data(), 1, s.size(), stdout);
            return 0;
        }
        std::vector<KmerGuts::SeqJob> jobs;
        FastaParser parser;
        parser.set_callback([&jobs](const std::string &id, const std::string &seq) {
            KmerGuts::SeqJob j;
            j.id = id;
            j.seq = seq;
            jobs.push_back(std::move(j));
            return 0;
        });
        std::ifstream in(fasta, std::ios::binary);
        if (!in) {
            std::fprintf(stderr, "cannot open %s\n", fasta.c_str());
            return 1;
        }
        char ch;
        while (in.get(ch))
            parser.parse_char(ch);
        parser.parse_complete();

        if (mode == "lookup") {
            auto mapping = std::make_shared<KmerPegMapping>(kgx_image_device(image->handle()));
            if (!qp["genus"].empty())
                mapping->load_genus_map(qp["genus"]);
            if (!qp["families"].empty())
                mapping->load_families(qp["families"]);
            const bool family_mode = qp["family_mode"] == "1";
            if (family_mode && !qp["nr"].empty())
                mapping->load_nr_families(kguts, qp["nr"]);
            std::vector<std::pair<std::string, std::string>> work;
            std::vector<std::string> seqs;
            for (auto &j : jobs) {
                work.emplace_back(j.id, j.seq);
                seqs.push_back(j.seq);
            }
            if (!family_mode) { /* /add first, ids encoded in order after the chunk */
                run_batch_on_device(kguts, seqs);
                std::vector<KmerPegMapping::encoded_id_t> ids;
                for (auto &j : jobs)
                    ids.push_back(mapping->encode_id(j.id));
                mapping->add_batch_mappings(kguts, ids);
            }
            LookupRequest req(mapping, family_mode, qp);
            std::ostringstream os;
            req.process_work(kguts, work, os);
            const std::string s = os.str();
            std::fwrite(s.data(), 1, s.size(), stdout);
            return 0;
        }
        if (mode == "matrix") {
            auto mapping = std::make_shared<KmerPegMapping>(kgx_image_device(image->handle()));
            std::vector<std::string> seqs;
            std::vector<std::pair<std::string, std::string>> work;
            for (auto &j : jobs) {
                seqs.push_back(j.seq);
                work.emplace_back(j.id, j.seq);
            }
            /* /add (add_request.cc:164-170 / 196-206): ids encoded in order */
            run_batch_on_device(kguts, seqs);
            std::vector<KmerPegMapping::encoded_id_t> ids;
            for (auto &j : jobs)
                ids.push_back(mapping->encode_id(j.id));
            mapping->add_batch_mappings(kguts, ids);
            MatrixRequest mx(mapping);
            mx.process_work(kguts, work);
            std::ostringstream os;
            mx.write_results(os);
            const std::string s = os.str();
            std::fwrite(s.data(), 1, s.size(), stdout);
            return 0;
        }
        const bool details = mode == "query_details";
        std::vector<std::shared_ptr<std::vector<KmerGuts::hit_in_sequence_t>>> hit_lists(jobs.size());
        for (size_t i = 0; i < jobs.size(); i++) {
            jobs[i].calls = std::make_shared<std::vector<KmerCall>>();
            jobs[i].otu_stats = std::make_shared<KmerOtuStats>();
            if (details || mode == "add") {
                auto hl = std::make_shared<std::vector<KmerGuts::hit_in_sequence_t>>();
                hit_lists[i] = hl;
                jobs[i].hit_cb = [hl](KmerGuts::hit_in_sequence_t h) { hl->push_back(h); };
            }
        }
        kguts.process_aa_batch(jobs);

        std::ostringstream os;
        for (size_t i = 0; i < jobs.size(); i++) {
            const std::string &id = jobs[i].id, &seq = jobs[i].seq;
            auto &calls = *jobs[i].calls;
            if (mode == "query_best") {
                int fi;
                std::string fn;
                float score, wscore, off = 0.0f;
                kguts.find_best_call(calls, fi, fn, score, wscore, off);
                if (!fn.empty())
                    os << id << "\t" << fn << "\t" << score << "\t" << wscore << "\n";
            } else if (mode == "add") {
                os << "PROTEIN-ID\t" << id << "\t" << seq.size() << "\n";
                for (auto &c : calls)
                    os << kguts.format_call(c);
                os << kguts.format_otu_stats(id, seq.size(), *jobs[i].otu_stats);
                int fi;
                std::string fn;
                /* uninitialised in the reference when there are no calls
                 * (add_request.cc:334); 0 here */
                float score, wscore, off = 0.0f;
                kguts.find_best_call(calls, fi, fn, score, wscore, off);
                if (fn.empty() || fn.find(" ?? ") != std::string::npos)
                    fn = "hypothetical protein";
                os << "BEST-CALL\t" << id << "\t" << fn << "\t" << score << "\t" << wscore << "\t"
                   << off << "\n";
            } else {
                os << "PROTEIN-ID\t" << id << "\t" << seq.size() << "\n";
                for (auto &c : calls)
                    os << kguts.format_call(c);
                if (details)
                    for (auto &h : *hit_lists[i])
                        os << kguts.format_hit(h);
                os << kguts.format_otu_stats(id, seq.size(), *jobs[i].otu_stats);
            }
        }
        const std::string s = os.str();
        std::fwrite(s.data(), 1, s.size(), stdout);
    } catch (const Error &e) {
        std::fprintf(stderr, "kgx_query: %s\n", e.what());
        return 1;
    }
    return 0;
}
