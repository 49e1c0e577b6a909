/*
 * oracle_query.cpp -- CPU oracle driver for the request-handler surface.
 *
 * TEST INFRASTRUCTURE ONLY.  Reads a kmer data directory (kmer.table.mem_map,
 * function.index, otu.index) and a FASTA file, runs the restated KmerGuts path
 * and prints exactly what the reference handlers print for each sequence:
 *
 *   mode=query          query_request.cc:103-151 (details=0, find_best_call=0)
 *   mode=query_details  query_request.cc:103-151 with details=1 (HIT lines)
 *   mode=query_best     query_request.cc:124-135 (find_best_call=1)
 *   mode=add            add_request.cc:305-353 (silent=0)
 *   mode=fq             the input is FASTQ: fq_process_request.cc:298-365 over
 *                       FamilyMapper; optional genus=, families=, nr= files
 *                       load the family DB (kmer.cc:341-493, nr_loader.cc)
 *   mode=lookup         /lookup (lookup_request.cc:153-400): family_mode=1 reads
 *                       the family DB (genus=, families=, nr=); otherwise the
 *                       FASTA is first /add-ed into kmer_to_id_; the request
 *                       parameters find_best_match, kmer_hit_threhsold,
 *                       allow_ambiguous_functions, target_genus, find_reps
 *   mode=matrix         /add of the FASTA into an empty mapping (add_request.cc:
 *                       164-170), then one /matrix request over the same FASTA
 *                       (matrix_request.cc:83-190): process_results' body
 *
 * usage: oracle_query DATA_DIR FASTA MODE [name=value ...]
 * The name=value pairs play the role of the request's query string
 * (krequest2.cc:112-124) and feed set_parameters (kguts.cc:244-268).
 */
#include "kmer_oracle.h"

#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

using namespace oracle;

extern "C" {
void *oracle_kmap_new(int mode);
void oracle_kmap_free(void *p);
void oracle_kmap_add(void *p, const uint64_t *kmers, const uint32_t *ids, uint64_t n);
void *oracle_matrix_new(void);
void oracle_matrix_free(void *p);
void oracle_matrix_add(void *px, void *pk, const uint32_t *seq_ids, const uint64_t *seq_lens,
                       uint64_t n_seq, const uint64_t *hit_off, const uint64_t *hit_kmers);
uint64_t oracle_matrix_pairs(void *px, uint32_t *id1, uint32_t *id2, uint64_t *count, float *score);
void *oracle_fq_new(const void *table, uint64_t num_sigs, const char *const *functions, uint64_t n_functions,
                    const char *genus_file, const char *families_file, const char *nr_fasta);
void oracle_fq_free(void *p);
char *oracle_fq_process(void *p, const char *fastq, uint64_t n);
void oracle_free(void *p);
void *oracle_lookup_new(const void *table, uint64_t num_sigs, const char *const *functions, uint64_t n_functions,
                        const char *genus_file, const char *families_file, const char *nr_fasta,
                        const char *add_fasta);
void oracle_lookup_free(void *p);
char *oracle_lookup_process(void *p, int family_mode, const char *const *names, const char *const *values,
                            uint64_t n_params, const char *fasta, uint64_t n);
}

/* KmerImage::map_image_file validation, kmer_image.cc:83-150 */
static bool load_image(const std::string &dir, std::vector<SigKmer> &table, uint64_t &num_sigs)
{
    std::string path = dir + "/kmer.table.mem_map";
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f)
        return false;
    std::fseek(f, 0, SEEK_END);
    long size = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    ImageHeader h;
    if (std::fread(&h, sizeof(h), 1, f) != 1) {
        std::fclose(f);
        return false;
    }
    if ((uint64_t)size != sizeof(SigKmer) * h.num_sigs + sizeof(ImageHeader) || h.version != 1 ||
        h.entry_size != sizeof(SigKmer)) {
        std::fclose(f);
        return false;
    }
    table.resize(h.num_sigs);
    size_t got = std::fread(table.data(), sizeof(SigKmer), h.num_sigs, f);
    std::fclose(f);
    num_sigs = h.num_sigs;
    return got == h.num_sigs;
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s DATA_DIR FASTA MODE [name=value ...]\n", argv[0]);
        return 2;
    }
    std::string dir = argv[1], fasta = argv[2], mode = argv[3];
    std::map<std::string, std::string> qp;
    for (int i = 4; i < argc; i++) {
        std::string a = argv[i];
        size_t eq = a.find('=');
        if (eq != std::string::npos)
            qp[a.substr(0, eq)] = a.substr(eq + 1);
    }
    std::vector<SigKmer> table;
    uint64_t num_sigs = 0;
    if (!load_image(dir, table, num_sigs)) {
        std::fprintf(stderr, "bad image in %s\n", dir.c_str());
        return 1;
    }
    std::vector<std::string> functions, otus;
    if (!load_index_file(dir + "/function.index", functions) ||
        !load_index_file(dir + "/otu.index", otus)) {
        std::fprintf(stderr, "missing/bad index files in %s\n", dir.c_str());
        return 1;
    }
    std::ifstream in(fasta, std::ios::binary);
    std::stringstream ss;
    ss << in.rdbuf();
    if (mode == "fq") {
        std::vector<const char *> fn;
        for (auto &f : functions)
            fn.push_back(f.c_str());
        void *q = oracle_fq_new(table.data(), num_sigs, fn.data(), fn.size(), qp["genus"].c_str(),
                                qp["families"].c_str(), qp["nr"].c_str());
        if (!q) {
            std::fprintf(stderr, "cannot load the family files\n");
            return 1;
        }
        const std::string text = ss.str();
        char *out = oracle_fq_process(q, text.data(), text.size());
        std::fwrite(out, 1, std::strlen(out), stdout);
        oracle_free(out);
        oracle_fq_free(q);
        return 0;
    }
    if (mode == "lookup") {
        std::vector<const char *> fn;
        for (auto &f : functions)
            fn.push_back(f.c_str());
        const bool family_mode = qp["family_mode"] == "1";
        /* the NR family load runs only for a family-mode server */
        void *q = oracle_lookup_new(table.data(), num_sigs, fn.data(), fn.size(), qp["genus"].c_str(),
                                    qp["families"].c_str(), family_mode ? qp["nr"].c_str() : "",
                                    family_mode ? "" : fasta.c_str());
        if (!q) {
            std::fprintf(stderr, "cannot load the family files\n");
            return 1;
        }
        std::vector<const char *> names, values;
        for (auto &kv : qp) {
            names.push_back(kv.first.c_str());
            values.push_back(kv.second.c_str());
        }
        const std::string text = ss.str();
        char *out = oracle_lookup_process(q, family_mode, names.data(), values.data(), names.size(), text.data(),
                                          text.size());
        std::fwrite(out, 1, std::strlen(out), stdout);
        oracle_free(out);
        oracle_lookup_free(q);
        return 0;
    }
    auto records = parse_fasta(ss.str());

    Scorer scorer(table.data(), num_sigs);
    /* set_parameters, kguts.cc:244-268: defaults, then std::stoi per known key;
     * std::invalid_argument only warns. */
    scorer.params = Params();
    {
        std::map<std::string, int *> pm = {{"order_constraint", &scorer.params.order_constraint},
                                           {"min_hits", &scorer.params.min_hits},
                                           {"min_weighted_hits", &scorer.params.min_weighted_hits},
                                           {"max_gap", &scorer.params.max_gap}};
        for (auto &kv : qp) {
            auto it = pm.find(kv.first);
            if (it == pm.end())
                continue;
            try {
                *it->second = std::stoi(kv.second);
            } catch (const std::invalid_argument &) {
                std::cerr << "Warning: invalid integer '" << kv.second << "' passed for parameter "
                          << kv.first << "\n";
            }
        }
    }

    std::ostringstream os;
    if (mode == "matrix") {
        /* KmerPegMapping::encode_id: ids from 0 in first-seen order (kmer.h:114-121) */
        std::map<std::string, uint32_t> peg_to_id;
        std::vector<std::string> id_to_peg;
        auto encode = [&](const std::string &p) {
            auto it = peg_to_id.find(p);
            if (it != peg_to_id.end())
                return it->second;
            uint32_t id = (uint32_t)id_to_peg.size();
            peg_to_id[p] = id;
            id_to_peg.push_back(p);
            return id;
        };
        std::vector<std::vector<uint64_t>> kmers(records.size());
        for (size_t r = 0; r < records.size(); r++) {
            std::vector<SeqHit> hits;
            scorer.process(records[r].second.c_str(), records[r].second.size(), nullptr, &hits, nullptr,
                           true);
            for (auto &h : hits)
                kmers[r].push_back(h.hit.which_kmer);
        }
        void *km = oracle_kmap_new(0);
        for (size_t r = 0; r < records.size(); r++) { /* /add */
            std::vector<uint32_t> ids(kmers[r].size(), encode(records[r].first));
            oracle_kmap_add(km, kmers[r].data(), ids.data(), ids.size());
        }
        void *mx = oracle_matrix_new();
        for (size_t r = 0; r < records.size(); r++) { /* /matrix */
            uint32_t id = encode(records[r].first);
            uint64_t len = records[r].second.size(), off[2] = {0, kmers[r].size()};
            oracle_matrix_add(mx, km, &id, &len, 1, off, kmers[r].data());
        }
        uint64_t n = oracle_matrix_pairs(mx, nullptr, nullptr, nullptr, nullptr);
        std::vector<uint32_t> a(n), b(n);
        std::vector<uint64_t> c(n);
        std::vector<float> sc(n);
        oracle_matrix_pairs(mx, a.data(), b.data(), c.data(), sc.data());
        for (uint64_t i = 0; i < n; i++)
            os << id_to_peg[a[i]] << "\t" << id_to_peg[b[i]] << "\t" << (unsigned long)c[i] << "\t" << sc[i]
               << "\n";
        oracle_matrix_free(mx);
        oracle_kmap_free(km);
        std::fwrite(os.str().data(), 1, os.str().size(), stdout);
        return 0;
    }
    const bool details = (mode == "query_details");
    for (auto &rec : records) {
        const std::string &id = rec.first, &seq = rec.second;
        std::vector<Call> calls;
        std::vector<SeqHit> hits;
        OtuStats stats;
        bool want_hits = details || mode == "add";
        scorer.process(seq.c_str(), seq.size(), &calls, want_hits ? &hits : nullptr, &stats, true);
        if (mode == "query_best") {
            int fi;
            std::string fn;
            float score, wscore, off = 0.0f;
            find_best_call(calls, functions, fi, fn, score, wscore, off);
            if (!fn.empty())
                os << id << "\t" << fn << "\t" << score << "\t" << wscore << "\n";
        } else if (mode == "add") {
            os << "PROTEIN-ID\t" << id << "\t" << seq.size() << "\n";
            for (auto &c : calls)
                os << format_call(c, functions);
            os << format_otu_stats(id, seq.size(), stats);
            int fi;
            std::string fn;
            /* best_call_score_offset is uninitialised in the reference when
             * there are no calls (add_request.cc:334); defined as 0 here. */
            float score, wscore, off = 0.0f;
            find_best_call(calls, functions, fi, fn, score, wscore, off);
            if (fn.empty() || fn.find(" ?? ") != std::string::npos)
                fn = "hypothetical protein";
            os << "BEST-CALL\t" << id << "\t" << fn << "\t" << score << "\t" << wscore << "\t" << off
               << "\n";
        } else {
            os << "PROTEIN-ID\t" << id << "\t" << seq.size() << "\n";
            for (auto &c : calls)
                os << format_call(c, functions);
            if (details)
                for (auto &h : hits)
                    os << format_hit(h, functions);
            os << format_otu_stats(id, seq.size(), stats);
        }
    }
    std::fwrite(os.str().data(), 1, os.str().size(), stdout);
    return 0;
}
