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

#include "kgx_handlers.h"

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
        std::ifstream in(fasta, std::ios::binary);
        if (!in) {
            std::fprintf(stderr, "cannot open %s\n", fasta.c_str());
            return 1;
        }
        std::stringstream ss;
        ss << in.rdbuf();
        const std::string body = ss.str();
        const work_list_t work = parse_fasta_body(body.data(), body.size());
        std::ostringstream os;
        if (mode == "lookup") {
            auto mapping = std::make_shared<KmerPegMapping>(kgx_image_device(image->handle()));
            if (!qp["genus"].empty())
                mapping->load_genus_map(qp["genus"]);
            if (!qp["families"].empty())
                mapping->load_families(qp["families"]);
            const bool family_mode = qp["family_mode"] == "1";
            if (family_mode && !qp["nr"].empty())
                mapping->load_nr_families(kguts, qp["nr"]);
            if (!family_mode) { /* a silent /add of the same FASTA first */
                std::ostringstream discard;
                add_request(kguts, *mapping, work, 1, discard);
            }
            lookup_request(kguts, mapping, family_mode, qp, work, os);
        } else if (mode == "matrix") {
            /* /add of the FASTA into an empty mapping, then one /matrix request */
            auto mapping = std::make_shared<KmerPegMapping>(kgx_image_device(image->handle()));
            std::ostringstream discard;
            add_request(kguts, *mapping, work, 1, discard);
            matrix_request(kguts, mapping, work, os);
        } else if (mode == "add") {
            KmerPegMapping mapping(kgx_image_device(image->handle()));
            add_request(kguts, mapping, work, 0, os);
        } else {
            query_request(kguts, work, mode == "query_details", mode == "query_best", os);
        }
        const std::string s = os.str();
        std::fwrite(s.data(), 1, s.size(), stdout);
    } catch (const Error &e) {
        std::fprintf(stderr, "kgx_query: %s\n", e.what());
        return 1;
    }
    return 0;
}
