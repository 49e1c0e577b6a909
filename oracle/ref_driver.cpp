/*
 * ref_driver.cpp -- C entry points over the parts of the reference that build
 * from their own sources with the stock toolchain (no stand-in headers):
 *
 *   kmer_encoder.cc (+ kguts.h, kmer_image.h, kmer_params.h, kmer_encoder.h)
 *   fasta_parser.cc (+ fasta_parser.h)
 *   trans_table.cc  (+ trans_table.h)
 *   kguts.h's header-only KmerOtuStats (finalize / std::sort tie order)
 *
 * TEST INFRASTRUCTURE ONLY.  Compiled by oracle/Makefile with
 * -I/root/reference straight from the read-only reference tree into
 * oracle/_ref/libref.so; used to pin the oracle restatement.  kguts.cc and
 * kmer_image.cc include boost headers that this image lacks, so they are not
 * built (DESIGN.md "Oracle").
 */
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kguts.h"
#include "kmer_encoder.h"
#include "fasta_parser.h"
#include "trans_table.h"

extern "C" {

/* KmerEncoder::encoded_aa_kmer (kmer_encoder.h:212-225) */
unsigned long long ref_encode(const char *kmer)
{
    static KmerEncoder enc;
    return enc.encoded_aa_kmer(kmer);
}

/* KmerEncoder::decoded_kmer (kmer_encoder.h:245-255) */
void ref_decode(unsigned long long key, char *out9)
{
    static KmerEncoder enc;
    enc.decoded_kmer(key, out9);
}

/* KmerEncoder::to_amino_acid_off (kmer_encoder.h:189-191); byte 255 is left
 * uninitialised by the constructor (kmer_encoder.cc:9), callers skip it. */
int ref_residue_code(int c)
{
    static KmerEncoder enc;
    return enc.to_amino_acid_off((uint8_t)c);
}

/* KmerOtuStats::finalize (kguts.h:214-218): fill otu_map with (otu, count)
 * pairs, finalize, and return otus_by_count in out_pairs (2*n ints). */
int ref_otu_finalize(const int *otus, const int *counts, int n, int *out_pairs)
{
    KmerOtuStats s;
    for (int i = 0; i < n; i++)
        s.otu_map[otus[i]] += counts[i];
    s.finalize();
    int k = 0;
    for (auto &p : s.otus_by_count) {
        out_pairs[2 * k] = p.first;
        out_pairs[2 * k + 1] = p.second;
        k++;
    }
    return k;
}

/* FastaParser (fasta_parser.h:38-165, fasta_parser.cc:1-36): parse text, then
 * return records as "id\tseq\n" lines in a malloc'd buffer. */
char *ref_fasta_parse(const char *text, unsigned long len)
{
    std::string out;
    FastaParser parser;
    parser.set_callback([&out](const std::string &id, const std::string &seq) {
        out += id;
        out += '\t';
        out += seq;
        out += '\n';
        return 0;
    });
    parser.set_error_callback([](const std::string &, int, const std::string) { return true; });
    for (unsigned long i = 0; i < len; i++)
        parser.parse_char(text[i]);
    parser.parse_complete();
    char *buf = (char *)std::malloc(out.size() + 1);
    std::memcpy(buf, out.data(), out.size());
    buf[out.size()] = 0;
    return buf;
}

void ref_free(void *p) { std::free(p); }

/* TranslationTable::make_table(11).translate (trans_table.cc:17-84) */
char *ref_translate11(const char *dna, unsigned long len)
{
    static TranslationTable t = TranslationTable::make_table(11);
    std::string s(dna, len);
    std::string p = t.translate(s.begin(), s.end());
    char *buf = (char *)std::malloc(p.size() + 1);
    std::memcpy(buf, p.data(), p.size());
    buf[p.size()] = 0;
    return buf;
}

}  /* extern "C" */
