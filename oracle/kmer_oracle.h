/*
 * kmer_oracle.h -- CPU restatement of close_kmers' k-mer encode -> hash-probe ->
 * hit-score path (KmerGuts::process_aa_seq over a KmerImage).
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the MI355X path in
 * close_kmers_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may link, load or run anything built from oracle/.  The
 * product library never includes this header.
 *
 * Parity status (see DESIGN.md "Oracle"): the reference's own kguts.cc and
 * kmer_image.cc include boost headers that this image lacks, so they are
 * unbuildable here.  This restatement is pinned by:
 *   - the reference's KmerEncoder (kmer_encoder.cc), KmerOtuStats (kguts.h),
 *     FastaParser (fasta_parser.cc) and TranslationTable (trans_table.cc),
 *     compiled from /root/reference into oracle/_ref/ (see oracle/Makefile);
 *   - the known-answer example in SCORING.txt:15-20,28-49,84-97.
 * The probe loop and the gather_hits/process_set_of_hits state machine are
 * restated line by line from kguts.cc (cited per function) and are otherwise
 * "parity partially pinned" (SCORING.txt's HIT->CALL example only).
 */
#ifndef KMER_ORACLE_H
#define KMER_ORACLE_H

#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace oracle {

/* kmer_params.h:5-19 */
constexpr int K = 8;
constexpr uint64_t CORE = 1280000000ULL;          /* 20^7 */
constexpr uint64_t MAX_ENCODED = 25600000000ULL;  /* 20^8 */
constexpr uint64_t EMPTY_KEY = MAX_ENCODED + 1;   /* kguts.cc:106-107 */
constexpr int MAX_HITS_PER_SEQ = 40000;           /* kmer_params.h:20 */

/* kmer_image.h:11-23 -- one 24-byte bucket of kmer.table.mem_map */
struct SigKmer {
    uint64_t which_kmer;
    int32_t otu_index;
    uint16_t avg_from_end;
    int32_t function_index;
    float function_wt;
};
static_assert(sizeof(SigKmer) == 24, "sig_kmer_t is 24 bytes");

/* kmer_image.h:11-15 */
struct ImageHeader {
    uint64_t num_sigs;
    uint64_t entry_size;
    int64_t version;
};

/* kguts.h:154-163 (KmerHit) -- the run buffer element */
struct RunHit {
    uint32_t oI;
    uint32_t pos;
    uint16_t avg;
    uint32_t fI;
    float wt;
};

/* kguts.h:166-183 */
struct Call {
    uint32_t start;
    uint32_t end;
    int32_t count;
    uint32_t function_index;
    float weighted_hits;
};

/* kguts.h:228-233 (hit_in_sequence_t): a copy of the bucket plus the offset */
struct SeqHit {
    SigKmer hit;
    uint32_t offset;
};

/* kguts.cc:236-242 */
struct Params {
    int order_constraint = 0;
    int min_hits = 5;
    int min_weighted_hits = 0;
    int max_gap = 200;
};

/* kguts.h:185-219 */
struct OtuStats {
    std::map<int, int> otu_map;
    std::vector<std::pair<int, int>> otus_by_count;
    void finalize();
};

/* Per-sequence scorer: one object per CPU thread, like one KmerGuts per pool
 * thread (threadpool.cc:33).  Mutable state mirrors kguts.h:263-293. */
class Scorer {
public:
    Scorer(const SigKmer *table, uint64_t num_sigs);
    Params params;
    /* process_aa_seq (kguts.cc:888-908); null pointers = not requested */
    void process(const char *seq, size_t len, std::vector<Call> *calls,
                 std::vector<SeqHit> *hits, OtuStats *otu, bool run_scorer);
    /* total probes (buckets examined) so far; for P-bar */
    uint64_t probes = 0;
    uint64_t windows = 0;

private:
    const SigKmer *table_;
    uint64_t num_sigs_;
    std::vector<RunHit> buf_;
    int num_hits_ = 0;
    uint32_t current_fI_ = 0;
    int64_t lookup(uint64_t key);
    void flush(std::vector<Call> *calls, OtuStats *otu);
};

unsigned char residue_code(char c);
uint64_t encode8(const unsigned char *codes);
void decode8(uint64_t key, char out[9]);

/* find_best_call (kguts.cc:1008-1199).  decision (optional): which branch
 * set the outputs -- [0] 0 no calls, 1 called, 2 ambiguous pair, 3 no call;
 * [1], [2] the function indices behind the call / the pair (vec[0], vec[1]
 * of :1134-1139), -1 where none -- so a caller without function names can
 * still tell the decisions apart */
void find_best_call(const std::vector<Call> &calls,
                    const std::vector<std::string> &functions, int &function_index,
                    std::string &function, float &score, float &weighted_score,
                    float &score_offset, int *decision = nullptr);

/* FastaParser framing (fasta_parser.h:38-144, fasta_parser.cc:30-36) */
std::vector<std::pair<std::string, std::string>> parse_fasta(const std::string &text);

/* TranslationTable::make_table(11).translate (trans_table.cc:65-84) */
std::string translate11(const std::string &dna);

/* load_indexed_ar (kguts.cc:544-575); returns false if the file is missing */
bool load_index_file(const std::string &path, std::vector<std::string> &out);

/* insert_kmer / find_empty_hash_entry (kguts.cc:166-171,202-222).
 * Returns 0, or 1 when the table would become half full (the reference exits). */
int insert_key(SigKmer *table, uint64_t num_sigs, uint64_t &loaded, uint64_t key,
               int32_t fI, int32_t oI, uint16_t avg, float wt);

/* format_call / format_hit / format_otu_stats (kguts.cc:939-973) */
std::string format_call(const Call &c, const std::vector<std::string> &functions);
std::string format_hit(const SeqHit &h, const std::vector<std::string> &functions);
std::string format_otu_stats(const std::string &id, size_t size, const OtuStats &s);

}  // namespace oracle

#endif
