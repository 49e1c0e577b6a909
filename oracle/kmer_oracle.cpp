/*
 * kmer_oracle.cpp -- CPU restatement of the KmerGuts hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see kmer_oracle.h).  Every function cites the
 * reference file:line it restates.  Built by oracle/Makefile into
 * oracle/_build/liboracle.so (ctypes API at the bottom of this file) and
 * linked into oracle/_build/oracle_query.
 */
#include "kmer_oracle.h"

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <sstream>
#include <thread>

namespace oracle {

static const char kAlpha[20] = {'A', 'C', 'D', 'E', 'F', 'G', 'H', 'I', 'K', 'L',
                                'M', 'N', 'P', 'Q', 'R', 'S', 'T', 'V', 'W', 'Y'};

/* to_amino_acid_off, kguts.cc:273-339: the 20 upper-case residues map to
 * 0..19, every other byte (lower case, X, *, B, Z, U, ...) to 20. */
unsigned char residue_code(char c)
{
    for (unsigned char i = 0; i < 20; i++)
        if (kAlpha[i] == c)
            return i;
    return 20;
}

/* encoded_kmer, kguts.cc:438-455: big-endian base-20 Horner over 8 codes. */
uint64_t encode8(const unsigned char *codes)
{
    uint64_t v = codes[0];
    for (int i = 1; i < K; i++)
        v = v * 20 + codes[i];
    return v;
}

/* decoded_kmer, kguts.cc:473-483 */
void decode8(uint64_t key, char out[9])
{
    out[K] = 0;
    for (int i = K - 1; i >= 0; i--) {
        out[i] = kAlpha[key % 20];
        key /= 20;
    }
}

/* KmerOtuStats::finalize, kguts.h:214-218: map entries appended, then
 * std::sort by count descending (less_second: rhs.second < lhs.second). */
void OtuStats::finalize()
{
    otus_by_count.insert(otus_by_count.begin(), otu_map.begin(), otu_map.end());
    std::sort(otus_by_count.begin(), otus_by_count.end(),
              [](const std::pair<int, int> &a, const std::pair<int, int> &b) {
                  return b.second < a.second;
              });
}

Scorer::Scorer(const SigKmer *table, uint64_t num_sigs)
    : table_(table), num_sigs_(num_sigs), buf_(MAX_HITS_PER_SEQ)
{
}

/* lookup_hash_entry, kguts.cc:585-602.  Linear probe from key % num_sigs,
 * stopping at the key or at any bucket whose key exceeds 20^8.  The reference
 * never terminates on a full table that lacks the key; we stop after
 * num_sigs buckets and report a miss. */
int64_t Scorer::lookup(uint64_t key)
{
    uint64_t h = key % num_sigs_;
    for (uint64_t n = 0; n < num_sigs_; n++) {
        probes++;
        uint64_t k = table_[h].which_kmer;
        if (k == key)
            return (int64_t)h;
        if (k > MAX_ENCODED)
            return -1;
        h = (h + 1) % num_sigs_;
    }
    return -1;
}

/* process_set_of_hits, kguts.cc:734-781. */
void Scorer::flush(std::vector<Call> *calls, OtuStats *otu)
{
    if (!calls && !otu)
        return; /* kguts.cc:737-738: no reset either */
    if (num_hits_ == 0) {
        /* Reachable only with min_hits <= 0 at the final flush, where the
         * reference reads hits[-2] (UB).  Defined here as "emit nothing". */
        return;
    }
    int count = 0;
    float wsum = 0.0f;
    int last = 0;
    for (int i = 0; i < num_hits_; i++) {
        if (buf_[i].fI == current_fI_) {
            last = i;
            count++;
            wsum += buf_[i].wt;
        }
    }
    if (count >= params.min_hits && wsum >= (float)params.min_weighted_hits) {
        if (calls)
            calls->push_back(Call{buf_[0].pos, buf_[last].pos + (K - 1), count,
                                  current_fI_, wsum});
        if (otu) {
            for (int i = 0; i <= last; i++)
                if (buf_[i].fI == current_fI_)
                    otu->otu_map[(int)buf_[i].oI]++;
        }
    }
    /* kguts.cc:772-780: carry a trailing same-function pair into a new run.
     * With one buffered hit the condition is false (that hit set current_fI). */
    if (num_hits_ >= 2 && buf_[num_hits_ - 2].fI != current_fI_ &&
        buf_[num_hits_ - 2].fI == buf_[num_hits_ - 1].fI) {
        current_fI_ = buf_[num_hits_ - 1].fI;
        RunHit a = buf_[num_hits_ - 2], b = buf_[num_hits_ - 1];
        buf_[0] = a;
        buf_[1] = b;
        num_hits_ = 2;
    } else {
        num_hits_ = 0;
    }
}

/* advance_past_ambig, kguts.cc:694-731 (KMER_SIZE == 8): while the window at
 * p holds a code-20 residue, jump past the rightmost such residue. */
static void skip_ambiguous(const unsigned char *codes, long &p, long bound)
{
    bool bad = true;
    while (p < bound && bad) {
        bad = false;
        for (int j = K - 1; j >= 0; j--) {
            if (codes[p + j] == 20) {
                p += j + 1;
                bad = true;
                break;
            }
        }
    }
}

/* process_aa_seq (kguts.cc:888-908) + gather_hits (kguts.cc:783-877). */
void Scorer::process(const char *seq, size_t len, std::vector<Call> *calls,
                     std::vector<SeqHit> *hits, OtuStats *otu, bool run_scorer)
{
    std::vector<unsigned char> codes(len + 1);
    for (size_t i = 0; i < len; i++)
        codes[i] = residue_code(seq[i]);
    /* kguts.cc:792 bounds the walk with strlen(), not the string's size */
    size_t slen = strnlen(seq, len);
    long bound = (long)slen - K; /* windows start at p < bound */
    long p = 0;
    num_hits_ = 0;
    skip_ambiguous(codes.data(), p, bound);
    uint64_t key = 0;
    if (p < bound)
        key = encode8(&codes[p]);
    while (p < bound) {
        windows++;
        int64_t slot = lookup(key);
        uint32_t pos = (uint32_t)p;
        if (slot >= 0) {
            const SigKmer &e = table_[slot];
            if (hits) { /* hit_cb runs before the run logic, kguts.cc:814-815 */
                SeqHit h;
                std::memset(&h, 0, sizeof(h));
                h.hit.which_kmer = e.which_kmer;
                h.hit.otu_index = e.otu_index;
                h.hit.avg_from_end = e.avg_from_end;
                h.hit.function_index = e.function_index;
                h.hit.function_wt = e.function_wt;
                h.offset = pos;
                hits->push_back(h);
            }
            if (run_scorer) {
                const uint16_t avg = e.avg_from_end;
                const uint32_t fI = (uint32_t)e.function_index;
                const uint32_t oI = (uint32_t)e.otu_index;
                const float wt = e.function_wt;
                /* gap rule, kguts.cc:821-831 (unsigned arithmetic) */
                if (num_hits_ > 0 &&
                    (uint32_t)(buf_[num_hits_ - 1].pos + (uint32_t)params.max_gap) < pos) {
                    if (num_hits_ >= params.min_hits)
                        flush(calls, otu);
                    else
                        num_hits_ = 0;
                }
                if (num_hits_ == 0)
                    current_fI_ = fI;
                /* order constraint, kguts.cc:838-842: labs() of an unsigned
                 * 32-bit difference */
                bool accept = true;
                if (params.order_constraint && num_hits_ > 0) {
                    const RunHit &prev = buf_[num_hits_ - 1];
                    uint32_t d = (uint32_t)(pos - prev.pos) -
                                 (uint32_t)((int)prev.avg - (int)avg);
                    accept = (fI == prev.fI) && d <= 20u;
                }
                if (accept) {
                    buf_[num_hits_] = RunHit{oI, pos, avg, fI, wt};
                    if (num_hits_ < MAX_HITS_PER_SEQ - 2)
                        num_hits_++;
                    /* pair switch, kguts.cc:852-856 */
                    if (num_hits_ > 1 && current_fI_ != fI &&
                        buf_[num_hits_ - 2].fI == buf_[num_hits_ - 1].fI)
                        flush(calls, otu);
                }
            }
        }
        /* advance, kguts.cc:859-871 */
        p++;
        if (p < bound) {
            if (codes[p + K - 1] < 20) {
                key = (key % CORE) * 20 + codes[p + K - 1];
            } else {
                p += K;
                skip_ambiguous(codes.data(), p, bound);
                if (p < bound)
                    key = encode8(&codes[p]);
            }
        }
    }
    if (run_scorer && num_hits_ >= params.min_hits)
        flush(calls, otu);
    num_hits_ = 0;
    if (otu)
        otu->finalize();
}

/* FastaParser::parse_char / parse_complete, fasta_parser.h:38-144,
 * fasta_parser.cc:30-36.  Callback fires on each '>' after data and once at
 * the end (possibly with an empty record). */
std::vector<std::pair<std::string, std::string>> parse_fasta(const std::string &text)
{
    enum { START, ID, DEFLINE, DATA, ID_OR_DATA } st = START;
    std::vector<std::pair<std::string, std::string>> out;
    std::string id, seq;
    for (char c : text) {
        if (c == '\r')
            continue;
        bool err = false;
        switch (st) {
        case START:
            if (c != '>')
                err = true;
            else
                st = ID;
            break;
        case ID:
            if (std::isblank((unsigned char)c))
                st = DEFLINE;
            else if (c == '\n')
                st = DATA;
            else
                id.push_back(c);
            break;
        case DEFLINE:
            if (c == '\n')
                st = DATA;
            break;
        case DATA:
            if (c == '\n')
                st = ID_OR_DATA;
            else if (std::isalpha((unsigned char)c) || c == '*')
                seq.push_back(c);
            else
                err = true;
            break;
        case ID_OR_DATA:
            if (c == '>') {
                out.emplace_back(id, seq);
                id.clear();
                seq.clear();
                st = ID;
            } else if (c == '\n') {
            } else if (std::isalpha((unsigned char)c)) {
                seq.push_back(c);
                st = DATA;
            } else {
                err = true;
            }
            break;
        }
        (void)err; /* the reference logs and continues (no error callback set) */
    }
    out.emplace_back(id, seq);
    return out;
}


/* TranslationTable code 11 (trans_table.cc:8-63, trans_table.h:45-83):
 * codon index e1*16 + e2*4 + e3 with A=0 C=1 G=2 T/U=3 (either case); any
 * other base -> index 64 -> 'X'. */
static const char *kAAs = "FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
static const char *kB1 = "TTTTTTTTTTTTTTTTCCCCCCCCCCCCCCCCAAAAAAAAAAAAAAAAGGGGGGGGGGGGGGGG";
static const char *kB2 = "TTTTCCCCAAAAGGGGTTTTCCCCAAAAGGGGTTTTCCCCAAAAGGGGTTTTCCCCAAAAGGGG";
static const char *kB3 = "TCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAG";

static int base_code(char c)
{
    switch (c) {
    case 'a': case 'A': return 0;
    case 'c': case 'C': return 1;
    case 'g': case 'G': return 2;
    case 't': case 'u': case 'T': case 'U': return 3;
    default: return 4;
    }
}

std::string translate11(const std::string &dna)
{
    static char table[65];
    static bool init = false;
    if (!init) {
        for (int i = 0; i < 64; i++)
            table[base_code(kB1[i]) * 16 + base_code(kB2[i]) * 4 + base_code(kB3[i])] = kAAs[i];
        table[64] = 'X';
        init = true;
    }
    std::string out;
    for (size_t i = 0; i + 3 <= dna.size(); i += 3) {
        int a = base_code(dna[i]), b = base_code(dna[i + 1]), c = base_code(dna[i + 2]);
        out.push_back((a < 4 && b < 4 && c < 4) ? table[a * 16 + b * 4 + c] : table[64]);
    }
    return out;
}

static const char *function_at(const std::vector<std::string> &f, int i)
{
    /* KmerGuts::function_at_index, kguts.h:361-366 */
    if (i < 0 || i >= (int)f.size())
        return "INVALID_OFFSET";
    return f[i].c_str();
}

/* find_best_call, kguts.cc:1008-1199 */
void find_best_call(const std::vector<Call> &calls, const std::vector<std::string> &functions,
                    int &function_index, std::string &function, float &score,
                    float &weighted_score, float &score_offset, int *decision)
{
    int dummy[3];
    int *d = decision ? decision : dummy;
    d[0] = 0;
    d[1] = d[2] = -1;
    function_index = -1;
    function = "";
    score = 0.0f;
    weighted_score = 0.0f;
    if (calls.empty())
        return; /* score_offset untouched, kguts.cc:1015-1018 */
    d[0] = 3;

    /* 1: collapse runs of adjacent calls with one function (:1023-1040) */
    std::vector<Call> collapsed;
    for (size_t i = 0; i < calls.size();) {
        Call cur = calls[i++];
        while (i < calls.size() && calls[i].function_index == cur.function_index) {
            cur.end = calls[i].end;
            cur.count += calls[i].count;
            cur.weighted_hits += calls[i].weighted_hits;
            i++;
        }
        collapsed.push_back(cur);
    }

    /* 2: F1 F2 F1 with |F2| < 5 and |F1|+|F1'| >= 10 -> one F1 (:1063-1086) */
    std::vector<Call> merged;
    for (size_t i = 0; i < collapsed.size();) {
        Call cur = collapsed[i++];
        while (i + 1 < collapsed.size() &&
               cur.function_index == collapsed[i + 1].function_index &&
               collapsed[i].count < 5 && cur.count + collapsed[i + 1].count >= 10) {
            cur.end = collapsed[i + 1].end;
            cur.count += collapsed[i + 1].count;
            cur.weighted_hits += collapsed[i + 1].weighted_hits;
            i += 2;
        }
        merged.push_back(cur);
    }

    /* 3: per-function totals in function-index order (:1108-1131) */
    struct Tot {
        int count;
        float weighted;
    };
    std::map<int, Tot> by_func;
    for (const Call &c : merged) {
        auto it = by_func.find((int)c.function_index);
        if (it == by_func.end())
            by_func.emplace((int)c.function_index, Tot{c.count, c.weighted_hits});
        else {
            it->second.count += c.count;
            it->second.weighted += c.weighted_hits;
        }
    }
    std::vector<std::pair<int, Tot>> vec(by_func.begin(), by_func.end());
    /* top two by weighted score; libstdc++ partial_sort fixes the tie order and
     * what lands at vec[2] (:1134-1139) */
    if (vec.size() > 1)
        std::partial_sort(vec.begin(), vec.begin() + 2, vec.end(),
                          [](const std::pair<int, Tot> &a, const std::pair<int, Tot> &b) {
                              return a.second.weighted > b.second.weighted;
                          });
    if (vec.size() == 1)
        score_offset = (float)vec[0].second.count;
    else
        score_offset = (float)(vec[0].second.count - vec[1].second.count);

    if (score_offset >= 5.0f) { /* code says >= 5 (SCORING.txt:77 says > 5) */
        d[0] = 1;
        d[1] = vec[0].first;
        function_index = vec[0].first;
        function = function_at(functions, function_index);
        score = (float)vec[0].second.count;
        weighted_score = vec[0].second.weighted;
        return;
    }
    function_index = -1;
    function = "";
    score = 0.0f;
    if (vec.size() >= 2) {
        std::string f1 = function_at(functions, vec[0].first);
        std::string f2 = function_at(functions, vec[1].first);
        if (f2 > f1)
            std::swap(f1, f2);
        if (vec.size() == 2) {
            d[0] = 2;
            d[1] = vec[0].first;
            d[2] = vec[1].first;
            function = f1 + " ?? " + f2;
            score = (float)vec[0].second.count;
        } else {
            float pair_offset = (float)(vec[1].second.count - vec[2].second.count);
            if (pair_offset > 5.0f) {
                d[0] = 2;
                d[1] = vec[0].first;
                d[2] = vec[1].first;
                function = f1 + " ?? " + f2;
                score = (float)vec[0].second.count;
                score_offset = pair_offset;
                weighted_score = vec[0].second.weighted;
            }
        }
    }
}

/* load_indexed_ar, kguts.cc:544-575: "%d\t" then fgets(1000); the last
 * character of each line (normally '\n') is dropped; the index must be dense. */
bool load_index_file(const std::string &path, std::vector<std::string> &out)
{
    FILE *f = std::fopen(path.c_str(), "r");
    if (!f)
        return false;
    out.clear();
    int j;
    char line[1000];
    while (std::fscanf(f, "%d\t", &j) == 1 && std::fgets(line, 1000, f)) {
        if (j != (int)out.size()) {
            std::fclose(f);
            return false; /* reference exits: "index must be dense and in order" */
        }
        size_t n = std::strlen(line);
        if (n > 0)
            line[n - 1] = 0;
        out.emplace_back(line);
    }
    std::fclose(f);
    return true;
}

/* insert_kmer + find_empty_hash_entry, kguts.cc:166-171,202-222 */
int insert_key(SigKmer *table, uint64_t num_sigs, uint64_t &loaded, uint64_t key, int32_t fI,
               int32_t oI, uint16_t avg, float wt)
{
    if (key > MAX_ENCODED)
        return 0;
    uint64_t h = key % num_sigs;
    while (table[h].which_kmer <= MAX_ENCODED)
        h = (h + 1) % num_sigs;
    loaded++;
    if ((int64_t)loaded >= (int64_t)num_sigs / 2)
        return 1; /* "Your Kmer hash is half-full" -> exit(1) in the reference */
    table[h].which_kmer = key;
    table[h].avg_from_end = avg;
    table[h].function_index = fI;
    table[h].otu_index = oI;
    table[h].function_wt = wt;
    return 0;
}

/* format_call, kguts.cc:939-947 */
std::string format_call(const Call &c, const std::vector<std::string> &functions)
{
    std::ostringstream oss;
    oss << "CALL\t" << c.start << "\t" << c.end << "\t" << c.count;
    oss << "\t" << c.function_index << "\t" << function_at(functions, (int)c.function_index);
    oss << "\t" << c.weighted_hits << "\n";
    return oss.str();
}

/* format_hit, kguts.cc:949-959 */
std::string format_hit(const SeqHit &h, const std::vector<std::string> &functions)
{
    char dc[K + 1];
    decode8(h.hit.which_kmer, dc);
    std::ostringstream oss;
    oss << "HIT\t" << h.offset << "\t" << dc << "\t" << h.hit.avg_from_end << "\t"
        << function_at(functions, h.hit.function_index) << "\t" << h.hit.function_wt << "\t"
        << h.hit.otu_index << "\n";
    return oss.str();
}

/* format_otu_stats, kguts.cc:961-973: at most five entries */
std::string format_otu_stats(const std::string &id, size_t size, const OtuStats &s)
{
    std::ostringstream oss;
    oss << "OTU-COUNTS\t" << id << "[" << size << "]";
    size_t n = std::min(s.otus_by_count.size(), (size_t)5);
    for (size_t i = 0; i < n; i++)
        oss << "\t" << s.otus_by_count[i].second << "-" << s.otus_by_count[i].first;
    oss << "\n";
    return oss.str();
}

}  // namespace oracle

/* ------------------------------------------------------------------------ */
/* ctypes API (tests / smoke / bench cpu_baseline only)                      */
/* ------------------------------------------------------------------------ */

using namespace oracle;

extern "C" {

/* 32-byte hit record: the bucket copy (pad zeroed) + offset + sequence index */
struct oracle_hit {
    SigKmer entry;
    uint32_t pos;
    uint32_t seq;
};
static_assert(sizeof(oracle_hit) == 32, "hit record is 32 bytes");
static_assert(sizeof(Call) == 20, "KmerCall is 20 bytes");

/* find_best_call's outputs for one sequence (kguts.cc:1008-1199; function
 * names are not loaded: every index reads as INVALID_OFFSET) */
struct oracle_best {
    int32_t function_index;
    float score, weighted_score, score_offset;
    int32_t offset_set; /* 0: score_offset left untouched (no calls, kguts.cc:1015-1018) */
    int32_t kind, fi0, fi1; /* find_best_call's decision argument */
};

struct oracle_result {
    uint64_t n_seq;
    uint64_t *hit_offsets; /* n_seq + 1 */
    oracle_hit *hits;
    uint64_t *call_offsets; /* n_seq + 1 */
    Call *calls;
    uint64_t *otu_offsets; /* n_seq + 1 */
    int32_t *otus;         /* pairs (otu_index, count), otus_by_count order */
    uint64_t probes;
    uint64_t windows;
    double seconds; /* processing loop only */
    oracle_best *best; /* n_seq entries with WANT_BEST, else NULL */
};

enum { WANT_HITS = 1, WANT_CALLS = 2, WANT_OTU = 4, WANT_BEST = 8 };

int oracle_process_batch(const void *table, uint64_t num_sigs, const int32_t *params4,
                         const char *residues, const uint64_t *offsets, uint64_t n_seq,
                         int want, int n_threads, oracle_result *out)
{
    if (n_threads < 1)
        n_threads = 1;
    std::memset(out, 0, sizeof(*out));
    out->n_seq = n_seq;
    struct PerSeq {
        std::vector<SeqHit> hits;
        std::vector<Call> calls;
        OtuStats otu;
        oracle_best best{};
    };
    const bool want_best = (want & WANT_BEST) != 0;
    const std::vector<std::string> no_names;
    std::vector<PerSeq> res(n_seq);
    std::vector<uint64_t> probes(n_threads, 0), windows(n_threads, 0);
    const SigKmer *tab = (const SigKmer *)table;

    auto worker = [&](int t) {
        Scorer s(tab, num_sigs);
        if (params4) {
            s.params.min_hits = params4[0];
            s.params.max_gap = params4[1];
            s.params.order_constraint = params4[2];
            s.params.min_weighted_hits = params4[3];
        }
        uint64_t lo = n_seq * t / n_threads, hi = n_seq * (t + 1) / n_threads;
        for (uint64_t i = lo; i < hi; i++) {
            PerSeq &r = res[i];
            s.process(residues + offsets[i], offsets[i + 1] - offsets[i],
                      (want & (WANT_CALLS | WANT_BEST)) ? &r.calls : nullptr,
                      (want & WANT_HITS) ? &r.hits : nullptr,
                      (want & WANT_OTU) ? &r.otu : nullptr,
                      (want & (WANT_CALLS | WANT_OTU | WANT_BEST)) != 0);
            if (want_best) { /* lookup_request.cc:203-210: per sequence, in the worker */
                std::string fn;
                float off = 0.0f;
                r.best.score_offset = std::numeric_limits<float>::quiet_NaN();
                off = r.best.score_offset;
                int dec[3];
                find_best_call(r.calls, no_names, r.best.function_index, fn, r.best.score, r.best.weighted_score,
                               off, dec);
                r.best.kind = dec[0];
                r.best.fi0 = dec[1];
                r.best.fi1 = dec[2];
                r.best.offset_set = !std::isnan(off);
                r.best.score_offset = r.best.offset_set ? off : 0.0f;
                if (!(want & WANT_CALLS))
                    r.calls.clear();
            }
        }
        probes[t] = s.probes;
        windows[t] = s.windows;
    };
    auto t0 = std::chrono::steady_clock::now();
    if (n_threads == 1) {
        worker(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < n_threads; t++)
            th.emplace_back(worker, t);
        for (auto &x : th)
            x.join();
    }
    auto t1 = std::chrono::steady_clock::now();
    out->seconds = std::chrono::duration<double>(t1 - t0).count();
    for (int t = 0; t < n_threads; t++) {
        out->probes += probes[t];
        out->windows += windows[t];
    }

    uint64_t nh = 0, nc = 0, no = 0;
    for (auto &r : res) {
        nh += r.hits.size();
        nc += r.calls.size();
        no += r.otu.otus_by_count.size();
    }
    out->hit_offsets = (uint64_t *)std::calloc(n_seq + 1, 8);
    out->call_offsets = (uint64_t *)std::calloc(n_seq + 1, 8);
    out->otu_offsets = (uint64_t *)std::calloc(n_seq + 1, 8);
    out->hits = (oracle_hit *)std::calloc(nh + 1, sizeof(oracle_hit));
    out->calls = (Call *)std::calloc(nc + 1, sizeof(Call));
    out->otus = (int32_t *)std::calloc(2 * no + 2, 4);
    uint64_t ih = 0, ic = 0, io = 0;
    for (uint64_t i = 0; i < n_seq; i++) {
        PerSeq &r = res[i];
        out->hit_offsets[i] = ih;
        out->call_offsets[i] = ic;
        out->otu_offsets[i] = io;
        for (auto &h : r.hits) {
            oracle_hit &o = out->hits[ih++];
            o.entry = h.hit;
            o.pos = h.offset;
            o.seq = (uint32_t)i;
        }
        for (auto &c : r.calls)
            out->calls[ic++] = c;
        for (auto &pr : r.otu.otus_by_count) {
            out->otus[2 * io] = pr.first;
            out->otus[2 * io + 1] = pr.second;
            io++;
        }
    }
    out->hit_offsets[n_seq] = ih;
    out->call_offsets[n_seq] = ic;
    out->otu_offsets[n_seq] = io;
    if (want_best) {
        out->best = (oracle_best *)std::calloc(n_seq + 1, sizeof(oracle_best));
        for (uint64_t i = 0; i < n_seq; i++)
            out->best[i] = res[i].best;
    }
    return 0;
}

void oracle_result_free(oracle_result *r)
{
    std::free(r->hit_offsets);
    std::free(r->hits);
    std::free(r->call_offsets);
    std::free(r->calls);
    std::free(r->otu_offsets);
    std::free(r->otus);
    std::free(r->best);
    std::memset(r, 0, sizeof(*r));
}

/* Sequential image build (the reference's writer order).  table must hold
 * num_sigs buckets; it is initialised here.  Returns the number of keys
 * stored, or -1 when the table would reach half full. */
int64_t oracle_build_table(void *table, uint64_t num_sigs, const uint64_t *keys,
                           const int32_t *fI, const int32_t *oI, const uint16_t *avg,
                           const float *wt, uint64_t n_keys)
{
    SigKmer *t = (SigKmer *)table;
    std::memset(t, 0, num_sigs * sizeof(SigKmer));
    for (uint64_t i = 0; i < num_sigs; i++)
        t[i].which_kmer = EMPTY_KEY;
    uint64_t loaded = 0;
    for (uint64_t i = 0; i < n_keys; i++)
        if (insert_key(t, num_sigs, loaded, keys[i], fI[i], oI[i], avg[i], wt[i]))
            return -1;
    return (int64_t)loaded;
}

/* find_best_call over a flat call list; names[n_names] are function.index
 * entries.  fn_buf receives the function string (NUL-terminated).
 * out3 = {score, weighted_score, score_offset}; *offset_set is 0 when
 * score_offset was left untouched (no calls). */
int oracle_find_best_call(const Call *calls, uint64_t n, const char *const *names, int n_names,
                          int32_t *function_index, char *fn_buf, uint64_t fn_cap, float *out3,
                          int *offset_set)
{
    std::vector<Call> v(calls, calls + n);
    std::vector<std::string> f;
    for (int i = 0; i < n_names; i++)
        f.emplace_back(names[i]);
    int fi;
    std::string fn;
    float score, wscore, off = -12345.0f;
    find_best_call(v, f, fi, fn, score, wscore, off);
    *function_index = fi;
    std::snprintf(fn_buf, fn_cap, "%s", fn.c_str());
    out3[0] = score;
    out3[1] = wscore;
    out3[2] = off;
    *offset_set = n > 0;
    return 0;
}

/* FASTA framing: records as "id\tseq\n" lines (malloc'd) */
char *oracle_fasta_parse(const char *text, uint64_t len)
{
    std::string out;
    for (auto &r : parse_fasta(std::string(text, len)))
        out += r.first + "\t" + r.second + "\n";
    char *b = (char *)std::malloc(out.size() + 1);
    std::memcpy(b, out.data(), out.size() + 1);
    return b;
}

char *oracle_translate11(const char *dna, uint64_t len)
{
    std::string p = translate11(std::string(dna, len));
    char *b = (char *)std::malloc(p.size() + 1);
    std::memcpy(b, p.data(), p.size() + 1);
    return b;
}

void oracle_free(void *p) { std::free(p); }

uint64_t oracle_encode8(const char *kmer)
{
    unsigned char c[K];
    for (int i = 0; i < K; i++) {
        c[i] = residue_code(kmer[i]);
        if (c[i] >= 20)
            return MAX_ENCODED + 1; /* encoded_aa_kmer, kguts.cc:457-471 */
    }
    return encode8(c);
}

void oracle_decode8(uint64_t key, char *out9) { decode8(key, out9); }

}  /* extern "C" */
