/*
 * handlers_oracle.cpp -- TEST INFRASTRUCTURE ONLY (never linked into the
 * product).  CPU restatement of the request-handler arithmetic that sits on
 * the hit stream, with the same standard containers the reference uses so
 * iteration and tie orders match:
 *
 *   oracle_kmap_*   KmerPegMapping::add_mapping (kmer.cc:173-210: append,
 *                   duplicates kept) and add_fam_mapping / fam_map_insert
 *                   (kmer.cc:212-256: std::find, push_back if absent)
 *   oracle_matrix_* MatrixRequest (matrix_request.cc:83-95 per-sequence loop,
 *                   on_hit 130-163, process_results 165-190; state
 *                   matrix_request.h:25-26)
 *   oracle_lookup_* LookupRequest (lookup_request.cc:33-79 parameters, 153-400
 *                   per-sequence loop and output, on_hit 446-482)
 *   oracle_fq_*     the fq path: FastqParser (fastq_parser.h:40-150,
 *                   fastq_parser.cc), DNASequence::get_possible_proteins
 *                   (dna_seq.cc:9-47, complement dna_seq.h:28-111),
 *                   FqProcessRequest::on_parsed_seq (fq_process_request.cc:
 *                   298-365) over FamilyMapper (family_mapper.cc:46-205,
 *                   287-330) and the family DB it reads (KmerPegMapping::
 *                   load_genus_map / load_families kmer.cc:341-493, the NR
 *                   family load nr_loader.cc:130-176)
 */
#include "kmer_oracle.h"

#include <cstdint>
#include <cstring>
#include <fstream>
#include <iostream>
#include <list>
#include <sstream>
#include <string>
#include <map>
#include <unordered_map>
#include <algorithm>
#include <utility>
#include <vector>
#include <cctype>
#include <cstdlib>
#include <functional>

namespace {

struct Kmap {
    int mode = 0; /* 0 append (kmer_to_id_), 1 set (kmer_to_family_id_) */
    std::unordered_map<uint64_t, std::vector<uint32_t>> m;
    void add(uint64_t kmer, uint32_t id)
    {
        auto &v = m[kmer];
        if (mode == 1 && std::find(v.begin(), v.end(), id) != v.end())
            return; /* fam_map_insert, kmer.cc:214-227 */
        v.push_back(id);
    }
};

struct Matrix {
    std::map<uint32_t, size_t> matrix_proteins;                         /* matrix_request.h:25 */
    std::map<std::pair<uint32_t, uint32_t>, unsigned long> distance;    /* matrix_request.h:26 */
};

/* ---- family DB (KmerPegMapping, kmer.h:58-66) -------------------------- */

struct FamilyData {
    std::string pgf, plf;
    unsigned long genus_id = 0;
    std::string function;
    uint32_t family_id = 0;
    unsigned long total_size = 0;
    unsigned short count = 0;
};

struct FamilyDb {
    std::map<std::string, std::string> genus_map;
    std::map<std::string, uint32_t> peg_to_id;
    std::vector<std::string> id_to_peg;
    std::unordered_map<uint32_t, FamilyData> family_data;
    std::map<std::pair<std::string, std::string>, uint32_t> family_key_to_id;
    std::unordered_map<uint32_t, uint32_t> peg_to_family;
    uint32_t next_family_id = 0;
    Kmap kmer_to_family;
    FamilyDb() { kmer_to_family.mode = 1; }

    uint32_t assign_new_peg_id(const std::string &peg) /* kmer.h:114-121 */
    {
        uint32_t id = (uint32_t)id_to_peg.size();
        peg_to_id[peg] = id;
        id_to_peg.push_back(peg);
        return id;
    }
    uint32_t encode_id(const std::string &peg) /* kmer.cc:273-286 */
    {
        auto it = peg_to_id.find(peg);
        return it != peg_to_id.end() ? it->second : assign_new_peg_id(peg);
    }
};

static std::vector<std::string> split_tabs(const std::string &line)
{
    /* boost::split(cols, line, is_any_of("\t")) without compression */
    std::vector<std::string> cols;
    size_t a = 0;
    for (;;) {
        size_t b = line.find('\t', a);
        cols.push_back(line.substr(a, b == std::string::npos ? std::string::npos : b - a));
        if (b == std::string::npos)
            break;
        a = b + 1;
    }
    return cols;
}

/* kmer.cc:341-358 */
static bool load_genus_map(FamilyDb &db, const std::string &path)
{
    std::ifstream gf(path);
    if (gf.fail())
        return false;
    std::string line;
    while (std::getline(gf, line)) {
        auto cols = split_tabs(line);
        db.genus_map[cols[0]] = cols.size() > 1 ? cols[1] : std::string();
    }
    return true;
}

/* kmer.cc:375-493 read with one thread (n-family-file-threads = 1): lines in
 * file order */
static bool load_families(FamilyDb &db, const std::string &path)
{
    std::ifstream f(path);
    if (f.fail())
        return false;
    const std::string zeros("00000000");
    std::string line;
    while (std::getline(f, line)) {
        auto cols = split_tabs(line);
        if (cols.size() < 9)
            continue;
        std::string pgf("PGF_");
        pgf += cols[0].substr(2);
        std::string plf("PLF_");
        unsigned long genus_id = 0;
        auto mapped = db.genus_map.find(cols[7]);
        if (mapped == db.genus_map.end()) {
            plf += cols[7];
        } else {
            plf += mapped->second;
            genus_id = std::stoul(mapped->second);
        }
        plf += "_";
        plf += zeros.substr(0, 8 - cols[8].size());
        plf += cols[8];
        uint32_t id = db.assign_new_peg_id(cols[3]);
        auto fkey = std::make_pair(pgf, plf);
        unsigned long seqlen = std::stoul(cols[4]);
        uint32_t fam_id;
        auto fit = db.family_key_to_id.find(fkey);
        if (fit == db.family_key_to_id.end()) {
            fam_id = db.next_family_id++;
            db.family_key_to_id[fkey] = fam_id;
            FamilyData d;
            d.pgf = pgf;
            d.plf = plf;
            d.genus_id = genus_id;
            d.function = cols[5];
            d.family_id = fam_id;
            d.total_size = seqlen;
            d.count = 1;
            db.family_data.emplace(fam_id, d);
        } else {
            fam_id = fit->second;
            auto &d = db.family_data[fam_id];
            d.total_size += seqlen;
            d.count++;
        }
        db.peg_to_family.insert(std::make_pair(id, fam_id));
    }
    return true;
}

/* ---- FamilyMapper (family_mapper.cc) -------------------------------------- */

struct AccScore { /* sequence_accumulated_score_t, family_mapper.h:33-49 */
    unsigned int hit_count = 0, hit_total = 0;
    float weighted_total = 0.0f;
};

struct BestMatch { /* family_mapper.h:20-28 */
    std::string gfam_id;
    float gfam_score;
    std::string lfam_id;
    float lfam_score;
    std::string function;
    float score;
};

struct FamilyMapper {
    FamilyDb *db;
    oracle::Scorer *scorer;
    const std::vector<std::string> *functions;
    std::unordered_map<uint32_t, AccScore> seq_score;
    unsigned int kmer_hit_threshold = 3;

    /* ingest_protein + find_best_family_match (family_mapper.cc:46-205) with
     * allow_ambiguous_functions_ = false (the constructor default fq uses) */
    BestMatch find_best_family_match(const std::string &seq)
    {
        seq_score.clear();
        std::vector<oracle::Call> calls;
        std::vector<oracle::SeqHit> hits;
        scorer->process(seq.c_str(), seq.size(), &calls, &hits, nullptr, true);
        for (auto &h : hits) { /* on_hit, family_mapper.cc:287-312 */
            auto ki = db->kmer_to_family.m.find(h.hit.which_kmer);
            if (ki == db->kmer_to_family.m.end())
                continue;
            const float weight = 1.0f / (float)ki->second.size();
            for (uint32_t ent : ki->second) {
                AccScore &a = seq_score[ent];
                a.hit_count++;
                a.hit_total++;
                a.weighted_total += weight;
            }
        }
        int fi;
        std::string fn;
        float score, wscore, off;
        oracle::find_best_call(calls, *functions, fi, fn, score, wscore, off);
        if (fn.empty() || fn.find(" ?? ") != std::string::npos)
            fn = "hypothetical protein";
        float best_lf_score = 0.0f, best_gf_score = 0.0f;
        std::string best_lf_fam, best_gf_fam;
        std::unordered_map<std::string, float> pgf_rollup;
        for (auto hit_ent : seq_score) {
            const AccScore &se = hit_ent.second;
            if (se.hit_total < kmer_hit_threshold)
                continue;
            auto fent = db->family_data.find(hit_ent.first);
            if (fent == db->family_data.end())
                continue;
            const FamilyData &fd = fent->second;
            if (fd.function == fn)
                pgf_rollup[fd.pgf] += se.weighted_total;
            else
                continue;
            if (se.weighted_total > best_lf_score) {
                best_lf_score = se.weighted_total;
                best_lf_fam = fd.plf;
            }
        }
        for (auto pgf_ent : pgf_rollup)
            if (pgf_ent.second > best_gf_score) {
                best_gf_score = pgf_ent.second;
                best_gf_fam = pgf_ent.first;
            }
        return BestMatch{best_gf_fam, best_gf_score, best_lf_fam, best_lf_score, fn, score};
    }
};

/* DNASequence complement (dna_seq.h:28-111) */
static char complement(char c)
{
    switch (c) {
    case 'a': return 't';
    case 'A': return 'T';
    case 'c': return 'g';
    case 'C': return 'G';
    case 'g': return 'c';
    case 'G': return 'C';
    case 't': case 'u': return 'a';
    case 'T': case 'U': return 'A';
    case 'm': return 'k';
    case 'M': return 'K';
    case 'r': return 'y';
    case 'R': return 'Y';
    case 'w': return 'w';
    case 'W': return 'W';
    case 's': return 'S';
    case 'S': return 'S';
    case 'y': return 'r';
    case 'Y': return 'R';
    case 'k': return 'm';
    case 'K': return 'M';
    case 'b': return 'v';
    case 'B': return 'V';
    case 'd': return 'h';
    case 'D': return 'H';
    case 'h': return 'd';
    case 'H': return 'D';
    case 'v': return 'b';
    case 'V': return 'B';
    case 'n': return 'n';
    case 'N': return 'N';
    default: return c;
    }
}

/* get_possible_proteins (dna_seq.cc:9-47): frames 1,2,3,-1,-2,-3, each split
 * on '*' with token_compress_on */
static std::list<std::pair<int, std::list<std::string>>> possible_proteins(const std::string &seq)
{
    std::string rev;
    for (auto it = seq.rbegin(); it != seq.rend(); ++it)
        rev.push_back(complement(*it));
    std::list<std::pair<int, std::list<std::string>>> ret;
    for (int frame : {1, 2, 3, -1, -2, -3}) {
        const std::string &m = frame < 0 ? rev : seq;
        size_t off = (size_t)std::abs(frame) - 1;
        std::string p = oracle::translate11(off <= m.size() ? m.substr(off) : std::string());
        std::list<std::string> l;
        /* boost::split, is_any_of("*"), token_compress_on: adjacent separators
         * form one; leading/trailing separators give empty tokens */
        std::string cur;
        size_t i = 0;
        while (i < p.size()) {
            if (p[i] == '*') {
                l.push_back(cur);
                cur.clear();
                while (i < p.size() && p[i] == '*')
                    i++;
            } else {
                cur.push_back(p[i++]);
            }
        }
        l.push_back(cur);
        ret.emplace_back(frame, l);
    }
    return ret;
}

/* FqProcessRequest::on_parsed_seq (fq_process_request.cc:298-365) */
static void fq_on_parsed_seq(const std::string &id, const std::string &seq, FamilyMapper &mapper,
                             std::ostream &os)
{
    if (id.empty())
        return;
    auto prots = possible_proteins(seq);
    double best_score = 0.0;
    int best_frame = 0;
    std::vector<std::pair<size_t, BestMatch>> best_matches;
    for (auto &fr : prots) {
        double score = 0.0;
        std::vector<std::pair<size_t, BestMatch>> matches;
        for (auto &prot : fr.second) {
            if (prot.length() > 10) {
                matches.emplace_back(prot.length(), mapper.find_best_family_match(prot));
                score += matches.back().second.score;
            }
            if (score > best_score) {
                best_score = score;
                best_frame = fr.first;
                best_matches = matches;
            }
        }
    }
    if (best_score > 0.0) {
        os << id << "\t" << best_frame << "\t" << best_score << "\t";
        bool first = true;
        for (auto &m : best_matches) {
            if (!first)
                os << "\t";
            first = false;
            const BestMatch &b = m.second;
            os << m.first << "\t" << b.gfam_id << "\t" << b.gfam_score << "\t" << b.lfam_id << "\t"
               << b.lfam_score << "\t" << b.function << "\t" << b.score;
        }
        os << std::endl;
    }
}

/* FastqParser (fastq_parser.h:40-150): one record per 4-line group; sequence
 * characters outside isalpha() are dropped (with an error message in the
 * reference); parse_complete() emits the current record */
static void parse_fastq(const std::string &text,
                        const std::function<void(const std::string &, const std::string &)> &cb)
{
    enum { S_START, S_ID, S_DEF, S_DATA, S_PLUS_START, S_PLUS, S_QUAL } st = S_START;
    std::string id, seq;
    for (char c : text) {
        switch (st) {
        case S_START:
            if (c == '@')
                st = S_ID;
            break;
        case S_ID:
            if (c == ' ' || c == '\t')
                st = S_DEF;
            else if (c == '\n')
                st = S_DATA;
            else
                id.push_back(c);
            break;
        case S_DEF:
            if (c == '\n')
                st = S_DATA;
            break;
        case S_DATA:
            if (c == '\n')
                st = S_PLUS_START;
            else if (std::isalpha((unsigned char)c))
                seq.push_back(c);
            break;
        case S_PLUS_START:
            if (c == '+')
                st = S_PLUS;
            break;
        case S_PLUS:
            if (c == '\n')
                st = S_QUAL;
            break;
        case S_QUAL:
            if (c == '\n') {
                cb(id, seq);
                id.clear();
                seq.clear();
                st = S_START;
            }
            break;
        }
    }
    cb(id, seq); /* parse_complete, fastq_parser.cc:29-35 */
}

/* std::stoi on a query-string value with only invalid_argument caught
 * (lookup_request.cc:47-58): absent or non-numeric values keep the default */
static bool stoi_param(const std::map<std::string, std::string> &p, const std::string &k, int &out)
{
    auto it = p.find(k);
    if (it == p.end())
        return false;
    try {
        out = std::stoi(it->second);
        return true;
    } catch (const std::invalid_argument &) {
        return false;
    }
}

struct LookupSession {
    FamilyDb db;
    Kmap kmer_to_id; /* mode 0 */
    const oracle::SigKmer *table = nullptr;
    std::vector<std::string> functions;
    oracle::Scorer *scorer = nullptr;
    ~LookupSession() { delete scorer; }
};

/* one /lookup request over FASTA records (lookup_request.cc) */
static std::string lookup_request(LookupSession &q, bool family_mode,
                                  const std::map<std::string, std::string> &params,
                                  const std::vector<std::pair<std::string, std::string>> &records)
{
    unsigned int kmer_hit_threshold = 3;
    int v;
    if (stoi_param(params, "kmer_hit_threhsold", v))
        kmer_hit_threshold = (unsigned int)v;
    bool find_best_match = false, find_reps = false, allow_ambiguous = false;
    if (stoi_param(params, "find_best_match", v))
        find_best_match = v != 0;
    if (stoi_param(params, "find_reps", v))
        find_reps = v != 0;
    if (stoi_param(params, "allow_ambiguous_functions", v))
        allow_ambiguous = v != 0;
    unsigned long target_genus_id = 0;
    {
        auto tg_it = params.find("target_genus");
        std::string tg = q.db.genus_map[tg_it == params.end() ? std::string() : tg_it->second];
        try {
            if (!tg.empty())
                target_genus_id = std::stoul(tg);
        } catch (const std::invalid_argument &) {
        }
    }
    std::unordered_map<uint32_t, AccScore> seq_score; /* lookup_request.h:43, one per request */
    std::ostringstream os;
    for (auto &rec : records) {
        const std::string &id = rec.first, &seq = rec.second;
        seq_score.clear();
        std::vector<oracle::Call> calls;
        std::vector<oracle::SeqHit> hits;
        const bool want_calls = find_best_match && family_mode;
        q.scorer->process(seq.c_str(), seq.size(), want_calls ? &calls : nullptr, &hits, nullptr, true);
        for (auto &h : hits) { /* on_hit, lookup_request.cc:446-482 */
            if (family_mode) {
                auto ki = q.db.kmer_to_family.m.find(h.hit.which_kmer);
                if (ki == q.db.kmer_to_family.m.end())
                    continue;
                const float weight = 1.0f / (float)ki->second.size();
                for (uint32_t ent : ki->second) {
                    AccScore &s = seq_score[ent];
                    s.hit_count++;
                    s.hit_total++;
                    s.weighted_total += weight;
                }
            } else {
                auto ki = q.kmer_to_id.m.find(h.hit.which_kmer);
                if (ki == q.kmer_to_id.m.end())
                    continue;
                for (uint32_t eid : ki->second)
                    seq_score[eid].hit_count++;
            }
        }
        if (find_best_match && family_mode) {
            int fi;
            std::string fn;
            float score, wscore, off;
            oracle::find_best_call(calls, q.functions, fi, fn, score, wscore, off);
            std::string ambig;
            bool do_ambig = false;
            if (fn.empty()) {
                fn = "hypothetical protein";
            } else {
                size_t where = fn.find(" ?? ");
                if (where != std::string::npos) {
                    if (allow_ambiguous) {
                        ambig = fn.substr(where + 4);
                        fn = fn.substr(0, where);
                        do_ambig = true;
                    } else {
                        fn = "hypothetical protein";
                    }
                }
            }
            float lf_score = 0.0f, gf_score = 0.0f;
            std::string lf_fam, lf_fn, gf_fam;
            std::unordered_map<std::string, float> pgf_rollup, pgf_rollup_ambig;
            for (auto hit_ent : seq_score) {
                const AccScore &se = hit_ent.second;
                if (se.hit_total < kmer_hit_threshold)
                    continue;
                auto fent = q.db.family_data.find(hit_ent.first);
                if (fent == q.db.family_data.end())
                    continue;
                const FamilyData &fd = fent->second;
                if (do_ambig) {
                    if (fd.function == fn)
                        pgf_rollup[fd.pgf] += se.weighted_total;
                    else if (fd.function == ambig)
                        pgf_rollup_ambig[fd.pgf] += se.weighted_total;
                    else
                        continue;
                } else {
                    if (fd.function == fn)
                        pgf_rollup[fd.pgf] += se.weighted_total;
                    else
                        continue;
                }
                if (se.weighted_total > lf_score && fd.genus_id == target_genus_id) {
                    lf_score = se.weighted_total;
                    lf_fam = fd.plf;
                    lf_fn = fd.function;
                }
            }
            auto *rollup = &pgf_rollup;
            if (do_ambig && lf_fn == ambig)
                rollup = &pgf_rollup_ambig;
            for (auto pgf_ent : *rollup)
                if (pgf_ent.second > gf_score) {
                    gf_score = pgf_ent.second;
                    gf_fam = pgf_ent.first;
                }
            os << id << "\t" << gf_fam << "\t" << gf_score << "\t" << lf_fam << "\t" << lf_score << "\t"
               << (do_ambig ? lf_fn : fn) << "\t" << score << "\t" << wscore << "\n";
        } else {
            typedef std::pair<uint32_t, AccScore> data_t;
            std::vector<data_t> vec;
            for (auto it : seq_score)
                vec.push_back(it);
            std::sort(vec.begin(), vec.end(), [](const data_t &l, const data_t &r) {
                return l.second.weighted_total > r.second.weighted_total;
            });
            os << id << "\n";
            for (auto it : vec) {
                const AccScore &se = it.second;
                if (se.hit_total < kmer_hit_threshold)
                    break;
                if (family_mode) {
                    const FamilyData &fd = q.db.family_data[it.first];
                    const float scaled = (float)se.hit_count / (float)fd.total_size;
                    os << se.hit_count << "\t" << se.hit_total << "\t" << se.weighted_total << "\t" << fd.pgf
                       << "\t" << fd.plf << "\t" << fd.total_size << "\t" << fd.count << "\t" << scaled << "\t"
                       << fd.function << "\n";
                    if (find_reps)
                        os << "///\n"; /* no family reps loaded */
                } else {
                    const std::string peg = it.first < q.db.id_to_peg.size() ? q.db.id_to_peg[it.first] : "";
                    os << peg << "\t" << se.hit_count;
                    auto fh = q.db.peg_to_family.find(it.first);
                    if (fh != q.db.peg_to_family.end()) {
                        const FamilyData &fd = q.db.family_data[fh->second];
                        os << "\t" << fd.pgf << "\t" << fd.plf << "\t" << fd.function << "\n";
                    } else {
                        os << "\n";
                    }
                }
            }
            os << "//\n";
        }
    }
    return os.str();
}

struct FqSession {
    FamilyDb db;
    const oracle::SigKmer *table = nullptr; /* the caller's, kept alive by it */
    std::vector<std::string> functions;
    oracle::Scorer *scorer = nullptr;
    ~FqSession() { delete scorer; }
};

}  // namespace

extern "C" {

void *oracle_kmap_new(int mode)
{
    Kmap *k = new Kmap;
    k->mode = mode;
    return k;
}

void oracle_kmap_free(void *p) { delete static_cast<Kmap *>(p); }

void oracle_kmap_add(void *p, const uint64_t *kmers, const uint32_t *ids, uint64_t n)
{
    Kmap *k = static_cast<Kmap *>(p);
    for (uint64_t i = 0; i < n; i++)
        k->add(kmers[i], ids[i]);
}

/* number of ids of `kmer`; copies up to cap of them into ids */
uint64_t oracle_kmap_lookup(void *p, uint64_t kmer, uint32_t *ids, uint64_t cap)
{
    Kmap *k = static_cast<Kmap *>(p);
    auto it = k->m.find(kmer);
    if (it == k->m.end())
        return 0;
    const auto &v = it->second;
    for (uint64_t i = 0; i < v.size() && i < cap; i++)
        ids[i] = v[i];
    return v.size();
}

uint64_t oracle_kmap_num_kmers(void *p) { return static_cast<Kmap *>(p)->m.size(); }

void *oracle_matrix_new(void) { return new Matrix; }
void oracle_matrix_free(void *p) { delete static_cast<Matrix *>(p); }

/* One batch of a /matrix request: sequence s has id seq_ids[s], length
 * seq_lens[s] and hits hit_kmers[hit_off[s] .. hit_off[s+1]) in position order. */
void oracle_matrix_add(void *px, void *pk, const uint32_t *seq_ids, const uint64_t *seq_lens,
                       uint64_t n_seq, const uint64_t *hit_off, const uint64_t *hit_kmers)
{
    Matrix *x = static_cast<Matrix *>(px);
    Kmap *k = static_cast<Kmap *>(pk);
    for (uint64_t s = 0; s < n_seq; s++) {
        const uint32_t id = seq_ids[s];
        x->matrix_proteins[id] = seq_lens[s]; /* matrix_request.cc:91 */
        for (uint64_t h = hit_off[s]; h < hit_off[s + 1]; h++) {
            auto ki = k->m.find(hit_kmers[h]);
            if (ki == k->m.end())
                continue; /* "no mapping for" on stderr, matrix_request.cc:159 */
            for (uint32_t eid : ki->second)
                if (eid != id && x->matrix_proteins.find(eid) != x->matrix_proteins.end())
                    x->distance[std::make_pair(id, eid)]++;
        }
    }
}

/* distance_ in map order with process_results' score (matrix_request.cc:
 * 179-186); returns the number of pairs, fills the arrays when non-null */
uint64_t oracle_matrix_pairs(void *px, uint32_t *id1, uint32_t *id2, uint64_t *count, float *score)
{
    Matrix *x = static_cast<Matrix *>(px);
    uint64_t i = 0;
    for (auto it = x->distance.begin(); it != x->distance.end(); ++it, ++i) {
        if (!id1)
            continue;
        const uint32_t e1 = it->first.first, e2 = it->first.second;
        id1[i] = e1;
        id2[i] = e2;
        count[i] = it->second;
        const size_t l1 = x->matrix_proteins[e1], l2 = x->matrix_proteins[e2];
        score[i] = (float)it->second / ((float)(l1 + l2));
    }
    return x->distance.size();
}

/* fq session over the caller's image table (not copied; it must outlive the
 * session), the function names and an optional family DB; genus / families
 * / nr may be null */
void *oracle_fq_new(const void *table, uint64_t num_sigs, const char *const *functions, uint64_t n_functions,
                    const char *genus_file, const char *families_file, const char *nr_fasta)
{
    FqSession *q = new FqSession;
    q->table = static_cast<const oracle::SigKmer *>(table);
    for (uint64_t i = 0; i < n_functions; i++)
        q->functions.push_back(functions[i]);
    q->scorer = new oracle::Scorer(q->table, num_sigs);
    if (genus_file && *genus_file && !load_genus_map(q->db, genus_file)) {
        delete q;
        return nullptr;
    }
    if (families_file && *families_file && !load_families(q->db, families_file)) {
        delete q;
        return nullptr;
    }
    if (nr_fasta && *nr_fasta) {
        /* NRLoader::thread_load in family mode (nr_loader.cc:130-176), one
         * thread: every hit of a protein with a family adds (kmer, family) */
        std::ifstream in(nr_fasta, std::ios::binary);
        std::stringstream ss;
        ss << in.rdbuf();
        for (auto &rec : oracle::parse_fasta(ss.str())) {
            uint32_t enc = q->db.encode_id(rec.first);
            auto fit = q->db.peg_to_family.find(enc);
            if (fit == q->db.peg_to_family.end())
                continue; /* "NO FAM FOR id=..." */
            std::vector<oracle::SeqHit> hits;
            q->scorer->process(rec.second.c_str(), rec.second.size(), nullptr, &hits, nullptr, false);
            for (auto &h : hits)
                q->db.kmer_to_family.add(h.hit.which_kmer, fit->second);
        }
    }
    return q;
}

void oracle_fq_free(void *p) { delete static_cast<FqSession *>(p); }

/* the fq request body for a FASTQ text (one FamilyMapper for the request) */
char *oracle_fq_process(void *p, const char *fastq, uint64_t n)
{
    FqSession *q = static_cast<FqSession *>(p);
    FamilyMapper mapper{&q->db, q->scorer, &q->functions, {}, 3};
    std::ostringstream os;
    parse_fastq(std::string(fastq, n), [&](const std::string &id, const std::string &seq) {
        fq_on_parsed_seq(id, seq, mapper, os);
    });
    const std::string s = os.str();
    char *b = static_cast<char *>(std::malloc(s.size() + 1));
    std::memcpy(b, s.c_str(), s.size() + 1);
    return b;
}

/* /lookup session: table (borrowed), functions, family DB files, and an
 * optional /add FASTA filling kmer_to_id_ first (add_request.cc:164-170) */
void *oracle_lookup_new(const void *table, uint64_t num_sigs, const char *const *functions, uint64_t n_functions,
                        const char *genus_file, const char *families_file, const char *nr_fasta,
                        const char *add_fasta)
{
    LookupSession *q = new LookupSession;
    q->table = static_cast<const oracle::SigKmer *>(table);
    for (uint64_t i = 0; i < n_functions; i++)
        q->functions.push_back(functions[i]);
    q->scorer = new oracle::Scorer(q->table, num_sigs);
    auto read_fasta = [](const char *path) {
        std::ifstream in(path, std::ios::binary);
        std::stringstream ss;
        ss << in.rdbuf();
        return oracle::parse_fasta(ss.str());
    };
    if ((genus_file && *genus_file && !load_genus_map(q->db, genus_file)) ||
        (families_file && *families_file && !load_families(q->db, families_file))) {
        delete q;
        return nullptr;
    }
    if (nr_fasta && *nr_fasta)
        for (auto &rec : read_fasta(nr_fasta)) {
            auto fit = q->db.peg_to_family.find(q->db.encode_id(rec.first));
            if (fit == q->db.peg_to_family.end())
                continue;
            std::vector<oracle::SeqHit> hits;
            q->scorer->process(rec.second.c_str(), rec.second.size(), nullptr, &hits, nullptr, false);
            for (auto &h : hits)
                q->db.kmer_to_family.add(h.hit.which_kmer, fit->second);
        }
    if (add_fasta && *add_fasta) {
        auto recs = read_fasta(add_fasta);
        std::vector<std::vector<uint64_t>> km(recs.size());
        for (size_t r = 0; r < recs.size(); r++) {
            std::vector<oracle::SeqHit> hits;
            q->scorer->process(recs[r].second.c_str(), recs[r].second.size(), nullptr, &hits, nullptr, true);
            for (auto &h : hits)
                km[r].push_back(h.hit.which_kmer);
        }
        for (size_t r = 0; r < recs.size(); r++) { /* ids encoded after the chunk (non-TBB add) */
            uint32_t eid = q->db.encode_id(recs[r].first);
            for (uint64_t k : km[r])
                q->kmer_to_id.add(k, eid);
        }
    }
    return q;
}

void oracle_lookup_free(void *p) { delete static_cast<LookupSession *>(p); }

/* names[i] = values[i] are the request's query-string parameters */
char *oracle_lookup_process(void *p, int family_mode, const char *const *names, const char *const *values,
                            uint64_t n_params, const char *fasta, uint64_t n)
{
    LookupSession *q = static_cast<LookupSession *>(p);
    std::map<std::string, std::string> params;
    for (uint64_t i = 0; i < n_params; i++)
        params[names[i]] = values[i];
    const std::string s = lookup_request(*q, family_mode != 0, params, oracle::parse_fasta(std::string(fasta, n)));
    char *b = static_cast<char *>(std::malloc(s.size() + 1));
    std::memcpy(b, s.c_str(), s.size() + 1);
    return b;
}

/* frames and >10-aa fragments of one read, as "frame:fragment" lines */
char *oracle_fq_fragments(const char *dna, uint64_t n)
{
    std::ostringstream os;
    for (auto &fr : possible_proteins(std::string(dna, n)))
        for (auto &prot : fr.second)
            if (prot.length() > 10)
                os << fr.first << ":" << prot << "\n";
    const std::string s = os.str();
    char *b = static_cast<char *>(std::malloc(s.size() + 1));
    std::memcpy(b, s.c_str(), s.size() + 1);
    return b;
}

}  /* extern "C" */
