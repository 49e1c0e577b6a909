/*
 * kguts_hip.cpp -- the KmerGuts-compatible facade over the kgx C ABI.
 * Host-side rules restated from the reference: find_best_call
 * (kguts.cc:984-1199), text formatting (kguts.cc:939-973), OTU sorting
 * (kguts.h:185-219), index files (kguts.cc:544-575), FASTA framing
 * (fasta_parser.h:38-165, fasta_parser.cc:21-36).
 */
#include "kguts_hip.h"

#include <algorithm>
#include <cctype>
#include <cstring>
#include <iostream>
#include <sstream>

namespace kgx {

namespace {
const char kResidues[21] = "ACDEFGHIKLMNPQRSTVWY";

[[noreturn]] void throw_last(int rc, const std::string &what)
{
    throw Error(rc, what + ": " + kgx_strerror(rc) + " (" + kgx_last_error() + ")");
}
}  // namespace

/* ---- KmerOtuStats ----------------------------------------------------------- */

void KmerOtuStats::write(FILE *fh) const
{
    std::fprintf(fh, "OTU-COUNTS\t%s[%d]", contig_id.c_str(), contig_len);
    for (const auto &p : otus_by_count)
        std::fprintf(fh, "\t%d-%d", p.second, p.first);
    std::fprintf(fh, "\n");
}

void KmerOtuStats::finalize()
{
    otus_by_count.insert(otus_by_count.begin(), otu_map.begin(), otu_map.end());
    std::sort(otus_by_count.begin(), otus_by_count.end(),
              [](const std::pair<int, int> &l, const std::pair<int, int> &r) {
                  return r.second < l.second;
              });
}

/* ---- KmerImage ---------------------------------------------------------------- */

KmerImage::KmerImage(const std::string &data_dir, int device) : data_dir_(data_dir)
{
    int rc = kgx_image_open(data_dir.c_str(), device, &img_);
    if (rc)
        throw_last(rc, "KmerImage(" + data_dir + ")");
}

KmerImage::KmerImage(kgx_image *adopted) : img_(adopted)
{
    if (!img_)
        throw Error(KGX_EINVAL, "KmerImage: null image");
}

KmerImage::~KmerImage() { kgx_image_close(img_); }

/* ---- index files ----------------------------------------------------------- */

bool load_index_file(const std::string &path, std::vector<std::string> &out)
{
    FILE *f = std::fopen(path.c_str(), "r");
    if (!f)
        return false;
    out.clear();
    int idx;
    char line[1000];
    /* fscanf("%d\t") skips any whitespace after the number; fgets keeps the
     * newline, which the reference then overwrites (even if it is not one) */
    while (std::fscanf(f, "%d\t", &idx) == 1 && std::fgets(line, sizeof(line), f)) {
        if (idx != (int)out.size()) {
            std::fclose(f);
            return false;
        }
        size_t n = std::strlen(line);
        out.emplace_back(line, n ? n - 1 : 0);
    }
    std::fclose(f);
    return true;
}

/* ---- KmerGuts ------------------------------------------------------------------ */

KmerGuts::KmerGuts(const std::string &kmer_dir, std::shared_ptr<KmerImage> image) : image_(image)
{
    if (!image_)
        throw Error(KGX_EINVAL, "KmerGuts: null image");
    if (!load_index_file(kmer_dir + "/function.index", functions_))
        throw Error(KGX_EIO, "could not load " + kmer_dir + "/function.index");
    if (!load_index_file(kmer_dir + "/otu.index", otus_))
        throw Error(KGX_EIO, "could not load " + kmer_dir + "/otu.index");
    set_default_parameters();
    int rc = kgx_ctx_create(image_->handle(), &ctx_);
    if (rc)
        throw_last(rc, "kgx_ctx_create");
}

KmerGuts::~KmerGuts() { kgx_ctx_destroy(ctx_); }

void KmerGuts::set_default_parameters()
{
    kgx_params p;
    kgx_params_default(&p);
    order_constraint = p.order_constraint;
    min_hits = p.min_hits;
    min_weighted_hits = p.min_weighted_hits;
    max_gap = p.max_gap;
}

void KmerGuts::set_parameters(const std::map<std::string, std::string> &params)
{
    std::vector<const char *> names, values;
    for (const auto &kv : params) {
        names.push_back(kv.first.c_str());
        values.push_back(kv.second.c_str());
    }
    kgx_params p;
    int rc = kgx_params_parse(&p, names.data(), values.data(), names.size());
    if (rc)
        throw std::out_of_range(kgx_last_error()); /* std::stoi's own exception */
    order_constraint = p.order_constraint;
    min_hits = p.min_hits;
    min_weighted_hits = p.min_weighted_hits;
    max_gap = p.max_gap;
}

void KmerGuts::process_aa_batch(std::vector<SeqJob> &jobs)
{
    const uint32_t n = (uint32_t)jobs.size();
    std::vector<uint64_t> off(n + 1, 0);
    uint32_t want = 0;
    for (uint32_t i = 0; i < n; i++) {
        off[i + 1] = off[i] + jobs[i].seq.size();
        if (jobs[i].hit_cb)
            want |= KGX_WANT_HITS;
        if (jobs[i].calls)
            want |= KGX_WANT_CALLS;
        if (jobs[i].otu_stats)
            want |= KGX_WANT_OTU;
    }
    std::string buf;
    buf.reserve(off[n]);
    for (auto &j : jobs)
        buf += j.seq;
    kgx_params p{min_hits, max_gap, order_constraint, min_weighted_hits};
    kgx_result r;
    int rc = kgx_process_batch(ctx_, &p, buf.data(), off.data(), n, want, &r);
    if (rc)
        throw_last(rc, "kgx_process_batch");
    for (uint32_t s = 0; s < n; s++) {
        SeqJob &j = jobs[s];
        if (j.hit_cb) {
            for (uint64_t i = r.hit_offsets[s]; i < r.hit_offsets[s + 1]; i++) {
                const kgx_hit &h = r.hits[i];
                sig_kmer_t e;
                e.which_kmer = h.which_kmer;
                e.otu_index = h.otu_index;
                e.avg_from_end = h.avg_from_end;
                e.pad = 0;
                e.function_index = h.function_index;
                e.function_wt = h.function_wt;
                j.hit_cb(hit_in_sequence_t(e, h.pos));
            }
        }
        if (j.calls) {
            for (uint64_t i = r.call_offsets[s]; i < r.call_offsets[s + 1]; i++) {
                const kgx_call &c = r.calls[i];
                j.calls->push_back(KmerCall(c.start, c.end, c.count, c.function_index, c.weighted_hits));
            }
        }
        if (j.otu_stats) {
            for (uint64_t i = r.otu_offsets[s]; i < r.otu_offsets[s + 1]; i++)
                j.otu_stats->otu_map[r.otus[i].otu_index] += r.otus[i].count;
            j.otu_stats->finalize(); /* process_aa_seq, kguts.cc:906-907 */
        }
        if (j.on_done)
            j.on_done();
    }
}

void KmerGuts::process_aa_seq(const std::string &id, const std::string &seq,
                              std::shared_ptr<std::vector<KmerCall>> calls,
                              std::function<void(hit_in_sequence_t)> hit_cb,
                              std::shared_ptr<KmerOtuStats> otu_stats)
{
    std::vector<SeqJob> jobs(1);
    jobs[0].id = id;
    jobs[0].seq = seq;
    jobs[0].calls = calls;
    jobs[0].hit_cb = hit_cb;
    jobs[0].otu_stats = otu_stats;
    process_aa_batch(jobs);
}

void KmerGuts::process_aa_seq_hits(const std::string &id, const std::string &seq,
                                   std::shared_ptr<std::vector<KmerCall>> calls,
                                   std::shared_ptr<std::vector<hit_in_sequence_t>> hits,
                                   std::shared_ptr<KmerOtuStats> otu_stats)
{
    /* kguts.cc:879-886 */
    auto cb = [hits](hit_in_sequence_t k) { hits->push_back(k); };
    process_aa_seq(id, seq, calls, cb, otu_stats);
}

const char *KmerGuts::function_at_index(int i) const
{
    if (i < 0 || i >= (int)functions_.size())
        return "INVALID_OFFSET";
    return functions_[i].c_str();
}

void KmerGuts::decoded_kmer(unsigned long long k, char *decoded)
{
    decoded[8] = 0;
    for (int i = 7; i >= 0; i--) {
        decoded[i] = kResidues[k % 20];
        k /= 20;
    }
}

unsigned long long KmerGuts::encoded_aa_kmer(const char *p)
{
    unsigned long long v = 0;
    for (int i = 0; i < 8; i++) {
        const char *hit = std::strchr(kResidues, p[i]);
        if (!p[i] || !hit)
            return 25600000000ULL + 1; /* MAX_ENCODED + 1 for any invalid residue */
        v = v * 20 + (unsigned long long)(hit - kResidues);
    }
    return v;
}

/* format_call / format_hit / format_otu_stats: iostream defaults (6
 * significant digits for floats), kguts.cc:939-973 */
std::string KmerGuts::format_call(const KmerCall &c)
{
    std::ostringstream o;
    o << "CALL\t" << c.start << "\t" << c.end << "\t" << c.count << "\t" << c.function_index << "\t"
      << function_at_index((int)c.function_index) << "\t" << c.weighted_hits << "\n";
    return o.str();
}

std::string KmerGuts::format_hit(const hit_in_sequence_t &h)
{
    char dc[9];
    decoded_kmer(h.hit.which_kmer, dc);
    std::ostringstream o;
    o << "HIT\t" << h.offset << "\t" << dc << "\t" << h.hit.avg_from_end << "\t"
      << function_at_index(h.hit.function_index) << "\t" << h.hit.function_wt << "\t"
      << h.hit.otu_index << "\n";
    return o.str();
}

std::string KmerGuts::format_otu_stats(const std::string &id, size_t size, KmerOtuStats &s)
{
    std::ostringstream o;
    o << "OTU-COUNTS\t" << id << "[" << size << "]";
    const size_t top = std::min<size_t>(s.otus_by_count.size(), 5);
    for (size_t i = 0; i < top; i++)
        o << "\t" << s.otus_by_count[i].second << "-" << s.otus_by_count[i].first;
    o << "\n";
    return o.str();
}

/* find_best_call, kguts.cc:1008-1199 -- a port of the SEED
 * km_process_hits_to_regions | km_pick_best_hit_in_peg pipeline. */
void KmerGuts::find_best_call(std::vector<KmerCall> &calls, int &function_index,
                              std::string &function, float &score, float &weighted_score,
                              float &score_offset)
{
    best_call(calls, [this](int i) { return function_at_index(i); }, function_index, function,
              score, weighted_score, score_offset);
}

void best_call(const std::vector<KmerCall> &calls, const std::function<const char *(int)> &name_of,
               int &function_index, std::string &function, float &score, float &weighted_score,
               float &score_offset)
{
    function_index = -1;
    function.clear();
    score = 0.0f;
    weighted_score = 0.0f;
    if (calls.empty())
        return; /* score_offset is left as the caller had it */

    /* adjacent calls of one function become one region */
    std::vector<KmerCall> regions;
    for (const KmerCall &c : calls) {
        if (!regions.empty() && regions.back().function_index == c.function_index) {
            KmerCall &r = regions.back();
            r.end = c.end;
            r.count += c.count;
            r.weighted_hits += c.weighted_hits;
        } else {
            regions.push_back(c);
        }
    }

    /* F1 | F2 | F1 with a weak interior (count < 5) and strong exterior
     * (counts summing to >= 10): drop F2 and join the F1 regions */
    std::vector<KmerCall> joined;
    size_t i = 0;
    while (i < regions.size()) {
        KmerCall cur = regions[i++];
        while (i + 1 < regions.size() && regions[i + 1].function_index == cur.function_index &&
               regions[i].count < 5 && cur.count + regions[i + 1].count >= 10) {
            cur.end = regions[i + 1].end;
            cur.count += regions[i + 1].count;
            cur.weighted_hits += regions[i + 1].weighted_hits;
            i += 2;
        }
        joined.push_back(cur);
    }

    /* per-function totals, ordered by function index (std::map) */
    typedef std::pair<int, std::pair<int, float>> total_t; /* fI -> (count, weighted) */
    std::map<int, std::pair<int, float>> totals;
    for (const KmerCall &c : joined) {
        auto ins = totals.emplace((int)c.function_index, std::make_pair(c.count, c.weighted_hits));
        if (!ins.second) {
            ins.first->second.first += c.count;
            ins.first->second.second += c.weighted_hits;
        }
    }
    std::vector<total_t> ranked(totals.begin(), totals.end());
    if (ranked.size() > 1)
        std::partial_sort(ranked.begin(), ranked.begin() + 2, ranked.end(),
                          [](const total_t &a, const total_t &b) {
                              return a.second.second > b.second.second;
                          });
    score_offset = ranked.size() == 1 ? (float)ranked[0].second.first
                                      : (float)(ranked[0].second.first - ranked[1].second.first);
    if (score_offset >= 5.0f) {
        function_index = ranked[0].first;
        function = name_of(function_index);
        score = (float)ranked[0].second.first;
        weighted_score = ranked[0].second.second;
        return;
    }
    /* ambiguous: optionally name the top two, lexically larger first */
    if (ranked.size() < 2)
        return;
    std::string a = name_of(ranked[0].first);
    std::string b = name_of(ranked[1].first);
    if (b > a)
        std::swap(a, b);
    if (ranked.size() == 2) {
        function = a + " ?? " + b;
        score = (float)ranked[0].second.first;
        return;
    }
    const float pair_offset = (float)(ranked[1].second.first - ranked[2].second.first);
    if (pair_offset > 5.0f) {
        function = a + " ?? " + b;
        score = (float)ranked[0].second.first;
        score_offset = pair_offset;
        weighted_score = ranked[0].second.second;
    }
}

/* ---- FastaParser --------------------------------------------------------------- */

FastaParser::FastaParser() { init_parse(); }

void FastaParser::init_parse()
{
    state_ = START;
    id_.clear();
    def_.clear();
    seq_.clear();
}

void FastaParser::emit()
{
    if (on_seq_)
        on_seq_(id_, seq_);
}

bool FastaParser::parse_char(char c)
{
    if (c == '\n')
        line_number_++;
    if (c == '\r')
        return true;
    std::string err;
    switch (state_) {
    case START:
        if (c == '>')
            state_ = ID;
        else
            err = "Missing >";
        break;
    case ID:
        if (std::isblank((unsigned char)c)) {
            def_.push_back(c);
            state_ = DEFLINE;
        } else if (c == '\n') {
            state_ = DATA;
        } else {
            id_.push_back(c);
        }
        break;
    case DEFLINE:
        if (c == '\n')
            state_ = DATA;
        else
            def_.push_back(c);
        break;
    case DATA:
        if (c == '\n')
            state_ = ID_OR_DATA;
        else if (std::isalpha((unsigned char)c) || c == '*')
            seq_.push_back(c);
        else
            err = std::string("Bad data character '") + c + "'";
        break;
    case ID_OR_DATA:
        if (c == '>') {
            emit();
            id_.clear();
            def_.clear();
            seq_.clear();
            state_ = ID;
        } else if (c == '\n') {
        } else if (std::isalpha((unsigned char)c)) {
            seq_.push_back(c);
            state_ = DATA;
        } else {
            err = std::string("Bad id or data character '") + c + "'";
        }
        break;
    }
    if (!err.empty()) {
        std::cerr << "Error found: " << err << " at line " << line_number_ << " id='" << id_ << "'"
                  << std::endl;
        if (on_error_)
            return on_error_(err, line_number_, id_);
    }
    return true;
}

void FastaParser::parse_complete()
{
    emit();
    id_.clear();
    def_.clear();
    seq_.clear();
}

/* ---- KmerPegMapping / MatrixRequest ------------------------------------ */

void run_batch_on_device(KmerGuts &kg, const std::vector<std::string> &seqs)
{
    std::vector<uint64_t> off(seqs.size() + 1, 0);
    std::string buf;
    for (size_t i = 0; i < seqs.size(); i++) {
        buf += seqs[i];
        off[i + 1] = buf.size();
    }
    kgx_params p{kg.min_hits, kg.max_gap, kg.order_constraint, kg.min_weighted_hits};
    kgx_result r;
    int rc = kgx_process_batch(kg.ctx(), &p, buf.data(), off.data(), (uint32_t)seqs.size(), 0, &r);
    if (rc)
        throw_last(rc, "kgx_process_batch");
}

KmerPegMapping::KmerPegMapping(int device) : device_(device)
{
    int rc = kgx_kmap_create(device, KGX_KMAP_APPEND, &kmer_to_id_);
    if (!rc)
        rc = kgx_kmap_create(device, KGX_KMAP_SET, &kmer_to_family_id_);
    if (rc) {
        kgx_kmap_destroy(kmer_to_id_);
        throw_last(rc, "kgx_kmap_create");
    }
}

KmerPegMapping::~KmerPegMapping()
{
    kgx_kmap_destroy(kmer_to_id_);
    kgx_kmap_destroy(kmer_to_family_id_);
}

KmerPegMapping::encoded_id_t KmerPegMapping::encode_id(const std::string &peg)
{
    auto it = peg_to_id_.find(peg);
    if (it != peg_to_id_.end())
        return it->second;
    const encoded_id_t id = (encoded_id_t)id_to_peg_.size();
    peg_to_id_[peg] = id;
    id_to_peg_.push_back(peg);
    return id;
}

std::string KmerPegMapping::decode_id(encoded_id_t id) const
{
    return id < id_to_peg_.size() ? id_to_peg_[id] : std::string();
}

void KmerPegMapping::add_batch_mappings(KmerGuts &kg, const std::vector<encoded_id_t> &ids)
{
    int rc = kgx_kmap_add_hits(kmer_to_id_, kg.ctx(), ids.data());
    if (rc)
        throw_last(rc, "kgx_kmap_add_hits");
}

void KmerPegMapping::add_batch_fam_mappings(KmerGuts &kg, const std::vector<encoded_family_id_t> &ids)
{
    int rc = kgx_kmap_add_hits(kmer_to_family_id_, kg.ctx(), ids.data());
    if (rc)
        throw_last(rc, "kgx_kmap_add_hits");
}

MatrixRequest::MatrixRequest(std::shared_ptr<KmerPegMapping> mapping) : mapping_(mapping)
{
    int rc = kgx_matrix_create(mapping_->kmer_to_id(), &mx_);
    if (rc)
        throw_last(rc, "kgx_matrix_create");
}

MatrixRequest::~MatrixRequest() { kgx_matrix_destroy(mx_); }

void MatrixRequest::process_work(KmerGuts &kg, const std::vector<std::pair<std::string, std::string>> &work)
{
    std::vector<KmerPegMapping::encoded_id_t> ids;
    std::vector<std::string> seqs;
    for (auto &w : work) {
        const KmerPegMapping::encoded_id_t eid = mapping_->encode_id(w.first);
        matrix_proteins_[eid] = w.second.size(); /* matrix_request.cc:91 */
        ids.push_back(eid);
        seqs.push_back(w.second);
    }
    run_batch_on_device(kg, seqs);
    int rc = kgx_matrix_add_hits(mx_, kg.ctx(), ids.data());
    if (rc)
        throw_last(rc, "kgx_matrix_add_hits");
}

void MatrixRequest::write_results(std::ostream &os)
{
    const kgx_pair_count *p = nullptr;
    uint64_t n = 0;
    int rc = kgx_matrix_pairs(mx_, &p, &n);
    if (rc)
        throw_last(rc, "kgx_matrix_pairs");
    for (uint64_t i = 0; i < n; i++) {
        const size_t l1 = matrix_proteins_[p[i].id1], l2 = matrix_proteins_[p[i].id2];
        const float score = (float)p[i].count / ((float)(l1 + l2));
        os << mapping_->decode_id(p[i].id1) << "\t" << mapping_->decode_id(p[i].id2) << "\t"
           << (unsigned long)p[i].count << "\t" << score << "\n";
    }
}

}  // namespace kgx

extern "C" int kgx_find_best_call(const kgx_call *calls, size_t n_calls, const char *const *names,
                                  int n_names, int32_t *function_index, char *function,
                                  size_t function_cap, float *score, float *weighted_score,
                                  float *score_offset, int *score_offset_set)
{
    if ((n_calls && !calls) || (n_names && !names) || !function_index || !score ||
        !weighted_score || !score_offset)
        return KGX_EINVAL;
    std::vector<kgx::KmerCall> v;
    v.reserve(n_calls);
    for (size_t i = 0; i < n_calls; i++)
        v.emplace_back(calls[i].start, calls[i].end, calls[i].count, calls[i].function_index,
                       calls[i].weighted_hits);
    auto name_of = [names, n_names](int i) -> const char * {
        return (i < 0 || i >= n_names) ? "INVALID_OFFSET" : names[i];
    };
    int fi;
    std::string fn;
    kgx::best_call(v, name_of, fi, fn, *score, *weighted_score, *score_offset);
    *function_index = fi;
    if (function && function_cap) {
        std::strncpy(function, fn.c_str(), function_cap - 1);
        function[function_cap - 1] = 0;
    }
    if (score_offset_set)
        *score_offset_set = n_calls > 0;
    return KGX_OK;
}
