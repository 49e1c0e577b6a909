/*
 * kgx_handlers.cpp -- request handlers and the HTTP request router over the
 * KmerGuts facade (see kgx_handlers.h).
 */
#include "kgx_handlers.h"

#include <algorithm>
#include <atomic>
#include <cctype>
#include <exception>
#include <charconv>
#include <cstring>
#include <emmintrin.h>
#include <regex>
#include <sstream>
#include <thread>

namespace kgx {

/* FastaParser's state machine (fasta_parser.h:45-133) one byte at a time:
 * the exact path, also for bodies with '\r', bad characters or odd framing */
static work_list_t parse_fasta_body_bytewise(const char *body, size_t n)
{
    work_list_t work;
    FastaParser parser;
    parser.set_callback([&work](const std::string &id, const std::string &seq) {
        work.emplace_back(id, seq);
        return 0;
    });
    for (size_t i = 0; i < n; i++)
        parser.parse_char(body[i]);
    parser.parse_complete();
    return work;
}

/* true when [p, le) holds only letters (C locale isalpha) and '*': 16 bytes
 * at a time (SSE2, the x86-64 baseline), then the tail */
static bool residue_line_ok(const char *p, const char *le)
{
    const __m128i lc = _mm_set1_epi8(0x20), a = _mm_set1_epi8('a'), z = _mm_set1_epi8(25),
                  star = _mm_set1_epi8('*');
    __m128i bad = _mm_setzero_si128();
    for (; le - p >= 16; p += 16) {
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(p));
        const __m128i t = _mm_sub_epi8(_mm_or_si128(c, lc), a);             /* letter: t in [0, 25] */
        const __m128i letter = _mm_cmpeq_epi8(_mm_min_epu8(t, z), t);       /* unsigned t <= 25 */
        const __m128i ok = _mm_or_si128(letter, _mm_cmpeq_epi8(c, star));
        bad = _mm_or_si128(bad, _mm_andnot_si128(ok, _mm_set1_epi8(-1)));
    }
    unsigned ok = _mm_movemask_epi8(bad) == 0;
    for (; p < le; p++) {
        const unsigned char c = (unsigned char)*p;
        ok &= (unsigned)((unsigned char)((c | 0x20) - 'a') < 26) | (unsigned)(c == '*');
    }
    return ok != 0;
}

/* Line-at-a-time parse of well-formed bodies, the common case, with the same
 * result as the state machine: every record starts with a header line
 * ('>' id [blank defline] '\n'), and every sequence line holds only letters
 * and '*' ('*' not first on a line other than the record's first line, where
 * the machine is still in DATA).  Blank lines are skipped, as in
 * ID_OR_DATA.  Anything else -- '\r', a bad character, a header right
 * after a header, a body not starting with '>' or ending inside a header --
 * returns false and the caller takes the bytewise path. */
static bool parse_fasta_body_lines(const char *body, size_t n, work_list_t &work)
{
    if (n == 0 || body[0] != '>' || std::memchr(body, '\r', n))
        return false;
    const char *p = body, *end = body + n;
    while (p < end) { /* p at a '>' */
        const char *eol = (const char *)std::memchr(p, '\n', end - p);
        if (!eol)
            return false; /* ends inside a header: leave it to the machine */
        const char *id_end = p + 1;
        while (id_end < eol && *id_end != ' ' && *id_end != '\t')
            id_end++;
        work.emplace_back(std::string(p + 1, id_end), std::string());
        std::string &seq = work.back().second;
        p = eol + 1;
        bool first_line = true;
        while (p < end && *p != '>') {
            eol = (const char *)std::memchr(p, '\n', end - p);
            const char *le = eol ? eol : end;
            const bool ok = residue_line_ok(p, le);
            if (!ok || (le > p && *p == '*' && !first_line))
                return false;
            seq.append(p, le);
            first_line = false;
            p = eol ? eol + 1 : end;
        }
        if (p < end && first_line)
            return false; /* '>' while the machine is in DATA: an error path */
    }
    return true;
}

/* parse_fasta_body_lines into the flat form (the same rules, record for
 * record); false: the byte machine's case */
static bool parse_fasta_flat_lines(const char *body, size_t n, FastaFlat &out)
{
    if (n == 0 || body[0] != '>' || std::memchr(body, '\r', n))
        return false;
    out.res.reserve(out.res.size() + n);
    const char *p = body, *end = body + n;
    while (p < end) { /* p at a '>' */
        const char *eol = (const char *)std::memchr(p, '\n', end - p);
        if (!eol)
            return false;
        const char *id_end = p + 1;
        while (id_end < eol && *id_end != ' ' && *id_end != '\t')
            id_end++;
        out.ids.append(p + 1, id_end);
        out.id_off.push_back(out.ids.size());
        p = eol + 1;
        bool first_line = true;
        while (p < end && *p != '>') {
            eol = (const char *)std::memchr(p, '\n', end - p);
            const char *le = eol ? eol : end;
            const bool ok = residue_line_ok(p, le);
            if (!ok || (le > p && *p == '*' && !first_line))
                return false;
            out.res.append(p, le);
            first_line = false;
            p = eol ? eol + 1 : end;
        }
        out.off.push_back(out.res.size());
        if (p < end && first_line)
            return false;
    }
    return true;
}

bool parse_fasta_piece_flat(const char *piece, size_t n, FastaFlat &out)
{
    return parse_fasta_flat_lines(piece, n, out);
}

FastaFlat flat_of(const work_list_t &work)
{
    FastaFlat f;
    for (const auto &w : work)
        f.add(w.first.data(), w.first.size(), w.second.data(), w.second.size());
    return f;
}

FastaFlat parse_fasta_body_flat(const char *body, size_t n)
{
    FastaFlat f;
    if (parse_fasta_flat_lines(body, n, f))
        return f;
    return flat_of(parse_fasta_body_bytewise(body, n));
}

std::vector<std::pair<size_t, size_t>> split_fasta_body(const char *body, size_t n, size_t pieces)
{
    std::vector<std::pair<size_t, size_t>> out;
    if (pieces < 2 || n == 0 || body[0] != '>')
        return out;
    size_t start = 0;
    for (size_t k = 1; k < pieces; k++) {
        size_t at = std::max(start + 1, k * (n / pieces));
        size_t cut = 0;
        while (at < n) {
            const char *nl = (const char *)std::memchr(body + at, '\n', n - at);
            if (!nl || nl + 1 >= body + n)
                break;
            const size_t c = (size_t)(nl - body) + 1;
            if (body[c] == '>') {
                /* the line before the cut must not be a header: a header right
                 * before '>' is an error path of the whole-body machine */
                size_t ls = c - 1;
                while (ls > start && body[ls - 1] != '\n')
                    ls--;
                if (body[ls] != '>') {
                    cut = c;
                    break;
                }
            }
            at = c;
        }
        if (!cut)
            break;
        out.emplace_back(start, cut);
        start = cut;
    }
    if (out.empty())
        return out;
    out.emplace_back(start, n);
    return out;
}

bool parse_fasta_piece(const char *piece, size_t n, work_list_t &work)
{
    return parse_fasta_body_lines(piece, n, work);
}

work_list_t parse_fasta_body(const char *body, size_t n)
{
    work_list_t work;
    if (parse_fasta_body_lines(body, n, work))
        return work;
    return parse_fasta_body_bytewise(body, n);
}

int param_int(const request_params_t &params, const std::string &name, int dflt)
{
    auto it = params.find(name);
    if (it == params.end())
        return dflt;
    try {
        return std::stoi(it->second);
    } catch (...) {
        return dflt;
    }
}

static std::vector<KmerGuts::SeqJob> jobs_for(const work_list_t &work)
{
    std::vector<KmerGuts::SeqJob> jobs(work.size());
    for (size_t i = 0; i < work.size(); i++) {
        jobs[i].id = work[i].first;
        jobs[i].seq = work[i].second;
        jobs[i].calls = std::make_shared<std::vector<KmerCall>>();
        jobs[i].otu_stats = std::make_shared<KmerOtuStats>();
    }
    return jobs;
}

void query_request(KmerGuts &kg, const work_list_t &work, int details, int find_best_call,
                   std::ostream &os)
{
    query_request(kg, flat_of(work), details, find_best_call, os);
}

void query_pass(KmerGuts &kg, const FastaFlat &batch, int details, int find_best_call, kgx_compact_result *cr)
{
    const uint32_t n = (uint32_t)batch.size();
    const bool want_hits = details && !find_best_call; /* HIT lines only without find_best_call */
    const uint32_t want = find_best_call ? KGX_WANT_BEST
                                         : (KGX_WANT_CALLS | KGX_WANT_OTU | (want_hits ? KGX_WANT_HITS : 0u));
    kgx_params p{kg.min_hits, kg.max_gap, kg.order_constraint, kg.min_weighted_hits};
    int rc;
    {
        StageClock clk(stage_stats().gpu_ns);
        rc = kgx_process_batch_compact(kg.ctx(), &p, batch.res.data(), batch.off.data(), n, want, cr);
    }
    stage_stats().gpu_passes++;
    if (rc)
        throw Error(rc, std::string("kgx_process_batch_compact: ") + kgx_strerror(rc) + " (" + kgx_last_error() + ")");
}

void query_text(KmerGuts &kg, const kgx_compact_result &cr, const FastaFlat &batch, uint32_t s0, uint32_t s1,
                const FastaFlat &ids, int details, int find_best_call, std::string &out)
{
    const bool want_hits = details && !find_best_call;
    const kgx_result &r = cr.r;
    out.reserve(out.size() + (size_t)(s1 - s0) * 96 + 64);
    std::vector<kgx_hit> seq_hits;
    char num[24];
    auto put_num = [&](long long v) {
        auto e = std::to_chars(num, num + sizeof num, v);
        out.append(num, e.ptr);
    };
    for (uint32_t s = s0; s < s1; s++) {
        const char *id = ids.ids.data() + ids.id_off[s - s0];
        const size_t id_len = ids.id_off[s - s0 + 1] - ids.id_off[s - s0];
        const uint64_t len = batch.off[s + 1] - batch.off[s];
        if (find_best_call) { /* query_request.cc:124-135, the device's decision */
            int fi;
            std::string fn;
            float score, wscore, off = 0.0f;
            kg.find_best_call(r.best[s], fi, fn, score, wscore, off);
            if (!fn.empty()) {
                std::ostringstream line; /* one line per call: the float format stays iostream's */
                line.write(id, (std::streamsize)id_len);
                line << "\t" << fn << "\t" << score << "\t" << wscore << "\n";
                out += line.str();
            }
            continue;
        }
        out += "PROTEIN-ID\t";
        out.append(id, id_len);
        out += '\t';
        put_num((long long)len);
        out += '\n';
        for (uint64_t c = r.call_offsets[s]; c < r.call_offsets[s + 1]; c++) {
            const kgx_call &k = r.calls[c];
            kg.append_call(out, KmerCall(k.start, k.end, k.count, k.function_index, k.weighted_hits));
        }
        if (want_hits) {
            const uint64_t nh = r.hit_offsets[s + 1] - r.hit_offsets[s];
            seq_hits.resize(nh);
            int rc;
            if (nh && (rc = kgx_compact_expand(&cr, batch.res.data(), batch.off.data(), s, s + 1, 0, seq_hits.data())))
                throw Error(rc, std::string("kgx_compact_expand: ") + kgx_last_error());
            for (const kgx_hit &h : seq_hits) {
                sig_kmer_t e;
                e.which_kmer = h.which_kmer;
                e.otu_index = h.otu_index;
                e.avg_from_end = h.avg_from_end;
                e.pad = 0;
                e.function_index = h.function_index;
                e.function_wt = h.function_wt;
                kg.append_hit(out, KmerGuts::hit_in_sequence_t(e, h.pos));
            }
        }
        /* KmerOtuStats::write's line (kguts.h:196-218): the device tallies
         * come in otus_by_count order; the top 5 */
        out += "OTU-COUNTS\t";
        out.append(id, id_len);
        out += '[';
        put_num((long long)len);
        out += ']';
        const uint64_t o0 = r.otu_offsets[s], o1 = std::min<uint64_t>(r.otu_offsets[s + 1], o0 + 5);
        for (uint64_t o = o0; o < o1; o++) {
            out += '\t';
            put_num(r.otus[o].count);
            out += '-';
            put_num(r.otus[o].otu_index);
        }
        out += '\n';
    }
}

void query_request(KmerGuts &kg, const FastaFlat &work, int details, int find_best_call, std::ostream &os)
{
    const uint32_t n = (uint32_t)work.size();
    if (n == 0)
        return;
    kgx_compact_result cr;
    query_pass(kg, work, details, find_best_call, &cr);
    std::string out;
    {
        StageClock clk(stage_stats().text_ns);
        query_text(kg, cr, work, 0, n, work, details, find_best_call, out);
    }
    os.write(out.data(), (std::streamsize)out.size());
}

/* ------------------------------------------------------------------------ */
/* ForkJoin                                                                  */
/* ------------------------------------------------------------------------ */

struct ForkJoin::Batch {
    const std::function<void(size_t)> *f;
    size_t k;
    std::atomic<size_t> next{0}, done{0};
    std::atomic<int> users{0}; /* helpers holding a pointer to the batch */
    std::mutex mu;
    std::condition_variable cv;
    std::mutex err_mu;
    std::exception_ptr err;
};

ForkJoin::ForkJoin(unsigned helpers)
{
    for (unsigned i = 0; i < helpers; i++)
        th_.emplace_back([this] { helper(); });
}

ForkJoin::~ForkJoin()
{
    {
        std::lock_guard<std::mutex> l(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_)
        t.join();
}

void ForkJoin::work(Batch &b)
{
    for (size_t i; (i = b.next.fetch_add(1)) < b.k;) {
        try {
            (*b.f)(i);
        } catch (...) {
            std::lock_guard<std::mutex> l(b.err_mu);
            if (!b.err)
                b.err = std::current_exception();
        }
        if (b.done.fetch_add(1) + 1 == b.k) {
            std::lock_guard<std::mutex> l(b.mu);
            b.cv.notify_all();
        }
    }
}

void ForkJoin::helper()
{
    for (;;) {
        Batch *b;
        {
            std::unique_lock<std::mutex> l(mu_);
            cv_.wait(l, [this] { return stop_ || !open_.empty(); });
            if (stop_)
                return;
            b = open_.front();
            b->users++;
        }
        work(*b);
        {
            std::lock_guard<std::mutex> l(mu_); /* every index is claimed: no one else takes it */
            auto it = std::find(open_.begin(), open_.end(), b);
            if (it != open_.end())
                open_.erase(it);
        }
        b->users--; /* the last touch: run() may return now */
    }
}

void ForkJoin::run(size_t k, const std::function<void(size_t)> &f)
{
    if (k == 0)
        return;
    if (k == 1 || th_.empty()) {
        for (size_t i = 0; i < k; i++)
            f(i);
        return;
    }
    Batch b;
    b.f = &f;
    b.k = k;
    {
        std::lock_guard<std::mutex> l(mu_);
        open_.push_back(&b);
    }
    for (size_t i = 1; i < std::min<size_t>(k, th_.size() + 1); i++)
        cv_.notify_one();
    work(b);
    {
        std::lock_guard<std::mutex> l(mu_);
        auto it = std::find(open_.begin(), open_.end(), &b);
        if (it != open_.end())
            open_.erase(it);
    }
    {
        std::unique_lock<std::mutex> l(b.mu);
        b.cv.wait(l, [&b] { return b.done.load() == b.k; });
    }
    while (b.users.load())
        std::this_thread::yield();
    if (b.err)
        std::rethrow_exception(b.err);
}

void add_request(KmerGuts &kg, KmerPegMapping &mapping, const work_list_t &work, int silent,
                 std::ostream &os)
{
    std::vector<KmerGuts::SeqJob> jobs = jobs_for(work);
    kg.process_aa_batch(jobs); /* the batch's hits stay on the device for the mapping */
    if (!silent) {
        std::string out;
        out.reserve(jobs.size() * 160);
        for (auto &j : jobs) { /* add_request.cc:134-161 */
            out += "PROTEIN-ID\t";
            out += j.id;
            out += '\t';
            out += std::to_string(j.seq.size());
            out += '\n';
            for (auto &c : *j.calls)
                kg.append_call(out, c);
            kg.append_otu_stats(out, j.id, j.seq.size(), *j.otu_stats);
            int fi;
            std::string fn;
            /* uninitialised in the reference when there are no calls
             * (add_request.cc:143-150, kguts.cc:1015-1018); 0 here */
            float score, wscore, off = 0.0f;
            kg.find_best_call(*j.calls, fi, fn, score, wscore, off);
            if (fn.empty() || fn.find(" ?? ") != std::string::npos)
                fn = "hypothetical protein";
            std::ostringstream line;
            line << "BEST-CALL\t" << j.id << "\t" << fn << "\t" << score << "\t" << wscore << "\t" << off
                 << "\n";
            out += line.str();
        }
        os.write(out.data(), (std::streamsize)out.size());
    }
    /* add_request.cc:164-170: ids encoded in request order, every hit's
     * k-mer mapped to its sequence's id */
    std::vector<KmerPegMapping::encoded_id_t> ids;
    ids.reserve(jobs.size());
    for (auto &j : jobs)
        ids.push_back(mapping.encode_id(j.id));
    mapping.add_batch_mappings(kg, ids);
}

void matrix_request(KmerGuts &kg, std::shared_ptr<KmerPegMapping> mapping, const work_list_t &work,
                    std::ostream &os)
{
    MatrixRequest mx(mapping);
    mx.process_work(kg, work);
    mx.write_results(os);
}

void lookup_request(KmerGuts &kg, std::shared_ptr<KmerPegMapping> mapping, bool family_mode,
                    const request_params_t &params, const work_list_t &work, std::ostream &os)
{
    LookupRequest req(mapping, family_mode, params);
    req.process_work(kg, work, os);
}

void fq_request(KmerGuts &kg, std::shared_ptr<KmerPegMapping> mapping, const char *body, size_t n,
                std::ostream &os)
{
    FqRequest req(kg, mapping);
    req.process(body, n, true, os);
}

/* ---- HTTP request framing (krequest2.cc) -------------------------------- */

bool parse_request_line(const std::string &line, HttpRequest &req)
{
    /* krequest2.cc:24 */
    static const std::regex request_regex("^([A-Z]+) ([^?#]*)(\\?([^#]*))?(#(.*))? HTTP/(\\d+\\.\\d+)");
    std::smatch m;
    if (!std::regex_match(line, m, request_regex))
        return false;
    req.method = m[1];
    req.path = m[2];
    req.parameters_raw = m[4];
    req.fragment = m[6];
    req.http_version = m[7];
    /* krequest2.cc:113-125: split on ';' or '&', keep "k=v" parts */
    size_t b = 0;
    const std::string &raw = req.parameters_raw;
    while (!raw.empty() && b <= raw.size()) {
        size_t e = raw.find_first_of(";&", b);
        if (e == std::string::npos)
            e = raw.size();
        const std::string part = raw.substr(b, e - b);
        const size_t eq = part.find('=');
        if (eq != std::string::npos)
            req.parameters[part.substr(0, eq)] = part.substr(eq + 1);
        b = e + 1;
    }
    return true;
}

void parse_header_line(const std::string &line, HttpRequest &req)
{
    /* krequest2.cc:176-186 */
    size_t x = line.find(':');
    std::string k = line.substr(0, x);
    std::string v;
    if (x != std::string::npos) {
        x++;
        while (x < line.size() && line[x] == ' ')
            x++;
        v = line.substr(x);
    }
    std::transform(k.begin(), k.end(), k.begin(), [](unsigned char c) { return std::tolower(c); });
    req.headers[k] = v;
}

/* ---- router --------------------------------------------------------------- */

class KmerRequestRouter::GutsLease {
public:
    explicit GutsLease(KmerRequestRouter &r, long only_slot = -1) : r_(r), kg_(r.acquire(only_slot)) {}
    ~GutsLease() { r_.release(kg_); }
    KmerGuts &operator*() { return *kg_; }

private:
    KmerRequestRouter &r_;
    KmerGuts *kg_;
};

namespace {

/* one replica per device slot: from the file (read once, copied to every
 * device) or, for the synthetic hook, built on the first device and copied
 * device to device to the others */
std::vector<std::shared_ptr<KmerImage>> open_images(const KmerRequestRouter::Options &opt,
                                                    const std::vector<int> &devs)
{
    std::vector<kgx_image *> raw(devs.size(), nullptr);
    int rc;
    if (opt.synthetic_keys) {
        uint64_t stored = 0;
        rc = kgx_image_build_synthetic(opt.synthetic_keys, opt.synthetic_sigs, devs[0], &raw[0], &stored);
        if (rc)
            throw Error(rc, std::string("kgx_image_build_synthetic: ") + kgx_last_error());
        std::vector<int> rcs(devs.size(), KGX_OK);
        std::vector<std::string> errs(devs.size());
        std::vector<std::thread> th;
        for (size_t i = 1; i < devs.size(); i++)
            th.emplace_back([&, i] {
                rcs[i] = kgx_image_replicate(raw[0], devs[i], &raw[i]);
                if (rcs[i])
                    errs[i] = kgx_last_error();
            });
        for (auto &t : th)
            t.join();
        for (size_t i = 1; i < devs.size(); i++)
            if (rcs[i]) {
                for (auto *im : raw)
                    kgx_image_close(im);
                throw Error(rcs[i], "kgx_image_replicate to device " + std::to_string(devs[i]) + ": " + errs[i]);
            }
    } else {
        rc = kgx_image_open_replicas(opt.kmer_data_dir.c_str(), devs.data(), (uint32_t)devs.size(), raw.data());
        if (rc)
            throw Error(rc, "KmerImage(" + opt.kmer_data_dir + "): " + kgx_strerror(rc) + " (" + kgx_last_error() +
                                ")");
    }
    std::vector<std::shared_ptr<KmerImage>> out;
    for (auto *im : raw)
        out.push_back(std::make_shared<KmerImage>(im));
    return out;
}

std::vector<int> device_list(const KmerRequestRouter::Options &opt)
{
    return opt.devices.empty() ? std::vector<int>{opt.device} : opt.devices;
}

} // namespace

KmerRequestRouter::KmerRequestRouter(const Options &opt)
    : opt_(opt), family_mode_(!opt.families_file.empty()) /* kser.cc:289 */,
      picker_(std::max<size_t>((size_t)std::max(1, opt.n_kmer_threads), device_list(opt).size()),
              device_list(opt).size())
{
    const std::vector<int> devs = device_list(opt_);
    images_ = open_images(opt_, devs);
    /* every device gets at least one worker; worker w on slot w % n (kgx_dispatch.h) */
    for (size_t w = 0; w < picker_.n_workers(); w++)
        pool_.emplace_back(new KmerGuts(opt_.kmer_data_dir, images_[picker_.slot_of(w)]));
    /* KGX_LOOKUP_BATCH=1: concurrent /lookup pieces share device passes
     * (LookupBatcher).  Off by default: at 16 clients 6.3e9 vs 7.5e9
     * residues/s with every piece its own pass (r8: ~5 pieces per shared pass,
     * but one pass at a time and its general path serialise what 16 workers'
     * small passes overlap) */
    if (const char *e = std::getenv("KGX_LOOKUP_BATCH"); e && std::atoi(e) != 0)
        lookup_batcher_.reset(new LookupBatcher());
    /* KGX_SERVER_PROBE_SERIALIZE=0: the workers' probes are not chained
     * behind one another (context option probe_serialize): a request piece's
     * probe may then overlap another's instead of waiting for it */
    if (const char *e = std::getenv("KGX_SERVER_PROBE_SERIALIZE"))
        for (auto &kg : pool_)
            if (int rc = kgx_ctx_set_option(kg->ctx(), "probe_serialize", std::atoi(e) != 0 ? 1 : 0))
                throw Error(rc, std::string("probe_serialize: ") + kgx_last_error());
    /* kserver.cc:40-130: the family DB goes into the root mapping, on the first device */
    auto root = std::make_shared<KmerPegMapping>(devs[0]);
    mapping_map_[""] = Mapping{root, std::make_shared<std::shared_mutex>()};
    if (!opt_.genus_mapping.empty())
        root->load_genus_map(opt_.genus_mapping);
    if (!opt_.families_file.empty())
        root->load_families(opt_.families_file);
    if (family_mode_)
        for (auto &nr : opt_.families_nr)
            root->load_nr_families(*pool_[0], nr); /* worker 0 is on slot 0: the mapping's device */
}

KmerRequestRouter::~KmerRequestRouter() = default;

std::vector<int> KmerRequestRouter::worker_devices() const
{
    std::vector<int> out;
    for (auto &kg : pool_)
        out.push_back(kgx_image_device(kg->image_->handle()));
    return out;
}

KmerGuts *KmerRequestRouter::acquire(long only_slot)
{
    std::unique_lock<std::mutex> lk(pool_mu_);
    long w = -1;
    pool_cv_.wait(lk, [&] { return (w = picker_.pick(only_slot)) >= 0; });
    picker_.lease((size_t)w);
    return pool_[(size_t)w].get();
}

void KmerRequestRouter::release(KmerGuts *kg)
{
    {
        std::lock_guard<std::mutex> lk(pool_mu_);
        for (size_t w = 0; w < pool_.size(); w++)
            if (pool_[w].get() == kg) {
                picker_.release(w);
                break;
            }
    }
    pool_cv_.notify_all(); /* a slot-restricted waiter may need this worker */
}

KmerRequestRouter::Mapping KmerRequestRouter::mapping_for(const std::string &key)
{
    /* krequest2.cc:416-425 creates unknown keys; the k-mer tables of every
     * mapping live on the first device */
    std::lock_guard<std::mutex> lk(mapping_mu_);
    /* (the root mapping "" always exists and is not counted) */
    if (mapping_map_.find(key) == mapping_map_.end() && mapping_map_.size() >= opt_.max_mappings + 1)
        return Mapping{}; /* over the cap: no new mapping */
    auto &m = mapping_map_[key];
    if (!m.map) {
        m.map = std::make_shared<KmerPegMapping>(device_list(opt_)[0]);
        m.mu = std::make_shared<std::shared_mutex>();
    }
    return m;
}

std::string KmerRequestRouter::header(const std::string &http_version, int code, const std::string &status)
{
    std::ostringstream os;
    os << "HTTP/" << http_version << " " << code << " " << status << "\n";
    os << "Content-type: text/plain\n";
    return os.str();
}

std::string KmerRequestRouter::respond(const std::string &http_version, int code,
                                       const std::string &status, const std::string &body)
{
    std::ostringstream os;
    os << header(http_version, code, status) << "Content-length: " << body.size() << "\n\n" << body;
    return os.str();
}

std::string KmerRequestRouter::handle(const HttpRequest &req, bool *quit)
{
    const std::string &ver = req.http_version;
    auto te = req.headers.find("transfer-encoding"); /* krequest2.cc:199-205 */
    if (te != req.headers.end() && te->second == "chunked")
        return respond(ver, 501, "Chunked encoding not implemented", "Chunked encoding not implemented\n");
    try {
        if (req.method == "GET") {
            static const std::regex genus_re("^/genus_lookup/([^/]+)$");
            std::smatch m;
            if (req.path == "/quit") {
                if (quit)
                    *quit = true;
                return respond(ver, 200, "OK", "OK, quitting\n");
            }
            if (req.path == "/version") {
                std::ostringstream os;
                if (!opt_.kmer_version.empty())
                    os << "kmer\t" << opt_.kmer_version << "\n";
                if (!opt_.families_version.empty())
                    os << "families\t" << opt_.families_version << "\n";
                os << "family-mode\t" << (family_mode_ ? "1" : "0") << "\n";
                return respond(ver, 200, "OK", os.str());
            }
            if (std::regex_match(req.path, m, genus_re)) {
                std::string id;
                Mapping root = mapping_for("");
                if (!root.map || !root.map->find_genus(m[1].str(), &id))
                    return respond(ver, 404, "Not Found", "genus not found\n");
                return respond(ver, 200, "OK", id + "\n");
            }
            if (req.path == "/server_stats") { /* stage clocks (StageStats); ?reset=1 zeroes them after */
                const std::string body = stage_stats().json();
                if (param_int(req.parameters, "reset", 0))
                    stage_stats().reset();
                return respond(ver, 200, "OK", body);
            }
            if (req.path == "/dump_sizes") {
                std::vector<std::pair<std::string, Mapping>> all;
                {
                    std::lock_guard<std::mutex> lk(mapping_mu_);
                    all.assign(mapping_map_.begin(), mapping_map_.end());
                }
                std::ostringstream os;
                os << "memory dump\n";
                for (auto &it : all) {
                    std::shared_lock<std::shared_mutex> rl(*it.second.mu);
                    os << "Mapping '" << it.first << "':\n";
                    it.second.map->dump_sizes(os);
                }
                return respond(ver, 200, "OK", os.str());
            }
            return respond(ver, 404, "Not found", "path not found\n");
        }
        if (req.method != "POST")
            return std::string(); /* the reference sends nothing for other methods */
        if (!req.headers.count("content-length"))
            return respond(ver, 500, "Missing content length", "Missing content length header\n");

        static const std::regex mapping_re("^/mapping/([^/]+)(/(add|matrix|lookup))$");
        std::string key, action = req.path;
        std::smatch m;
        if (std::regex_match(req.path, m, mapping_re)) {
            key = m[1];
            action = m[2];
        }
        const char *body = req.body.data();
        const size_t n = req.body.size();
        std::ostringstream os;
        if (action == "/query") {
            const int details = param_int(req.parameters, "details", 0);
            const int fbc = param_int(req.parameters, "find_best_call", 0);
            os << header(ver, 200, "OK") << "\n";
            /* a large body is cut into pieces at record starts that run on
             * several workers at once and are written in request order -- the
             * reference's 1-MiB chunks on its thread pool (krequest2.cc:41,
             * query_request.cc:62-160) -- when every piece parses line by line */
            const size_t n_pieces = std::min(pool_.size(), n / kPieceBytes);
            std::vector<std::pair<size_t, size_t>> cuts;
            std::vector<FastaFlat> works;
            bool ok;
            /* only while few /query bodies are in flight: under load the
             * requests themselves keep the cores busy, and a helper holding a
             * sub-piece while descheduled would stretch its request's tail */
            struct InFlight {
                std::atomic<int> &c;
                int now;
                explicit InFlight(std::atomic<int> &c_) : c(c_), now(++c_) {}
                ~InFlight() { --c; }
            } in_flight(query_in_flight_);
            const size_t n_sub = in_flight.now <= (int)fj_.helpers() ? std::min<size_t>(fj_.helpers() + 1, n / kSplitBytes)
                                                                      : 0;
            if (n_pieces < 2 && n_sub >= 2) {
                /* one GPU pass for the body; its parse and its text in
                 * sub-pieces on the ForkJoin helpers */
                FastaFlat batch;
                std::vector<uint64_t> seq_base, res_base;
                {
                    StageClock clk(stage_stats().parse_ns);
                    cuts = split_fasta_body(body, n, n_sub);
                    works.resize(cuts.size());
                    std::vector<char> good(cuts.size(), 0);
                    fj_.run(cuts.size(), [&](size_t i) {
                        good[i] = parse_fasta_piece_flat(body + cuts[i].first, cuts[i].second - cuts[i].first,
                                                         works[i]);
                    });
                    ok = !cuts.empty() && std::all_of(good.begin(), good.end(), [](char c) { return c != 0; });
                    if (ok) {
                        seq_base.assign(works.size() + 1, 0);
                        res_base.assign(works.size() + 1, 0);
                        for (size_t i = 0; i < works.size(); i++) {
                            seq_base[i + 1] = seq_base[i] + works[i].size();
                            res_base[i + 1] = res_base[i] + works[i].res.size();
                        }
                        batch.res.resize(res_base.back());
                        batch.off.resize(seq_base.back() + 1);
                        fj_.run(works.size(), [&](size_t i) {
                            const FastaFlat &w = works[i];
                            std::memcpy(&batch.res[res_base[i]], w.res.data(), w.res.size());
                            for (size_t j = 1; j <= w.size(); j++)
                                batch.off[seq_base[i] + j] = w.off[j] + res_base[i];
                        });
                    }
                }
                if (ok) {
                    if (batch.size() == 0)
                        return os.str();
                    GutsLease kg(*this);
                    (*kg).set_parameters(req.parameters);
                    kgx_compact_result cr;
                    query_pass(*kg, batch, details, fbc, &cr);
                    std::vector<std::string> outs(works.size());
                    {
                        StageClock clk(stage_stats().text_ns);
                        fj_.run(works.size(), [&](size_t i) {
                            query_text(*kg, cr, batch, (uint32_t)seq_base[i], (uint32_t)seq_base[i + 1], works[i],
                                       details, fbc, outs[i]);
                        });
                    }
                    std::string all = os.str();
                    size_t total = all.size();
                    for (auto &o : outs)
                        total += o.size();
                    all.reserve(total);
                    for (auto &o : outs)
                        all += o;
                    return all;
                }
                works.clear();
            }
            {
                StageClock clk(stage_stats().parse_ns);
                cuts = n_pieces >= 2 ? split_fasta_body(body, n, n_pieces) : decltype(cuts)();
                works.resize(cuts.size());
                ok = !cuts.empty();
                for (size_t i = 0; ok && i < cuts.size(); i++)
                    ok = parse_fasta_piece_flat(body + cuts[i].first, cuts[i].second - cuts[i].first, works[i]);
            }
            if (!ok) {
                GutsLease kg(*this);
                (*kg).set_parameters(req.parameters);
                FastaFlat work;
                {
                    StageClock clk(stage_stats().parse_ns);
                    work = parse_fasta_body_flat(body, n);
                }
                query_request(*kg, work, details, fbc, os);
                return os.str();
            }
            std::vector<std::string> outs(works.size());
            std::vector<std::string> errs(works.size());
            std::vector<std::thread> ths;
            for (size_t i = 0; i < works.size(); i++)
                ths.emplace_back([&, i] {
                    try {
                        GutsLease kg(*this);
                        (*kg).set_parameters(req.parameters);
                        std::ostringstream po;
                        query_request(*kg, works[i], details, fbc, po);
                        outs[i] = po.str();
                    } catch (const std::exception &e) {
                        errs[i] = e.what();
                    }
                });
            for (auto &t : ths)
                t.join();
            for (auto &e : errs)
                if (!e.empty())
                    throw Error(KGX_EDEVICE, e);
            std::string all = os.str();
            for (auto &o : outs)
                all += o;
            return all;
        }
        if (action != "/add" && action != "/matrix" && action != "/lookup" && action != "/fq_lookup")
            return respond(ver, 404, "Not found", "path not found\n");
        if (action == "/fq_lookup" && n == 0) /* fq_process_request.cc:42-46 */
            return respond(ver, 200, "OK", "data done\n");

        Mapping mp = mapping_for(key);
        if (!mp.map)
            return respond(ver, 503, "Service Unavailable", "too many mappings\n");
        /* /add and /matrix assign peg ids and read the device k-mer tables
         * of the mapping (its device: slot 0) -- one at a time per mapping;
         * /lookup and /fq_lookup only read the mapping, on any device */
        const bool writes = action == "/add" || action == "/matrix";
        std::unique_lock<std::shared_mutex> wl(*mp.mu, std::defer_lock);
        std::shared_lock<std::shared_mutex> rl(*mp.mu, std::defer_lock);
        if (writes)
            wl.lock();
        else
            rl.lock();
        GutsLease kg(*this, writes ? 0 : -1);
        (*kg).set_parameters(req.parameters);
        auto mapping = mp.map;
        if (action == "/fq_lookup") {
            os << header(ver, 200, "OK") << "\n";
            fq_request(*kg, mapping, body, n, os);
            return os.str();
        }
        if (action == "/lookup") { /* lookup_request.cc:146-150 */
            FastaFlat flat;
            {
                StageClock clk(stage_stats().parse_ns);
                flat = parse_fasta_body_flat(body, n);
            }
            os << header(ver, 200, "OK") << "\n";
            LookupRequest lr(mapping, family_mode_, req.parameters);
            lr.set_batcher(lookup_batcher_.get());
            lr.process_flat(*kg, flat.res.data(), flat.off.data(), flat.ids.data(), flat.id_off.data(), flat.size(),
                            os);
            return os.str();
        }
        work_list_t work;
        {
            StageClock clk(stage_stats().parse_ns);
            work = parse_fasta_body(body, n);
        }
        if (action == "/add") { /* krequest2.cc:429-436 */
            os << header(ver, 200, "OK") << "\n";
            add_request(*kg, *mapping, work, param_int(req.parameters, "silent", 0), os);
        } else if (action == "/matrix") { /* matrix_request.cc:166-170 */
            os << "HTTP/1.1 200 OK\nContent-type: text/plain\n\n";
            matrix_request(*kg, mapping, work, os);
        } else { /* lookup_request.cc:146-150 */
            os << header(ver, 200, "OK") << "\n";
            lookup_request(*kg, mapping, family_mode_, req.parameters, work, os);
        }
        return os.str();
    } catch (const std::exception &e) { /* krequest2.cc:206-220 */
        const std::string msg = std::string("Caught exception ") + e.what() + "\n";
        return respond(ver, 500, "Failed", msg);
    }
}

} // namespace kgx
