/*
 * kguts_hip.cpp -- the KmerGuts-compatible facade over the kgx C ABI.
 * Host-side rules restated from the reference: find_best_call
 * (kguts.cc:984-1199), text formatting (kguts.cc:939-973), OTU sorting
 * (kguts.h:185-219), index files (kguts.cc:544-575), FASTA framing
 * (fasta_parser.h:38-165, fasta_parser.cc:21-36).
 */
#include "kguts_hip.h"
#include "kgx_score_map.h"

#include <algorithm>
#include <x86intrin.h>
#include <charconv>
#include <cmath>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cctype>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <thread>

namespace kgx {

namespace {
const char kResidues[21] = "ACDEFGHIKLMNPQRSTVWY";

[[noreturn]] void throw_last(int rc, const std::string &what)
{
    throw Error(rc, what + ": " + kgx_strerror(rc) + " (" + kgx_last_error() + ")");
}
}  // namespace

/* ---- stage clocks -------------------------------------------------------------- */

namespace {
uint64_t now_ns()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}
}  // namespace

StageStats &stage_stats()
{
    static StageStats s;
    return s;
}

void StageStats::reset()
{
    for (auto *a : {&requests, &bytes_in, &bytes_out, &gpu_passes, &recv_ns, &parse_ns, &gpu_ns, &text_ns, &handle_ns,
                    &send_ns, &batched_pieces, &batched_passes})
        a->store(0);
    for (auto &a : text_cycles)
        a.store(0);
}

std::string StageStats::json() const
{
    char b[768];
    const double r = (double)std::max<uint64_t>(1, requests.load());
    std::snprintf(b, sizeof b,
                  "{\"requests\": %llu, \"bytes_in\": %llu, \"bytes_out\": %llu, \"gpu_passes\": %llu, "
                  "\"batched_pieces\": %llu, \"batched_passes\": %llu, "
                  "\"ms_per_request\": {\"recv\": %.4f, \"parse\": %.4f, \"gpu\": %.4f, \"text\": %.4f, \"handle\": %.4f, "
                  "\"send\": %.4f}, \"text_cycles\": [%llu, %llu, %llu, %llu, %llu]}\n",
                  (unsigned long long)requests.load(), (unsigned long long)bytes_in.load(),
                  (unsigned long long)bytes_out.load(), (unsigned long long)gpu_passes.load(),
                  (unsigned long long)batched_pieces.load(), (unsigned long long)batched_passes.load(),
                  recv_ns.load() / r * 1e-6,
                  parse_ns.load() / r * 1e-6, gpu_ns.load() / r * 1e-6, text_ns.load() / r * 1e-6,
                  handle_ns.load() / r * 1e-6,
                  send_ns.load() / r * 1e-6, (unsigned long long)text_cycles[0].load(),
                  (unsigned long long)text_cycles[1].load(), (unsigned long long)text_cycles[2].load(),
                  (unsigned long long)text_cycles[3].load(), (unsigned long long)text_cycles[4].load());
    return b;
}

StageClock::StageClock(std::atomic<uint64_t> &acc) : acc_(acc), t0_(now_ns()) {}
StageClock::~StageClock() { acc_ += now_ns() - t0_; }

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

KmerImage::KmerImage(kgx_image *borrowed, bool owned) : img_(borrowed), owned_(owned)
{
    if (!img_)
        throw Error(KGX_EINVAL, "KmerImage: null image");
}

KmerImage::~KmerImage()
{
    if (owned_)
        kgx_image_close(img_);
}

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

bool KmerGuts::default_service()
{
    const char *e = std::getenv("KGX_SVC");
    return !(e && std::atoi(e) == 0);
}

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
    /* compact hits: each sequence's hit_in_sequence_t are built as its
     * callbacks replay (no 32-B record per hit for the whole batch) */
    kgx_compact_result cr;
    int rc;
    {
        StageClock clk(stage_stats().gpu_ns);
        rc = kgx_process_batch_compact(ctx_, &p, buf.data(), off.data(), n, want, &cr);
    }
    stage_stats().gpu_passes++;
    if (rc)
        throw_last(rc, "kgx_process_batch_compact");
    const kgx_result &r = cr.r;
    std::vector<kgx_hit> seq_hits;
    for (uint32_t s = 0; s < n; s++) {
        SeqJob &j = jobs[s];
        if (j.hit_cb) {
            const uint64_t nh = r.hit_offsets[s + 1] - r.hit_offsets[s];
            seq_hits.resize(nh);
            if (nh && (rc = kgx_compact_expand(&cr, buf.data(), off.data(), s, s + 1, 0, seq_hits.data())))
                throw_last(rc, "kgx_compact_expand");
            for (uint64_t i = 0; i < nh; i++) {
                const kgx_hit &h = seq_hits[i];
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

/* ---- SeqCoalescer ------------------------------------------------------- */

SeqCoalescer::SeqCoalescer()
{
    if (const char *e = std::getenv("KGX_COALESCE_INFLIGHT"))
        max_inflight = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("KGX_COALESCE_RESIDUES"))
        max_residues = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));
    if (const char *e = std::getenv("KGX_COALESCE_SPIN_US"))
        spin_us = std::max(0, std::atoi(e));
}

void SeqCoalescer::submit(kgx_ctx *ctx, Req &r)
{
    using clock = std::chrono::steady_clock;
    {
        std::lock_guard<std::mutex> lk(mu_);
        queue_.push_back(&r);
        queued_.store(queue_.size(), std::memory_order_relaxed);
    }
    /* a waiter spins (a pass takes tens of us; a futex wake-up costs several)
     * and sleeps only after spin_us; it wakes for its own result or to lead */
    const auto spin_end = clock::now() + std::chrono::microseconds(spin_us);
    for (uint32_t spin = 0;; spin++) {
        if (r.done.load(std::memory_order_acquire))
            return;
        const bool can_lead = inflight_.load(std::memory_order_relaxed) < max_inflight &&
                              queued_.load(std::memory_order_relaxed) > 0;
        if (!can_lead && ((spin & 63u) != 0 || clock::now() < spin_end)) {
#if defined(__x86_64__)
            __builtin_ia32_pause();
#endif
            continue;
        }
        std::unique_lock<std::mutex> lk(mu_);
        if (r.done.load(std::memory_order_acquire))
            return;
        if (inflight_.load(std::memory_order_relaxed) < max_inflight && !queue_.empty()) {
            /* lead a pass: the queue's head and every queued call with the
             * same parameters, in arrival order, up to max_residues */
            std::vector<Req *> batch;
            uint64_t res = 0;
            const kgx_params p0 = queue_.front()->params;
            for (auto it = queue_.begin(); it != queue_.end();) {
                Req *q = *it;
                const bool same = q->params.min_hits == p0.min_hits && q->params.max_gap == p0.max_gap &&
                                  q->params.order_constraint == p0.order_constraint &&
                                  q->params.min_weighted_hits == p0.min_weighted_hits;
                if (same && (batch.empty() || res + q->seq->size() <= max_residues)) {
                    batch.push_back(q);
                    res += q->seq->size();
                    it = queue_.erase(it);
                } else {
                    ++it;
                }
            }
            queued_.store(queue_.size(), std::memory_order_relaxed);
            inflight_.fetch_add(1, std::memory_order_relaxed);
            lk.unlock();
            run_batch(ctx, batch);
            lk.lock();
            inflight_.fetch_sub(1, std::memory_order_relaxed);
            passes++;
            calls += batch.size();
            /* the callers served, and a sleeping queue head to lead the next
             * pass (spinning callers see the flags themselves) */
            for (Req *q : batch) {
                q->done.store(true, std::memory_order_release);
                if (q->sleeping)
                    q->cv.notify_one();
            }
            if (!queue_.empty() && queue_.front()->sleeping)
                queue_.front()->cv.notify_one();
            continue;
        }
        if (clock::now() < spin_end)
            continue; /* someone else leads: keep spinning */
        r.sleeping = true;
        r.cv.wait(lk, [&] {
            return r.done.load(std::memory_order_acquire) ||
                   (inflight_.load(std::memory_order_relaxed) < max_inflight && !queue_.empty());
        });
        r.sleeping = false;
    }
}

void SeqCoalescer::run_batch(kgx_ctx *ctx, std::vector<Req *> &batch)
{
    const uint32_t n = (uint32_t)batch.size();
    std::vector<uint64_t> off(n + 1, 0);
    uint32_t want = 0;
    for (uint32_t i = 0; i < n; i++) {
        off[i + 1] = off[i] + batch[i]->seq->size();
        want |= batch[i]->want;
    }
    std::string buf;
    buf.reserve(off[n]);
    for (Req *q : batch)
        buf += *q->seq;
    kgx_compact_result cr;
    /* per-sequence callers: the one-launch path where it applies */
    (void)kgx_ctx_set_option(ctx, "small_fused", 1);
    int rc = kgx_process_batch_compact(ctx, &batch[0]->params, buf.data(), off.data(), n, want, &cr);
    (void)kgx_ctx_set_option(ctx, "small_fused", 0);
    const kgx_result &r = cr.r;
    for (uint32_t i = 0; i < n && !rc; i++) {
        Req &q = *batch[i];
        if (q.want & KGX_WANT_HITS) {
            q.out.hits.resize(r.hit_offsets[i + 1] - r.hit_offsets[i]);
            if (!q.out.hits.empty())
                rc = kgx_compact_expand(&cr, buf.data(), off.data(), i, i + 1, 0, q.out.hits.data());
        }
        if (q.want & KGX_WANT_CALLS)
            q.out.calls.assign(r.calls + r.call_offsets[i], r.calls + r.call_offsets[i + 1]);
        if (q.want & KGX_WANT_OTU)
            q.out.otus.assign(r.otus + r.otu_offsets[i], r.otus + r.otu_offsets[i + 1]);
    }
    if (rc) {
        const std::string err = kgx_last_error();
        for (Req *q : batch) {
            q->rc = rc;
            q->err = err;
        }
    }
}

void KmerGuts::process_aa_seq(const std::string &id, const std::string &seq,
                              std::shared_ptr<std::vector<KmerCall>> calls,
                              std::function<void(hit_in_sequence_t)> hit_cb,
                              std::shared_ptr<KmerOtuStats> otu_stats)
{
    const uint32_t want = (hit_cb ? KGX_WANT_HITS : 0u) | (calls ? KGX_WANT_CALLS : 0u) | (otu_stats ? KGX_WANT_OTU : 0u);
    if (coalesce && service && want) {
        /* the image's resident call service: no launch on this call's path
         * (KGX_EBUSY: not a call it serves, or every slot taken -> below) */
        thread_local std::vector<kgx_hit> hbuf;
        thread_local std::vector<kgx_call> cbuf;
        thread_local std::vector<kgx_otu> obuf;
        const uint64_t W = seq.size() >= 9 ? seq.size() - 8 : 0;
        if (hbuf.size() < W)
            hbuf.resize(W);
        if (cbuf.size() < W)
            cbuf.resize(W);
        if (otu_stats && obuf.size() < W)
            obuf.resize(W);
        const kgx_params p{min_hits, max_gap, order_constraint, min_weighted_hits};
        uint64_t nh = 0, nc = 0, no = 0;
        const int rc = kgx_svc_call(image_->handle(), &p, seq.data(), seq.size(), want, hbuf.data(), hbuf.size(), &nh,
                                    cbuf.data(), cbuf.size(), &nc, obuf.data(), obuf.size(), &no);
        if (rc == KGX_OK) {
            /* replay on the calling thread, in position order (kguts.cc:814-815) */
            if (hit_cb)
                for (uint64_t i = 0; i < nh; i++) {
                    const kgx_hit &h = hbuf[i];
                    sig_kmer_t e;
                    e.which_kmer = h.which_kmer;
                    e.otu_index = h.otu_index;
                    e.avg_from_end = h.avg_from_end;
                    e.pad = 0;
                    e.function_index = h.function_index;
                    e.function_wt = h.function_wt;
                    hit_cb(hit_in_sequence_t(e, h.pos));
                }
            if (calls)
                for (uint64_t i = 0; i < nc; i++) {
                    const kgx_call &c = cbuf[i];
                    calls->push_back(KmerCall(c.start, c.end, c.count, c.function_index, c.weighted_hits));
                }
            if (otu_stats) {
                for (uint64_t i = 0; i < no; i++)
                    otu_stats->otu_map[obuf[i].otu_index] += obuf[i].count;
                otu_stats->finalize(); /* kguts.cc:906-907 */
            }
            return;
        }
        if (rc == KGX_EDEVICE) {
            /* no answer within 10 s leaves the service "broken" (every later
             * call KGX_EBUSY): replace it, so one stall does not turn the
             * service off for the rest of the process; this call takes the
             * batch path below */
            uint64_t broken = 0;
            if (kgx_svc_stat(image_->handle(), "broken", &broken) != KGX_OK || !broken)
                throw_last(rc, "kgx_svc_call");
            (void)kgx_svc_stop(image_->handle());
        } else if (rc != KGX_EBUSY) {
            throw_last(rc, "kgx_svc_call");
        }
    }
    if (coalesce) {
        SeqCoalescer::Req q;
        q.seq = &seq;
        q.params = kgx_params{min_hits, max_gap, order_constraint, min_weighted_hits};
        q.want = want;
        image_->coalescer().submit(ctx_, q);
        if (q.rc)
            throw Error(q.rc, "process_aa_seq: " + std::string(kgx_strerror(q.rc)) + " (" + q.err + ")");
        /* replay on the calling thread, in position order (kguts.cc:814-815) */
        if (hit_cb)
            for (const kgx_hit &h : q.out.hits) {
                sig_kmer_t e;
                e.which_kmer = h.which_kmer;
                e.otu_index = h.otu_index;
                e.avg_from_end = h.avg_from_end;
                e.pad = 0;
                e.function_index = h.function_index;
                e.function_wt = h.function_wt;
                hit_cb(hit_in_sequence_t(e, h.pos));
            }
        if (calls)
            for (const kgx_call &c : q.out.calls)
                calls->push_back(KmerCall(c.start, c.end, c.count, c.function_index, c.weighted_hits));
        if (otu_stats) {
            for (const kgx_otu &o : q.out.otus)
                otu_stats->otu_map[o.otu_index] += o.count;
            otu_stats->finalize(); /* kguts.cc:906-907 */
        }
        return;
    }
    /* one pass of one sequence: the one-launch path where it applies */
    struct Fused {
        kgx_ctx *c;
        explicit Fused(kgx_ctx *x) : c(x) { (void)kgx_ctx_set_option(c, "small_fused", 1); }
        ~Fused() { (void)kgx_ctx_set_option(c, "small_fused", 0); }
    } fused(ctx_);
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
/* iostream's default formatting of the numbers in the handler lines */
static void append_u64(std::string &out, unsigned long long v)
{
    char b[24];
    auto r = std::to_chars(b, b + sizeof b, v);
    out.append(b, r.ptr);
}

static void append_i64(std::string &out, long long v)
{
    char b[24];
    auto r = std::to_chars(b, b + sizeof b, v);
    out.append(b, r.ptr);
}

/* operator<<(float) with precision 6 and no floatfield is "%.*g" of the
 * value widened to double (libstdc++ num_put::_M_insert_float); to_chars in
 * general format with a precision is specified as printf's %.6g, at a quarter
 * of snprintf's cost.  Integral values below 1e6 in magnitude -- the scores
 * (counts) and the zeros of most output lines -- print as %.6g prints them,
 * their digits (and "-0" for negative zero), without the float formatter.
 * kgx_format_g6 exports it; tests/test_abi_host.py checks it against
 * printf's %.6g. */
static size_t format_g6(char *b, size_t cap, float v)
{
    const double d = (double)v;
    if (d == 0.0) {
        if (std::signbit(d)) {
            b[0] = '-';
            b[1] = '0';
            return 2;
        }
        b[0] = '0';
        return 1;
    }
    if (d > -1e6 && d < 1e6 && d == (double)(long long)d)
        return (size_t)(std::to_chars(b, b + cap, (long long)d).ptr - b);
    /* 1e-4 <= |v| < 1e6 (the scores): with 10^e <= |v| < 10^(e+1), |v| *
     * 10^(5-e) is exact in a double (24 + at most 21 bits), so rounding it
     * to an integer (nearbyint: to nearest, ties to even) gives printf's six
     * significant digits; fixed notation, trailing zeros dropped */
    static const double p10[] = {1e-4, 1e-3, 1e-2, 1e-1, 1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9};
    const double a = std::fabs(d);
    if (cap >= 16 && a >= 1e-4 && a < 1e6) {
        int e = 5;
        while (a < p10[e + 4])
            e--;
        long long r = (long long)std::nearbyint(a * p10[5 - e + 4]);
        if (r == 1000000) { /* rounded up to 10^(e+1) */
            if (e == 5)
                return (size_t)(std::to_chars(b, b + cap, d, std::chars_format::general, 6).ptr - b);
            r = 100000;
            e++;
        }
        char dig[6];
        for (int i = 5; i >= 0; i--, r /= 10)
            dig[i] = (char)('0' + r % 10);
        size_t n = 0;
        if (d < 0)
            b[n++] = '-';
        int last = 5; /* the last significant digit kept */
        while (last > 0 && last > e && dig[last] == '0')
            last--;
        if (e >= 0) {
            for (int i = 0; i <= e; i++)
                b[n++] = dig[i];
            if (last > e) {
                b[n++] = '.';
                for (int i = e + 1; i <= last; i++)
                    b[n++] = dig[i];
            }
        } else {
            b[n++] = '0';
            b[n++] = '.';
            for (int i = 0; i < -e - 1; i++)
                b[n++] = '0';
            for (int i = 0; i <= last; i++)
                b[n++] = dig[i];
        }
        return n;
    }
    return (size_t)(std::to_chars(b, b + cap, d, std::chars_format::general, 6).ptr - b);
}

static void append_f32(std::string &out, float v)
{
    char b[48];
    out.append(b, format_g6(b, sizeof b, v));
}

extern "C" size_t kgx_format_g6(float v, char *out, size_t cap)
{
    char b[48];
    const size_t n = format_g6(b, sizeof b, v);
    if (out && cap) {
        const size_t k = std::min(n, cap - 1);
        std::memcpy(out, b, k);
        out[k] = 0;
    }
    return n;
}

void KmerGuts::append_call(std::string &out, const KmerCall &c) const
{
    out += "CALL\t";
    append_u64(out, c.start);
    out += '\t';
    append_u64(out, c.end);
    out += '\t';
    append_i64(out, c.count);
    out += '\t';
    append_u64(out, c.function_index);
    out += '\t';
    out += function_at_index((int)c.function_index);
    out += '\t';
    append_f32(out, c.weighted_hits);
    out += '\n';
}

void KmerGuts::append_hit(std::string &out, const hit_in_sequence_t &h) const
{
    char dc[9];
    decoded_kmer(h.hit.which_kmer, dc);
    out += "HIT\t";
    append_u64(out, h.offset);
    out += '\t';
    out += dc;
    out += '\t';
    append_u64(out, h.hit.avg_from_end);
    out += '\t';
    out += function_at_index(h.hit.function_index);
    out += '\t';
    append_f32(out, h.hit.function_wt);
    out += '\t';
    append_i64(out, h.hit.otu_index);
    out += '\n';
}

void KmerGuts::append_otu_stats(std::string &out, const std::string &id, size_t size,
                                const KmerOtuStats &s) const
{
    out += "OTU-COUNTS\t";
    out += id;
    out += '[';
    append_u64(out, size);
    out += ']';
    const size_t top = std::min<size_t>(s.otus_by_count.size(), 5);
    for (size_t i = 0; i < top; i++) {
        out += '\t';
        append_i64(out, s.otus_by_count[i].second);
        out += '-';
        append_i64(out, s.otus_by_count[i].first);
    }
    out += '\n';
}

std::string KmerGuts::format_call(const KmerCall &c)
{
    std::string o;
    append_call(o, c);
    return o;
}

std::string KmerGuts::format_hit(const hit_in_sequence_t &h)
{
    std::string o;
    append_hit(o, h);
    return o;
}

std::string KmerGuts::format_otu_stats(const std::string &id, size_t size, KmerOtuStats &s)
{
    std::string o;
    append_otu_stats(o, id, size, s);
    return o;
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

void KmerGuts::find_best_call(const kgx_best_call &best, int &function_index, std::string &function,
                              float &score, float &weighted_score, float &score_offset)
{
    best_call(best, [this](int i) { return function_at_index(i); }, function_index, function, score,
              weighted_score, score_offset);
}

void best_call(const kgx_best_call &b, const std::function<const char *(int)> &name_of, int &function_index,
               std::string &function, float &score, float &weighted_score, float &score_offset)
{
    function_index = b.kind == 1 ? b.fi0 : -1;
    function.clear();
    score = b.score;
    weighted_score = b.weighted_score;
    if (b.kind != 0)
        score_offset = b.score_offset; /* kind 0: left as the caller had it */
    if (b.kind == 1) {
        function = name_of(b.fi0);
    } else if (b.kind == 2) { /* the lexically larger name first (kguts.cc:1176-1179) */
        std::string f1 = name_of(b.fi0), f2 = name_of(b.fi1);
        if (f2 > f1)
            std::swap(f1, f2);
        function = f1 + " ?? " + f2;
    }
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

std::string KmerPegMapping::lookup_genus(const std::string &genus)
{
    std::lock_guard<std::mutex> lk(genus_mu_);
    return genus_map_[genus];
}

bool KmerPegMapping::find_genus(const std::string &genus, std::string *id) const
{
    std::lock_guard<std::mutex> lk(genus_mu_);
    auto it = genus_map_.find(genus);
    if (it == genus_map_.end())
        return false;
    *id = it->second;
    return true;
}

KmerPegMapping::family_data_t KmerPegMapping::family_at(encoded_family_id_t id) const
{
    auto it = family_data_.find(id);
    return it == family_data_.end() ? family_data_t{} : it->second;
}

std::string KmerPegMapping::decode_id(encoded_id_t id) const
{
    return id < id_to_peg_.size() ? id_to_peg_[id] : std::string();
}

void KmerPegMapping::dump_sizes(std::ostream &os) const
{
    os << "kmer_to_id_: size=" << kgx_kmap_num_kmers(kmer_to_id_) << "\n";
    os << "kmer_to_id_: content size=" << kgx_kmap_num_values(kmer_to_id_) << "\n";
    os << "peg_to_id_: size=" << peg_to_id_.size() << "\n";
    os << "id_to_peg_: size=" << id_to_peg_.size() << "\n";
    os << "genome_to_id_: size=0\n";
    os << "id_to_genome_: size=0\n";
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

/* ---- family DB, FamilyMapper, FqRequest ---------------------------------- */

KmerPegMapping::encoded_id_t KmerPegMapping::assign_new_peg_id(const std::string &peg)
{
    const encoded_id_t id = (encoded_id_t)id_to_peg_.size();
    peg_to_id_[peg] = id;
    id_to_peg_.push_back(peg);
    return id;
}

static std::vector<std::string> split_tabs(const std::string &line)
{
    std::vector<std::string> cols; /* boost::split(cols, line, is_any_of("\t")) */
    size_t a = 0;
    for (;;) {
        size_t b = line.find('\t', a);
        cols.push_back(line.substr(a, b == std::string::npos ? std::string::npos : b - a));
        if (b == std::string::npos)
            return cols;
        a = b + 1;
    }
}

void KmerPegMapping::load_genus_map(const std::string &genus_file)
{
    std::ifstream gf(genus_file);
    if (gf.fail())
        throw Error(KGX_EIO, "Error opening gnus file " + genus_file);
    std::string line;
    while (std::getline(gf, line)) {
        auto cols = split_tabs(line);
        genus_map_[cols[0]] = cols.size() > 1 ? cols[1] : std::string();
    }
}

void KmerPegMapping::load_families(const std::string &families_file)
{
    std::ifstream f(families_file);
    if (f.fail())
        throw Error(KGX_EIO, "Failure opening families file " + families_file);
    const std::string zeros("00000000");
    std::string line;
    while (std::getline(f, line)) {
        auto cols = split_tabs(line);
        if (cols.size() < 9)
            continue;
        std::string pgf = "PGF_" + cols[0].substr(2);
        std::string plf("PLF_");
        unsigned long genus_id = 0;
        auto mapped = genus_map_.find(cols[7]);
        if (mapped == genus_map_.end()) {
            plf += cols[7];
        } else {
            plf += mapped->second;
            genus_id = std::stoul(mapped->second);
        }
        plf += "_";
        plf += zeros.substr(0, 8 - cols[8].size());
        plf += cols[8];
        const encoded_id_t id = assign_new_peg_id(cols[3]);
        const unsigned long seqlen = std::stoul(cols[4]);
        auto fkey = std::make_pair(pgf, plf);
        encoded_family_id_t fam_id;
        auto fit = family_key_to_id_.find(fkey);
        if (fit == family_key_to_id_.end()) {
            fam_id = next_family_id_++;
            family_key_to_id_[fkey] = fam_id;
            family_data_.emplace(fam_id, family_data_t{pgf, plf, genus_id, cols[5], fam_id, seqlen, 1});
        } else {
            fam_id = fit->second;
            family_data_t &d = family_data_[fam_id];
            d.total_size += seqlen;
            d.count++;
        }
        peg_to_family_.insert(std::make_pair(id, fam_id));
    }
}

void KmerPegMapping::load_nr_families(KmerGuts &kg, const std::string &nr_fasta, size_t batch)
{
    std::ifstream in(nr_fasta, std::ios::binary);
    if (!in)
        throw Error(KGX_EIO, "cannot open " + nr_fasta);
    std::vector<std::string> seqs;
    std::vector<encoded_family_id_t> fams;
    auto flush = [&]() {
        if (seqs.empty())
            return;
        run_batch_on_device(kg, seqs);
        add_batch_fam_mappings(kg, fams);
        seqs.clear();
        fams.clear();
    };
    FastaParser parser;
    parser.set_callback([&](const std::string &id, const std::string &seq) {
        auto fit = peg_to_family_.find(encode_id(id));
        if (fit == peg_to_family_.end())
            return 0; /* "NO FAM FOR id=..." (nr_loader.cc:150-156) */
        seqs.push_back(seq);
        fams.push_back(fit->second);
        if (seqs.size() >= batch)
            flush();
        return 0;
    });
    char ch;
    while (in.get(ch))
        parser.parse_char(ch);
    parser.parse_complete();
    flush();
}

FamilyMapper::FamilyMapper(KmerGuts &kg, std::shared_ptr<KmerPegMapping> mapping) : kg_(kg), mapping_(mapping) {}

FamilyMapper::best_match_t FamilyMapper::find_best_family_match(const kgx_rollup_row *rows, size_t n_rows,
                                                                 std::vector<KmerCall> &calls)
{
    int fi;
    std::string fn;
    float score, wscore, off = 0.0f;
    kg_.find_best_call(calls, fi, fn, score, wscore, off);
    return match_from(rows, n_rows, fn, score);
}

FamilyMapper::best_match_t FamilyMapper::find_best_family_match(const kgx_rollup_row *rows, size_t n_rows,
                                                                 const kgx_best_call &best)
{
    int fi;
    std::string fn;
    float score, wscore, off = 0.0f;
    kg_.find_best_call(best, fi, fn, score, wscore, off);
    return match_from(rows, n_rows, fn, score);
}

FamilyMapper::best_match_t FamilyMapper::match_from(const kgx_rollup_row *rows, size_t n_rows, std::string fn,
                                                    float score)
{
    /* ingest_protein clears seq_score_ (family_mapper.cc:48); on_hit's
     * operator[] calls (family_mapper.cc:287-312) leave the ids in
     * first-touch order, which is the rows' order */
    seq_score_.clear();
    for (size_t j = 0; j < n_rows; j++) {
        sequence_accumulated_score_t &s = seq_score_[rows[j].id];
        s.hit_count = rows[j].hit_count;
        s.hit_total = rows[j].hit_total;
        s.weighted_total = rows[j].weighted_total;
    }
    if (fn.empty() || fn.find(" ?? ") != std::string::npos)
        fn = "hypothetical protein"; /* allow_ambiguous_functions_ = false */
    float best_lf = 0.0f, best_gf = 0.0f;
    std::string lf, gf;
    std::unordered_map<std::string, float> pgf_rollup;
    for (auto hit_ent : seq_score_) {
        const sequence_accumulated_score_t &se = hit_ent.second;
        if (se.hit_total < kmer_hit_threshold_)
            continue;
        auto fent = mapping_->family_data_.find(hit_ent.first);
        if (fent == mapping_->family_data_.end())
            continue;
        const KmerPegMapping::family_data_t &fd = fent->second;
        if (fd.function != fn)
            continue;
        pgf_rollup[fd.pgf] += se.weighted_total;
        if (se.weighted_total > best_lf) {
            best_lf = se.weighted_total;
            lf = fd.plf;
        }
    }
    for (auto pgf_ent : pgf_rollup)
        if (pgf_ent.second > best_gf) {
            best_gf = pgf_ent.second;
            gf = pgf_ent.first;
        }
    return best_match_t{gf, best_gf, lf, best_lf, fn, score};
}

std::ostream &operator<<(std::ostream &os, const FamilyMapper::best_match_t &m)
{
    /* family_mapper.h:70-75 */
    os << m.gfam_id << "\t" << m.gfam_score << "\t" << m.lfam_id << "\t" << m.lfam_score << "\t" << m.function
       << "\t" << m.score;
    return os;
}

/* ---- LookupBatcher ------------------------------------------------------- */

struct LookupBatcher::Piece {
    uint32_t seq0 = 0, n = 0;
    uint64_t res0 = 0;
    Out *out = nullptr;
    int rc = KGX_OK;
    std::string err;
    bool done = false;
};

/* a staging area: pieces' residues and rebased offsets, contiguous, in
 * pinned host memory (the pass reads them by DMA, no staging copy) */
struct LookupBatcher::Area {
    char *res = nullptr;
    uint64_t *off = nullptr;
    uint64_t res_used = 0;
    uint32_t seq_used = 0, copying = 0;
    std::vector<Piece *> pieces;
    kgx_kmap *map = nullptr;
    int mode = 0;
    kgx_params p{};
    uint32_t want = 0;
    ~Area()
    {
        if (res)
            kgx_host_free(res);
        if (off)
            kgx_host_free(off);
    }
    bool fits(kgx_kmap *m, int md, const kgx_params &q, uint32_t w, uint64_t nres, uint32_t n, uint64_t max_res,
              uint32_t max_seq) const
    {
        if (pieces.empty())
            return true;
        return m == map && md == mode && w == want && q.min_hits == p.min_hits && q.max_gap == p.max_gap &&
               q.order_constraint == p.order_constraint && q.min_weighted_hits == p.min_weighted_hits &&
               res_used + nres <= max_res && seq_used + n <= max_seq;
    }
};

LookupBatcher::LookupBatcher(uint64_t max_residues, uint32_t max_seqs) : max_res_(max_residues), max_seq_(max_seqs)
{
    for (auto &a : area_)
        a.reset(new Area);
}

LookupBatcher::~LookupBatcher() = default;

void LookupBatcher::run_alone(KmerGuts &kg, kgx_kmap *map, int mode, const kgx_params &p, uint32_t want,
                              const char *res, const uint64_t *off, uint32_t n, Out &out)
{
    kgx_result r;
    int rc = kgx_process_batch(kg.ctx(), &p, res, off, n, want, &r);
    if (rc)
        throw_last(rc, "kgx_process_batch");
    kgx_rollup_result ru;
    if ((rc = kgx_kmap_rollup(map, kg.ctx(), mode, &ru)))
        throw_last(rc, "kgx_kmap_rollup");
    if (want & KGX_WANT_BEST)
        out.best.assign(r.best, r.best + n);
    out.roff.assign(ru.offsets, ru.offsets + n + 1);
    out.rows.assign(ru.rows, ru.rows + ru.offsets[n]);
}

void LookupBatcher::run(KmerGuts &kg, kgx_kmap *map, int mode, const kgx_params &p, uint32_t want,
                        const char *res, const uint64_t *off, uint32_t n, Out &out)
{
    const uint64_t nres = n ? off[n] - off[0] : 0;
    std::unique_lock<std::mutex> lk(mu_);
    /* alone (no other request inside), too large for an area, or a map the
     * worker's device cannot roll up in its own pass: the piece's own pass */
    const bool alone = active_ == 0 && !busy_ && area_[open_]->pieces.empty();
    if (alone || n == 0 || nres > max_res_ || n > max_seq_ ||
        kgx_kmap_device(map) != kgx_image_device(kg.image_->handle())) {
        active_++;
        lk.unlock();
        alone_++;
        try {
            run_alone(kg, map, mode, p, want, res, off, n, out);
        } catch (...) {
            lk.lock();
            active_--;
            throw;
        }
        lk.lock();
        active_--;
        return;
    }
    active_++;
    /* a place in the open area (wait while it holds other parameters or is full) */
    while (!area_[open_]->fits(map, mode, p, want, nres, n, max_res_, max_seq_))
        cv_.wait(lk);
    Area &A = *area_[open_];
    if (!A.res) { /* first use: both areas' pinned buffers */
        for (auto &a : area_) {
            void *r = nullptr, *o = nullptr;
            if (kgx_host_alloc(max_res_ + 64, &r) || kgx_host_alloc(((uint64_t)max_seq_ + 1) * 8, &o)) {
                if (r)
                    kgx_host_free(r);
                active_--;
                throw_last(KGX_ENOMEM, "lookup batcher: pinned staging");
            }
            a->res = static_cast<char *>(r);
            a->off = static_cast<uint64_t *>(o);
        }
    }
    Piece pc;
    pc.seq0 = A.seq_used;
    pc.res0 = A.res_used;
    pc.n = n;
    pc.out = &out;
    if (A.pieces.empty()) {
        A.map = map;
        A.mode = mode;
        A.p = p;
        A.want = want;
    }
    A.pieces.push_back(&pc);
    A.seq_used += n;
    A.res_used += nres;
    A.copying++;
    lk.unlock();
    /* the piece into place (each request copies its own, at once) */
    std::memcpy(A.res + pc.res0, res + off[0], nres);
    for (uint32_t i = 0; i < n; i++)
        A.off[pc.seq0 + i] = pc.res0 + (off[i] - off[0]);
    lk.lock();
    A.copying--;
    cv_.notify_all();
    Area *mine = &A;
    while (!pc.done) {
        /* no pass running and our area complete: lead it, the other area
         * (empty: its pass is over) opening for the next pieces */
        if (!busy_ && mine == area_[open_].get() && mine->copying == 0) {
            busy_ = true;
            open_ ^= 1;
            lk.unlock();
            lead(kg, *mine);
            lk.lock();
            for (Piece *q : mine->pieces)
                q->done = true;
            mine->pieces.clear();
            mine->seq_used = 0;
            mine->res_used = 0;
            busy_ = false;
            cv_.notify_all();
        } else {
            cv_.wait(lk);
        }
    }
    active_--;
    if (pc.rc)
        throw Error(pc.rc, "lookup batcher: " + pc.err);
}

void LookupBatcher::lead(KmerGuts &kg, Area &a)
{
    const uint32_t N = a.seq_used;
    a.off[N] = a.res_used;
    kgx_result r;
    kgx_rollup_result ru;
    const int rc = kgx_lookup(kg.ctx(), a.map, a.mode, &a.p, a.res, a.off, N, a.want, &r, &ru);
    passes_++;
    batched_ += a.pieces.size();
    stage_stats().batched_passes++;
    stage_stats().batched_pieces += a.pieces.size();
    const std::string err = rc ? kgx_last_error() : "";
    for (Piece *q : a.pieces) {
        q->rc = rc;
        if (rc) {
            q->err = err;
            continue;
        }
        Out &o = *q->out;
        if (a.want & KGX_WANT_BEST)
            o.best.assign(r.best + q->seq0, r.best + q->seq0 + q->n);
        const uint64_t r0 = ru.offsets[q->seq0], r1 = ru.offsets[q->seq0 + q->n];
        o.roff.resize((size_t)q->n + 1);
        for (uint32_t i = 0; i <= q->n; i++)
            o.roff[i] = ru.offsets[q->seq0 + i] - r0;
        o.rows.assign(ru.rows + r0, ru.rows + r1);
    }
}

/* ---- LookupRequest ------------------------------------------------------- */

static bool stoi_param(const std::map<std::string, std::string> &p, const char *k, int &out)
{
    /* std::stoi with only std::invalid_argument caught (lookup_request.cc:47-58) */
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

namespace {

/* Helper threads for a request's text stage: run(parts, fn) calls fn(0 ..
 * parts-1) once each, on the caller and on whichever helpers are idle (with
 * none idle the caller runs every part itself).  KGX_TEXT_HELPERS threads
 * (default 0: none; r8 at 16 clients on the box's 16-CPU share: 8.59e9
 * residues/s with none, 7.76e9 with 4, 7.34e9 with 8 -- the parts cost more
 * CPU than the share has spare), started on first use and never joined (a
 * process may exit with them waiting). */
class TextHelpers {
public:
    static TextHelpers &get()
    {
        static TextHelpers *h = new TextHelpers();
        return *h;
    }
    uint32_t size() const { return n_; }
    void run(uint32_t parts, const std::function<void(uint32_t)> &fn)
    {
        Job job{&fn, parts};
        const bool shared = n_ && parts > 1;
        if (shared) {
            std::lock_guard<std::mutex> g(mu_);
            jobs_.push_back(&job);
        }
        if (shared)
            cv_.notify_all();
        for (;;) {
            uint32_t p;
            {
                std::lock_guard<std::mutex> g(mu_);
                p = job.next < parts ? job.next++ : parts;
                if (job.next == parts && shared)
                    drop(&job);
            }
            if (p == parts)
                break;
            fn(p);
            std::lock_guard<std::mutex> g(mu_);
            job.done++;
        }
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return job.done == parts; });
    }

private:
    struct Job {
        const std::function<void(uint32_t)> *fn;
        uint32_t parts;
        uint32_t next = 0, done = 0;
    };
    TextHelpers()
    {
        const char *e = std::getenv("KGX_TEXT_HELPERS");
        n_ = (uint32_t)std::max(0, std::min(64, e ? std::atoi(e) : 0));
        for (uint32_t i = 0; i < n_; i++)
            std::thread([this] { loop(); }).detach();
    }
    void drop(Job *j)
    {
        auto it = std::find(jobs_.begin(), jobs_.end(), j);
        if (it != jobs_.end())
            jobs_.erase(it);
    }
    void loop()
    {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return !jobs_.empty(); });
            Job *j = jobs_.front(); /* a queued job has parts left */
            const uint32_t p = j->next++;
            if (j->next == j->parts)
                jobs_.pop_front();
            lk.unlock();
            (*j->fn)(p);
            lk.lock();
            if (++j->done == j->parts)
                done_cv_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::deque<Job *> jobs_;
    uint32_t n_ = 0;
};

}  // namespace

LookupRequest::LookupRequest(std::shared_ptr<KmerPegMapping> mapping, bool family_mode,
                             const std::map<std::string, std::string> &params)
    : mapping_(mapping), family_mode_(family_mode)
{
    int v;
    if (stoi_param(params, "kmer_hit_threhsold", v))
        kmer_hit_threshold_ = (unsigned int)v;
    if (stoi_param(params, "find_best_match", v))
        find_best_match_ = v != 0;
    if (stoi_param(params, "find_reps", v))
        find_reps_ = v != 0;
    if (stoi_param(params, "allow_ambiguous_functions", v))
        allow_ambiguous_functions_ = v != 0;
    auto tg_it = params.find("target_genus");
    const std::string tg = mapping_->lookup_genus(tg_it == params.end() ? std::string() : tg_it->second);
    try {
        if (!tg.empty())
            target_genus_id_ = std::stoul(tg);
    } catch (const std::invalid_argument &) {
    }
}

void LookupRequest::process_work(KmerGuts &kg, const std::vector<std::pair<std::string, std::string>> &work,
                                 std::ostream &os)
{
    std::string ids, res;
    std::vector<uint64_t> id_off{0}, off{0};
    for (const auto &w : work) {
        ids += w.first;
        id_off.push_back(ids.size());
        res += w.second;
        off.push_back(res.size());
    }
    process_flat(kg, res.data(), off.data(), ids.data(), id_off.data(), work.size(), os);
}

void LookupRequest::process_flat(KmerGuts &kg, const char *res, const uint64_t *off, const char *ids,
                                 const uint64_t *id_off, size_t n_work, std::ostream &os)
{
    /* pieces that keep the batch's hits on the device (one small-batch pass
     * each: at most 2M residues, 65,536 sequences) */
    const FlatWork fw{res, off, ids, id_off};
    size_t a = 0;
    while (a < n_work) {
        size_t b = a + 1;
        while (b < n_work && off[b + 1] - off[a] <= (uint64_t(1) << 21) && b - a < 65536)
            b++;
        process_piece(kg, fw, a, b, os);
        a = b;
    }
}

void LookupRequest::best_match_lines(KmerGuts &kg, const FlatWork &fw, size_t w0, uint32_t a, uint32_t b,
                                     const kgx_best_call *best, const uint64_t *roff, const kgx_rollup_row *rows,
                                     ScoreMap &smap, std::string &out) const
{
    typedef FamilyMapper::sequence_accumulated_score_t acc_t;
    /* the per-sequence strings live across the part's sequences: their
     * buffers are reused, not allocated per line */
    std::string id, fn, ambig, lf_fam, lf_fn, gf_fam;
    static const bool clocks = std::getenv("KGX_TEXT_CLOCKS") != nullptr;
    uint64_t cyc[5] = {0, 0, 0, 0, 0}, t_last = clocks ? __rdtsc() : 0;
    auto tick = [&](int k) {
        if (clocks) {
            const uint64_t t = __rdtsc();
            cyc[k] += t - t_last;
            t_last = t;
        }
    };
    /* a block's family lookups and name fetches first: independent of each
     * other, so their cache misses overlap instead of stalling one by one */
    constexpr uint32_t BLK = 16;
    std::vector<const KmerPegMapping::family_data_t *> fdv;
    uint64_t fd0 = 0;
    for (uint32_t s = a; s < b; s++) {
        if ((s - a) % BLK == 0) {
            const uint32_t e = std::min(b, s + BLK);
            fd0 = roff[s];
            fdv.resize(roff[e] - fd0);
            for (uint64_t j = fd0; j < roff[e]; j++) {
                auto it = mapping_->family_data_.find(rows[j].id);
                fdv[j - fd0] = it == mapping_->family_data_.end() ? nullptr : &it->second;
            }
            for (uint32_t q = s; q < e; q++)
                kg.prefetch_call_names(best[q]);
        }
        const size_t ia = fw.id_off[w0 + s], ib = fw.id_off[w0 + s + 1];
        id.assign(fw.ids + ia, ib - ia);
        /* smap as the reference's operator[] calls leave it: the ids in
         * first-touch order into the request's one map (cleared per sequence,
         * its bucket count kept), so its iteration order is the reference's */
        if (!smap.empty())
            smap.clear();
        for (uint64_t j = roff[s]; j < roff[s + 1]; j++) {
            const kgx_rollup_row &row = rows[j];
            acc_t &e = smap[row.id];
            e.hit_count = row.hit_count;
            e.hit_total = row.hit_total;
            e.weighted_total = row.weighted_total;
        }
        tick(0);
        {
            int fi;
            float score, wscore, offs = 0.0f;
            ambig.clear();
            kg.find_best_call(best[s], fi, fn, score, wscore, offs);
            bool do_ambig = false;
            if (fn.empty()) {
                fn.assign("hypothetical protein");
            } else {
                const size_t where = fn.find(" ?? ");
                if (where != std::string::npos) {
                    if (allow_ambiguous_functions_) {
                        ambig = fn.substr(where + 4);
                        fn = fn.substr(0, where);
                        do_ambig = true;
                    } else {
                        fn = "hypothetical protein";
                    }
                }
            }
            tick(1);
            float lf_score = 0.0f, gf_score = 0.0f;
            lf_fam.clear();
            lf_fn.clear();
            gf_fam.clear();
            /* fresh maps per sequence, as the reference declares them
             * (lookup_request.cc:259): their iteration order -- the tie
             * order of the family pick below -- depends on it (an empty
             * map allocates nothing) */
            std::unordered_map<std::string, float> pgf_rollup, pgf_rollup_ambig;
            for (const auto &hit_ent : smap) {
                const acc_t &se = hit_ent.second;
                if (se.hit_total < kmer_hit_threshold_)
                    continue;
                /* the entry's family, looked up with the block (a search of
                 * the sequence's rows; past 32 rows the map again) */
                const KmerPegMapping::family_data_t *fdp = nullptr;
                if (roff[s + 1] - roff[s] <= 32) {
                    for (uint64_t j = roff[s]; j < roff[s + 1]; j++)
                        if (rows[j].id == hit_ent.first) {
                            fdp = fdv[j - fd0];
                            break;
                        }
                } else {
                    auto fent = mapping_->family_data_.find(hit_ent.first);
                    fdp = fent == mapping_->family_data_.end() ? nullptr : &fent->second;
                }
                if (!fdp)
                    continue;
                const KmerPegMapping::family_data_t &fd = *fdp;
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
                if (se.weighted_total > lf_score && fd.genus_id == target_genus_id_) {
                    lf_score = se.weighted_total;
                    lf_fam = fd.plf;
                    lf_fn = fd.function;
                }
            }
            tick(2);
            auto *rollup = (do_ambig && lf_fn == ambig) ? &pgf_rollup_ambig : &pgf_rollup;
            for (const auto &pgf_ent : *rollup)
                if (pgf_ent.second > gf_score) {
                    gf_score = pgf_ent.second;
                    gf_fam = pgf_ent.first;
                }
            tick(3);
            /* the iostream line (lookup_request.cc), floats as operator<< prints them (%.6g) */
            out += id;
            out += '\t';
            out += gf_fam;
            out += '\t';
            append_f32(out, gf_score);
            out += '\t';
            out += lf_fam;
            out += '\t';
            append_f32(out, lf_score);
            out += '\t';
            out += do_ambig ? lf_fn : fn;
            out += '\t';
            append_f32(out, score);
            out += '\t';
            append_f32(out, wscore);
            out += '\n';
        }
        tick(4);
    }
    if (clocks)
        for (int k = 0; k < 5; k++)
            stage_stats().text_cycles[k] += cyc[k];
}

void LookupRequest::process_piece(KmerGuts &kg, const FlatWork &fw, size_t w0, size_t w1, std::ostream &os)
{
    const uint32_t n = (uint32_t)(w1 - w0);
    if (n == 0)
        return;
    const bool want_calls = find_best_match_ && family_mode_;
    kgx_params p{kg.min_hits, kg.max_gap, kg.order_constraint, kg.min_weighted_hits};
    kgx_result r;
    /* find_best_call runs on the device (KGX_WANT_BEST): only its decision
     * per sequence comes back, not the calls; the hits stay on the device,
     * where on_hit's rollups run (kgx_kmap_rollup) */
    const uint64_t g0 = now_ns(); /* gpu stage: the pass and the rollups */
    /* on_hit (lookup_request.cc:446-482) over kmer_to_family_id_ or kmer_to_id_ */
    kgx_kmap *map = family_mode_ ? mapping_->kmer_to_family_id() : mapping_->kmer_to_id();
    const int mode = family_mode_ ? KGX_ROLLUP_FAMILY : KGX_ROLLUP_PEG;
    const uint32_t want = want_calls ? KGX_WANT_BEST : 0u;
    kgx_rollup_result ru;
    /* the pass and the rollup enqueued together with one host wait
     * (kgx_lookup: the small-batch path with the rollup queued behind it)
     * when the map is on the worker's device; KGX_LOOKUP_ONE_WAIT=0: the
     * pass, then the rollup, a wait each (HTTP family /lookup at 16 clients
     * 9.05e9 vs 8.35e9 residues/s, r8 s20) */
    static const bool one_wait = [] {
        const char *e = std::getenv("KGX_LOOKUP_ONE_WAIT");
        return !e || std::atoi(e) != 0;
    }();
    int rc;
    const kgx_best_call *best = nullptr;
    const uint64_t *roff = nullptr;
    const kgx_rollup_row *rows = nullptr;
    LookupBatcher::Out out;
    if (batcher_) { /* a pass shared with concurrent requests' pieces */
        batcher_->run(kg, map, mode, p, want, fw.res, fw.off + w0, n, out);
        stage_stats().gpu_passes++;
        best = out.best.data();
        roff = out.roff.data();
        rows = out.rows.data();
    } else if (one_wait && kgx_kmap_device(map) == kgx_image_device(kg.image_->handle())) {
        rc = kgx_lookup(kg.ctx(), map, mode, &p, fw.res, fw.off + w0, n, want, &r, &ru);
        stage_stats().gpu_passes++;
        if (rc)
            throw_last(rc, "kgx_lookup");
        best = r.best;
        roff = ru.offsets;
        rows = ru.rows;
    } else {
        rc = kgx_process_batch(kg.ctx(), &p, fw.res, fw.off + w0, n, want, &r);
        stage_stats().gpu_passes++;
        if (rc)
            throw_last(rc, "kgx_process_batch");
        rc = kgx_kmap_rollup(map, kg.ctx(), mode, &ru);
        if (rc)
            throw_last(rc, "kgx_kmap_rollup");
        best = r.best;
        roff = ru.offsets;
        rows = ru.rows;
    }
    stage_stats().gpu_ns += now_ns() - g0;
    StageClock text_clock(stage_stats().text_ns); /* the scoring and the output lines, to the end */
    typedef FamilyMapper::sequence_accumulated_score_t acc_t;
    if (want_calls) {
        /* the lines in parts on the text helpers (KGX_TEXT_HELPERS): part k
         * starts from a map grown as the request's seq_score_ would be at
         * its first sequence, so every map iterates as the reference's one
         * does; the parts' text is written in order */
        TextHelpers &th = TextHelpers::get();
        const uint32_t P = std::max<uint32_t>(1u, std::min<uint32_t>(th.size() + 1, n / 768));
        std::vector<uint32_t> cut(P + 1);
        for (uint32_t k = 0; k <= P; k++)
            cut[k] = (uint32_t)((uint64_t)n * k / P);
        std::vector<size_t> most(P);
        size_t m = seq_score_most_;
        for (uint32_t k = 0, q = 0; k < P; k++) {
            most[k] = m;
            for (; q < cut[k + 1]; q++)
                m = std::max<size_t>(m, (size_t)(roff[q + 1] - roff[q]));
        }
        std::vector<std::string> outs(P);
        th.run(P, [&](uint32_t k) {
            if (k == 0) {
                best_match_lines(kg, fw, w0, cut[0], cut[1], best, roff, rows, seq_score_, outs[0]);
                return;
            }
            ScoreMap score;
            grow_to(score, most[k]);
            best_match_lines(kg, fw, w0, cut[k], cut[k + 1], best, roff, rows, score, outs[k]);
        });
        for (const std::string &o : outs)
            os.write(o.data(), (std::streamsize)o.size());
        if (P > 1) {
            seq_score_.clear();
            grow_to(seq_score_, m);
        }
        seq_score_most_ = m;
        return;
    }
    std::string id;
    for (uint32_t s = 0; s < n; s++) {
        const size_t ia = fw.id_off[w0 + s], ib = fw.id_off[w0 + s + 1];
        id.assign(fw.ids + ia, ib - ia);
        /* seq_score_ as the reference's operator[] calls leave it: the ids in
         * first-touch order into the request's one map (cleared per sequence,
         * its bucket count kept), so its iteration order is the reference's */
        if (!seq_score_.empty())
            seq_score_.clear();
        for (uint64_t j = roff[s]; j < roff[s + 1]; j++) {
            const kgx_rollup_row &row = rows[j];
            acc_t &e = seq_score_[row.id];
            e.hit_count = row.hit_count;
            e.hit_total = row.hit_total;
            e.weighted_total = row.weighted_total;
        }
        {
            typedef std::pair<KmerPegMapping::encoded_id_t, acc_t> data_t;
            std::vector<data_t> vec(seq_score_.begin(), seq_score_.end());
            std::sort(vec.begin(), vec.end(), [](const data_t &l, const data_t &rr) {
                return l.second.weighted_total > rr.second.weighted_total;
            });
            os << id << "\n";
            for (auto &it : vec) {
                const acc_t &se = it.second;
                if (se.hit_total < kmer_hit_threshold_)
                    break;
                if (family_mode_) {
                    const KmerPegMapping::family_data_t fd = mapping_->family_at(it.first);
                    const float scaled = (float)se.hit_count / (float)fd.total_size;
                    os << se.hit_count << "\t" << se.hit_total << "\t" << se.weighted_total << "\t" << fd.pgf << "\t"
                       << fd.plf << "\t" << fd.total_size << "\t" << fd.count << "\t" << scaled << "\t"
                       << fd.function << "\n";
                    if (find_reps_)
                        os << "///\n"; /* no family reps DB loaded */
                } else {
                    os << mapping_->decode_id(it.first) << "\t" << se.hit_count;
                    auto fh = mapping_->peg_to_family_.find(it.first);
                    if (fh != mapping_->peg_to_family_.end()) {
                        const KmerPegMapping::family_data_t fd = mapping_->family_at(fh->second);
                        os << "\t" << fd.pgf << "\t" << fd.plf << "\t" << fd.function << "\n";
                    } else {
                        os << "\n";
                    }
                }
            }
            os << "//\n";
        }
    }
}

FqRequest::FqRequest(KmerGuts &kg, std::shared_ptr<KmerPegMapping> mapping) : kg_(kg), mapping_(mapping) {}

void FqRequest::process(const std::string &block, bool finished, std::ostream &os)
{
    process(block.data(), block.size(), finished, os);
}

namespace {

enum { FQ_START, FQ_ID, FQ_DEF, FQ_DATA, FQ_PLUS_START, FQ_PLUS, FQ_QUAL };

/* every byte a letter (isalpha in the C locale: A-Z, a-z): a branch-free
 * reduction the compiler vectorises */
inline bool all_letters(const char *s, size_t n)
{
    unsigned bad = 0;
    for (size_t i = 0; i < n; i++)
        bad |= (unsigned)((unsigned char)((unsigned char)s[i] | 0x20u) - (unsigned char)'a') >= 26u;
    return bad == 0;
}

inline bool is_letter(char c) { return (unsigned char)((unsigned char)c | 0x20u) - (unsigned char)'a' < 26u; }

/* FastqParser::parse_char (fastq_parser.h:40-150), line-at-a-time, over
 * [p, end): the id runs to the first blank, sequence lines keep isalpha()
 * characters only (others are reported there and dropped), '+' and quality
 * lines are skipped; a record is emitted at the quality line's newline.  The
 * current record's residues are built in place at the end of `bases` (the
 * caller sizes it: at most one byte per byte parsed); `state` and `id` carry
 * the parser across calls. */
void fq_parse(const char *p, const char *end, int &state, std::string &id, char *bases, size_t &n_bases,
              std::vector<uint64_t> &roff, std::string &id_chars, std::vector<uint64_t> &id_off)
{
    size_t nb = n_bases;
    while (p < end) {
        switch (state) {
        case FQ_START:
            if (*p++ == '@')
                state = FQ_ID;
            break;
        case FQ_ID: {
            const char *q = p;
            while (q < end && *q != ' ' && *q != '\t' && *q != '\n')
                q++;
            id.append(p, (size_t)(q - p));
            if (q < end)
                state = *q == '\n' ? FQ_DATA : FQ_DEF;
            p = q < end ? q + 1 : end;
            break;
        }
        case FQ_DEF:
        case FQ_PLUS:
        case FQ_QUAL: {
            const char *nl = static_cast<const char *>(std::memchr(p, '\n', (size_t)(end - p)));
            if (!nl) {
                p = end;
                break;
            }
            p = nl + 1;
            if (state == FQ_QUAL) { /* emit */
                id_chars += id;
                id_off.push_back(id_chars.size());
                roff.push_back(nb);
                id.clear();
                state = FQ_START;
            } else {
                state = state == FQ_DEF ? FQ_DATA : FQ_QUAL;
            }
            break;
        }
        case FQ_DATA: {
            const char *nl = static_cast<const char *>(std::memchr(p, '\n', (size_t)(end - p)));
            const char *stop = nl ? nl : end;
            const size_t L = (size_t)(stop - p);
            if (all_letters(p, L)) { /* the usual line: copied whole */
                std::memcpy(bases + nb, p, L);
                nb += L;
            } else {
                for (const char *q = p; q < stop; q++)
                    if (is_letter(*q))
                        bases[nb++] = *q;
            }
            p = stop;
            if (nl) {
                p = nl + 1;
                state = FQ_PLUS_START;
            }
            break;
        }
        case FQ_PLUS_START:
            if (*p++ == '+')
                state = FQ_PLUS;
            break;
        }
    }
    n_bases = nb;
}

/* a place to cut a FASTQ block for a parallel parse: a line that starts
 * with '@' and whose next-but-one line starts with '+' (a record start in
 * any well-formed file), searched from p for up to 1 MiB; null if none */
const char *fq_cut_after(const char *p, const char *end)
{
    const char *limit = std::min(end, p + (1 << 20));
    while (p < limit) {
        const char *nl = static_cast<const char *>(std::memchr(p, '\n', (size_t)(limit - p)));
        if (!nl || nl + 1 >= end)
            return nullptr;
        const char *l0 = nl + 1;
        if (*l0 == '@') {
            const char *n1 = static_cast<const char *>(std::memchr(l0, '\n', (size_t)(end - l0)));
            const char *n2 = n1 ? static_cast<const char *>(std::memchr(n1 + 1, '\n', (size_t)(end - n1 - 1))) : nullptr;
            if (!n2)
                return nullptr;
            if (n2 + 1 < end && n2[1] == '+')
                return l0;
        }
        p = l0;
    }
    return nullptr;
}

}  // namespace

FqRequest::FqPart::~FqPart()
{
    if (bases)
        kgx_host_free(bases);
}

void FqRequest::FqPart::begin(size_t need, int st, const std::string &carried_id, const std::string &carried_bases)
{
    if (need > cap) {
        if (bases)
            kgx_host_free(bases);
        bases = nullptr;
        cap = 0;
        void *q = nullptr;
        const size_t want = need + need / 8 + 4096;
        int rc = kgx_host_alloc(want, &q);
        if (rc)
            throw_last(rc, "kgx_host_alloc");
        bases = static_cast<char *>(q);
        cap = want;
    }
    state = st;
    id = carried_id;
    std::memcpy(bases, carried_bases.data(), carried_bases.size());
    len = carried_bases.size();
    roff.assign(1, 0);
    id_off.assign(1, 0);
    id_chars.clear();
}

void FqRequest::FqPart::parse(const char *a, const char *b)
{
    fq_parse(a, b, state, id, bases, len, roff, id_chars, id_off);
}

FqRequest::FqBlock FqRequest::FqPart::view() const
{
    FqBlock v;
    v.res = bases;
    v.roff = roff.data();
    v.ids = id_chars.data();
    v.id_off = id_off.data();
    v.n = id_off.size() - 1;
    return v;
}

/* The block is cut into parts of about kPartBytes at record starts
 * (fq_cut_after).  Worker threads parse the parts ahead, in order, into
 * pinned buffers (a ring of a few per worker); this thread takes them in
 * order and runs each through the GPU (its bases go to the device by DMA from
 * the part's buffer) and the frame choice, so parsing overlaps the device
 * work.  Part 0 continues the carried parser state; the others start
 * speculatively in the start state, and a part is used only if the exact
 * sequential parse reaches its first byte in that state with nothing pending
 * (the previous record emitted).  Otherwise the rest of the block is parsed
 * again here from the true state.  So the reads, and the output, are the
 * sequential parse's.  One FamilyMapper serves the whole block, as the
 * reference keeps one per block (fq_process_request.cc:241). */
void FqRequest::process(const char *text, size_t n, bool finished, std::ostream &os)
{
    /* KGX_FQ_PART_KB: the part size, for tests of the parallel parse */
    const size_t kPartBytes = [] {
        const char *e = std::getenv("KGX_FQ_PART_KB");
        return e ? std::max<size_t>(4, std::strtoull(e, nullptr, 10)) << 10 : size_t(32) << 20;
    }();
    const bool timing = std::getenv("KGX_FQ_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    const char *end = text + n;
    std::vector<const char *> cuts{text};
    const size_t want_parts = n / kPartBytes;
    /* the first part is an eighth of the others: nothing overlaps its parse
     * (r5k: 4.4-5.9 ms of a 66-ms block waiting for a 32-MB first part) */
    if (want_parts > 1)
        if (const char *c = fq_cut_after(text + kPartBytes / 8, end))
            cuts.push_back(c);
    for (size_t i = 1; i < want_parts; i++) {
        const char *c = fq_cut_after(text + n * i / want_parts, end);
        if (c && c > cuts.back())
            cuts.push_back(c);
    }
    cuts.push_back(end);
    const size_t K = cuts.size() - 1;
    FamilyMapper mapper(kg_, mapping_);
    double parse_wait_ms = 0.0, device_ms = 0.0;
    /* the final part: the block's end state goes back to the request */
    auto finish_part = [&](FqPart &pt) {
        if (finished) { /* parse_complete() emits the last record */
            pt.id_chars += pt.id;
            pt.id_off.push_back(pt.id_chars.size());
            pt.roff.push_back(pt.len);
            pt.id.clear();
            state_ = FQ_START;
            id_.clear();
            seq_.clear();
        } else { /* the cut record's residues wait for the next block */
            state_ = pt.state;
            id_ = pt.id;
            seq_.assign(pt.bases + pt.roff.back(), pt.len - pt.roff.back());
        }
    };
    auto run_part = [&](const FqPart &pt) {
        const auto d0 = std::chrono::steady_clock::now();
        process_block(pt.view(), mapper, os);
        device_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - d0).count();
    };
    if (K == 1) {
        if (parts_.empty())
            parts_.emplace_back(new FqPart);
        FqPart &pt = *parts_[0];
        pt.begin(seq_.size() + n, state_, id_, seq_);
        pt.parse(text, end);
        finish_part(pt);
        run_part(pt);
    } else {
        const size_t W = std::min<size_t>(K, std::max<size_t>(1, std::min<size_t>(15, std::thread::hardware_concurrency() - 1)));
        const size_t R = std::min(K, 2 * W + 2); /* parts in flight */
        while (parts_.size() < R)
            parts_.emplace_back(new FqPart);
        std::mutex mu;
        std::condition_variable cv;
        size_t next = 0, consumed = 0;
        bool abort = false;
        std::vector<size_t> ready(R, SIZE_MAX); /* ring slot -> the part it holds, parsed */
        std::string err;
        const int carried_state = state_;
        const std::string carried_id = id_, carried_seq = seq_;
        auto worker = [&]() {
            for (;;) {
                size_t k;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    if (abort || next >= K)
                        return;
                    k = next++;
                    cv.wait(lk, [&] { return abort || k < consumed + R; });
                    if (abort)
                        return;
                }
                FqPart &pt = *parts_[k % R];
                try {
                    const size_t span = (size_t)(cuts[k + 1] - cuts[k]);
                    if (k == 0)
                        pt.begin(carried_seq.size() + span, carried_state, carried_id, carried_seq);
                    else
                        pt.begin(span, FQ_START, std::string(), std::string());
                    pt.parse(cuts[k], cuts[k + 1]);
                } catch (const std::exception &e) {
                    std::lock_guard<std::mutex> lk(mu);
                    err = e.what();
                    abort = true;
                    cv.notify_all();
                    return;
                }
                std::lock_guard<std::mutex> lk(mu);
                ready[k % R] = k;
                cv.notify_all();
            }
        };
        std::vector<std::thread> pool;
        for (size_t w = 0; w < W; w++)
            pool.emplace_back(worker);
        auto stop_workers = [&]() {
            {
                std::lock_guard<std::mutex> lk(mu);
                abort = true;
            }
            cv.notify_all();
            for (auto &th : pool)
                th.join();
            pool.clear();
        };
        /* parts rotate over three contexts, two parts ahead of the one being
         * collected: part k + 2's bases go up by DMA while part k + 1 is sized
         * and its lookup enqueued and part k is collected, so the next probe
         * never waits for an upload (with two contexts and the upload inside
         * the launch, each part's 16-MB H2D ran with the GPU idle: 1.06 ms
         * per part against a 0.46-ms probe, r5j) */
        kgx_ctx *ctxs[3] = {kg_.ctx(), twin_ctx(), twin2_ctx()};
        auto wait_part = [&](size_t k) -> FqPart & {
            const auto w0 = std::chrono::steady_clock::now();
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return ready[k % R] == k || !err.empty(); });
            if (!err.empty())
                throw std::runtime_error(err);
            parse_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
            return *parts_[k % R];
        };
        auto release = [&](size_t k) {
            std::lock_guard<std::mutex> lk(mu);
            ready[k % R] = SIZE_MAX;
            consumed = k + 1;
            cv.notify_all();
        };
        struct Slot {
            FqPart *pt = nullptr;
            bool tail = false; /* the exact re-parse of the rest of the block: the last part */
            FqLaunched l;
        };
        /* part j, given part j - 1 (prev): the speculative part when the
         * exact parse of prev ends at a record start with nothing pending,
         * else the rest of the block parsed again from prev's end state */
        auto next_part = [&](const FqPart &prev, size_t j) -> Slot {
            Slot sl;
            const bool holds = prev.state == FQ_START && prev.id.empty() && prev.len == prev.roff.back();
            if (holds) {
                sl.pt = &wait_part(j);
                if (j + 1 == K)
                    finish_part(*sl.pt);
                return sl;
            }
            stop_workers();
            if (!tail_)
                tail_.reset(new FqPart);
            tail_->begin((size_t)(end - cuts[j]) + (prev.len - prev.roff.back()), prev.state, prev.id,
                         std::string(prev.bases + prev.roff.back(), prev.len - prev.roff.back()));
            tail_->parse(cuts[j], end);
            finish_part(*tail_);
            sl.pt = tail_.get();
            sl.tail = true;
            return sl;
        };
        auto upload = [&](Slot &sl, kgx_ctx *ctx) {
            const FqBlock v = sl.pt->view();
            sl.l = FqLaunched{};
            sl.l.ctx = ctx;
            sl.l.n_reads = (uint32_t)v.n_reads();
            if (sl.l.n_reads) {
                if (int rc = kgx_fq_upload(ctx, v.residues(), v.roff, sl.l.n_reads))
                    throw_last(rc, "kgx_fq_upload");
                start_fragments(ctx);
            }
        };
        auto launch = [&](Slot &sl) {
            const auto l0 = std::chrono::steady_clock::now();
            launch_uploaded(sl.l);
            device_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - l0).count();
        };
        try {
            Slot sl[3];
            size_t have = 1; /* parts 0 .. have-1 are prepared (uploaded) */
            bool last_known = false; /* the last prepared part is the block's last */
            sl[0].pt = &wait_part(0);
            upload(sl[0], ctxs[0]);
            launch(sl[0]);
            if (K > 1) {
                sl[1] = next_part(*sl[0].pt, 1);
                upload(sl[1], ctxs[1]);
                have = 2;
                last_known = sl[1].tail || K == 2;
            } else {
                last_known = true;
            }
            for (size_t k = 0; k < have; k++) {
                Slot &cur = sl[k % 3];
                if (k + 1 < have) {
                    Slot &nxt = sl[(k + 1) % 3];
                    if (!last_known && k + 2 < K) { /* part k + 2 up while k + 1 launches and k finishes */
                        sl[(k + 2) % 3] = next_part(*nxt.pt, k + 2);
                        upload(sl[(k + 2) % 3], ctxs[(k + 2) % 3]);
                        have = k + 3;
                        last_known = sl[(k + 2) % 3].tail || k + 3 == K;
                    }
                    launch(nxt);
                }
                const auto f0 = std::chrono::steady_clock::now();
                finish_block(cur.pt->view(), cur.l, mapper, os);
                device_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - f0).count();
                if (!cur.tail)
                    release(k);
            }
        } catch (...) {
            stop_workers();
            throw;
        }
        stop_workers();
    }
    if (timing)
        std::fprintf(stderr, "[fq] block %.1f MB in %zu part(s): %.3f ms, waiting for the parse %.3f ms, device + "
                             "frame choice %.3f ms\n",
                     n / 1e6, K,
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                     parse_wait_ms, device_ms);
}

void FqRequest::process_reads(const std::vector<std::pair<std::string, std::string>> &reads, std::ostream &os)
{
    size_t nb = 0;
    for (auto &r : reads)
        nb += r.second.size();
    FqPart pt;
    pt.begin(nb, FQ_START, std::string(), std::string());
    for (auto &r : reads) {
        pt.id_chars += r.first;
        pt.id_off.push_back(pt.id_chars.size());
        std::memcpy(pt.bases + pt.len, r.second.data(), r.second.size());
        pt.len += r.second.size();
        pt.roff.push_back(pt.len);
    }
    FamilyMapper mapper(kg_, mapping_);
    process_block(pt.view(), mapper, os);
}

void FqRequest::process_block(const FqBlock &blk, FamilyMapper &mapper, std::ostream &os)
{
    FqLaunched l = launch_block(blk, kg_.ctx());
    finish_block(blk, l, mapper, os);
}

kgx_ctx *FqRequest::twin2_ctx()
{
    if (!twin2_) {
        int rc = kgx_ctx_create(kg_.image_->handle(), &twin2_);
        if (rc)
            throw_last(rc, "kgx_ctx_create");
    }
    return twin2_;
}

kgx_ctx *FqRequest::twin_ctx()
{
    if (!twin_) {
        int rc = kgx_ctx_create(kg_.image_->handle(), &twin_);
        if (rc)
            throw_last(rc, "kgx_ctx_create");
    }
    return twin_;
}

FqRequest::~FqRequest()
{
    if (twin_)
        kgx_ctx_destroy(twin_);
    if (twin2_)
        kgx_ctx_destroy(twin2_);
}

/* the block's reads -> fragments -> lookup, one GPU batch on ctx: returns
 * once the fragment pass has sized the batch and the lookup is enqueued */
FqRequest::FqLaunched FqRequest::launch_block(const FqBlock &blk, kgx_ctx *ctx)
{
    FqLaunched l;
    l.ctx = ctx;
    l.n_reads = (uint32_t)blk.n_reads();
    if (l.n_reads == 0)
        return l;
    if (int rc = kgx_fq_upload(ctx, blk.residues(), blk.roff, l.n_reads))
        throw_last(rc, "kgx_fq_upload");
    start_fragments(ctx);
    launch_uploaded(l);
    return l;
}

/* the fragment pass over the reads just uploaded to ctx, enqueued behind the
 * upload: a part's pass runs while the GPU still probes the part before it */
void FqRequest::start_fragments(kgx_ctx *ctx)
{
    /* fragments as anchors into the bases: the probe translates their windows
     * itself and no residue goes through HBM (the context keeps residues when
     * its probe cannot take anchors) */
    int rc = kgx_ctx_set_option(ctx, "fq_residues", 0);
    if (rc)
        throw_last(rc, "kgx_ctx_set_option");
    if ((rc = kgx_fq_fragments_uploaded_start(ctx)))
        throw_last(rc, "kgx_fq_fragments_uploaded_start");
}

void FqRequest::launch_uploaded(FqLaunched &l)
{
    if (l.n_reads == 0)
        return;
    kgx_ctx *ctx = l.ctx;
    int rc = kgx_fq_fragments_finish(ctx, &l.fr); /* the pass start_fragments enqueued */
    if (rc)
        throw_last(rc, "kgx_fq_fragments_finish");
    kgx_params p{kg_.min_hits, kg_.max_gap, kg_.order_constraint, kg_.min_weighted_hits};
    /* Calls are sparse over fragments (most fragments of a read are noise),
     * so the calls come back and find_best_call runs on the host for the
     * fragments that have any: a per-fragment device decision (KGX_WANT_BEST)
     * would copy 24 B for every fragment (measured: 8.3M -> 6.7M reads/s).
     * The hits stay on the device for the rollups. */
    rc = kgx_fq_run_device(ctx, &p, &l.fr, KGX_WANT_CALLS, nullptr);
    if (rc)
        throw_last(rc, "kgx_fq_run_device");
}

void FqRequest::finish_block(const FqBlock &blk, FqLaunched &l, FamilyMapper &mapper, std::ostream &os)
{
    const uint32_t n_reads = l.n_reads;
    if (n_reads == 0)
        return;
    /* KGX_FQ_TIMING=1: per-phase wall times on stderr */
    static const bool timing = std::getenv("KGX_FQ_TIMING") != nullptr && std::getenv("KGX_FQ_TIMING")[0] == '2';
    auto t_last = std::chrono::steady_clock::now();
    kgx_ctx *ctx = l.ctx;
    auto mark = [&](const char *what) {
        if (!timing)
            return;
        kgx_ctx_synchronize(ctx);
        auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[fq] %-12s %8.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(now - t_last).count());
        t_last = now;
    };
    kgx_fragments &fr = l.fr;
    const uint32_t want = KGX_WANT_CALLS;
    int rc;
    /* Without family lists a fragment's match depends on its calls alone,
     * and a read without calls scores 0 in every frame: no output and no
     * FamilyMapper state (seq_score_ stays empty).  Only then may reads
     * without calls be skipped and hits stay on the device; with families
     * loaded every fragment is replayed, since each one grows seq_score_ and
     * so shapes the iteration order later reads see. */
    const bool families = kgx_kmap_num_kmers(mapping_->kmer_to_family_id()) > 0;
    mark("lookup");
    if (!families) {
        /* only the reads with a call in some fragment come back (sparse):
         * the others produce no output and no mapper state */
        kgx_fq_called cr;
        if ((rc = kgx_fq_called_reads(ctx, &fr, &cr)))
            throw_last(rc, "kgx_fq_called_reads");
        mark("collect");
        std::vector<KmerCall> calls;
        std::vector<std::pair<size_t, FamilyMapper::best_match_t>> best_matches, matches;
        std::vector<uint32_t> match_len, best_len;
        for (uint32_t i = 0; i < cr.n; i++) {
            const uint32_t r = cr.reads[i];
            if (blk.id_len(r) == 0)
                continue;
            double best_score = 0.0;
            int best_frame = 0;
            best_matches.clear();
            best_len.clear();
            uint64_t g = cr.frag_offsets[i];
            for (int fs = 0; fs < 6; fs++) {
                const int frame = fs < 3 ? fs + 1 : -(fs - 2);
                const uint64_t g_end = g + cr.frame_counts[(size_t)i * 6 + fs];
                double score = 0.0;
                matches.clear();
                match_len.clear();
                for (; g < g_end; g++) {
                    calls.clear();
                    for (uint64_t c = cr.call_offsets[g]; c < cr.call_offsets[g + 1]; c++)
                        calls.emplace_back(cr.calls[c].start, cr.calls[c].end, cr.calls[c].count,
                                           cr.calls[c].function_index, cr.calls[c].weighted_hits);
                    matches.emplace_back(0, mapper.find_best_family_match(nullptr, 0, calls));
                    match_len.push_back(cr.frag_len[g]);
                    score += matches.back().second.score;
                    if (score > best_score) {
                        best_score = score;
                        best_frame = frame;
                        best_matches = matches;
                        best_len = match_len;
                    }
                }
            }
            if (best_score > 0.0) {
                os.write(blk.id(r), (std::streamsize)blk.id_len(r));
                os << "\t" << best_frame << "\t" << best_score << "\t";
                for (size_t k = 0; k < best_matches.size(); k++) {
                    if (k)
                        os << "\t";
                    os << (size_t)best_len[k] << "\t" << best_matches[k].second;
                }
                os << std::endl;
            }
        }
        mark("host loop");
        return;
    }
    /* fragments per (read, frame): fragment g of read r, frame slot k */
    std::vector<uint32_t> fcount((size_t)n_reads * 6);
    if ((rc = kgx_ctx_synchronize(ctx)) || (rc = kgx_memcpy_d2h(fcount.data(), fr.frame_counts, fcount.size() * 4)))
        throw_last(rc, "fragment counts");
    kgx_result res;
    rc = kgx_device_batch_collect(ctx, want, &res);
    if (rc)
        throw_last(rc, "kgx_device_batch_collect");
    mark("collect");
    /* on_hit's rollups of every fragment (family_mapper.cc:287-312) on the device */
    kgx_rollup_result ru;
    if ((rc = kgx_kmap_rollup(mapping_->kmer_to_family_id(), ctx, KGX_ROLLUP_FAMILY, &ru)))
        throw_last(rc, "kgx_kmap_rollup");
    /* fragment lengths (printed for matches) are needed only for reads with
     * calls: fetch their offset slices, or all offsets when there are many */
    std::vector<uint64_t> rfirst(n_reads + 1, 0);
    for (uint32_t r = 0; r < n_reads; r++) {
        uint64_t k = 0;
        for (int f = 0; f < 6; f++)
            k += fcount[(size_t)r * 6 + f];
        rfirst[r + 1] = rfirst[r] + k;
    }
    std::vector<uint32_t> called;
    for (uint32_t r = 0; r < n_reads; r++)
        if (res.call_offsets[rfirst[r + 1]] != res.call_offsets[rfirst[r]])
            called.push_back(r);
    std::vector<uint64_t> frag_off;
    const bool all_offsets = called.size() > 1024;
    if (all_offsets) {
        frag_off.resize(fr.n_fragments + 1);
        if ((rc = kgx_memcpy_d2h(frag_off.data(), fr.offsets, frag_off.size() * 8)))
            throw_last(rc, "fragment offsets");
    }
    std::vector<uint64_t> slice;
    mark("family lists");
    /* on_parsed_seq (fq_process_request.cc:298-365), reads in order */
    std::vector<KmerCall> calls;
    std::vector<std::pair<size_t, FamilyMapper::best_match_t>> best_matches, matches;
    std::vector<uint64_t> match_frag, best_frag;
    size_t next_called = 0;
    for (uint32_t r = 0; r < n_reads; r++) {
        const bool has_calls = next_called < called.size() && called[next_called] == r;
        if (has_calls)
            next_called++;
        if (blk.id_len(r) == 0)
            continue;
        if (!families && !has_calls)
            continue; /* no calls in any frame: no output, no mapper state */
        double best_score = 0.0;
        int best_frame = 0;
        best_matches.clear();
        best_frag.clear();
        uint64_t g = rfirst[r];
        for (int fs = 0; fs < 6; fs++) {
            const int frame = fs < 3 ? fs + 1 : -(fs - 2);
            const uint64_t g_end = g + fcount[(size_t)r * 6 + fs];
            double score = 0.0;
            matches.clear();
            match_frag.clear();
            for (; g < g_end; g++) {
                calls.clear();
                for (uint64_t c = res.call_offsets[g]; c < res.call_offsets[g + 1]; c++)
                    calls.emplace_back(res.calls[c].start, res.calls[c].end, res.calls[c].count,
                                       res.calls[c].function_index, res.calls[c].weighted_hits);
                matches.emplace_back(0, mapper.find_best_family_match(ru.rows + ru.offsets[g], ru.offsets[g + 1] - ru.offsets[g], calls));
                match_frag.push_back(g);
                score += matches.back().second.score;
                if (score > best_score) {
                    best_score = score;
                    best_frame = frame;
                    best_matches = matches;
                    best_frag = match_frag;
                }
            }
        }
        if (best_score > 0.0) {
            /* the lengths of the printed fragments */
            const uint64_t f0 = rfirst[r], f1 = rfirst[r + 1];
            const uint64_t *offs = frag_off.data();
            if (!all_offsets) {
                slice.resize(f1 - f0 + 1);
                if ((rc = kgx_memcpy_d2h(slice.data(), fr.offsets + f0, slice.size() * 8)))
                    throw_last(rc, "fragment offsets");
                offs = slice.data() - f0;
            }
            os.write(blk.id(r), (std::streamsize)blk.id_len(r));
            os << "\t" << best_frame << "\t" << best_score << "\t";
            for (size_t i = 0; i < best_matches.size(); i++) {
                const uint64_t g2 = best_frag[i];
                if (i)
                    os << "\t";
                os << (size_t)(offs[g2 + 1] - offs[g2]) << "\t" << best_matches[i].second;
            }
            os << std::endl;
        }
    }
    mark("host loop");
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

/* ---- C ABI of the fq request handler (include/kgx.h kgx_fq_*) ------------- */

namespace kgx {
int fail(int code, const std::string &msg); /* kgx_runtime.cpp: sets kgx_last_error() */
}

struct kgx_fq {
    std::unique_ptr<kgx::KmerGuts> kg;
    std::shared_ptr<kgx::KmerPegMapping> mapping;
    std::unique_ptr<kgx::FqRequest> req;
    std::string text;
};

extern "C" {

int kgx_fq_create(kgx_image *img, const char *data_dir, const char *genus_file, const char *families_file,
                  const char *nr_fasta, kgx_fq **out)
{
    if (!img || !data_dir || !out)
        return kgx::fail(KGX_EINVAL, "null argument");
    kgx_fq *q = new kgx_fq;
    try {
        auto image = std::make_shared<kgx::KmerImage>(img, false);
        q->kg.reset(new kgx::KmerGuts(data_dir, image));
        q->mapping = std::make_shared<kgx::KmerPegMapping>(kgx_image_device(img));
        if (genus_file && *genus_file)
            q->mapping->load_genus_map(genus_file);
        if (families_file && *families_file)
            q->mapping->load_families(families_file);
        if (nr_fasta && *nr_fasta)
            q->mapping->load_nr_families(*q->kg, nr_fasta);
        q->req.reset(new kgx::FqRequest(*q->kg, q->mapping));
    } catch (const kgx::Error &e) {
        delete q;
        return kgx::fail(e.code(), e.what());
    } catch (const std::exception &e) {
        delete q;
        return kgx::fail(KGX_EINVAL, e.what());
    }
    *out = q;
    return KGX_OK;
}

int kgx_fq_destroy(kgx_fq *q)
{
    delete q;
    return KGX_OK;
}

int kgx_fq_process(kgx_fq *q, const char *fastq, uint64_t n, int finished, const char **text, uint64_t *text_len)
{
    if (!q || (n && !fastq) || !text || !text_len)
        return kgx::fail(KGX_EINVAL, "null argument");
    try {
        std::ostringstream os;
        q->req->process(fastq ? fastq : "", (size_t)n, finished != 0, os);
        q->text = os.str();
    } catch (const kgx::Error &e) {
        return kgx::fail(e.code(), e.what());
    } catch (const std::exception &e) {
        return kgx::fail(KGX_EINVAL, e.what());
    }
    *text = q->text.data();
    *text_len = q->text.size();
    return KGX_OK;
}

}  // extern "C"
