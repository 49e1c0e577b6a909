/*
 * kguts_hip.h -- C++ facade with the KmerGuts / KmerImage surface of the
 * reference (kguts.h:146-372, kmer_image.h:25-39, fasta_parser.h:8-165),
 * backed by the HIP engine behind include/kgx.h.
 *
 * Drop-in contract: the same class names, method names,
 * argument meaning and ownership as the reference; hit_cb runs synchronously,
 * in ascending position order, on the calling thread before process_aa_seq
 * returns; calls / otu_stats are appended to the caller's objects.  One
 * KmerGuts per host thread over one shared KmerImage (threadpool.cc:18-44).
 * Differences: failures throw kgx::Error instead of exit(); and
 * process_aa_batch() runs a whole work list (lookup_request.cc:153) in one GPU
 * pass -- per-sequence calls work but pay a launch round trip each.
 */
#ifndef KGUTS_HIP_H
#define KGUTS_HIP_H

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <unordered_map>
#include <ostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "kgx.h"

namespace kgx {

/*
 * Request-path stage clocks (kgx_server's GET /server_stats): nanoseconds
 * summed over every thread that spent them -- recv / send / handle by the
 * connection threads, parse by the router, gpu by the facade around each GPU
 * pass (host buffers in, results on the host: staging, H2D, kernels, D2H)
 * and the k-mer table lookups; handle - parse - gpu is the host rollups and
 * the text output.  A large /query's pieces run on several workers at once,
 * so their gpu time can add up to more than the request's handle time.
 */
struct StageStats {
    std::atomic<uint64_t> requests{0}, bytes_in{0}, bytes_out{0}, gpu_passes{0};
    std::atomic<uint64_t> recv_ns{0}, parse_ns{0}, gpu_ns{0}, text_ns{0}, handle_ns{0}, send_ns{0};
    /* /lookup pieces that shared a pass (LookupBatcher) and those passes */
    std::atomic<uint64_t> batched_pieces{0}, batched_passes{0};
    /* KGX_TEXT_CLOCKS=1: TSC cycles of the family /lookup text's steps (rows
     * into the map, best call, family loop, family pick, line) */
    std::atomic<uint64_t> text_cycles[5] = {};
    void reset();
    std::string json() const;
};
StageStats &stage_stats();
/* adds the scope's wall time to one clock */
class StageClock {
public:
    explicit StageClock(std::atomic<uint64_t> &acc);
    ~StageClock();
    StageClock(const StageClock &) = delete;
    StageClock &operator=(const StageClock &) = delete;

private:
    std::atomic<uint64_t> &acc_;
    uint64_t t0_;
};

class Error : public std::runtime_error {
public:
    Error(int code, const std::string &msg) : std::runtime_error(msg), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

typedef kgx_sig_kmer sig_kmer_t; /* kmer_image.h:17-23 */

/* KmerCall, kguts.h:166-183 */
class KmerCall {
public:
    unsigned int start;
    unsigned int end;
    int count;
    unsigned int function_index;
    float weighted_hits;

    KmerCall() : start(0), end(0), count(0), function_index(0), weighted_hits(0.0f) {}
    KmerCall(unsigned int s, unsigned int e, int c, unsigned int f, float w)
        : start(s), end(e), count(c), function_index(f), weighted_hits(w) {}
};

/* KmerOtuStats, kguts.h:185-219 */
class KmerOtuStats {
public:
    std::string contig_id;
    int contig_len = 0;
    std::map<int, int> otu_map;
    std::vector<std::pair<int, int>> otus_by_count;

    void write(FILE *fh) const;
    /* appends otu_map to otus_by_count, then sorts by count, descending */
    void finalize();
};

/*
 * Coalescing of concurrent per-sequence calls.  The reference's pool keeps one
 * KmerGuts per worker thread, each calling process_aa_seq once per sequence
 * (threadpool.cc:33-60, lookup_request.cc:153-172).  On a GPU one sequence is
 * far too little work for a pass, so calls that arrive on an image while
 * another pass is in flight are queued and run together: a caller that finds
 * fewer than max_inflight passes running becomes the leader, takes every
 * queued call with its parameters (up to max_residues residues) and runs them
 * as one batch on its own context; each caller waits until its slice is
 * done (spinning first, then sleeping), then replays its hit_cb / calls /
 * OTU stats on its own thread, in position order, before returning
 * (kguts.cc:814-815, 888-908).
 */
class SeqCoalescer {
public:
    struct Slice {
        std::vector<kgx_hit> hits;
        std::vector<kgx_call> calls;
        std::vector<kgx_otu> otus;
    };
    /* one pending call */
    struct Req {
        const std::string *seq = nullptr;
        kgx_params params{};
        uint32_t want = 0;
        Slice out;
        std::atomic<bool> done{false};
        int rc = KGX_OK;
        std::string err;
        bool sleeping = false;      /* under the queue's mutex */
        std::condition_variable cv; /* a sleeping caller's wake-up: done, or lead the next pass */
    };
    /* max_inflight / max_residues from KGX_COALESCE_INFLIGHT /
     * KGX_COALESCE_RESIDUES when set */
    SeqCoalescer();
    /* runs r on ctx, joining whatever is queued meanwhile; returns when r is
     * done (its slice filled, or r.rc set) */
    void submit(kgx_ctx *ctx, Req &r);
    int max_inflight = 8;
    uint64_t max_residues = 1 << 16;
    int spin_us = 200; /* a waiting caller spins this long before it sleeps */
    /* statistics: passes run and calls served */
    uint64_t passes = 0, calls = 0;

private:
    void run_batch(kgx_ctx *ctx, std::vector<Req *> &batch);
    std::mutex mu_;
    std::deque<Req *> queue_;
    std::atomic<size_t> queued_{0};   /* queue_.size(), for spinning callers */
    std::atomic<int> inflight_{0};
};

/* KmerImage (kmer_image.h:25-39): the read-only signature table, resident in
 * the HBM of one device.  Validation as kmer_image.cc:128-147. */
class KmerImage {
public:
    explicit KmerImage(const std::string &data_dir, int device = 0);
    /* adopt an image built elsewhere (e.g. kgx_image_build_synthetic) */
    explicit KmerImage(kgx_image *adopted);
    /* a borrowed image (closed by its owner, not here) */
    KmerImage(kgx_image *borrowed, bool owned);
    ~KmerImage();
    KmerImage(const KmerImage &) = delete;
    KmerImage &operator=(const KmerImage &) = delete;

    kgx_image *handle() const { return img_; }
    uint64_t num_sigs() const { return kgx_image_num_sigs(img_); }
    const std::string &data_dir() const { return data_dir_; }
    /* the queue that coalesces the image's concurrent process_aa_seq calls */
    SeqCoalescer &coalescer() { return coalescer_; }

private:
    SeqCoalescer coalescer_;
    kgx_image *img_ = nullptr;
    std::string data_dir_;
    bool owned_ = true;
};

class KmerGuts {
public:
    /* kguts.h:228-233 */
    struct hit_in_sequence_t {
        sig_kmer_t hit;
        unsigned int offset;
        hit_in_sequence_t(const sig_kmer_t &h, unsigned int o) : hit(h), offset(o) {}
    };

    /* one entry of a batched work list */
    struct SeqJob {
        std::string id;
        std::string seq;
        std::shared_ptr<std::vector<KmerCall>> calls;
        std::function<void(hit_in_sequence_t)> hit_cb;
        std::shared_ptr<KmerOtuStats> otu_stats;
        /* runs after this job's hits / calls / OTU are delivered and before the
         * next job's: the handler's per-sequence tail (e.g. the result block
         * after process_aa_seq in lookup_request.cc:174-400) moves here */
        std::function<void()> on_done;
    };

    /* kguts.cc:35-58: loads <dir>/function.index and <dir>/otu.index */
    KmerGuts(const std::string &kmer_dir, std::shared_ptr<KmerImage> image);
    ~KmerGuts();
    KmerGuts(const KmerGuts &) = delete;
    KmerGuts &operator=(const KmerGuts &) = delete;

    /* parameters, public like the reference (kguts.h:290-293) */
    int order_constraint;
    int min_hits;
    int min_weighted_hits;
    int max_gap;
    void set_default_parameters();
    void set_parameters(const std::map<std::string, std::string> &params);

    void process_aa_seq(const std::string &id, const std::string &seq,
                        std::shared_ptr<std::vector<KmerCall>> calls,
                        std::function<void(hit_in_sequence_t)> hit_cb,
                        std::shared_ptr<KmerOtuStats> otu_stats);
    void process_aa_seq_hits(const std::string &id, const std::string &seq,
                             std::shared_ptr<std::vector<KmerCall>> calls,
                             std::shared_ptr<std::vector<hit_in_sequence_t>> hits,
                             std::shared_ptr<KmerOtuStats> otu_stats);
    /* every job as process_aa_seq would, in order, with one GPU pass */
    void process_aa_batch(std::vector<SeqJob> &jobs);
    /* process_aa_seq joins the image's queue of concurrent calls (default
     * on; SeqCoalescer); off: one GPU pass per call on this object's context */
    bool coalesce = true;
    /* with coalesce: calls the image's resident call service serves
     * (kgx_svc_call: one sequence, hits / calls, order_constraint 0) skip the
     * queue and the launch; default on, KGX_SVC=0 turns it off */
    bool service = default_service();
    static bool default_service();

    void find_best_call(std::vector<KmerCall> &calls, int &function_index, std::string &function,
                        float &score, float &weighted_score, float &score_offset);
    /* the same outputs from the device's decision (KGX_WANT_BEST) */
    void find_best_call(const kgx_best_call &best, int &function_index, std::string &function,
                        float &score, float &weighted_score, float &score_offset);

    std::string format_call(const KmerCall &c);
    std::string format_hit(const hit_in_sequence_t &h);
    std::string format_otu_stats(const std::string &id, size_t size, KmerOtuStats &otu_stats);
    /* the same lines appended to out, without a stream per line: the
     * handlers' bulk output path (numbers as iostream prints them: decimal
     * integers, floats as "%.6g") */
    void append_call(std::string &out, const KmerCall &c) const;
    void append_hit(std::string &out, const hit_in_sequence_t &h) const;
    void append_otu_stats(std::string &out, const std::string &id, size_t size,
                          const KmerOtuStats &otu_stats) const;

    const char *function_at_index(int i) const;
    /* the name(s) a best call will print, toward the cache (the text stage
     * asks a block of sequences ahead) */
    void prefetch_call_names(const kgx_best_call &b) const
    {
        for (int k = 0; k < (b.kind == 2 ? 2 : b.kind == 1 ? 1 : 0); k++) {
            const int i = k ? b.fi1 : b.fi0;
            if (i >= 0 && (size_t)i < functions_.size())
                __builtin_prefetch(functions_[i].data());
        }
    }
    int function_count() const { return (int)functions_.size(); }
    static void decoded_kmer(unsigned long long encodedK, char *decoded);
    static unsigned long long encoded_aa_kmer(const char *p);

    std::shared_ptr<KmerImage> image_;
    kgx_ctx *ctx() const { return ctx_; }

private:
    kgx_ctx *ctx_ = nullptr;
    std::vector<std::string> functions_;
    std::vector<std::string> otus_;
};

/* FastaParser (fasta_parser.h:8-165): the framing that turns request bytes
 * into the (id, seq) pairs fed to KmerGuts. */
class FastaParser {
public:
    FastaParser();
    void set_callback(std::function<int(const std::string &, const std::string &)> cb) { on_seq_ = cb; }
    void set_error_callback(std::function<bool(const std::string &, int, const std::string)> cb)
    {
        on_error_ = cb;
    }
    void init_parse();
    bool parse_char(char c);
    void parse_complete();

private:
    enum State { START, ID, DEFLINE, DATA, ID_OR_DATA };
    int line_number_ = 1;
    State state_ = START;
    std::string id_, def_, seq_;
    std::function<int(const std::string &, const std::string &)> on_seq_;
    std::function<bool(const std::string &, int, const std::string)> on_error_;
    void emit();
};

/*
 * KmerPegMapping (kmer.h:25-157), the parts the request handlers use: the peg
 * id dictionary (encode_id / decode_id; ids assigned from 0 in first-seen
 * order, assign_new_peg_id kmer.h:114-121) on the host, and kmer_to_id_ /
 * kmer_to_family_id_ as device tables (include/kgx.h kgx_kmap).
 */
class KmerPegMapping {
public:
    typedef unsigned int encoded_id_t;
    typedef unsigned int encoded_family_id_t;
    explicit KmerPegMapping(int device = 0);
    ~KmerPegMapping();
    KmerPegMapping(const KmerPegMapping &) = delete;
    KmerPegMapping &operator=(const KmerPegMapping &) = delete;

    encoded_id_t encode_id(const std::string &peg);
    std::string decode_id(encoded_id_t id) const; /* "" when unknown, kmer.cc:288-295 */
    /* GET /dump_sizes body for this mapping (kmer.cc:510-524); the genome
     * tables are never filled by the request path, so they print 0 */
    void dump_sizes(std::ostream &os) const;
    /* add_mapping (kmer.cc:173-210) for every hit of kg's last batch, in
     * order: sequence s contributes ids[s] (add_request.cc:164-170) */
    void add_batch_mappings(KmerGuts &kg, const std::vector<encoded_id_t> &ids);
    /* add_fam_mapping (kmer.cc:212-256) likewise, into kmer_to_family_id_ */
    void add_batch_fam_mappings(KmerGuts &kg, const std::vector<encoded_family_id_t> &fam_ids);
    kgx_kmap *kmer_to_id() const { return kmer_to_id_; }
    kgx_kmap *kmer_to_family_id() const { return kmer_to_family_id_; }
    int device() const { return device_; }

    /* family data (kmer.h:58-66) */
    struct family_data_t {
        std::string pgf;
        std::string plf;
        unsigned long genus_id;
        std::string function;
        encoded_family_id_t family_id;
        unsigned long total_size; /* in aa */
        unsigned short count;
    };
    std::map<std::string, std::string> genus_map_;
    std::unordered_map<encoded_family_id_t, family_data_t> family_data_;
    /* genus_map_[genus] (kmer.h:136 lookup_genus: an unknown genus is
     * inserted with an empty id, which later GET /genus_lookup requests
     * see) and genus_map_.find (krequest2.cc:311-316), safe beside
     * concurrent /lookup requests */
    std::string lookup_genus(const std::string &genus);
    bool find_genus(const std::string &genus, std::string *id) const;
    /* family_data_[id] without inserting: the default record when unknown
     * (the reference's operator[] inserts one into a TBB map, which no
     * output shows), safe beside concurrent readers */
    family_data_t family_at(encoded_family_id_t id) const;
    std::map<std::pair<std::string, std::string>, encoded_family_id_t> family_key_to_id_;
    std::unordered_map<encoded_id_t, encoded_family_id_t> peg_to_family_;
    encoded_id_t assign_new_peg_id(const std::string &peg); /* kmer.h:114-121 */
    /* kmer.cc:341-358; throws kgx::Error when the file cannot be read */
    void load_genus_map(const std::string &genus_file);
    /* kmer.cc:375-493 with one reader thread (families in file order) */
    void load_families(const std::string &families_file);
    /* NRLoader family mode (nr_loader.cc:130-176) over a protein FASTA: every
     * hit of a protein with a family adds (k-mer, family) to
     * kmer_to_family_id_, proteins in file order, batched on the GPU */
    void load_nr_families(KmerGuts &kg, const std::string &nr_fasta, size_t batch = 100000);

private:
    mutable std::mutex genus_mu_;
    encoded_family_id_t next_family_id_ = 0;
    int device_;
    std::map<std::string, encoded_id_t> peg_to_id_;
    std::vector<std::string> id_to_peg_;
    kgx_kmap *kmer_to_id_ = nullptr;
    kgx_kmap *kmer_to_family_id_ = nullptr;
};

/*
 * MatrixRequest (matrix_request.cc:83-190): one /matrix request over a
 * mapping.  process_work() is the per-chunk worker loop (every sequence of
 * the chunk is encoded, its length recorded and its hits counted against
 * the proteins seen so far, in one GPU pass); write_results() prints
 * process_results' body (matrix_request.cc:171-187).
 */
class MatrixRequest {
public:
    explicit MatrixRequest(std::shared_ptr<KmerPegMapping> mapping);
    ~MatrixRequest();
    MatrixRequest(const MatrixRequest &) = delete;
    MatrixRequest &operator=(const MatrixRequest &) = delete;
    void process_work(KmerGuts &kg, const std::vector<std::pair<std::string, std::string>> &work);
    void write_results(std::ostream &os);

private:
    std::shared_ptr<KmerPegMapping> mapping_;
    kgx_matrix *mx_ = nullptr;
    std::map<KmerPegMapping::encoded_id_t, size_t> matrix_proteins_;
};

/*
 * FamilyMapper (family_mapper.cc:46-205, 287-330) in family mode with
 * allow_ambiguous_functions_ = false, over results computed in batches: the
 * caller supplies a fragment's on_hit rollups (computed on the device from
 * its hits and their kmer_to_family_id_ lists) and its calls.  seq_score_ is one
 * std::unordered_map kept across calls (cleared per protein), as in the
 * reference, so iteration -- and with it tie and summation order -- matches.
 */
class FamilyMapper {
public:
    struct best_match_t {
        std::string gfam_id;
        float gfam_score;
        std::string lfam_id;
        float lfam_score;
        std::string function;
        float score;
    };
    struct sequence_accumulated_score_t {
        unsigned int hit_count = 0;
        unsigned int hit_total = 0;
        float weighted_total = 0.0f;
    };
    FamilyMapper(KmerGuts &kg, std::shared_ptr<KmerPegMapping> mapping);
    /* rows: the fragment's on_hit rollups (kgx_kmap_rollup over
     * kmer_to_family_id_, KGX_ROLLUP_FAMILY), in first-touch order */
    best_match_t find_best_family_match(const kgx_rollup_row *rows, size_t n_rows, std::vector<KmerCall> &calls);
    /* the same with find_best_call decided on the device (KGX_WANT_BEST) */
    best_match_t find_best_family_match(const kgx_rollup_row *rows, size_t n_rows, const kgx_best_call &best);
    unsigned int kmer_hit_threshold_ = 3;

private:
    /* seq_score_ from the fragment's rollups, then the family rollup for the
     * called function (family_mapper.cc:46-205) */
    best_match_t match_from(const kgx_rollup_row *rows, size_t n_rows, std::string fn, float score);
    KmerGuts &kg_;
    std::shared_ptr<KmerPegMapping> mapping_;
    std::unordered_map<KmerPegMapping::encoded_id_t, sequence_accumulated_score_t> seq_score_;
};
std::ostream &operator<<(std::ostream &os, const FamilyMapper::best_match_t &m);

/*
 * LookupRequest (lookup_request.cc): one /lookup request.  The request's
 * query-string parameters are read as in lookup_request.cc:33-79
 * (kmer_hit_threhsold -- sic --, find_best_match, find_reps,
 * allow_ambiguous_functions, target_genus).  process_work() is the worker
 * loop over a chunk (lookup_request.cc:153-400): the chunk's lookups run as
 * one GPU batch and the per-sequence rollups (on_hit 446-482) on the device
 * (kgx_kmap_rollup); the rows go into one seq_score_ map for the request in
 * first-touch order, and the selection and output run on the host in order.  No family
 * reps DB is loaded, so find_reps prints only the "///" separators.
 */
/*
 * LookupBatcher: the device side of concurrent /lookup requests' pieces in
 * shared passes -- the reference's pool runs one chunk per worker
 * (lookup_request.cc:153-172); here, while other requests are in flight, a
 * piece is copied into the open staging area (pinned, two areas: one
 * filling while the other's pass runs) and the first waiting request whose
 * area is complete leads ONE pass + rollup (kgx_lookup) for every piece in
 * it on its own worker's context; each piece then gets its own best calls
 * and rollup rows back.  A request alone (nothing in flight), a piece too
 * large for an area, or a map on another device than the worker runs its
 * own pass (the small-batch path + kgx_kmap_rollup).  Sequences are
 * independent, so the results are the same bytes either way.  The server
 * takes it with KGX_LOOKUP_BATCH=1 (measured slower than a pass per piece
 * for 1-MiB bodies at 16 clients: one shared pass at a time serialises what
 * the workers' own small passes overlap).
 */
class LookupBatcher {
public:
    /* pieces of a pass: at most max_residues residues and max_seqs sequences */
    explicit LookupBatcher(uint64_t max_residues = 16u << 20, uint32_t max_seqs = 1u << 20);
    ~LookupBatcher();
    LookupBatcher(const LookupBatcher &) = delete;
    LookupBatcher &operator=(const LookupBatcher &) = delete;
    /* a piece's device results: best calls (want KGX_WANT_BEST), rollup
     * offsets (n + 1, from 0) and rows */
    struct Out {
        std::vector<kgx_best_call> best;
        std::vector<uint64_t> roff;
        std::vector<kgx_rollup_row> rows;
    };
    /* the n sequences res[off[i], off[i+1]) through a pass (throws kgx::Error) */
    void run(KmerGuts &kg, kgx_kmap *map, int mode, const kgx_params &p, uint32_t want, const char *res,
             const uint64_t *off, uint32_t n, Out &out);
    /* passes run, pieces they carried, pieces run alone */
    uint64_t passes() const { return passes_; }
    uint64_t batched() const { return batched_; }
    uint64_t alone() const { return alone_; }
    /* a piece's own pass (the small-batch path, then kgx_kmap_rollup) */
    static void run_alone(KmerGuts &kg, kgx_kmap *map, int mode, const kgx_params &p, uint32_t want,
                          const char *res, const uint64_t *off, uint32_t n, Out &out);

private:
    struct Piece;
    struct Area;
    void lead(KmerGuts &kg, Area &a);
    std::mutex mu_;
    std::condition_variable cv_;
    std::unique_ptr<Area> area_[2];
    int open_ = 0;
    bool busy_ = false;
    int active_ = 0; /* requests inside run() */
    uint64_t max_res_;
    uint32_t max_seq_;
    std::atomic<uint64_t> passes_{0}, batched_{0}, alone_{0};
};

class LookupRequest {
public:
    LookupRequest(std::shared_ptr<KmerPegMapping> mapping, bool family_mode,
                  const std::map<std::string, std::string> &params);
    /* the device side through a batcher shared with concurrent requests
     * (null: every piece its own pass) */
    void set_batcher(LookupBatcher *b) { batcher_ = b; }
    void process_work(KmerGuts &kg, const std::vector<std::pair<std::string, std::string>> &work,
                      std::ostream &os);

    /* the same over a flat work list: sequence i's residues res[off[i],
     * off[i+1]), its id ids[id_off[i], id_off[i+1]) */
    void process_flat(KmerGuts &kg, const char *res, const uint64_t *off, const char *ids, const uint64_t *id_off,
                      size_t n, std::ostream &os);

private:
    struct FlatWork {
        const char *res;
        const uint64_t *off;
        const char *ids;
        const uint64_t *id_off;
    };
    typedef std::unordered_map<KmerPegMapping::encoded_id_t, FamilyMapper::sequence_accumulated_score_t> ScoreMap;
    /* sequences [w0, w1) as one GPU pass, their rollups on the device */
    void process_piece(KmerGuts &kg, const FlatWork &fw, size_t w0, size_t w1, std::ostream &os);
    /* the find_best_match lines of the piece's sequences [a, b) into out,
     * `smap` in the state seq_score_ would be in at sequence a */
    void best_match_lines(KmerGuts &kg, const FlatWork &fw, size_t w0, uint32_t a, uint32_t b,
                          const kgx_best_call *best, const uint64_t *roff, const kgx_rollup_row *rows,
                          ScoreMap &smap, std::string &out) const;
    std::shared_ptr<KmerPegMapping> mapping_;
    bool family_mode_;
    unsigned int kmer_hit_threshold_ = 3;
    bool find_best_match_ = false;
    bool allow_ambiguous_functions_ = false;
    bool find_reps_ = false;
    unsigned long target_genus_id_ = 0;
    ScoreMap seq_score_;
    size_t seq_score_most_ = 0; /* the most rows seq_score_ has held (its bucket count follows from it) */
    LookupBatcher *batcher_ = nullptr;
};

/*
 * FqProcessRequest (fq_process_request.cc:230-365): FASTQ in, per read the
 * best frame's family matches out.  process() runs a block: the reads'
 * 6-frame fragments, their lookup and scoring on the GPU in one batch, then
 * on_parsed_seq's frame choice and FamilyMapper in read order on the host
 * (one FamilyMapper per block, as process_data constructs one,
 * fq_process_request.cc:241).
 */
class FqRequest {
public:
    FqRequest(KmerGuts &kg, std::shared_ptr<KmerPegMapping> mapping);
    ~FqRequest();
    FqRequest(const FqRequest &) = delete;
    FqRequest &operator=(const FqRequest &) = delete;
    /* one block of FASTQ text; `finished` = the request's last block
     * (parse_complete).  Output lines are appended to os. */
    void process(const std::string &fastq_block, bool finished, std::ostream &os);
    void process(const char *fastq_block, size_t n, bool finished, std::ostream &os);
    /* reads already parsed (id, DNA) */
    void process_reads(const std::vector<std::pair<std::string, std::string>> &reads, std::ostream &os);

private:
    /* parsed reads, flat (a view): read r's id is ids[id_off[r], id_off[r+1]),
     * its bases res[roff[r], roff[r+1]) */
    struct FqBlock {
        const char *res = nullptr;
        const uint64_t *roff = nullptr;
        const char *ids = nullptr;
        const uint64_t *id_off = nullptr;
        size_t n = 0;
        const char *residues() const { return res; }
        size_t n_reads() const { return n; }
        const char *id(size_t r) const { return ids + id_off[r]; }
        size_t id_len(size_t r) const { return (size_t)(id_off[r + 1] - id_off[r]); }
    };
    /* one part of a block, parsed: its reads' bases in pinned host memory
     * (kgx_host_alloc; the device copies them from there), offsets, ids, and
     * the parser state at its end.  Kept across blocks (buffers reused). */
    struct FqPart {
        int state = 0;
        std::string id;
        char *bases = nullptr;
        size_t cap = 0, len = 0;
        std::vector<uint64_t> roff{0}, id_off{0};
        std::string id_chars;
        FqPart() = default;
        FqPart(const FqPart &) = delete;
        FqPart &operator=(const FqPart &) = delete;
        ~FqPart();
        /* empty, from a parser state, room for `need` bases */
        void begin(size_t need, int state, const std::string &carried_id, const std::string &carried_bases);
        void parse(const char *a, const char *b);
        FqBlock view() const;
    };
    void process_block(const FqBlock &blk, FamilyMapper &mapper, std::ostream &os);
    /* process_block in two halves: launch sizes the block's fragments and
     * enqueues their lookup on ctx; finish collects the results and writes the
     * block's lines.  Between the two the host may launch the next block on
     * another context. */
    struct FqLaunched {
        kgx_ctx *ctx = nullptr;
        uint32_t n_reads = 0;
        kgx_fragments fr{};
    };
    FqLaunched launch_block(const FqBlock &blk, kgx_ctx *ctx);
    /* after kgx_fq_upload on ctx: enqueue the fragment pass over those reads */
    void start_fragments(kgx_ctx *ctx);
    /* launch_block's second half, after kgx_fq_upload and start_fragments of
     * l's reads on l.ctx: the pass's sizes, then the lookup enqueued */
    void launch_uploaded(FqLaunched &l);
    void finish_block(const FqBlock &blk, FqLaunched &l, FamilyMapper &mapper, std::ostream &os);
    kgx_ctx *twin_ctx(); /* a second context on the image, created on first use */
    kgx_ctx *twin_ = nullptr;
    kgx_ctx *twin2_ctx(); /* a third, for the multi-part pipeline */
    kgx_ctx *twin2_ = nullptr;
    KmerGuts &kg_;
    std::shared_ptr<KmerPegMapping> mapping_;
    /* FastqParser state (fastq_parser.h:40-150) */
    int state_ = 0;
    std::string id_, seq_;
    std::vector<std::unique_ptr<FqPart>> parts_;
    /* the exact re-parse after a rejected speculative cut: kept, so its pinned
     * buffer is allocated once, not per fallback */
    std::unique_ptr<FqPart> tail_;
};

/* one host-buffer batch through kg's context, device results only (no D2H):
 * what KmerPegMapping / MatrixRequest read from (kgx_kmap_add_hits,
 * kgx_matrix_add_hits) */
void run_batch_on_device(KmerGuts &kg, const std::vector<std::string> &seqs);

/* find_best_call (kguts.cc:1008-1199) with an explicit function-name lookup */
void best_call(const std::vector<KmerCall> &calls, const std::function<const char *(int)> &name_of,
               int &function_index, std::string &function, float &score, float &weighted_score,
               float &score_offset);

/* find_best_call's outputs from a device decision (kgx_best_call) */
void best_call(const kgx_best_call &b, const std::function<const char *(int)> &name_of, int &function_index,
               std::string &function, float &score, float &weighted_score, float &score_offset);

/* load_indexed_ar (kguts.cc:544-575): "%d\t<name>\n" lines, dense and in
 * order; returns false when the file cannot be opened or is not dense. */
bool load_index_file(const std::string &path, std::vector<std::string> &out);

}  // namespace kgx

#endif
