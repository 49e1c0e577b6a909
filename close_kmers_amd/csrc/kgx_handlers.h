/*
 * kgx_handlers.h -- the kserver request surface over the KmerGuts facade.
 *
 * Request handlers (the per-chunk worker loops of query_request.cc,
 * add_request.cc, matrix_request.cc, lookup_request.cc and
 * fq_process_request.cc) as functions of (KmerGuts, mapping, parameters,
 * request body) writing the response body, and the HTTP request router of
 * krequest2.cc:273-489 (KmerRequestRouter) that picks a handler and the
 * keyed mapping for a request.  The router is transport-free: kgx_server
 * feeds it requests read from a socket, an embedding server (the
 * reference's boost.asio loop) can feed it its own.
 *
 * Each handler runs a request body as one work list: one GPU pass for the
 * body's sequences, then the per-sequence output in request order.  The
 * reference splits a body into 1-MiB chunks and writes each chunk's output
 * as it completes; the concatenated output is the same, because every line
 * depends only on its own sequence and on state updated in request order.
 */
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <ostream>
#include <shared_mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "kgx_dispatch.h"
#include "kguts_hip.h"

namespace kgx {

typedef std::vector<std::pair<std::string, std::string>> work_list_t;
typedef std::map<std::string, std::string> request_params_t;

/* FastaParser over a whole body: (id, seq) pairs in input order */
work_list_t parse_fasta_body(const char *body, size_t n);

/* cut points [begin, end) of at most `pieces` pieces of a FASTA body, each
 * starting at a record's '>' that follows a sequence or blank line; empty
 * when the body cannot be cut (too small, not starting with '>') */
std::vector<std::pair<size_t, size_t>> split_fasta_body(const char *body, size_t n, size_t pieces);
/* the line-at-a-time parse of one piece; false when the piece needs the
 * byte machine (then the whole body must be parsed as one) */
bool parse_fasta_piece(const char *piece, size_t n, work_list_t &work);

/* A parsed body, flat (no string per record): record i's id is
 * ids[id_off[i], id_off[i+1]), its residues res[off[i], off[i+1]) -- the
 * batch layout kgx_process_batch takes as is. */
struct FastaFlat {
    std::string ids, res;
    std::vector<uint64_t> id_off{0}, off{0};
    size_t size() const { return off.size() - 1; }
    std::string id(size_t i) const { return ids.substr(id_off[i], id_off[i + 1] - id_off[i]); }
    void add(const char *id, size_t id_len, const char *seq, size_t seq_len)
    {
        ids.append(id, id_len);
        id_off.push_back(ids.size());
        res.append(seq, seq_len);
        off.push_back(res.size());
    }
};
/* parse_fasta_piece / parse_fasta_body into the flat form (same records) */
bool parse_fasta_piece_flat(const char *piece, size_t n, FastaFlat &out);
FastaFlat parse_fasta_body_flat(const char *body, size_t n);
FastaFlat flat_of(const work_list_t &work);

/* the reference reads integer flags with std::stoi and keeps the default
 * when the value is absent or not a number (query_request.cc:92-100) */
int param_int(const request_params_t &params, const std::string &name, int dflt);

/* /query (query_request.cc:103-151): details=1 adds HIT lines,
 * find_best_call=1 prints one best-call line per sequence with a call */
void query_request(KmerGuts &kg, const work_list_t &work, int details, int find_best_call,
                   std::ostream &os);
/* the same over a flat batch: one GPU pass, the lines written straight from
 * the result CSR (calls, device OTU tallies already in otus_by_count order,
 * device find_best_call decisions) -- no per-sequence objects */
void query_request(KmerGuts &kg, const FastaFlat &work, int details, int find_best_call, std::ostream &os);

/* query_request in its two halves: the GPU pass over the whole flat batch
 * (res / off; ids unused) into *cr, valid until the next pass on kg -- then
 * the text of sequences [s0, s1) appended to out, their ids taken from
 * `ids` (a piece whose record 0 is sequence s0).  Text of disjoint ranges may
 * be written on several threads at once. */
void query_pass(KmerGuts &kg, const FastaFlat &batch, int details, int find_best_call, kgx_compact_result *cr);
void query_text(KmerGuts &kg, const kgx_compact_result &cr, const FastaFlat &batch, uint32_t s0, uint32_t s1,
                const FastaFlat &ids, int details, int find_best_call, std::string &out);

/*
 * ForkJoin -- a few host threads shared by all requests: run(k, f) calls
 * f(0) ... f(k-1), the caller taking indices too, and returns when all have
 * returned (the first exception is rethrown on the caller).  Concurrent
 * run()s share the helpers; a run never waits on another's work, so nothing
 * deadlocks when every helper is busy -- the caller then does it all.
 */
class ForkJoin {
public:
    explicit ForkJoin(unsigned helpers);
    ~ForkJoin();
    ForkJoin(const ForkJoin &) = delete;
    ForkJoin &operator=(const ForkJoin &) = delete;
    unsigned helpers() const { return (unsigned)th_.size(); }
    void run(size_t k, const std::function<void(size_t)> &f);

private:
    struct Batch;
    void helper();
    static void work(Batch &b);
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<Batch *> open_; /* batches with unclaimed indices */
    bool stop_ = false;
};

/* /add (add_request.cc:115-170): per sequence PROTEIN-ID / CALL / OTU-COUNTS /
 * BEST-CALL unless silent, then every hit's k-mer is mapped to the
 * sequence's id in mapping.kmer_to_id_ (ids encoded in request order) */
void add_request(KmerGuts &kg, KmerPegMapping &mapping, const work_list_t &work, int silent,
                 std::ostream &os);

/* /matrix (matrix_request.cc:83-190): pair counts against the proteins seen
 * earlier in the same request and present in mapping.kmer_to_id_ */
void matrix_request(KmerGuts &kg, std::shared_ptr<KmerPegMapping> mapping, const work_list_t &work,
                    std::ostream &os);

/* /lookup (lookup_request.cc:153-400) */
void lookup_request(KmerGuts &kg, std::shared_ptr<KmerPegMapping> mapping, bool family_mode,
                    const request_params_t &params, const work_list_t &work, std::ostream &os);

/* /fq_lookup (fq_process_request.cc:230-365): FASTQ body */
void fq_request(KmerGuts &kg, std::shared_ptr<KmerPegMapping> mapping, const char *body, size_t n,
                std::ostream &os);

/* one parsed HTTP request (krequest2.cc:24-29, 92-213) */
struct HttpRequest {
    std::string method, path, parameters_raw, fragment, http_version;
    request_params_t parameters;            /* split on ';' and '&', "k=v" parts only */
    std::map<std::string, std::string> headers; /* keys lower-cased */
    std::string body;
};

/* the request line "METHOD path[?params][#frag] HTTP/x.y" (krequest2.cc:24,
 * 92-131); false when it does not match */
bool parse_request_line(const std::string &line, HttpRequest &req);
/* one header line "Key: value" ('\r' stripped by the caller) */
void parse_header_line(const std::string &line, HttpRequest &req);

/*
 * KmerRequestRouter (krequest2.cc:273-489 + kserver.cc:40-130): owns the
 * image replicas (one per listed device), a pool of KmerGuts (one per
 * worker, like threadpool.cc:33-36; worker w on replica w % n_devices) and
 * the keyed mappings ("" = the root mapping, which carries the family DB).
 * handle() returns the full response bytes.  Thread-safe: requests run
 * concurrently up to the pool size; each mapping has a reader/writer lock --
 * /add writes it (one at a time, so request-order id assignment stays
 * deterministic; the reference's TBB maps make concurrent /add safe),
 * /matrix, /lookup and /fq_lookup read it concurrently.  Workers are dealt
 * by WorkerPicker (kgx_dispatch.h), so the pieces of a large /query and
 * concurrent requests spread over the devices; /add and /matrix run on a
 * worker of the mappings' device (their k-mer tables live there).
 */
class KmerRequestRouter {
public:
    struct Options {
        std::string kmer_data_dir;
        int device = 0;
        /* one image replica per entry (the file read once, or the synthetic
         * image built on the first and copied device to device); empty =
         * {device}.  The mappings' device tables live on devices[0]. */
        std::vector<int> devices;
        int n_kmer_threads = 1;
        std::string kmer_version, families_version; /* "" = not given */
        std::string genus_mapping, families_file;
        std::vector<std::string> families_nr;
        /* benchmark hook: when synthetic_keys > 0 the image is built in HBM
         * by kgx_image_build_synthetic (synthetic_keys keys in synthetic_sigs
         * buckets) instead of loading kmer_data_dir/kmer.table.mem_map; the
         * directory still provides function.index and otu.index */
        uint64_t synthetic_keys = 0, synthetic_sigs = 0;
        /* distinct /mapping/<key> keys that may be created besides the root
         * mapping (each holds device k-mer tables); a request for a new key
         * past the cap answers 503 */
        size_t max_mappings = 1024;
    };
    explicit KmerRequestRouter(const Options &opt);
    ~KmerRequestRouter();

    bool family_mode() const { return family_mode_; }
    /* *quit is set for GET /quit (after the response is built) */
    std::string handle(const HttpRequest &req, bool *quit);

    /* "HTTP/ver code status\nContent-type: text/plain\n" (krequest2.cc:491-495) */
    static std::string header(const std::string &http_version, int code, const std::string &status);
    /* header + Content-length + body (krequest2.cc:497-503) */
    static std::string respond(const std::string &http_version, int code, const std::string &status,
                               const std::string &body);

    /* the device each worker runs on (for tests / logs) */
    std::vector<int> worker_devices() const;

private:
    static constexpr size_t kPieceBytes = 1 << 20; /* krequest2.cc:41 */
    /* a body under 2 pieces: parsed and written in sub-pieces of at least
     * this size on the ForkJoin helpers, around one GPU pass */
    static constexpr size_t kSplitBytes = 192 << 10;
    static constexpr unsigned kHelpers = 3;
    class GutsLease;
    struct Mapping {
        std::shared_ptr<KmerPegMapping> map;
        std::shared_ptr<std::shared_mutex> mu; /* /add: exclusive, other handlers: shared */
    };
    /* only_slot >= 0: a worker on that device slot */
    KmerGuts *acquire(long only_slot = -1);
    void release(KmerGuts *kg);
    Mapping mapping_for(const std::string &key);

    Options opt_;
    bool family_mode_;
    std::vector<std::shared_ptr<KmerImage>> images_; /* one per device slot */
    std::vector<std::unique_ptr<KmerGuts>> pool_;
    WorkerPicker picker_;
    std::mutex pool_mu_;
    std::condition_variable pool_cv_;
    std::mutex mapping_mu_; /* the mapping map itself */
    std::map<std::string, Mapping> mapping_map_;
    ForkJoin fj_{kHelpers};
    std::unique_ptr<LookupBatcher> lookup_batcher_; /* /lookup pieces of concurrent requests, shared passes */
    std::atomic<int> query_in_flight_{0};
};

} // namespace kgx
