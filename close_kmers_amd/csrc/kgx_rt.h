/*
 * kgx_rt.h -- host runtime internals shared by the C ABI translation units
 * (kgx_runtime.cpp: images, contexts, batches; kgx_tables.cpp: k-mer -> id
 * tables and /matrix pair counting).  Not part of the public ABI.
 */
#ifndef KGX_RT_H
#define KGX_RT_H

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kgx_internal.h"

namespace kgx {

/* sets the thread's kgx_last_error() text and returns code */
int fail(int code, const std::string &msg);
bool is_gfx950(int dev);

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return ::kgx::fail(KGX_EDEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

/* How a thread waits for its own stream (kgx_set_host_wait): KGX_WAIT_SPIN
 * (hipStreamSynchronize: the runtime polls), KGX_WAIT_SLEEP (hipStreamQuery
 * every poll_us, the thread asleep in between) or KGX_WAIT_BLOCK (a
 * blocking-sync event: the thread sleeps until the device signals).  A
 * server of many workers under a CPU share (the box's 16 CPUs) spends that
 * share spinning in the default; the two others hand it to the text and
 * socket work.  Process-wide; KGX_HOST_WAIT=spin|sleep[:us]|block sets the
 * starting mode. */
extern std::atomic<int> g_host_wait_mode;
extern std::atomic<uint32_t> g_host_wait_us;
hipError_t host_wait(hipStream_t s);
/* the host spins on a completion word the device stores (small batches):
 * the same modes, polling `done` instead of the stream */
hipError_t host_wait_word(const volatile uint32_t *done, uint32_t token, hipStream_t s);

/* grow-only device buffer, freed with its owner */
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    DevBuf(DevBuf &&o) noexcept : p(o.p), cap(o.cap)
    {
        o.p = nullptr;
        o.cap = 0;
    }
    DevBuf &operator=(DevBuf &&o) noexcept
    {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
        return *this;
    }
    ~DevBuf() { release(); }
    hipError_t reserve(size_t bytes)
    {
        if (bytes <= cap)
            return hipSuccess;
        if (p)
            (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 256);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess)
            cap = want;
        return e;
    }
    void release()
    {
        if (p)
            (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

/* grow-only pinned host array (hipHostMalloc): the staging and result
 * buffers of the host-buffer path, so H2D / D2H run at DMA speed instead of
 * through the runtime's pageable bounce buffers.  Contents are not
 * initialised on growth. */
template <class T> struct PinnedVec {
    T *p = nullptr;
    size_t n = 0, cap = 0;
    mutable void *dp = nullptr; /* p's device address, looked up once per allocation */
    PinnedVec() = default;
    PinnedVec(const PinnedVec &) = delete;
    PinnedVec &operator=(const PinnedVec &) = delete;
    ~PinnedVec()
    {
        if (p)
            (void)hipHostFree(p);
    }
    hipError_t resize(size_t m)
    {
        if (m > cap) {
            T *q = nullptr;
            const size_t want = std::max<size_t>(m + m / 4, 64);
            hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&q), want * sizeof(T), hipHostMallocDefault);
            if (e != hipSuccess)
                return e;
            if (p) {
                std::memcpy(q, p, n * sizeof(T));
                (void)hipHostFree(p);
            }
            p = q;
            cap = want;
            dp = nullptr;
        }
        n = m;
        return hipSuccess;
    }
    T *data() { return p; }
    const T *data() const { return p; }
    /* the device's address of element i (pinned host memory is mapped) */
    hipError_t device_ptr(size_t i, void **out) const
    {
        if (!dp) {
            hipError_t e = hipHostGetDevicePointer(&dp, p, 0);
            if (e != hipSuccess) {
                dp = nullptr;
                return e;
            }
        }
        *out = static_cast<char *>(dp) + i * sizeof(T);
        return hipSuccess;
    }
    size_t size() const { return n; }
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
};

inline uint64_t windows_of(uint64_t len) { return len >= 9 ? len - 8 : 0; }

/* [p, p + n) lies in one pinned, device-mapped host allocation (kgx_host_alloc,
 * hipHostMalloc, hipHostRegister): the device may read it by DMA directly */
bool host_pinned_range(const void *p, uint64_t n, const void **device_address = nullptr);

/* one pass over a whole host batch, split into enqueue and collect
 * (kgx_runtime.cpp): the upload by pull kernels on `up` (recording up_done)
 * when given, else on the context's stream */
class HostPool;
/* stage: the threads that copy pageable residues into the context's pinned
 * staging (null: the context's own stage pool) */
int one_pass_enqueue(kgx_ctx *c, const kgx_params *params, const char *residues, const uint64_t *seq_offsets,
                     uint32_t n_seq, uint32_t want, hipStream_t up, hipEvent_t up_done, HostPool *stage = nullptr);
int one_pass_collect(kgx_ctx *c, const kgx_params *params, const char *residues, const uint64_t *seq_offsets,
                     uint32_t n_seq, uint32_t want, kgx_result *out);

/* host CPUs this process may keep busy: the affinity mask, capped by a
 * cgroup v2 quota (cpu.max) -- on the GPU box the mask shows the whole
 * machine while the quota is 16 */
unsigned host_cpu_budget();

/* memcpy by up to 8 host threads for large copies (host staging into pinned
 * buffers runs at several times one core's copy rate) */
inline void parallel_memcpy(void *dst, const void *src, size_t n)
{
    const size_t T = std::min<size_t>(8, n >> 23); /* one thread per 8 MiB, up to 8 */
    if (T <= 1) {
        std::memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> pool;
    for (size_t t = 0; t < T; t++)
        pool.emplace_back([=]() {
            const size_t a = n * t / T, b = n * (t + 1) / T;
            std::memcpy(static_cast<char *>(dst) + a, static_cast<const char *>(src) + a, b - a);
        });
    for (auto &th : pool)
        th.join();
}

/* A few persistent host threads for work that overlaps device streams (the
 * compact host path's hit expansion).  submit() queues a task; wait() blocks
 * until every queued task has finished and returns the first nonzero code a
 * task returned (then clears it). */
class HostPool {
  public:
    explicit HostPool(unsigned n)
    {
        for (unsigned i = 0; i < n; i++)
            th_.emplace_back([this] { run(); });
    }
    HostPool(const HostPool &) = delete;
    HostPool &operator=(const HostPool &) = delete;
    ~HostPool()
    {
        {
            std::lock_guard<std::mutex> l(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_)
            t.join();
    }
    unsigned size() const { return (unsigned)th_.size(); }
    void submit(std::function<int()> f)
    {
        {
            std::lock_guard<std::mutex> l(mu_);
            q_.push_back(std::move(f));
            pending_++;
        }
        cv_.notify_one();
    }
    int wait()
    {
        std::unique_lock<std::mutex> l(mu_);
        idle_.wait(l, [this] { return pending_ == 0; });
        const int rc = rc_;
        rc_ = 0;
        if (rc)
            fail(rc, msg_); /* the task's error text on the waiting thread */
        return rc;
    }

  private:
    void run()
    {
        for (;;) {
            std::function<int()> f;
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [this] { return stop_ || !q_.empty(); });
                if (q_.empty())
                    return;
                f = std::move(q_.front());
                q_.pop_front();
            }
            const int rc = f();
            const char *why = rc ? kgx_last_error() : nullptr; /* the failing thread's text */
            std::lock_guard<std::mutex> l(mu_);
            if (rc && !rc_) {
                rc_ = rc;
                msg_ = why ? why : "";
            }
            if (--pending_ == 0)
                idle_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::deque<std::function<int()>> q_;
    std::mutex mu_;
    std::condition_variable cv_, idle_;
    size_t pending_ = 0;
    int rc_ = 0;
    std::string msg_;
    bool stop_ = false;
};

/* a fragment pass enqueued by fq_fragments_enqueue, finished by fq_fragments_finish */
struct FqPending {
    bool active = false;
    bool desc = false;
    uint32_t n_reads = 0;
    uint64_t max_frag = 0, max_res = 0;
    const uint8_t *bases = nullptr;
    uint64_t bound = 0;
};
int fq_fragments_enqueue(kgx_ctx *c, const uint8_t *d_bases, const uint64_t *d_read_off, uint32_t n_reads,
                         uint64_t n_bases, uint64_t bound);
int fq_fragments_finish(kgx_ctx *c, kgx_fragments *out);
/* n_bases: the bytes the reads span (bounds the output); bound: bytes
 * readable from d_bases (the DNA probe's limit) */
int fq_fragments(kgx_ctx *c, const uint8_t *d_bases, const uint64_t *d_read_off, uint32_t n_reads,
                 uint64_t n_bases, uint64_t bound, kgx_fragments *out);
/* kgx_stage_probe over fragments left as DNA (launch_probe_dna) */
int stage_probe_dna(kgx_ctx *c, const uint8_t *bases, uint64_t n_bases, const uint64_t *anchors,
                    const uint64_t *d_off);
/* kgx_stage_plan's buffers and bookkeeping without the plan kernels */
int plan_reserve(kgx_ctx *c, const uint64_t *d_off, uint32_t n_seq, uint64_t n_residues);
/* whether this context's probe can take fragments as DNA */
bool probe_takes_dna(const kgx_ctx *c);
/* the lookup's plan over fragments of at least 9 residues each (every
 * fragment a fragment pass emits has >= 11): window base = residue offset - 8
 * per earlier fragment, no scan; tile owners and the longest fragment as
 * launch_plan writes them (kgx_fq.hip) */
hipError_t launch_fq_plan(const uint64_t *off, uint32_t n, uint64_t *wbase, uint32_t *tile_seq, uint32_t tile_windows,
                          uint32_t *status, uint32_t *block_max, hipStream_t stream);

struct SvcState;
/* stops and frees the image's call service (kgx_svc.cpp), if any */
void svc_shutdown(kgx_image *img);
/* the same, and keeps the image's service lock until the returned guard
 * goes: a call arriving meanwhile waits for it before it starts a new
 * service, so no instance is created over a table being replaced */
std::unique_lock<std::mutex> svc_shutdown_hold(kgx_image *img);
/* kgx_kmap_rollup in two steps: the device work enqueued on c's stream (no
 * host wait once an earlier rollup on c gave a size), then the wait, the size
 * check (passes 2-3 again when short) and the result */
int rollup_enqueue(kgx_kmap *m, kgx_ctx *c, int mode);
int lookup_small(kgx_ctx *c, kgx_kmap *m, int mode, const kgx_params *params, const char *residues,
                 const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want, kgx_result *out, bool *taken);
/* kgx_device_batch_collect's counts (and best calls) round trip enqueued on
 * c's stream ahead of the collect, which then only waits */
int collect_counts_enqueue(kgx_ctx *c, uint32_t want);
int rollup_finish(kgx_kmap *m, kgx_ctx *c, int mode, kgx_rollup_result *out);

/* kgx_kmap_rollup's device scratch and host results (kgx_tables.hip), per
 * context: grow-only, no allocation per call once warm */
struct RollupScratch {
    DevBuf tcount, tbase, hseq, hstart, hlen, sfirst, send, ev_id, ev_w, flag, rowdata, rows2, rowcnt, rowoff, tmp;
    PinnedVec<uint64_t> h_n; /* [0] hits, [1] events, [2] rows */
    PinnedVec<uint64_t> h_off;
    PinnedVec<kgx_rollup_row> h_rows;
    uint64_t hint = 0;          /* the previous rollup's event count: the next one's size */
    uint64_t cap = 0;           /* the enqueued rollup's event capacity (0: not yet sized) */
    uint64_t presize_misses = 0;
    bool enqueued = false;
};

}  // namespace kgx

struct kgx_image {
    int device = 0;
    uint64_t num_sigs = 0;
    int layout = KGX_LAYOUT_AOS24;
    kgx_sig_kmer *d_table = nullptr;   /* AOS24: the file's buckets */
    kgx::packed_bucket *d_packed = nullptr; /* PACKED16 */
    /* kgx_image_set_line_index: the PACKED16 records again, 4 buckets a line,
     * each key's home at the start of line (key mod n_lines); the probes read
     * it instead of d_packed, which stays for downloads, saves and filters */
    kgx::packed_bucket *d_lines = nullptr;
    uint64_t n_lines = 0;
    uint32_t lines_load = 0; /* keys per 64 lines it was built for */
    uint64_t *d_filter = nullptr;           /* presence filter (kgx_image_set_filter) */
    uint32_t filter_log2_words = 0;
    /* probe order across the image's contexts: the probe is bound by random
     * HBM requests, so two probes at once only share that rate; run back to
     * back instead, each context's other kernels (plan, score, gather, fq
     * translation) overlap the next context's probe */
    std::mutex probe_mu;
    hipEvent_t last_probe = nullptr; /* end of the latest probe enqueued */
    hipStream_t probe_stream = nullptr; /* contexts' chained probes with option probe_stream */
    /* the resident call service (kgx_svc.cpp), created on the first kgx_svc_call */
    std::mutex svc_mu; /* creation, configuration and shutdown; a call takes no lock */
    std::atomic<kgx::SvcState *> svc{nullptr};
    /* callers inside kgx_svc_call, counted per thread shard, each shard on a
     * line of its own: a call writes no line that other callers write
     * (kgx_svc.cpp: enter / shutdown_locked) */
    struct alignas(64) SvcUsers {
        std::atomic<uint32_t> n{0};
    };
    SvcUsers svc_users[32];
    uint32_t svc_slots = 32, svc_idle_us = 1000, svc_life_us = 1000;
    bool svc_configured = false; /* kgx_svc_config was called (env defaults no longer apply) */
    const void *resident() const
    {
        return layout == KGX_LAYOUT_PACKED16 ? static_cast<const void *>(d_packed) : d_table;
    }
    uint64_t resident_bytes() const
    {
        return num_sigs * (layout == KGX_LAYOUT_PACKED16 ? sizeof(kgx::packed_bucket) : sizeof(kgx_sig_kmer));
    }
    /* what the probes read: the line index when there is one */
    const void *probe_table() const { return d_lines ? static_cast<const void *>(d_lines) : resident(); }
    uint64_t probe_buckets() const { return d_lines ? 4 * n_lines : num_sigs; }
    uint32_t home_shift() const { return d_lines ? 2u : 0u; }
};

struct kgx_ctx {
    kgx_image *img = nullptr;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipEvent_t probe_done = nullptr; /* recorded after each of this context's probes */
    int probe_serialize = 1;          /* option "probe_serialize" */
    int probe_stream = 0;             /* chained probes on the image's probe stream (option "probe_stream") */
    hipEvent_t probe_ready = nullptr; /* this context's inputs are ready for its probe */
    /* a pool's /lookup: the stream the pass's score runs on after its probe
     * (null: the context's stream), behind score_gate recorded after the probe */
    hipStream_t score_stream = nullptr;
    hipEvent_t score_gate = nullptr;
    /* device scratch */
    kgx::DevBuf residues, offsets, wbase, tile_seq, hit_mask, hits, calls, hit_count, call_count,
        dense_hoff, dense_coff, dense_hits, dense_calls, plan_ws, ranges;
    /* plan status word (1 = the last plan's offsets were bad, batch emptied) */
    kgx::DevBuf plan_status;
    /* the one-launch plan's look-back states (zero between launches) */
    kgx::DevBuf plan_look;
    int plan_fused = 0; /* option "plan_fused": 0 = three kernels, 1 = one look-back launch, 2 = one workgroup */
    kgx::PinnedVec<uint32_t> h_plan_status;
    /* current plan */
    uint32_t n_seq = 0;
    uint64_t n_residues = 0;
    uint64_t max_tiles = 0;
    uint32_t tile_windows = 64u * kgx::PROBE_J_DEFAULT;
    uint64_t hit_slots = 0; /* slots per hit plane: cold plane at hits + hit_slots */
    const uint64_t *d_off = nullptr;
    bool have_hits = false; /* the tiled hits of the current plan are on the device */
    uint32_t hit_format = kgx::HIT_PLANES; /* of the current plan's hits (set by the probe) */
    bool have_best = false; /* best[] holds find_best_call of the current plan */
    bool defer_best = false; /* kgx_stage_score leaves best[] to the small path's collect */
    kgx::DevBuf best, best_ws, bc_calls, bc_start, bc_count; /* KGX_WANT_BEST / kgx_find_best_calls */
    kgx::PinnedVec<kgx_best_call> h_best;
    /* fq fragments (kgx_fq.hip) */
    kgx::DevBuf fq_bases, fq_roff, fq_nfrag, fq_fbase, fq_tmp, fq_res, fq_off, fq_read, fq_frame, fq_start,
        fq_anchor, fq_nres;
    kgx::DevBuf fq_look; /* fq_fused: tile counter | tile states */
    kgx::PinnedVec<uint64_t> h_fq_tot; /* fragments, residues of the last fq batch */
    kgx::FqPending fq_pend;             /* an enqueued fragment pass awaiting its finish */
    /* kgx_fq_upload: reads whose H2D is enqueued, awaiting kgx_fq_fragments_uploaded */
    struct {
        bool active = false;
        uint32_t n_reads = 0;
        uint64_t n_bases = 0;
    } fq_up;
    kgx::PinnedVec<uint64_t> h_fq_roff; /* the uploaded reads' relative offsets (pinned: the copy is async) */
    /* kgx_fq_called_reads */
    kgx::DevBuf fqc_flag, fqc_reads, fqc_nsel, fqc_nfrag, fqc_ncall, fqc_fo, fqc_co, fqc_fc, fqc_len, fqc_coff,
        fqc_calls;
    kgx::PinnedVec<uint32_t> h_fqc_n, h_fqc_reads, h_fqc_fc, h_fqc_len;
    kgx::PinnedVec<uint64_t> h_fqc_tot, h_fqc_fo, h_fqc_coff;
    kgx::PinnedVec<kgx_call> h_fqc_calls;
    /* tuning options */
    int probe_variant = kgx::PROBE_AUTO;
    int probe_j = kgx::PROBE_J_DEFAULT;
    int probe_lds_kb = 0;  /* LDS reserved per probe workgroup, caps its occupancy (option "probe_lds_kb") */
    int probe_persist = 0; /* line probe grid cap in workgroups per CU, waves stride over tiles (option "probe_persist") */
    int fq_residues = 1;   /* 1: kgx_fq_fragments writes residues; 0: anchors (kgx_fq_run_device) */
    int fq_count = 1;      /* fq count pass: 1 = lane-per-read stop scan, 0 = wave-per-read translation */
    int fq_probe_j = 1;    /* tile of the DNA probe (fragments as anchors), 64 x J windows; 0 = probe_j */
    int fq_plan = 1;       /* 1: this context's fragments are planned elementwise (fq_plan_kernel); 0: launch_plan */
    int fq_fused = 1;      /* anchors: count + scan + emit in one look-back pass (fq_anchor_fused_kernel); 0: four launches */
    int score_variant = 0; /* 0 = hybrid, 1 = wave-parallel, 2 = lane only (option "score_variant", kgx_internal.h) */
    int score_wave_tiles = 16; /* probe tiles of windows per scorer wave (option "score_wave_tiles") */
    int probe_filter = 1; /* use the image's presence filter when it has one */
    int use_line_index = 1; /* option "line_index": 0 = probe the reference slots even when the image has a line index */
    int probe_nt = 0;       /* option "probe_nt": 1 = the line probe's hit stores non-temporal */
    uint64_t microbench_span = 0; /* bytes of the table the random-read ceiling covers; 0 = all */
    int microbench_ilp = 8;       /* independent reads in flight per lane */
    int microbench_wgs = 8;       /* 256-thread workgroups per CU */
    /* host results */
    std::vector<uint64_t> h_hoff, h_coff, h_ooff;
    kgx::PinnedVec<kgx_hit> h_hits;
    kgx::PinnedVec<kgx_call> h_calls;
    kgx::PinnedVec<kgx_otu> h_otus;
    kgx::PinnedVec<uint32_t> h_ocount;
    /* KGX_WANT_OTU: device tallies (otu_kernel) */
    kgx::DevBuf otu_ws, otus, otu_count, dense_ooff, dense_otus;
    bool have_otus = false;
    kgx::PinnedVec<uint32_t> h_hcount, h_ccount;
    kgx::PinnedVec<char> h_res;
    /* host-buffer batches in chunks (option "host_chunks"): chunks alternate
     * between this context and a twin over the same image, so one chunk's
     * gather + D2H overlaps the next chunk's H2D + kernels */
    int host_chunks = 6;
    int host_copy = 1; /* chunk D2H: 0 = DMA (hipMemcpyAsync), 1 = device stores into mapped memory */
    int host_copy_blocks = 64; /* workgroups of the store copy (option "host_copy_blocks") */
    kgx_ctx *twin = nullptr;
    kgx::PinnedVec<uint64_t> h_off_stage, h_dense_hoff, h_dense_coff, h_dense_ooff, h_nwin;
    /* compact chunk D2H (option "host_hits16", PACKED16 images): a chunk's
     * hits cross PCIe as their 16-byte table records plus the chunk's hit
     * mask, and host threads expand them into kgx_hit (position = mask bit)
     * while the next chunk streams */
    int host_hits16 = 1;
    int host_threads = 12; /* expansion threads (option "host_threads") */
    std::unique_ptr<kgx::HostPool> pool;
    /* chunk staging (pageable caller buffer -> pinned) in parts on
     * stage_threads threads (option "stage_threads", 1 = the calling thread) */
    int stage_threads = 8; /* option "stage_threads": r4ag, 3.57-3.65 vs 3.71-3.90 ms per batch with 4 */
    std::unique_ptr<kgx::HostPool> stage_pool;
    kgx::PinnedVec<uint4> h_hits16;
    kgx::PinnedVec<uint64_t> h_mask;
    std::vector<uint64_t> h_wstart;     /* chunk-relative first window of each sequence */
    std::vector<hipEvent_t> chunk_done; /* per chunk: its records and mask are on the host */
    std::vector<hipEvent_t> chunk_counts; /* per chunk: its counts are on the host */
    std::vector<hipEvent_t> chunk_gathered; /* per chunk: its dense buffers are complete */
    hipStream_t copy_stream = nullptr; /* bulk chunk D2H, apart from the contexts' kernels */
    /* streamed schedule, option "host_upload_stream" 1: every chunk's residues
     * and offsets go up on a stream of their own into a region of the
     * batch's own (up_res / up_off), as soon as they are staged, instead of
     * behind the previous chunk's kernels on the context's stream.  Off by
     * default: with the runtime's 4 hardware queues per process the upload
     * stream shares one with a stream that waits on events, and measured no
     * faster (r4l/r4m: 3.66-4.21 vs 3.76-4.09 ms per 30M-residue batch; with
     * 16 queues the uploads do run early, 3.60-3.90 ms) */
    int host_upload_stream = 0;
    int host_score_variant = 1; /* streamed chunks' scorer (option "host_score_variant"; -1: score_variant) */
    hipStream_t up_stream = nullptr;
    kgx::DevBuf up_res, up_off;
    kgx::DevBuf dense_mask, dense_best; /* a chunk's mask / best calls for its bulk copy */
    /* streamed schedule (option "host_stream", compact records only): device
     * CSR offsets, bulk copies sized on the device into host regions sized
     * from the rates below (records per window seen so far, x 1.25) */
    int host_stream_chunks = 1;
    int host_taper = 1; /* first and last chunk half-size (option "host_taper") */
    double rate_hits = 0.35, rate_calls = 0.05, rate_otus = 0.05;
    uint64_t stream_fallbacks = 0; /* batches rerun exact after a region overflowed */
    /* option "pinned_input" (default 1): a streamed host batch whose residues
     * already sit in pinned memory (kgx_host_alloc, hipHostMalloc /
     * hipHostRegister) goes to the device by DMA straight from the caller's
     * buffer, with no staging copy on the host; a device scan flags NUL bytes
     * (the host-side strlen cut, kguts.cc:792) and such a batch reruns staged */
    int pinned_input = 1;
    bool one_pass_pinned = false; /* the enqueued one-pass batch reads caller-pinned residues */
    uint64_t pinned_batches = 0, nul_reruns = 0;
    uint32_t counts_enqueued = 0; /* want + 1 of an enqueued collect_counts_enqueue, else 0 */
    kgx::PinnedVec<uint32_t> h_nul;
    std::vector<hipEvent_t> chunk_h2d; /* per chunk: its staged residues are on the device */
    kgx::DevBuf dense_counts, cscan_ws;
    kgx::PinnedVec<uint32_t> h_counts;
    kgx::PinnedVec<uint32_t> h_hits12; /* 12-B records (3 words per hit, no key) */
    int host_rec12 = 1; /* streamed: 12-B records, key re-encoded on the host (option "host_rec12") */
    int host_h2d_first = 1; /* streamed: chunk k's D2H waits for chunk k+1's H2D (option "host_h2d_first") */
    /* streamed: every chunk staged into its own region of h_res_all / h_off_all
     * (option "host_stage_all"), not into the context's h_res behind the H2D of
     * the chunk two before */
    int host_stage_all = 0; /* r4ak: 3.61-3.70 vs 3.49-3.73 ms per batch, no gain */
    kgx::PinnedVec<char> h_res_all;
    /* streamed: chunk copies by DMA (hipMemcpyAsync of each region whole, at
     * its host-sized room) instead of the counted device-store copy (option
     * "host_stream_dma") */
    int host_stream_dma = 0;
    kgx::PinnedVec<uint64_t> h_off_all;
    /* small host batches (<= small_batch residues, option "small_batch", 0 =
     * off): planned on the host, read by the device from the mapped staging
     * blob, results stored into mapped memory: one host wait per batch */
    int64_t small_batch = 1 << 21; /* 2M residues: a 1-MiB request body and then some */
    int small_wave = 1; /* small batches: the wave scorer instead of the hybrid (option "small_wave") */
    int small_wave_tiles = 1; /* small batches: probe tiles per scorer wave (option "small_wave_tiles") */
    kgx::PinnedVec<uint4> h_small; /* offsets | window bases | tile owners | status | residues */
    kgx::PinnedVec<uint32_t> h_done; /* the fused small gather's completion token */
    kgx::DevBuf small_blocks_done;    /* its workgroup counter (zero between launches) */
    /* one-launch small batches (option "small_fused"; kgx_fused.hip): mapped
     * window bases, per-sequence result regions, counts and tokens */
    int small_fused = 0;
    int fused_inline = 1; /* a tiny fused batch travels in the kernel arguments (option "fused_inline") */
    uint64_t fused_batches = 0, small_batches = 0; /* kgx_ctx_stat */
    kgx::PinnedVec<uint64_t> h_fwb;
    kgx::PinnedVec<kgx_hit> h_fhits;
    kgx::PinnedVec<kgx_call> h_fcalls;
    kgx::PinnedVec<uint32_t> h_fcounts, h_fdone;
    kgx::PinnedVec<uint64_t> h_fdbg; /* KGX_FUSED_DEBUG phase stamps */
    uint32_t small_token = 0;
    int host_nt = 1;    /* expansion with streaming stores (option "host_nt") */
    kgx::PinnedVec<kgx_call> h_calls_region;
    kgx::PinnedVec<kgx_otu> h_otus_region;
    int counts_first = 1; /* chunk k's bulk D2H waits for chunk k+1's counts (option "counts_first") */
    /* compact results (kgx_process_batch_compact): the call leaves the hits as
     * records + mask; compact_segs say where each chunk's landed (element
     * offsets into h_hits12 / h_hits16 and h_mask, resolved to pointers once
     * the pinned arrays stop growing) */
    int compact_out = 0;
    struct CompactSeg {
        uint32_t s0, s1, words;
        uint64_t hit_begin, rec_at, mask_at;
    };
    std::vector<CompactSeg> compact_segs;
    std::vector<kgx_hit_chunk> compact_chunks;
    /* option "host_profile": per-chunk timing events and the last call's profile */
    int host_profile = 0;
    std::vector<hipEvent_t> prof_ev; /* 4 per chunk: H2D start, H2D end, device end, gathered */
    std::vector<hipEvent_t> prof_done; /* per chunk: bulk copy done (timing events on the copy stream) */
    kgx_host_profile last_profile{};
    /* kgx_kmap_rollup */
    std::unique_ptr<kgx::RollupScratch> rollup;
};

namespace kgx {
/* what c's probes read: the image's line index unless option "line_index" is 0 */
inline bool ctx_lines(const kgx_ctx *c) { return c->img->d_lines && c->use_line_index; }
inline const void *ctx_probe_table(const kgx_ctx *c)
{
    return ctx_lines(c) ? static_cast<const void *>(c->img->d_lines) : c->img->resident();
}
inline uint64_t ctx_probe_buckets(const kgx_ctx *c) { return ctx_lines(c) ? 4 * c->img->n_lines : c->img->num_sigs; }
inline uint32_t ctx_home_shift(const kgx_ctx *c) { return ctx_lines(c) ? 2u : 0u; }
/* one chunk of compact records -> kgx_hit for sequences [a, b) of it:
 * out[j - out_base] for CSR hit j (hoff: the batch's hit offsets);
 * kgx_hit.seq = s + seq_base; nt = streaming stores */
int expand_chunk(const kgx_hit_chunk &ch, const uint64_t *hoff, const char *residues, const uint64_t *seq_offsets,
                 uint32_t a, uint32_t b, kgx_hit *out, uint64_t out_base, uint32_t seq_base, bool nt);
/* kgx_compact_expand with a choice of streaming stores */
int compact_expand(const kgx_compact_result *r, const char *residues, const uint64_t *seq_offsets, uint32_t s_begin,
                   uint32_t s_end, uint32_t seq_base, kgx_hit *out, bool nt);
}  // namespace kgx

#endif
