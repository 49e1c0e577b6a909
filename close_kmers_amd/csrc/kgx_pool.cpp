/*
 * kgx_pool.cpp -- one query batch split across the GPUs of a node.
 *
 * The reference runs a thread pool of KmerGuts workers over one shared,
 * read-only KmerImage (threadpool.cc:18-44) and feeds it one chunk of a
 * request per task (lookup_request.cc:138-172, krequest2.cc:41).  Sequences
 * are independent (KmerGuts state is per sequence, kguts.h:263-266), so the
 * batch shards with no exchange step: a kgx_pool holds contexts over image
 * replicas (one per GPU), cuts a batch into contiguous residue-balanced
 * shards, runs shard i on context i from its own host thread, and
 * concatenates the per-shard CSR results in input order.  No collective.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cctype>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <cstdio>

#include <pthread.h>
#include <sched.h>

#include "kgx_rt.h"

using namespace kgx;

unsigned kgx::host_cpu_budget()
{
    static const unsigned budget = [] {
        cpu_set_t set;
        unsigned n = 0;
        if (sched_getaffinity(0, sizeof(set), &set) == 0)
            n = (unsigned)CPU_COUNT(&set);
        if (n == 0)
            n = std::max(1u, std::thread::hardware_concurrency());
        if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[64] = {0};
            unsigned long long period = 0;
            if (std::fscanf(f, "%63s %llu", q, &period) == 2 && std::string(q) != "max" && period) {
                const unsigned long long quota = std::strtoull(q, nullptr, 10);
                n = std::min<unsigned>(n, (unsigned)std::max<unsigned long long>(1, quota / period));
            }
            std::fclose(f);
        }
        return n;
    }();
    return budget;
}

namespace {

/* "0-31,128-159" -> the CPUs it names, in set (false: unreadable) */
bool parse_cpulist(const char *text, cpu_set_t &set)
{
    CPU_ZERO(&set);
    const char *p = text;
    bool any = false;
    while (*p) {
        while (*p == ',' || *p == ' ' || *p == '\n')
            p++;
        if (!*p)
            break;
        char *end = nullptr;
        const long a = std::strtol(p, &end, 10);
        if (end == p || a < 0)
            return false;
        long b = a;
        p = end;
        if (*p == '-') {
            b = std::strtol(p + 1, &end, 10);
            if (end == p + 1 || b < a)
                return false;
            p = end;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; c++)
            CPU_SET((int)c, &set);
        any = true;
    }
    return any;
}

/* the CPUs of node that this process may use (empty: none, or no such node) */
bool node_cpus(int node, cpu_set_t &out)
{
    CPU_ZERO(&out);
    if (node < 0)
        return false;
    char path[96];
    std::snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    FILE *f = std::fopen(path, "r");
    if (!f)
        return false;
    char buf[4096] = {0};
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    cpu_set_t nodeset, mine;
    if (!parse_cpulist(buf, nodeset) || sched_getaffinity(0, sizeof mine, &mine) != 0)
        return false;
    CPU_AND(&out, &nodeset, &mine);
    return CPU_COUNT(&out) > 0;
}

}  // namespace

struct kgx_pool {
    std::vector<kgx_ctx *> ctxs;
    std::vector<int> numa; /* per context: the node its thread is bound to, -1 unbound */
    /* one persistent host thread per context: job generation counter */
    std::vector<std::thread> threads;
    std::mutex mu;
    std::condition_variable cv_job, cv_done;
    uint64_t generation = 0;
    uint32_t pending = 0;
    bool quit = false;
    std::function<void(uint32_t)> job; /* run by every worker i < job_width */
    uint32_t job_width = 0;
    /* the concatenated result */
    std::vector<uint64_t> hoff, coff, ooff;
    std::unique_ptr<kgx_hit[]> hits; /* grow-only (no zeroing of GBs per batch) */
    uint64_t hits_cap = 0;
    std::vector<kgx_hit_chunk> chunks; /* kgx_pool_process_batch_compact */
    /* kgx_hit expansion of the shards' compact records (KGX_POOL_EXPAND_THREADS, default 16) */
    std::unique_ptr<kgx::HostPool> xpool;
    unsigned expand_threads = 16;
    std::vector<kgx_call> calls;
    std::vector<kgx_otu> otus;
    std::vector<kgx_best_call> best;
    std::vector<uint64_t> roff; /* kgx_pool_lookup's rollup rows */
    std::vector<kgx_rollup_row> rows;
    /* Shards per device: a host batch runs its chunks on a context and its
     * twin, with copies and event waits across their streams, and a process's
     * streams share a few hardware queues (4), so past two batches at once on
     * one device they queue behind each other's waits: 8 contexts of one
     * device took 38-41 ms per C5 batch against 31 with 2 (r5e, r5i), gated
     * to two at a time or not.  So a batch is cut into at most `per_device`
     * shards per device (KGX_POOL_PER_DEVICE, default 2), run on the first
     * contexts of each device; /lookup's one-pass shards take twice that
     * (no twins: 4 contexts measured best, r5e) */
    uint32_t per_device = 2;
    /* kgx_pool_lookup: per device a stream for the shards' uploads (lowest
     * priority: a queue of its own), and an event per shard */
    std::vector<hipStream_t> up_stream;
    std::vector<hipEvent_t> up_done;
    /* per device three streams made in a row before the contexts: the
     * shards' plans and probes one after another, their scores (behind each
     * probe, an event), and their rollups (behind each probe too).  The
     * runtime spreads a process's streams over a few hardware queues
     * (GPU_MAX_HW_QUEUES, 4), so streams made in a row rarely share one, and a
     * shard's score and rollup run beside the next shard's probe instead of
     * holding it back in a shared queue.  The shards' contexts lend their
     * buffers; their own streams stay idle.  (r5x: passes and rollups on the
     * contexts' streams, 1.86-2.09 ms for the same batch by which of them the
     * runtime put on one queue; r5z/r6b: 2.08-2.10 ms with these streams,
     * deterministic; more hardware queues than 4 measured slower still.) */
    std::vector<hipStream_t> pass_stream, score_stream, roll_stream;
    /* kgx_pool_lookup stages a pageable batch shard after shard from one
     * thread, so each shard's copy into pinned memory gets all the process's
     * CPUs (a context's own stage pool has its share: cpus / contexts) */
    std::unique_ptr<HostPool> lookup_stage;
    std::vector<hipEvent_t> pass_done, roll_done;
    std::vector<uint32_t> runners(uint32_t per) const
    {
        std::vector<uint32_t> out, used;
        for (uint32_t i = 0; i < (uint32_t)ctxs.size(); i++) {
            const int d = kgx_image_device(ctxs[i]->img);
            if ((int)used.size() <= d)
                used.resize((size_t)d + 1, 0);
            if (used[(size_t)d] < per) {
                used[(size_t)d]++;
                out.push_back(i);
            }
        }
        return out;
    }

    void worker(uint32_t i)
    {
        /* numa.cc:13-42: the worker on its device's node, before it allocates
         * (pinned staging lands on the node of the thread that first touches it) */
        if (numa[i] >= 0) {
            cpu_set_t set;
            if (!node_cpus(numa[i], set) || pthread_setaffinity_np(pthread_self(), sizeof set, &set) != 0)
                numa[i] = -1;
        }
        uint64_t seen = 0;
        for (;;) {
            std::function<void(uint32_t)> fn;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_job.wait(lk, [&] { return quit || generation != seen; });
                if (quit)
                    return;
                seen = generation;
                if (i >= job_width)
                    continue;
                fn = job;
            }
            fn(i);
            {
                std::lock_guard<std::mutex> lk(mu);
                if (--pending == 0)
                    cv_done.notify_all();
            }
        }
    }

    /* fn(i) for i < width on the workers, concurrently; returns when all are done */
    void run(uint32_t width, std::function<void(uint32_t)> fn)
    {
        std::unique_lock<std::mutex> lk(mu);
        job = std::move(fn);
        job_width = width;
        pending = width;
        generation++;
        cv_job.notify_all();
        cv_done.wait(lk, [&] { return pending == 0; });
    }
};

extern "C" {

int kgx_shard_cuts(const uint64_t *seq_offsets, uint32_t n_seq, uint32_t n_shards, uint32_t *cuts)
{
    if (!cuts || n_shards == 0 || (n_seq && !seq_offsets))
        return fail(KGX_EINVAL, "bad shard arguments");
    cuts[0] = 0;
    cuts[n_shards] = n_seq;
    if (n_seq == 0) {
        for (uint32_t i = 1; i < n_shards; i++)
            cuts[i] = 0;
        return KGX_OK;
    }
    const uint64_t r0 = seq_offsets[0], total = seq_offsets[n_seq] - r0;
    for (uint32_t i = 1; i < n_shards; i++) {
        /* 128-bit product: total * i can exceed 2^64 only for absurd sizes, but stay exact */
        const uint64_t target = r0 + (uint64_t)((unsigned __int128)total * i / n_shards);
        const uint32_t s = (uint32_t)(std::lower_bound(seq_offsets, seq_offsets + n_seq, target) - seq_offsets);
        cuts[i] = std::max(cuts[i - 1], s);
    }
    return KGX_OK;
}

int kgx_pool_create(kgx_image *const *images, uint32_t n_images, uint32_t n_ctx, kgx_pool **out)
{
    if (!images || !out || n_images == 0 || n_ctx == 0)
        return fail(KGX_EINVAL, "a pool needs images and contexts");
    *out = nullptr;
    kgx_pool *p = new kgx_pool;
    for (uint32_t i = 0; i < n_images; i++) {
        const int d = images[i] ? kgx_image_device(images[i]) : -1;
        if (d < 0)
            continue;
        if ((int)p->pass_stream.size() <= d)
            p->pass_stream.resize((size_t)d + 1, nullptr);
        if ((int)p->roll_stream.size() <= d) {
            p->roll_stream.resize((size_t)d + 1, nullptr);
            p->score_stream.resize((size_t)d + 1, nullptr);
        }
        if (!p->pass_stream[(size_t)d]) {
            hipStream_t st[3] = {nullptr, nullptr, nullptr};
            bool ok = hipSetDevice(d) == hipSuccess;
            for (int k = 0; k < 3 && ok; k++)
                ok = hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking) == hipSuccess;
            if (!ok) {
                for (hipStream_t x : st)
                    if (x)
                        (void)hipStreamDestroy(x);
                for (auto *v : {&p->pass_stream, &p->score_stream, &p->roll_stream})
                    for (hipStream_t x : *v)
                        if (x)
                            (void)hipStreamDestroy(x);
                delete p;
                return fail(KGX_EDEVICE, "pool: stream creation failed");
            }
            p->pass_stream[(size_t)d] = st[0];
            p->score_stream[(size_t)d] = st[1];
            p->roll_stream[(size_t)d] = st[2];
        }
    }
    for (uint32_t i = 0; i < n_ctx; i++) {
        kgx_ctx *c = nullptr;
        int rc = images[i % n_images] ? kgx_ctx_create(images[i % n_images], &c) : fail(KGX_EINVAL, "null image");
        if (rc) {
            for (auto *x : p->ctxs)
                kgx_ctx_destroy(x);
            for (auto *v : {&p->pass_stream, &p->score_stream, &p->roll_stream})
                for (hipStream_t x : *v)
                    if (x)
                        (void)hipStreamDestroy(x);
            delete p;
            return rc;
        }
        p->ctxs.push_back(c);
    }
    /* the contexts' host threads share the process's CPUs: staging and
     * expansion threads per context sized so the pool keeps about as many
     * busy as there are CPUs (8 contexts x 8 stagers on a 16-CPU share ran
     * slower than 2 contexts, r4x_bench_pool) */
    const unsigned cpus = host_cpu_budget();
    for (kgx_ctx *c : p->ctxs) {
        c->stage_threads = (int)std::max(1u, std::min<unsigned>((unsigned)c->stage_threads, cpus / n_ctx));
        c->host_threads = (int)std::max(1u, std::min<unsigned>((unsigned)c->host_threads, cpus / n_ctx));
    }
    p->expand_threads = std::max(1u, std::min(p->expand_threads, cpus));
    if (const char *e = std::getenv("KGX_POOL_PER_DEVICE"))
        p->per_device = (uint32_t)std::max(1L, std::strtol(e, nullptr, 10));
    if (const char *e = std::getenv("KGX_POOL_EXPAND_THREADS"))
        p->expand_threads = (unsigned)std::min(256L, std::max(1L, std::strtol(e, nullptr, 10)));
    /* each context's NUMA node, worked out here (the HIP call) and bound
     * by its thread */
    const char *ne = std::getenv("KGX_POOL_NUMA");
    const bool bind = !ne || std::atoi(ne) != 0;
    p->numa.assign(n_ctx, -1);
    for (uint32_t i = 0; i < n_ctx && bind; i++) {
        cpu_set_t set;
        const int node = kgx_device_numa_node(kgx_image_device(p->ctxs[i]->img));
        if (node_cpus(node, set))
            p->numa[i] = node;
    }
    for (uint32_t i = 0; i < n_ctx; i++)
        p->threads.emplace_back([p, i] { p->worker(i); });
    /* the binding is read back only after the threads have started */
    p->run(n_ctx, [](uint32_t) {});
    *out = p;
    return KGX_OK;
}

int kgx_pool_map_select(const int32_t *ctx_device, uint32_t n_ctx, const int32_t *map_device, uint32_t n_maps,
                        int32_t *pick)
{
    if (n_ctx && (!ctx_device || !pick || (n_maps && !map_device)))
        return fail(KGX_EINVAL, "null argument");
    for (uint32_t i = 0; i < n_ctx; i++) {
        pick[i] = -1;
        for (uint32_t j = 0; j < n_maps && pick[i] < 0; j++)
            if (map_device[j] >= 0 && map_device[j] == ctx_device[i])
                pick[i] = (int32_t)j;
        if (pick[i] < 0)
            return fail(KGX_EINVAL, "pool lookup: no map on device " + std::to_string(ctx_device[i]));
    }
    return KGX_OK;
}

int kgx_pool_numa_node(const kgx_pool *p, uint32_t i)
{
    return p && i < p->numa.size() ? p->numa[i] : -1;
}

int kgx_device_numa_node(int device)
{
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    for (char *q = bus; *q; q++)
        *q = (char)std::tolower((unsigned char)*q);
    char path[160];
    std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE *f = std::fopen(path, "r");
    if (!f)
        return -1;
    int node = -1;
    if (std::fscanf(f, "%d", &node) != 1)
        node = -1;
    std::fclose(f);
    return node;
}

int kgx_numa_node_cpus(int node, uint32_t *cpus, uint32_t cap)
{
    cpu_set_t set;
    if (!node_cpus(node, set))
        return 0;
    uint32_t k = 0;
    for (int c = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &set)) {
            if (cpus && k < cap)
                cpus[k] = (uint32_t)c;
            k++;
        }
    return (int)k;
}

int kgx_device_memory(int device, uint64_t *free_bytes, uint64_t *total_bytes)
{
    if (!free_bytes || !total_bytes)
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(device));
    size_t f = 0, t = 0;
    HIP_TRY(hipMemGetInfo(&f, &t));
    *free_bytes = f;
    *total_bytes = t;
    return KGX_OK;
}

int kgx_pool_destroy(kgx_pool *p)
{
    if (!p)
        return KGX_OK;
    {
        std::lock_guard<std::mutex> lk(p->mu);
        p->quit = true;
    }
    p->cv_job.notify_all();
    for (auto &t : p->threads)
        t.join();
    for (auto *c : p->ctxs)
        kgx_ctx_destroy(c);
    for (size_t d = 0; d < p->up_stream.size(); d++)
        if (p->up_stream[d]) {
            (void)hipSetDevice((int)d);
            (void)hipStreamSynchronize(p->up_stream[d]);
            (void)hipStreamDestroy(p->up_stream[d]);
        }
    for (hipEvent_t e : p->up_done)
        (void)hipEventDestroy(e);
    for (auto *v : {&p->pass_stream, &p->score_stream, &p->roll_stream})
        for (size_t d = 0; d < v->size(); d++)
            if ((*v)[d]) {
                (void)hipSetDevice((int)d);
                (void)hipStreamSynchronize((*v)[d]);
                (void)hipStreamDestroy((*v)[d]);
            }
    for (auto *v : {&p->pass_done, &p->roll_done})
        for (hipEvent_t e : *v)
            (void)hipEventDestroy(e);
    delete p;
    return KGX_OK;
}

uint32_t kgx_pool_size(const kgx_pool *p) { return p ? (uint32_t)p->ctxs.size() : 0; }

kgx_ctx *kgx_pool_ctx(kgx_pool *p, uint32_t i) { return p && i < p->ctxs.size() ? p->ctxs[i] : nullptr; }

}  // extern "C"

namespace {

/* phase 1 of a pool batch: the shards, each on its context, all at once,
 * results left compact in the contexts (kgx_process_batch_compact); then the
 * concatenation's offsets (hoff/coff/ooff) and the per-shard bases */
struct PoolRun {
    std::vector<uint32_t> run; /* shard i runs on context run[i] */
    uint32_t K = 0;
    std::vector<uint32_t> cuts;
    std::vector<kgx_compact_result> part;
    std::vector<uint64_t> hb, cb, ob;
    uint64_t nwin = 0;
};

int pool_shards(kgx_pool *p, const kgx_params *params, const char *residues, const uint64_t *seq_offsets,
                uint32_t n_seq, uint32_t want, PoolRun &R)
{
    if (!p || (!seq_offsets && n_seq))
        return fail(KGX_EINVAL, "null argument");
    for (uint32_t s = 0; s < n_seq; s++)
        if (seq_offsets[s + 1] < seq_offsets[s])
            return fail(KGX_EINVAL, "seq_offsets not monotone");
    R.run = p->runners(p->per_device);
    R.K = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)R.run.size(), n_seq));
    const uint32_t K = R.K;
    R.cuts.assign(K + 1, 0);
    int rc = kgx_shard_cuts(seq_offsets, n_seq, K, R.cuts.data());
    if (rc)
        return rc;
    /* A shard's offsets stay absolute: kgx_process_batch reads residues from
     * seq_offsets[first] on. */
    R.part.assign(K, kgx_compact_result{});
    std::vector<int> rcs(K, KGX_OK);
    std::vector<std::string> errs(K);
    p->run(K, [&](uint32_t i) {
        rcs[i] = kgx_process_batch_compact(p->ctxs[R.run[i]], params, residues, seq_offsets + R.cuts[i],
                                           R.cuts[i + 1] - R.cuts[i], want, &R.part[i]);
        if (rcs[i])
            errs[i] = kgx_last_error();
    });
    for (uint32_t i = 0; i < K; i++)
        if (rcs[i])
            return fail(rcs[i], "pool shard " + std::to_string(i) + ": " + errs[i]);
    R.hb.assign(K + 1, 0);
    R.cb.assign(K + 1, 0);
    R.ob.assign(K + 1, 0);
    R.nwin = 0;
    for (uint32_t i = 0; i < K; i++) {
        const uint32_t n = R.cuts[i + 1] - R.cuts[i];
        const kgx_result &r = R.part[i].r;
        R.hb[i + 1] = R.hb[i] + r.hit_offsets[n];
        R.cb[i + 1] = R.cb[i] + r.call_offsets[n];
        R.ob[i + 1] = R.ob[i] + r.otu_offsets[n];
        R.nwin += r.n_windows;
    }
    p->hoff.resize((size_t)n_seq + 1);
    p->coff.resize((size_t)n_seq + 1);
    p->ooff.resize((size_t)n_seq + 1);
    p->hoff[0] = p->coff[0] = p->ooff[0] = 0;
    const bool want_best = (want & KGX_WANT_BEST) != 0;
    p->calls.resize(R.cb[K]);
    p->otus.resize(R.ob[K]);
    p->best.resize(want_best ? n_seq : 0);
    /* offsets, calls, OTUs and best calls into place (small: no hit records) */
    p->run(K, [&](uint32_t i) {
        const kgx_result &r = R.part[i].r;
        const uint32_t s0 = R.cuts[i], n = R.cuts[i + 1] - R.cuts[i];
        for (uint32_t s = 1; s <= n; s++) {
            p->hoff[s0 + s] = R.hb[i] + r.hit_offsets[s];
            p->coff[s0 + s] = R.cb[i] + r.call_offsets[s];
            p->ooff[s0 + s] = R.ob[i] + r.otu_offsets[s];
        }
        if (R.cb[i + 1] > R.cb[i])
            std::memcpy(p->calls.data() + R.cb[i], r.calls, (R.cb[i + 1] - R.cb[i]) * sizeof(kgx_call));
        if (R.ob[i + 1] > R.ob[i])
            std::memcpy(p->otus.data() + R.ob[i], r.otus, (R.ob[i + 1] - R.ob[i]) * sizeof(kgx_otu));
        if (want_best && n)
            std::memcpy(p->best.data() + s0, r.best, n * sizeof(kgx_best_call));
    });
    return KGX_OK;
}

void pool_fill(kgx_pool *p, const PoolRun &R, uint32_t n_seq, uint32_t want, kgx_result *out)
{
    out->n_seq = n_seq;
    out->hit_offsets = p->hoff.data();
    out->hits = nullptr;
    out->call_offsets = p->coff.data();
    out->calls = p->calls.data();
    out->otu_offsets = p->ooff.data();
    out->otus = p->otus.data();
    out->n_windows = R.nwin;
    out->best = (want & KGX_WANT_BEST) ? p->best.data() : nullptr;
}

/* every shard's hits as kgx_hit, each record written once, straight into its
 * place in the concatenation (kgx_hit.seq = batch index) */
int pool_expand(kgx_pool *p, const PoolRun &R, const char *residues, const uint64_t *seq_offsets)
{
    const uint64_t nh = R.hb[R.K];
    if (nh > p->hits_cap) {
        p->hits.reset(new kgx_hit[nh + nh / 4]); /* grow-only, not initialised */
        p->hits_cap = nh + nh / 4;
    }
    if (!nh)
        return KGX_OK;
    /* pieces of about nh / (4 T) hits, never across a shard, on the pool's
     * expansion threads (the contexts' own threads are idle by now) */
    if (!p->xpool)
        p->xpool.reset(new HostPool(p->expand_threads));
    const uint64_t piece = std::max<uint64_t>(4096, nh / (4ull * p->xpool->size()));
    kgx_hit *base = p->hits.get();
    for (uint32_t i = 0; i < R.K; i++) {
        const uint32_t s0 = R.cuts[i], n = R.cuts[i + 1] - R.cuts[i];
        const uint64_t *ho = R.part[i].r.hit_offsets;
        uint32_t a = 0;
        while (a < n) {
            const uint64_t target = ho[a] + piece;
            uint32_t b = (uint32_t)(std::lower_bound(ho + a + 1, ho + n, target) - ho);
            b = std::min(std::max(b, a + 1), n);
            const kgx_compact_result *cr = &R.part[i];
            kgx_hit *dst = base + R.hb[i] + ho[a];
            p->xpool->submit([cr, residues, seq_offsets, s0, a, b, dst]() -> int {
                return compact_expand(cr, residues, seq_offsets + s0, a, b, s0, dst, true);
            });
            a = b;
        }
    }
    const int rc = p->xpool->wait();
    return rc ? fail(rc, std::string("pool expansion: ") + kgx_last_error()) : KGX_OK;
}

}  // namespace

extern "C" {

int kgx_pool_process_batch(kgx_pool *p, const kgx_params *params, const char *residues,
                           const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want, kgx_result *out)
{
    if (!p || !out)
        return fail(KGX_EINVAL, "null argument");
    PoolRun R;
    int rc = pool_shards(p, params, residues, seq_offsets, n_seq, want, R);
    if (rc)
        return rc;
    if ((want & KGX_WANT_HITS) && (rc = pool_expand(p, R, residues, seq_offsets)))
        return rc;
    pool_fill(p, R, n_seq, want, out);
    out->hits = (want & KGX_WANT_HITS) ? p->hits.get() : nullptr;
    return KGX_OK;
}

int kgx_pool_process_batch_compact(kgx_pool *p, const kgx_params *params, const char *residues,
                                   const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want,
                                   kgx_compact_result *out)
{
    if (!p || !out)
        return fail(KGX_EINVAL, "null argument");
    PoolRun R;
    int rc = pool_shards(p, params, residues, seq_offsets, n_seq, want, R);
    if (rc)
        return rc;
    pool_fill(p, R, n_seq, want, &out->r);
    out->n_chunks = 0;
    out->chunks = nullptr;
    if (!(want & KGX_WANT_HITS))
        return KGX_OK;
    bool all_compact = true;
    for (uint32_t i = 0; i < R.K; i++)
        if (R.part[i].n_chunks == 0 && R.hb[i + 1] > R.hb[i])
            all_compact = false;
    if (!all_compact) {
        if ((rc = pool_expand(p, R, residues, seq_offsets)))
            return rc;
        out->r.hits = p->hits.get();
        return KGX_OK;
    }
    /* every shard's chunks, renumbered into the batch: no record moves */
    p->chunks.clear();
    for (uint32_t i = 0; i < R.K; i++)
        for (uint32_t k = 0; k < R.part[i].n_chunks; k++) {
            kgx_hit_chunk ch = R.part[i].chunks[k];
            ch.seq_begin += R.cuts[i];
            ch.seq_end += R.cuts[i];
            ch.hit_begin += R.hb[i];
            p->chunks.push_back(ch);
        }
    out->n_chunks = (uint32_t)p->chunks.size();
    out->chunks = p->chunks.data();
    return KGX_OK;
}

int kgx_lookup(kgx_ctx *c, kgx_kmap *map, int mode, const kgx_params *params, const char *residues,
               const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want, kgx_result *out, kgx_rollup_result *rollup)
{
    if (!c || !map || !out || !rollup || (!seq_offsets && n_seq))
        return fail(KGX_EINVAL, "null argument");
    if (want & (KGX_WANT_HITS | KGX_WANT_OTU))
        return fail(KGX_EINVAL, "lookup: want within KGX_WANT_CALLS | KGX_WANT_BEST (the hits stay on the device)");
    if (kgx_kmap_device(map) != kgx_image_device(c->img))
        return fail(KGX_EINVAL, "lookup: the map is on another device than the context");
    for (uint32_t s = 0; s < n_seq; s++)
        if (seq_offsets[s + 1] < seq_offsets[s])
            return fail(KGX_EINVAL, "seq_offsets not monotone");
    bool small = false;
    int rc = lookup_small(c, map, mode, params, residues, seq_offsets, n_seq, want, out, &small);
    if (small) {
        if (!rc)
            rc = rollup_finish(map, c, mode, rollup);
        if (rc)
            (void)hipStreamSynchronize(c->stream);
        return rc;
    }
    if (!rc)
        rc = one_pass_enqueue(c, params, residues, seq_offsets, n_seq, want, nullptr, nullptr);
    if (!rc)
        rc = collect_counts_enqueue(c, want);
    if (!rc)
        rc = rollup_enqueue(map, c, mode);
    if (!rc) {
        const uint64_t reruns = c->nul_reruns;
        rc = one_pass_collect(c, params, residues, seq_offsets, n_seq, want, out);
        if (!rc && c->nul_reruns != reruns) /* the pass ran again, staged: so does its rollup */
            rc = rollup_enqueue(map, c, mode);
    }
    if (!rc)
        rc = rollup_finish(map, c, mode, rollup);
    if (rc)
        (void)hipStreamSynchronize(c->stream); /* nothing of the call left running */
    return rc;
}

int kgx_pool_lookup(kgx_pool *p, kgx_kmap *const *maps, uint32_t n_maps, int mode, const kgx_params *params,
                    const char *residues, const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want,
                    kgx_result *out, kgx_rollup_result *rollup)
{
    if (!p || !out || !rollup || !maps || n_maps == 0 || (!seq_offsets && n_seq))
        return fail(KGX_EINVAL, "null argument");
    if (want & (KGX_WANT_HITS | KGX_WANT_OTU))
        return fail(KGX_EINVAL, "pool lookup: want within KGX_WANT_CALLS | KGX_WANT_BEST (the hits stay on the device)");
    for (uint32_t s = 0; s < n_seq; s++)
        if (seq_offsets[s + 1] < seq_offsets[s])
            return fail(KGX_EINVAL, "seq_offsets not monotone");
    /* each context's map: the one on its device */
    const std::vector<uint32_t> run = p->runners(2 * p->per_device);
    const uint32_t K = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)run.size(), n_seq));
    std::vector<kgx_kmap *> mine(K, nullptr);
    {
        std::vector<int32_t> cdev(K), mdev(n_maps), pick(K);
        for (uint32_t i = 0; i < K; i++)
            cdev[i] = kgx_image_device(p->ctxs[run[i]]->img);
        for (uint32_t j = 0; j < n_maps; j++)
            mdev[j] = maps[j] ? kgx_kmap_device(maps[j]) : -1;
        int rc = kgx_pool_map_select(cdev.data(), K, mdev.data(), n_maps, pick.data());
        if (rc)
            return rc;
        for (uint32_t i = 0; i < K; i++)
            mine[i] = maps[pick[i]];
    }
    /* residue shares: a device's first and last shards half the others'.
     * Its pipeline fills with the first shard's upload and drains with the
     * last one's score and rollup, the GPU part idle meanwhile; the inner
     * shards overlap both (r5z: even quarters, 175 us fill and 290 us drain
     * of a 2.1-ms call) */
    std::vector<double> share(K, 2.0);
    {
        static const double edge = [] {
            const char *e = std::getenv("KGX_POOL_EDGE_SHARE");
            return e ? std::max(0.05, std::min(8.0, std::atof(e))) : 1.0;
        }();
        std::vector<int> first(64, -1), last(64, -1);
        for (uint32_t i = 0; i < K; i++) {
            const int d = kgx_image_device(p->ctxs[run[i]]->img);
            if (d >= 0 && d < 64) {
                if (first[(size_t)d] < 0)
                    first[(size_t)d] = (int)i;
                last[(size_t)d] = (int)i;
            }
        }
        for (int d = 0; d < 64; d++)
            if (first[(size_t)d] >= 0 && first[(size_t)d] != last[(size_t)d]) {
                share[(size_t)first[(size_t)d]] = edge;
                share[(size_t)last[(size_t)d]] = edge;
            }
    }
    std::vector<uint32_t> cuts(K + 1, 0);
    {
        const uint64_t r0 = n_seq ? seq_offsets[0] : 0, total = n_seq ? seq_offsets[n_seq] - r0 : 0;
        double sum = 0, acc = 0;
        for (double w : share)
            sum += w;
        cuts[K] = n_seq;
        for (uint32_t i = 1; i < K; i++) {
            acc += share[i - 1];
            const uint64_t target = r0 + (uint64_t)((double)total * (acc / sum));
            const uint32_t s = n_seq ? (uint32_t)(std::lower_bound(seq_offsets, seq_offsets + n_seq, target) -
                                                  seq_offsets)
                                     : 0;
            cuts[i] = std::min(n_seq, std::max(cuts[i - 1], s));
        }
    }
    int rc = KGX_OK;
    /* every shard is ONE pass on its context (its hits stay on the device
     * for the rollup: host_chunks 1 for the call), then its rollups */
    std::vector<kgx_result> part(K, kgx_result{});
    std::vector<kgx_rollup_result> ru(K, kgx_rollup_result{});
    static const bool timing = std::getenv("KGX_POOL_TIMING") != nullptr;
    const auto T0 = std::chrono::steady_clock::now();
    std::vector<int> rcs(K, KGX_OK);
    std::vector<std::string> errs(K);
    /* every shard's upload and pass enqueued from this thread, in shard
     * order: the uploads one after another at the link's full rate on the
     * device's upload stream, each shard's pass behind its own upload (an
     * event), and a hardware queue shared by two shards' streams holds them
     * in shard order, so no shard's kernels wait behind a later shard's
     * upload (r5q: per-shard threads enqueueing at once left shard 0's probe
     * behind shard 2's upload).  Each shard's rollup follows its pass on the
     * context's stream (sized by the context's previous rollup); the collects
     * and the rollups' checks then run on the pool's threads. */
    while (p->up_done.size() < K) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        p->up_done.push_back(e);
    }
    for (auto *v : {&p->pass_done, &p->roll_done})
        while (v->size() < K) {
            hipEvent_t e;
            HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            v->push_back(e);
        }
    for (uint32_t i = 0; i < K; i++) {
        kgx_ctx *c = p->ctxs[run[i]];
        const int dev = kgx_image_device(c->img);
        HIP_TRY(hipSetDevice(dev));
        if ((int)p->up_stream.size() <= dev)
            p->up_stream.resize((size_t)dev + 1, nullptr);
        if (!p->up_stream[(size_t)dev]) {
            int least = 0, greatest = 0;
            hipStream_t st = nullptr;
            if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
                hipStreamCreateWithPriority(&st, hipStreamNonBlocking, least) != hipSuccess) {
                (void)hipGetLastError();
                HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            }
            p->up_stream[(size_t)dev] = st;
        }
        /* a shard's sequences on the host path's scorer (option
         * host_score_variant: the wave scorer; the lane scorer's longest
         * chain sets a shard's score time whatever its size) */
        const int sv = c->score_variant;
        if (c->host_score_variant >= 0)
            c->score_variant = c->host_score_variant;
        /* the pass (and its counts' copy) on the device's pass stream, the
         * rollup on its rollup stream behind it; the context's own stream
         * gets nothing (a wait on it could sit in the pass stream's queue) */
        hipStream_t own = c->stream, ps = p->pass_stream[(size_t)dev], ss = p->score_stream[(size_t)dev],
                    rs = p->roll_stream[(size_t)dev];
        c->stream = ps;
        c->score_stream = ss;
        if (!p->lookup_stage)
            p->lookup_stage.reset(new HostPool(std::max(1u, host_cpu_budget())));
        rcs[i] = one_pass_enqueue(c, params, residues, seq_offsets + cuts[i], cuts[i + 1] - cuts[i], want,
                                  p->up_stream[(size_t)dev], p->up_done[i], p->lookup_stage.get());
        c->score_variant = sv;
        c->score_stream = nullptr;
        c->stream = ss; /* the counts and best calls behind the score */
        if (!rcs[i])
            rcs[i] = collect_counts_enqueue(c, want);
        if (!rcs[i] && (hipEventRecord(p->pass_done[i], ss) != hipSuccess ||
                        hipStreamWaitEvent(rs, c->score_gate, 0) != hipSuccess))
            rcs[i] = fail(KGX_EDEVICE, "pool lookup: pass event");
        c->stream = rs; /* the rollup behind the probe */
        if (!rcs[i])
            rcs[i] = rollup_enqueue(mine[i], c, mode);
        if (!rcs[i] && hipEventRecord(p->roll_done[i], rs) != hipSuccess)
            rcs[i] = fail(KGX_EDEVICE, "pool lookup: rollup event");
        c->stream = own;
        if (rcs[i]) {
            errs[i] = kgx_last_error();
            /* the shards enqueued so far still run: drain them before returning
             * (their uploads too, which may still read the caller's pinned
             * residues or the shared staging buffer) */
            for (auto *v : {&p->up_stream, &p->pass_stream, &p->score_stream, &p->roll_stream})
                for (hipStream_t x : *v)
                    if (x)
                        (void)hipStreamSynchronize(x);
            return fail(rcs[i], "pool lookup shard " + std::to_string(i) + ": " + errs[i]);
        }
    }
    p->run(K, [&](uint32_t i) {
        kgx_ctx *c = p->ctxs[run[i]];
        const auto t0 = std::chrono::steady_clock::now();
        const uint64_t reruns = c->nul_reruns;
        if (hipEventSynchronize(p->pass_done[i]) != hipSuccess ||
            hipEventSynchronize(p->roll_done[i]) != hipSuccess) { /* the shard's pass and rollup */
            rcs[i] = fail(KGX_EDEVICE, "pool lookup: rollup wait");
            errs[i] = kgx_last_error();
            return;
        }
        rcs[i] = one_pass_collect(c, params, residues, seq_offsets + cuts[i], cuts[i + 1] - cuts[i], want, &part[i]);
        const auto t1 = std::chrono::steady_clock::now();
        if (!rcs[i] && c->nul_reruns != reruns) /* the pass ran again, staged: so does its rollup */
            rcs[i] = rollup_enqueue(mine[i], c, mode);
        if (!rcs[i])
            rcs[i] = rollup_finish(mine[i], c, mode, &ru[i]);
        if (timing) {
            const auto t2 = std::chrono::steady_clock::now();
            auto us = [&](std::chrono::steady_clock::time_point a) {
                return std::chrono::duration<double, std::micro>(a - T0).count();
            };
            std::fprintf(stderr, "[pool] lookup shard %u: batch %.1f-%.1f us, rollup -%.1f us\n", i, us(t0), us(t1),
                         us(t2));
        }
        if (rcs[i])
            errs[i] = kgx_last_error();
    });
    for (uint32_t i = 0; i < K; i++)
        if (rcs[i])
            return fail(rcs[i], "pool lookup shard " + std::to_string(i) + ": " + errs[i]);
    /* concatenation in input order: offsets, calls, best calls, rows */
    std::vector<uint64_t> hb(K + 1, 0), cb(K + 1, 0), rb(K + 1, 0);
    uint64_t nwin = 0, nev = 0;
    for (uint32_t i = 0; i < K; i++) {
        const uint32_t n = cuts[i + 1] - cuts[i];
        hb[i + 1] = hb[i] + part[i].hit_offsets[n];
        cb[i + 1] = cb[i] + part[i].call_offsets[n];
        rb[i + 1] = rb[i] + ru[i].offsets[n];
        nwin += part[i].n_windows;
        nev += ru[i].n_events;
    }
    const bool want_best = (want & KGX_WANT_BEST) != 0;
    p->hoff.resize((size_t)n_seq + 1);
    p->coff.resize((size_t)n_seq + 1);
    p->ooff.assign((size_t)n_seq + 1, 0);
    p->roff.resize((size_t)n_seq + 1);
    p->hoff[0] = p->coff[0] = p->roff[0] = 0;
    p->calls.resize(cb[K]);
    p->best.resize(want_best ? n_seq : 0);
    p->rows.resize(rb[K]);
    p->run(K, [&](uint32_t i) {
        const uint32_t s0 = cuts[i], n = cuts[i + 1] - cuts[i];
        for (uint32_t s = 1; s <= n; s++) {
            p->hoff[s0 + s] = hb[i] + part[i].hit_offsets[s];
            p->coff[s0 + s] = cb[i] + part[i].call_offsets[s];
            p->roff[s0 + s] = rb[i] + ru[i].offsets[s];
        }
        if (cb[i + 1] > cb[i])
            std::memcpy(p->calls.data() + cb[i], part[i].calls, (cb[i + 1] - cb[i]) * sizeof(kgx_call));
        if (rb[i + 1] > rb[i])
            std::memcpy(p->rows.data() + rb[i], ru[i].rows, (rb[i + 1] - rb[i]) * sizeof(kgx_rollup_row));
        if (want_best && n)
            std::memcpy(p->best.data() + s0, part[i].best, n * sizeof(kgx_best_call));
    });
    out->n_seq = n_seq;
    out->hit_offsets = p->hoff.data();
    out->hits = nullptr;
    out->call_offsets = p->coff.data();
    out->calls = p->calls.data();
    out->otu_offsets = p->ooff.data();
    out->otus = nullptr;
    out->n_windows = nwin;
    out->best = want_best ? p->best.data() : nullptr;
    rollup->n_seq = n_seq;
    rollup->offsets = p->roff.data();
    rollup->rows = p->rows.data();
    rollup->n_events = nev;
    return KGX_OK;
}

}  // extern "C"
