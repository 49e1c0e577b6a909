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
#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kgx_rt.h"

using namespace kgx;

struct kgx_pool {
    std::vector<kgx_ctx *> ctxs;
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
    std::vector<kgx_hit> hits;
    std::vector<kgx_call> calls;
    std::vector<kgx_otu> otus;
    std::vector<kgx_best_call> best;

    void worker(uint32_t i)
    {
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
    for (uint32_t i = 0; i < n_ctx; i++) {
        kgx_ctx *c = nullptr;
        int rc = images[i % n_images] ? kgx_ctx_create(images[i % n_images], &c) : fail(KGX_EINVAL, "null image");
        if (rc) {
            for (auto *x : p->ctxs)
                kgx_ctx_destroy(x);
            delete p;
            return rc;
        }
        p->ctxs.push_back(c);
    }
    for (uint32_t i = 0; i < n_ctx; i++)
        p->threads.emplace_back([p, i] { p->worker(i); });
    *out = p;
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
    delete p;
    return KGX_OK;
}

uint32_t kgx_pool_size(const kgx_pool *p) { return p ? (uint32_t)p->ctxs.size() : 0; }

kgx_ctx *kgx_pool_ctx(kgx_pool *p, uint32_t i) { return p && i < p->ctxs.size() ? p->ctxs[i] : nullptr; }

int kgx_pool_process_batch(kgx_pool *p, const kgx_params *params, const char *residues,
                           const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want, kgx_result *out)
{
    if (!p || !out || (!seq_offsets && n_seq))
        return fail(KGX_EINVAL, "null argument");
    for (uint32_t s = 0; s < n_seq; s++)
        if (seq_offsets[s + 1] < seq_offsets[s])
            return fail(KGX_EINVAL, "seq_offsets not monotone");
    const uint32_t K = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)p->ctxs.size(), n_seq));
    std::vector<uint32_t> cuts(K + 1);
    int rc = kgx_shard_cuts(seq_offsets, n_seq, K, cuts.data());
    if (rc)
        return rc;

    /* phase 1: every shard on its own context, all at once.  A shard's
     * offsets stay absolute: kgx_process_batch reads residues from
     * seq_offsets[first] on. */
    std::vector<kgx_result> part(K);
    std::vector<int> rcs(K, KGX_OK);
    std::vector<std::string> errs(K);
    p->run(K, [&](uint32_t i) {
        rcs[i] = kgx_process_batch(p->ctxs[i], params, residues, seq_offsets + cuts[i], cuts[i + 1] - cuts[i],
                                   want, &part[i]);
        if (rcs[i])
            errs[i] = kgx_last_error();
    });
    for (uint32_t i = 0; i < K; i++)
        if (rcs[i])
            return fail(rcs[i], "pool shard " + std::to_string(i) + ": " + errs[i]);

    /* phase 2: offsets of the concatenation, then every shard copies its part */
    const bool need_hits = (want & KGX_WANT_HITS) != 0;
    const bool want_best = (want & KGX_WANT_BEST) != 0;
    std::vector<uint64_t> hb(K + 1, 0), cb(K + 1, 0), ob(K + 1, 0);
    uint64_t nwin = 0;
    for (uint32_t i = 0; i < K; i++) {
        const uint32_t n = cuts[i + 1] - cuts[i];
        hb[i + 1] = hb[i] + part[i].hit_offsets[n];
        cb[i + 1] = cb[i] + part[i].call_offsets[n];
        ob[i + 1] = ob[i] + part[i].otu_offsets[n];
        nwin += part[i].n_windows;
    }
    p->hoff.resize((size_t)n_seq + 1);
    p->coff.resize((size_t)n_seq + 1);
    p->ooff.resize((size_t)n_seq + 1);
    p->hits.resize(need_hits ? hb[K] : 0);
    p->calls.resize(cb[K]);
    p->otus.resize(ob[K]);
    p->best.resize(want_best ? n_seq : 0);
    p->hoff[0] = p->coff[0] = p->ooff[0] = 0;
    p->run(K, [&](uint32_t i) {
        const kgx_result &r = part[i];
        const uint32_t s0 = cuts[i], n = cuts[i + 1] - cuts[i];
        for (uint32_t s = 1; s <= n; s++) {
            p->hoff[s0 + s] = hb[i] + r.hit_offsets[s];
            p->coff[s0 + s] = cb[i] + r.call_offsets[s];
            p->ooff[s0 + s] = ob[i] + r.otu_offsets[s];
        }
        const uint64_t nh = hb[i + 1] - hb[i];
        if (need_hits && nh) {
            kgx_hit *dst = p->hits.data() + hb[i];
            std::memcpy(dst, r.hits, nh * sizeof(kgx_hit));
            for (uint64_t h = 0; h < nh; h++)
                dst[h].seq += s0; /* batch index, not shard index */
        }
        if (cb[i + 1] > cb[i])
            std::memcpy(p->calls.data() + cb[i], r.calls, (cb[i + 1] - cb[i]) * sizeof(kgx_call));
        if (ob[i + 1] > ob[i])
            std::memcpy(p->otus.data() + ob[i], r.otus, (ob[i + 1] - ob[i]) * sizeof(kgx_otu));
        if (want_best && n)
            std::memcpy(p->best.data() + s0, r.best, n * sizeof(kgx_best_call));
    });
    out->n_seq = n_seq;
    out->hit_offsets = p->hoff.data();
    out->hits = need_hits ? p->hits.data() : nullptr;
    out->call_offsets = p->coff.data();
    out->calls = p->calls.data();
    out->otu_offsets = p->ooff.data();
    out->otus = p->otus.data();
    out->n_windows = nwin;
    out->best = want_best ? p->best.data() : nullptr;
    return KGX_OK;
}

}  // extern "C"
