/*
 * kgx_svc.cpp -- the resident call service: KmerGuts::process_aa_seq for one
 * sequence without a kernel launch per call.
 *
 * The reference's worker pool calls process_aa_seq once per sequence from T
 * threads, one KmerGuts each (threadpool.cc:18-44, lookup_request.cc:153-172,
 * kguts.cc:888-908).  A launch per call costs ~6 us of host time inside the
 * runtime and those launches serialise across the pool's threads, so the pool
 * topped out at 170K calls/s whatever T (r3g).  Here workgroups of svc_kernel
 * (kgx_fused.hip) stay resident, one per slot; a caller takes a free slot,
 * writes its residues (16-B chunks of 12 residues tagged with the request
 * number, so the polling wave can take the first ones with the header line),
 * length, want mask and parameters into the slot (device memory through a
 * large BAR, else mapped host memory), stores the slot's request number, and
 * spins until the
 * device stores the same number into the slot's done word, behind the hit
 * and call records (fused_small_body: probe, ordered compaction, wave
 * scorer).  No runtime call is on a call's path.
 *
 * Instances: the kernel leaves life_us after its start (a bound on how long
 * it holds its hardware queue, which other streams may share) or on stop.
 * The host keeps two instances enqueued on the service's stream while calls
 * arrive, so when one leaves the next is already dispatched; callers top the
 * queue up (hipEventQuery on the oldest, at most every 200 us) and, should a
 * request wait more than 100 us, at once.  Without calls nothing is
 * enqueued, so the service leaves the GPU within 2 x life_us of the last call.  A
 * request written while an instance was leaving stays pending in its slot and
 * the next instance serves it (a workgroup starts from the slot's done word).
 * kgx_image_close / set_layout / set_filter stop the service first, and an
 * atexit hook stops every live one, so no instance outlives the process.
 */
#include <hip/hip_runtime.h>

#include <atomic>
#include <cctype>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <set>
#include <string>
#include <thread>

#if defined(__x86_64__)
#include <emmintrin.h>
#endif
#include <sys/prctl.h>
#include <time.h>

#include "kgx_rt.h"

namespace kgx {

struct SvcState {
    int device = 0;
    uint32_t slots = 32;
    uint64_t idle_us = 1000, life_us = 1000;
    hipStream_t stream = nullptr;
    char *host = nullptr; /* one mapped, coherent block: hdr | out | dbg | res | hits | calls */
    /* large-BAR devices: the request side (hdr | res) in fine-grained device
     * memory instead, which the host writes through the BAR (posted stores)
     * and the polling wave reads from HBM, not across PCIe; the replies stay
     * in host memory, where the host polls them */
    char *reqmem = nullptr;
    SvcSlotHdr *hdr = nullptr;
    SvcSlotOut *out = nullptr;
    SvcSlotDbg *dbg = nullptr;
    uint8_t *res = nullptr;
    kgx_hit *hits = nullptr;
    kgx_call *calls = nullptr;
    kgx_otu *otus = nullptr;
    /* their device addresses */
    SvcSlotHdr *d_hdr = nullptr;
    SvcSlotOut *d_out = nullptr;
    SvcSlotDbg *d_dbg = nullptr;
    uint8_t *d_res = nullptr;
    kgx_hit *d_hits = nullptr;
    kgx_call *d_calls = nullptr;
    kgx_otu *d_otus = nullptr;
    const void *table = nullptr;
    uint64_t num_sigs = 0; /* buckets of the probe table */
    uint32_t home_shift = 0;
    /* the host side of each slot, a line apiece: a call touches only its
     * own slot's line (a pool's threads each settle on a slot of their own,
     * take_slot), never one that every caller writes */
    struct alignas(64) Slot {
        std::atomic<uint32_t> busy{0};
        uint32_t seq = 0;                /* the last request number (its holder's) */
        std::atomic<uint64_t> n_calls{0}; /* calls served through the slot (its holder counts) */
    };
    Slot slot[SVC_MAX_SLOTS];
    std::mutex mu;                    /* instances */
    std::deque<hipEvent_t> running;   /* end of each enqueued instance */
    std::vector<hipEvent_t> spare;
    std::atomic<int64_t> next_check{0};
    std::atomic<uint64_t> n_launches{0}, n_busy{0};
    /* KGX_SVC_DEBUG=1: the device's phase stamps per call, summed (ns):
     * [0] request stored -> done seen on the host (wall), [1..5] the device
     * phases (stamps 0->1 residues, 1->2 probe, 2->3 compaction, 3->4 stores
     * + scorer, and [5] 3->6 the record stores alone) */
    bool debug = false;
    std::atomic<uint64_t> phase_ns[16] = {};
    /* KGX_SVC_SLEEP_US: a caller sleeps this long before it spins for its
     * answer (the device needs >= ~10 us per call), so a pool of spinning
     * callers holds fewer CPUs; 0 = spin only */
    uint32_t sleep_us = 0;
    std::atomic<bool> broken{false}; /* a launch failed or a call timed out: callers take other paths */
    std::atomic<uint64_t> n_abandoned{0}; /* slots given up after a 10-s wait (never handed out again) */
    int priority = 0; /* the stream's priority (hipDeviceGetStreamPriorityRange: lower = higher) */
    /* the probe's loads by 4-lane quads, one 64-B line per window in one
     * instruction for 16 windows (the default), or KGX_SVC_PROBE=thread: a
     * thread's four 16-B loads of its own window's line -- four address
     * translations per line instead of one: probe phase 4.1 vs 3.8 us per
     * 300-aa call over the 114-GB line index (r7c) */
    int quad_probe = 1;
    /* residue chunks the polling wave reads with the header
     * (KGX_SVC_POLL_CHUNKS, at most SVC_POLL_CHUNKS): 28 = 336 residues.
     * Read with the header they save the residues' own round trip after it
     * (host wall per 300-aa call 11.25 vs 11.9 us, r7f); more chunks per
     * poll measured no better (60: 11.3-11.6) */
    uint32_t poll_chunks = 28;
    /* a call unanswered this long marks the service broken (KGX_SVC_TIMEOUT_MS,
     * default 10 s) */
    int64_t timeout_ns = 10000000000ll;
    /* test injection (KGX_SVC_TEST_DROP=n): the next n requests are written
     * but never posted, as if the device had stalled on them */
    std::atomic<int> drop{0};
    bool leaked = false; /* drain timed out: the state stays allocated */
};

namespace {

std::mutex g_live_mu;
std::set<SvcState *> g_live;
bool g_atexit = false;

int64_t now_ns()
{
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

constexpr size_t align64(size_t x) { return (x + 63) & ~size_t(63); }

/* a request's residues as the device reads them (kgx_internal.h,
 * SVC_RES_CHUNKS): chunk c = residues [12 c, 12 c + 12) and the request
 * number, one 16-B store each (written, never read, by the host); the bytes
 * from cut to len read 'X' */
inline void put_chunks(uint8_t *dst, const char *seq, uint64_t cut, uint64_t len, uint32_t q)
{
    const uint64_t n = (len + 11) / 12;
    for (uint64_t c = 0; c < n; c++) {
        alignas(16) uint8_t b[16];
        const uint64_t i0 = 12 * c;
        if (i0 + 12 <= cut) {
            std::memcpy(b, seq + i0, 12);
        } else {
            for (uint64_t j = 0; j < 12; j++) {
                const uint64_t i = i0 + j;
                b[j] = i < cut ? (uint8_t)seq[i] : i < len ? (uint8_t)'X' : (uint8_t)0;
            }
        }
        std::memcpy(b + 12, &q, 4);
#if defined(__x86_64__)
        _mm_store_si128(reinterpret_cast<__m128i *>(dst + 16 * c), _mm_load_si128(reinterpret_cast<const __m128i *>(b)));
#else
        std::memcpy(dst + 16 * c, b, 16);
#endif
    }
}

/* orders the host's stores to the request lines before what follows and, for
 * device memory written through the write-combining BAR, pushes them out */
inline void wc_fence()
{
#if defined(__x86_64__)
    __builtin_ia32_sfence();
#else
    std::atomic_thread_fence(std::memory_order_seq_cst);
#endif
}

std::atomic<uint32_t> g_threads{0};

/* the calling thread's number, fixed at its first call: it picks the
 * thread's user shard and its first-choice slot */
uint32_t thread_index()
{
    thread_local uint32_t t = ~0u;
    if (t == ~0u)
        t = g_threads.fetch_add(1, std::memory_order_relaxed);
    return t;
}

/* a caller's hold on the service: shutdown waits until none is left */
struct SvcUse {
    std::atomic<uint32_t> *n = nullptr;
    SvcState *s = nullptr;
    SvcUse() = default;
    SvcUse(const SvcUse &) = delete;
    SvcUse &operator=(const SvcUse &) = delete;
    ~SvcUse()
    {
        if (n)
            n->fetch_sub(1, std::memory_order_release);
    }
};

/* keep two instances enqueued (mu held) */
int top_up(SvcState *s)
{
    while (!s->running.empty()) {
        const hipError_t q = hipEventQuery(s->running.front());
        if (q == hipErrorNotReady)
            break;
        if (q != hipSuccess) {
            s->broken = true;
            return fail(KGX_EDEVICE, std::string("call service: ") + hipGetErrorString(q));
        }
        s->spare.push_back(s->running.front());
        s->running.pop_front();
    }
    while (s->running.size() < 2) {
        hipEvent_t ev = nullptr;
        if (!s->spare.empty()) {
            ev = s->spare.back();
            s->spare.pop_back();
        } else {
            HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        }
        /* wall clock at 100 MHz: 100 ticks per us */
        hipError_t e = launch_svc(s->d_hdr, s->d_out, s->d_dbg, s->d_res, s->d_hits, s->d_calls, s->d_otus, s->slots,
                                  s->table,
                                  s->num_sigs, s->life_us * 100, s->quad_probe, s->stream, s->home_shift,
                                  s->poll_chunks);
        if (e == hipSuccess)
            e = hipEventRecord(ev, s->stream);
        if (e != hipSuccess) {
            s->spare.push_back(ev);
            s->broken = true;
            return fail(KGX_EDEVICE, std::string("call service launch: ") + hipGetErrorString(e));
        }
        s->running.push_back(ev);
        s->n_launches++;
    }
    return KGX_OK;
}

/* every workgroup of every enqueued instance leaves; the slots stay.  No
 * unbounded runtime wait: every slot's stop word is raised and the host waits
 * -- at most 2 s -- until each slot's workgroups of every instance launched
 * have counted themselves out (SvcSlotOut.left); only then is the stream
 * synchronised, which returns at once.  false: some workgroup did not leave
 * (a stalled instance), and the caller must not free what it may touch. */
bool drain(SvcState *s)
{
    std::lock_guard<std::mutex> lk(s->mu);
    for (uint32_t i = 0; i < s->slots; i++)
        __atomic_store_n(&s->hdr[i].stop, 1u, __ATOMIC_RELEASE);
    wc_fence();
    const uint32_t launched = (uint32_t)s->n_launches.load();
    const int64_t t0 = now_ns();
    for (uint32_t i = 0; i < s->slots; i++)
        while (__atomic_load_n(&s->out[i].left, __ATOMIC_ACQUIRE) != launched) {
            if (now_ns() - t0 > 2000000000ll)
                return false;
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    (void)hipStreamSynchronize(s->stream);
    for (hipEvent_t e : s->running)
        s->spare.push_back(e);
    s->running.clear();
    for (uint32_t i = 0; i < s->slots; i++)
        __atomic_store_n(&s->hdr[i].stop, 0u, __ATOMIC_RELEASE);
    wc_fence();
    return true;
}

std::atomic<uint64_t> g_leaked{0};

void destroy(SvcState *s)
{
    if (!s)
        return;
    {
        std::lock_guard<std::mutex> lk(g_live_mu);
        g_live.erase(s);
    }
    (void)hipSetDevice(s->device);
    if (s->stream && !drain(s)) {
        /* an instance that never left may still read the slots and write
         * the replies: keep its memory and stream (leaked, counted) */
        s->leaked = true;
        g_leaked++;
        return;
    }
    for (hipEvent_t e : s->spare)
        (void)hipEventDestroy(e);
    if (s->stream)
        (void)hipStreamDestroy(s->stream);
    if (s->reqmem)
        (void)hipFree(s->reqmem);
    if (s->host)
        (void)hipHostFree(s->host);
    delete s;
}

/* Process exit with services alive (the reference's server ends from a
 * signal with its workers live, kserver.cc:206-214).  No runtime call here:
 * by the time exit handlers run, the calling thread's thread_local objects
 * are gone, and a profiler's HIP wrappers keep theirs there (r5a: rocprofv3
 * aborted in hipStreamSynchronize from this hook, "get_stream_stack() must be
 * non nullptr", and the process hung).  Every slot's stop word is raised by a
 * plain store, and the hook waits -- at most 1 s -- until each slot's
 * workgroups of every instance launched have counted themselves out
 * (SvcSlotOut.left, a system-scope add in svc_kernel), so no persistent grid
 * outlives the process.  Streams and pinned memory go with the process. */
void stop_all_at_exit()
{
    std::lock_guard<std::mutex> lk(g_live_mu);
    for (SvcState *s : g_live)
        for (uint32_t i = 0; i < s->slots; i++)
            __atomic_store_n(&s->hdr[i].stop, 1u, __ATOMIC_RELEASE);
    wc_fence();
    const int64_t t0 = now_ns();
    for (SvcState *s : g_live) {
        const uint32_t launched = (uint32_t)s->n_launches.load();
        for (uint32_t i = 0; i < s->slots; i++)
            while (__atomic_load_n(&s->out[i].left, __ATOMIC_ACQUIRE) != launched && now_ns() - t0 < 1000000000ll)
                std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

int create(kgx_image *img, uint32_t slots, uint64_t idle_us, uint64_t life_us, SvcState **out)
{
    if (img->layout != KGX_LAYOUT_PACKED16 || !img->d_packed)
        return fail(KGX_EBUSY, "call service: PACKED16 images only");
    HIP_TRY(hipSetDevice(img->device));
    SvcState *s = new SvcState;
    s->device = img->device;
    s->slots = slots;
    s->idle_us = idle_us;
    s->life_us = life_us;
    s->table = img->probe_table();
    s->num_sigs = img->probe_buckets();
    s->home_shift = img->home_shift();
    const size_t b_hdr = align64(slots * sizeof(SvcSlotHdr)), b_out = align64(slots * sizeof(SvcSlotOut)),
                 b_dbg = align64(slots * sizeof(SvcSlotDbg)), b_res = align64((size_t)slots * SVC_RES_STRIDE),
                 b_hits = align64((size_t)slots * FUSED_MAX_WINDOWS * sizeof(kgx_hit)),
                 b_calls = align64((size_t)slots * FUSED_MAX_WINDOWS * sizeof(kgx_call)),
                 b_otus = align64((size_t)slots * FUSED_MAX_WINDOWS * sizeof(kgx_otu));
    const size_t total = b_hdr + b_out + b_dbg + b_res + b_hits + b_calls + b_otus;
    void *h = nullptr, *d = nullptr;
    hipError_t e = hipHostMalloc(&h, total, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess)
        e = hipHostGetDevicePointer(&d, h, 0);
    if (e == hipSuccess) {
        /* the service's stream gets a hardware queue of its own: a queue is a
         * FIFO, so a batch kernel whose stream shared the service's queue
         * waited behind the enqueued persistent instances (r3z: 2,000-protein
         * batches beside 8 service callers, median 3.0 ms / max 28 ms vs 1.3 ms
         * alone).  The runtime keeps a queue pool per stream priority, so the
         * high-priority stream never shares with the contexts' (normal)
         * streams; KGX_SVC_PRIORITY=normal restores the old placement. */
        int least = 0, greatest = 0;
        const char *pe = std::getenv("KGX_SVC_PRIORITY");
        const bool normal = pe && std::string(pe) == "normal";
        if (!normal && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && greatest != least)
            e = hipStreamCreateWithPriority(&s->stream, hipStreamNonBlocking, greatest);
        else
            e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
        s->priority = normal ? 0 : greatest;
    }
    s->host = static_cast<char *>(h);
    if (e != hipSuccess) {
        destroy(s);
        return fail(KGX_EDEVICE, std::string("call service: ") + hipGetErrorString(e));
    }
    /* the residue chunks too: a chunk's tag must never match a request of
     * this service before the host wrote it, and a new service's request
     * numbers start again at 1 (on memory an earlier service may have used) */
    std::memset(h, 0, b_hdr + b_out + b_dbg + b_res);
    const char *dbg_env = std::getenv("KGX_SVC_DEBUG");
    s->debug = dbg_env && std::atoi(dbg_env) != 0;
    if (const char *pr = std::getenv("KGX_SVC_PROBE"))
        s->quad_probe = std::string(pr) != "thread";
    if (const char *pc = std::getenv("KGX_SVC_POLL_CHUNKS"))
        s->poll_chunks = (uint32_t)std::min<long>(SVC_POLL_CHUNKS, std::max(0L, std::atol(pc)));
    if (const char *sl = std::getenv("KGX_SVC_SLEEP_US"))
        s->sleep_us = (uint32_t)std::max(0, std::atoi(sl));
    if (const char *to = std::getenv("KGX_SVC_TIMEOUT_MS"))
        s->timeout_ns = std::max<int64_t>(1, std::atoll(to)) * 1000000ll;
    if (const char *dr = std::getenv("KGX_SVC_TEST_DROP"))
        s->drop = std::max(0, std::atoi(dr));
    char *hp = static_cast<char *>(h), *dp = static_cast<char *>(d);
    s->hdr = reinterpret_cast<SvcSlotHdr *>(hp);
    s->d_hdr = reinterpret_cast<SvcSlotHdr *>(dp);
    s->out = reinterpret_cast<SvcSlotOut *>(hp + b_hdr);
    s->d_out = reinterpret_cast<SvcSlotOut *>(dp + b_hdr);
    s->dbg = reinterpret_cast<SvcSlotDbg *>(hp + b_hdr + b_out);
    s->d_dbg = reinterpret_cast<SvcSlotDbg *>(dp + b_hdr + b_out);
    const size_t o_res = b_hdr + b_out + b_dbg;
    s->res = reinterpret_cast<uint8_t *>(hp + o_res);
    s->d_res = reinterpret_cast<uint8_t *>(dp + o_res);
    int large_bar = 0;
    const char *dm = std::getenv("KGX_SVC_DEVMEM");
    if ((!dm || std::atoi(dm) != 0) &&
        hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, img->device) == hipSuccess && large_bar) {
        void *r = nullptr;
        /* on the service's stream: a device-wide synchronisation would wait
         * for every batch in flight on the device */
        if (hipExtMallocWithFlags(&r, b_hdr + b_res, hipDeviceMallocFinegrained) == hipSuccess &&
            hipMemsetAsync(r, 0, b_hdr + b_res, s->stream) == hipSuccess &&
            hipStreamSynchronize(s->stream) == hipSuccess) {
            s->reqmem = static_cast<char *>(r); /* one address for the host and the device */
            s->hdr = s->d_hdr = reinterpret_cast<SvcSlotHdr *>(s->reqmem);
            s->res = s->d_res = reinterpret_cast<uint8_t *>(s->reqmem + b_hdr);
        } else {
            (void)hipGetLastError();
            if (r)
                (void)hipFree(r);
        }
    }
    s->hits = reinterpret_cast<kgx_hit *>(hp + o_res + b_res);
    s->d_hits = reinterpret_cast<kgx_hit *>(dp + o_res + b_res);
    s->calls = reinterpret_cast<kgx_call *>(hp + o_res + b_res + b_hits);
    s->d_calls = reinterpret_cast<kgx_call *>(dp + o_res + b_res + b_hits);
    s->otus = reinterpret_cast<kgx_otu *>(hp + o_res + b_res + b_hits + b_calls);
    s->d_otus = reinterpret_cast<kgx_otu *>(dp + o_res + b_res + b_hits + b_calls);
    {
        std::lock_guard<std::mutex> lk(g_live_mu);
        g_live.insert(s);
        if (!g_atexit) {
            std::atexit(stop_all_at_exit);
            g_atexit = true;
        }
    }
    *out = s;
    return KGX_OK;
}

constexpr uint32_t kShards = sizeof(kgx_image::svc_users) / sizeof(kgx_image::svc_users[0]);

/* the image's service, created on first use with its configuration, held
 * by `use` until the caller returns.  No lock on the way in: the caller
 * counts itself in its shard, then reads the service pointer; shutdown
 * clears the pointer, then waits for every shard to read 0.  Both pairs are
 * sequentially consistent, so a caller either sees the pointer cleared (and
 * takes the lock, behind the shutdown) or is counted before shutdown looks. */
int enter(kgx_image *img, SvcUse &use)
{
    std::atomic<uint32_t> &n = img->svc_users[thread_index() % kShards].n;
    for (;;) {
        n.fetch_add(1, std::memory_order_seq_cst);
        if (SvcState *s = img->svc.load(std::memory_order_seq_cst)) {
            use.n = &n;
            use.s = s;
            return KGX_OK;
        }
        n.fetch_sub(1, std::memory_order_release);
        std::lock_guard<std::mutex> lk(img->svc_mu);
        if (!img->svc.load(std::memory_order_relaxed)) {
            /* KGX_SVC_LIFE_US: a default for experiments, for images that
             * kgx_svc_config never configured */
            uint64_t life = img->svc_life_us;
            if (const char *e = std::getenv("KGX_SVC_LIFE_US"); e && !img->svc_configured)
                life = std::max<uint64_t>(10, std::strtoull(e, nullptr, 10));
            SvcState *s = nullptr;
            if (int rc = create(img, img->svc_slots, img->svc_idle_us, life, &s))
                return rc;
            img->svc.store(s, std::memory_order_seq_cst);
        }
    }
}

/* detach and free the image's service (svc_mu held): new callers create a
 * fresh one after the lock is released; callers already inside keep the old
 * one's instances serving them until they return, then it is drained and
 * freed */
void shutdown_locked(kgx_image *img)
{
    SvcState *s = img->svc.exchange(nullptr, std::memory_order_seq_cst);
    if (!s)
        return;
    for (;;) {
        uint32_t inside = 0;
        for (uint32_t i = 0; i < kShards; i++)
            inside += img->svc_users[i].n.load(std::memory_order_seq_cst);
        if (!inside)
            break;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    destroy(s);
}

/* the thread's own slot when it is free (a pool of at most `slots` threads
 * keeps one slot each), else the first free one after it */
bool take_slot(SvcState *s, uint32_t &slot)
{
    const uint32_t first = thread_index() % s->slots;
    for (uint32_t k = 0; k < s->slots; k++) {
        const uint32_t i = (first + k) % s->slots;
        std::atomic<uint32_t> &b = s->slot[i].busy;
        if (b.load(std::memory_order_relaxed) == 0 && b.exchange(1, std::memory_order_acquire) == 0) {
            slot = i;
            return true;
        }
    }
    return false;
}

void give_slot(SvcState *s, uint32_t slot) { s->slot[slot].busy.store(0, std::memory_order_release); }

}  // namespace

void svc_shutdown(kgx_image *img)
{
    std::lock_guard<std::mutex> lk(img->svc_mu);
    shutdown_locked(img);
}

std::unique_lock<std::mutex> svc_shutdown_hold(kgx_image *img)
{
    std::unique_lock<std::mutex> lk(img->svc_mu);
    shutdown_locked(img);
    return lk;
}

}  // namespace kgx

using namespace kgx;

extern "C" {

int kgx_svc_config(kgx_image *img, uint32_t slots, uint32_t idle_us, uint32_t life_us)
{
    if (!img)
        return fail(KGX_EINVAL, "null image");
    if (slots < 1 || slots > SVC_MAX_SLOTS || idle_us < 10 || life_us < idle_us)
        return fail(KGX_EINVAL, "call service: 1..64 slots, idle_us >= 10, life_us >= idle_us");
    /* one critical section: no call in between starts a service with the old settings */
    std::lock_guard<std::mutex> lk(img->svc_mu);
    shutdown_locked(img);
    img->svc_configured = true;
    img->svc_slots = slots;
    img->svc_idle_us = idle_us;
    img->svc_life_us = life_us;
    return KGX_OK;
}

int kgx_svc_stop(kgx_image *img)
{
    if (!img)
        return fail(KGX_EINVAL, "null image");
    svc_shutdown(img);
    return KGX_OK;
}

int kgx_svc_stat(kgx_image *img, const char *name, uint64_t *value)
{
    if (!img || !name || !value)
        return fail(KGX_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(img->svc_mu);
    const SvcState *s = img->svc.load(std::memory_order_acquire);
    const std::string n(name);
    if (n == "slots")
        *value = img->svc_slots;
    else if (n == "calls")
    {
        uint64_t c = 0;
        for (uint32_t i = 0; s && i < s->slots; i++)
            c += s->slot[i].n_calls.load(std::memory_order_relaxed);
        *value = c;
    }
    else if (n == "launches")
        *value = s ? s->n_launches.load() : 0;
    else if (n == "busy")
        *value = s ? s->n_busy.load() : 0;
    else if (n == "abandoned") /* slots given up after a 10-s wait */
        *value = s ? s->n_abandoned.load() : 0;
    else if (n == "broken") /* 1: the service turns every call away until kgx_svc_stop */
        *value = s && s->broken ? 1 : 0;
    else if (n == "priority") /* the service stream's priority + 100 (lower = higher priority) */
        *value = s ? (uint64_t)(s->priority + 100) : 0;
    else if (n == "leaked") /* services whose drain timed out (their memory kept), process-wide */
        *value = g_leaked.load();
    else if (n == "devmem") /* 1: requests travel through device memory (large BAR) */
        *value = s && s->reqmem ? 1 : 0;
    else if ((n.size() == 8 || n.size() == 9) && n.compare(0, 7, "phase_n") == 0 &&
             std::isdigit((unsigned char)n[7]) && (n.size() == 8 || std::isdigit((unsigned char)n[8])) &&
             std::stoul(n.substr(7)) < 16) /* "phase_n0".."phase_n15" */
        *value = s ? s->phase_ns[std::stoul(n.substr(7))].load() : 0;
    else
        return fail(KGX_EINVAL, "unknown service statistic " + n);
    return KGX_OK;
}

int kgx_svc_call(kgx_image *img, const kgx_params *params, const char *seq, uint64_t len, uint32_t want,
                 kgx_hit *hits, uint64_t hits_cap, uint64_t *n_hits, kgx_call *calls, uint64_t calls_cap,
                 uint64_t *n_calls, kgx_otu *otus, uint64_t otus_cap, uint64_t *n_otus)
{
    if (!img || (len && !seq) || !n_hits || !n_calls || ((want & KGX_WANT_OTU) && !n_otus))
        return fail(KGX_EINVAL, "null argument");
    kgx_params p;
    if (params)
        p = *params;
    else
        kgx_params_default(&p);
    /* what fused_small_body serves (the rest takes the batch paths) */
    if (len > SVC_MAX_RES || want == 0 || (want & ~(KGX_WANT_HITS | KGX_WANT_CALLS | KGX_WANT_OTU)) ||
        p.order_constraint != 0 || p.min_hits < 1)
        return fail(KGX_EBUSY, "call service: not a call it serves (length, want mask or parameters)");
    const uint64_t W = windows_of(len);
    if (((want & KGX_WANT_HITS) && hits_cap < W) || ((want & KGX_WANT_CALLS) && calls_cap < W) ||
        ((want & KGX_WANT_OTU) && otus_cap < W))
        return fail(KGX_EINVAL, "call service: result capacity below the sequence's window count");
    if ((want & KGX_WANT_HITS && W && !hits) || (want & KGX_WANT_CALLS && W && !calls) ||
        (want & KGX_WANT_OTU && W && !otus))
        return fail(KGX_EINVAL, "null result buffer");
    SvcUse use;
    int rc = enter(img, use);
    if (rc)
        return rc;
    SvcState *s = use.s;
    if (s->broken)
        return fail(KGX_EBUSY, "call service: unavailable after a launch failure");
    uint32_t slot = 0;
    if (!take_slot(s, slot)) {
        s->n_busy++;
        return fail(KGX_EBUSY, "call service: every slot is in use");
    }
    /* the request: residues (cut at the first NUL as the batch paths do,
     * kguts.cc:792) in 16-B chunks tagged with the request number, then the
     * header, then the request number */
    uint32_t q = s->slot[slot].seq + 1;
    if (q == 0 || q == __atomic_load_n(&s->out[slot].done, __ATOMIC_RELAXED))
        q++;
    s->slot[slot].seq = q;
    const void *z = len ? std::memchr(seq, 0, len) : nullptr;
    const uint64_t keep = z ? (uint64_t)(static_cast<const char *>(z) - seq) : len;
    const uint64_t cut = z && keep ? keep - 1 : keep;
    put_chunks(s->res + (size_t)slot * SVC_RES_STRIDE, seq, cut, len, q);
    SvcSlotHdr &h = s->hdr[slot];
    h.len = (uint32_t)len;
    h.want = want;
    h.prm = p;
    h.debug = s->debug ? 1u : 0u;
    /* device memory is written through a write-combining BAR mapping: the
     * fences order the request's bytes before its number and push it out */
    if (s->reqmem)
        wc_fence();
    const bool post = s->drop.load(std::memory_order_relaxed) <= 0 || s->drop.fetch_sub(1) <= 0;
    if (post) {
        __atomic_store_n(&h.copy, q, __ATOMIC_RELEASE);
        __atomic_store_n(&h.req, q, __ATOMIC_RELEASE);
    }
    if (s->reqmem)
        wc_fence();
    /* keep instances enqueued (cheap: one clock read unless 200 us passed) */
    const int64_t t0 = now_ns();
    if (t0 >= s->next_check.load(std::memory_order_relaxed)) {
        std::unique_lock<std::mutex> lk(s->mu, std::try_to_lock);
        if (lk.owns_lock()) {
            s->next_check.store(t0 + 200000, std::memory_order_relaxed);
            if ((rc = top_up(s))) {
                give_slot(s, slot); /* nothing will serve it; the holder's next request overwrites it */
                return rc;
            }
        }
    }
    const volatile uint32_t *done = &s->out[slot].done;
    if (s->sleep_us) {
        thread_local bool slack = false;
        if (!slack) { /* hrtimer sleeps of a few us need a small timer slack */
            (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
            slack = true;
        }
        const struct timespec ts = {0, (long)s->sleep_us * 1000};
        nanosleep(&ts, nullptr);
    }
    bool nudged = false;
    for (uint32_t spin = 1; *done != q; spin++) {
        if ((spin & 1023u) == 0) {
            const int64_t dt = now_ns() - t0;
            if (!nudged && dt > 100000) { /* 100 us: no instance is serving the slots */
                std::lock_guard<std::mutex> lk(s->mu);
                if ((rc = top_up(s))) {
                    give_slot(s, slot);
                    return rc;
                }
                nudged = true;
            }
            if (dt > s->timeout_ns) {
                /* 10 s: the slot is abandoned (a late answer could still land
                 * in it, so it is never handed out again) and the service
                 * turns every later call away, to the batch paths, until
                 * kgx_svc_stop / kgx_svc_config replaces it */
                s->n_abandoned++;
                s->broken = true;
                return fail(KGX_EDEVICE, "call service: no answer within the timeout (10 s)");
            }
            if (s->broken.load(std::memory_order_relaxed)) {
                /* another call found the service broken: do not wait out the
                 * timeout too (the slot is abandoned the same way) */
                s->n_abandoned++;
                return fail(KGX_EBUSY, "call service: broken while this call waited");
            }
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (s->debug) {
        const uint64_t *st = s->dbg[slot].stamp;
        s->phase_ns[0] += (uint64_t)(now_ns() - t0);
        for (int k = 1; k <= 4; k++)
            s->phase_ns[k] += (st[k] - st[k - 1]) * 10; /* 100 MHz ticks */
        s->phase_ns[5] += (st[6] - st[3]) * 10; /* compaction end -> thread 0's record stores issued */
        s->phase_ns[14] += (st[5] - st[4]) * 10; /* the system fence: the results' host stores drained */
        if (want & KGX_WANT_OTU) {
            s->phase_ns[6] += (st[4] - st[7]) * 10; /* the OTU tally alone */
            s->phase_ns[7] += (st[4] - st[8]) * 10; /* ... its sort by count */
            s->phase_ns[15] += st[17] - st[16]; /* the sort's shader clock cycles */
        } else if (st[9] >= st[6] && st[9] <= st[4]) {
            s->phase_ns[6] += (st[9] - st[6]) * 10; /* the scorer's first 64-hit chunk */
            s->phase_ns[7] += (st[4] - st[9]) * 10; /* its other chunks and the final flush */
        }
        s->phase_ns[8] += st[10] * 1000; /* probe rounds (x1000: read back per call like the times) */
        if (st[11] >= st[1] && st[11] <= st[2])
            s->phase_ns[9] += (st[11] - st[1]) * 10; /* the probe's first round */
        if (st[12] >= st[1] && st[13] >= st[12] && st[13] <= st[11]) {
            s->phase_ns[10] += (st[12] - st[1]) * 10; /* keys and homes */
            s->phase_ns[11] += (st[13] - st[12]) * 10; /* thread 0's first-round loads */
        }
        if (!(want & KGX_WANT_OTU) && st[14] >= st[6] && st[15] >= st[14] && st[9] >= st[15]) {
            s->phase_ns[12] += (st[14] - st[6]) * 10; /* the first chunk's runs and members */
            s->phase_ns[13] += (st[15] - st[14]) * 10; /* ... its sums */
        }
    }
    const SvcSlotOut &o = s->out[slot];
    const uint32_t nh = o.nh, nc = o.nc, no = (want & KGX_WANT_OTU) ? o.no : 0u;
    if (nh == 0xFFFFFFFFu) {
        /* the device gave up on residue chunks that never arrived (svc_kernel's
         * 1-s bound): not computed, take the batch path */
        give_slot(s, slot);
        return fail(KGX_EBUSY, "call service: the request's residues did not reach the device");
    }
    if (nh > W || nc > W || no > W) {
        give_slot(s, slot);
        return fail(KGX_EDEVICE, "call service: more records than windows");
    }
    *n_hits = (want & KGX_WANT_HITS) ? nh : 0;
    *n_calls = (want & KGX_WANT_CALLS) ? nc : 0;
    if (*n_hits)
        std::memcpy(hits, s->hits + (size_t)slot * FUSED_MAX_WINDOWS, *n_hits * sizeof(kgx_hit));
    if (*n_calls)
        std::memcpy(calls, s->calls + (size_t)slot * FUSED_MAX_WINDOWS, *n_calls * sizeof(kgx_call));
    if (want & KGX_WANT_OTU) {
        *n_otus = no;
        if (no)
            std::memcpy(otus, s->otus + (size_t)slot * FUSED_MAX_WINDOWS, no * sizeof(kgx_otu));
    } else if (n_otus) {
        *n_otus = 0;
    }
    std::atomic<uint64_t> &nc_slot = s->slot[slot].n_calls;
    nc_slot.store(nc_slot.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
    give_slot(s, slot);
    return KGX_OK;
}

}  // extern "C"
