/*
 * kgx_runtime.cpp -- host side of the C ABI (include/kgx.h): image loading
 * and replication into HBM, per-thread contexts, batch orchestration, host
 * OTU tallies.
 *
 * Replaces KmerImage (kmer_image.cc:41-108) and the per-sequence loop of
 * KmerGuts::process_aa_seq (kguts.cc:888-908) with batched HIP launches.
 */
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <cerrno>
#include <ctime>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <atomic>
#include <fcntl.h>
#include <mutex>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "kgx_rt.h"

using namespace kgx;

namespace kgx {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg)
{
    g_last_error = msg;
    return code;
}

bool is_gfx950(int dev)
{
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return false;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

/* KGX_TIMING=1: phase wall times of the host-buffer path on stderr */
struct PhaseTimer {
    kgx_ctx *c;
    bool on;
    std::chrono::steady_clock::time_point t;
    explicit PhaseTimer(kgx_ctx *ctx) : c(ctx), on(std::getenv("KGX_TIMING") != nullptr), t(std::chrono::steady_clock::now()) {}
    void mark(const char *what)
    {
        if (!on)
            return;
        (void)hipStreamSynchronize(c->stream);
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[kgx] %-10s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

namespace {

int wait_mode_from_env(uint32_t *us)
{
    *us = 20;
    const char *e = std::getenv("KGX_HOST_WAIT");
    if (!e)
        return KGX_WAIT_SPIN;
    const std::string v(e);
    if (v.rfind("sleep", 0) == 0) {
        if (v.size() > 6 && v[5] == ':')
            *us = (uint32_t)std::max(1, std::atoi(v.c_str() + 6));
        return KGX_WAIT_SLEEP;
    }
    return v == "block" ? KGX_WAIT_BLOCK : KGX_WAIT_SPIN;
}

uint32_t g_env_wait_us = 20;

void sleep_us(uint32_t us)
{
    timespec ts{0, (long)us * 1000};
    nanosleep(&ts, nullptr);
}

}  // namespace

std::atomic<int> g_host_wait_mode{wait_mode_from_env(&g_env_wait_us)};
std::atomic<uint32_t> g_host_wait_us{g_env_wait_us};

hipError_t host_wait(hipStream_t s)
{
    const int mode = g_host_wait_mode.load(std::memory_order_relaxed);
    if (mode == KGX_WAIT_SLEEP) {
        const uint32_t us = g_host_wait_us.load(std::memory_order_relaxed);
        for (;;) {
            const hipError_t q = hipStreamQuery(s);
            if (q != hipErrorNotReady)
                return q;
            sleep_us(us);
        }
    }
    if (mode == KGX_WAIT_BLOCK) {
        /* one blocking-sync event per thread and device, never destroyed (a
         * thread_local destructor must not call the runtime at exit, §10) */
        thread_local hipEvent_t ev[64] = {};
        int dev = 0;
        hipError_t e = hipStreamGetDevice(s, &dev);
        if (e != hipSuccess || dev < 0 || dev >= 64)
            return e != hipSuccess ? e : hipStreamSynchronize(s);
        if (!ev[dev]) {
            int cur = 0;
            if ((e = hipGetDevice(&cur)) != hipSuccess || (cur != dev && (e = hipSetDevice(dev)) != hipSuccess))
                return e;
            e = hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming | hipEventBlockingSync);
            if (cur != dev)
                (void)hipSetDevice(cur);
            if (e != hipSuccess) {
                ev[dev] = nullptr;
                return e;
            }
        }
        if ((e = hipEventRecord(ev[dev], s)) != hipSuccess)
            return e;
        return hipEventSynchronize(ev[dev]);
    }
    return hipStreamSynchronize(s);
}

hipError_t host_wait_word(const volatile uint32_t *done, uint32_t token, hipStream_t s)
{
    const int mode = g_host_wait_mode.load(std::memory_order_relaxed);
    if (mode == KGX_WAIT_BLOCK)
        return host_wait(s); /* the stream drains after the word's store */
    const uint32_t us = g_host_wait_us.load(std::memory_order_relaxed);
    const auto w0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 1; *done != token; spin++) {
        if (mode == KGX_WAIT_SLEEP || (spin & 255u) == 0) { /* a fault or a lost store still ends the wait */
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess)
                break;
            if (q != hipErrorNotReady)
                return q;
            if (mode == KGX_WAIT_SLEEP)
                sleep_us(us);
            /* past 50 us of spinning the CPU goes to whoever else is
             * runnable (a server's other workers, its socket threads) */
            else if (std::chrono::steady_clock::now() - w0 > std::chrono::microseconds(50))
                sched_yield();
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
    return hipSuccess;
}

}  // namespace kgx

/* [p, p + n) lies in one pinned, device-mapped host allocation */
bool kgx::host_pinned_range(const void *p, uint64_t n, const void **device_address)
{
    if (!p || n == 0)
        return false;
    hipPointerAttribute_t a{}, b{};
    const char *first = static_cast<const char *>(p), *last = first + n - 1;
    if (hipPointerGetAttributes(&a, first) != hipSuccess || a.type != hipMemoryTypeHost || !a.devicePointer ||
        hipPointerGetAttributes(&b, last) != hipSuccess || b.type != hipMemoryTypeHost || !b.devicePointer) {
        (void)hipGetLastError(); /* an unregistered pointer is not an error here */
        return false;
    }
    const bool one = static_cast<const char *>(b.devicePointer) - static_cast<const char *>(a.devicePointer) ==
                     (std::ptrdiff_t)(n - 1);
    if (one && device_address)
        *device_address = a.devicePointer;
    return one;
}


extern "C" {

const char *kgx_version(void) { return "close_kmers_amd 0.1 (gfx950)"; }

const char *kgx_last_error(void) { return g_last_error.c_str(); }

const char *kgx_strerror(int code)
{
    switch (code) {
    case KGX_OK: return "ok";
    case KGX_EINVAL: return "invalid argument";
    case KGX_EIO: return "i/o error";
    case KGX_EFORMAT: return "image format mismatch";
    case KGX_ENOMEM: return "out of memory";
    case KGX_EDEVICE: return "device error";
    case KGX_ERANGE: return "out of supported range";
    case KGX_EFULL: return "hash table half full";
    case KGX_EBUSY: return "call service busy or not applicable";
    default: return "unknown error";
    }
}

int kgx_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    int good = 0;
    for (int d = 0; d < n; d++)
        good += is_gfx950(d) ? 1 : 0;
    return good;
}

int kgx_set_host_wait(int mode, uint32_t poll_us)
{
    if (mode != KGX_WAIT_SPIN && mode != KGX_WAIT_SLEEP && mode != KGX_WAIT_BLOCK)
        return fail(KGX_EINVAL, "host wait mode: KGX_WAIT_SPIN, KGX_WAIT_SLEEP or KGX_WAIT_BLOCK");
    g_host_wait_us.store(poll_us ? std::min<uint32_t>(poll_us, 100000) : 20u);
    g_host_wait_mode.store(mode);
    return KGX_OK;
}

int kgx_get_host_wait(uint32_t *poll_us)
{
    if (poll_us)
        *poll_us = g_host_wait_us.load();
    return g_host_wait_mode.load();
}

int kgx_params_default(kgx_params *p)
{
    if (!p)
        return fail(KGX_EINVAL, "null params");
    /* set_default_parameters, kguts.cc:236-242 */
    p->order_constraint = 0;
    p->min_hits = 5;
    p->min_weighted_hits = 0;
    p->max_gap = 200;
    return KGX_OK;
}

int kgx_params_parse(kgx_params *p, const char *const *names, const char *const *values, size_t n)
{
    if (!p || (n && (!names || !values)))
        return fail(KGX_EINVAL, "null argument");
    kgx_params_default(p);
    /* set_parameters, kguts.cc:244-268: std::stoi; invalid_argument warns */
    for (size_t i = 0; i < n; i++) {
        int32_t *dst = nullptr;
        std::string k = names[i] ? names[i] : "";
        if (k == "order_constraint")
            dst = &p->order_constraint;
        else if (k == "min_hits")
            dst = &p->min_hits;
        else if (k == "min_weighted_hits")
            dst = &p->min_weighted_hits;
        else if (k == "max_gap")
            dst = &p->max_gap;
        if (!dst)
            continue;
        try {
            *dst = std::stoi(values[i] ? values[i] : "");
        } catch (const std::invalid_argument &) {
            std::fprintf(stderr, "Warning: invalid integer '%s' passed for parameter %s\n",
                         values[i] ? values[i] : "", k.c_str());
        } catch (const std::out_of_range &) {
            return fail(KGX_ERANGE, "parameter " + k + " out of int range");
        }
    }
    return KGX_OK;
}

/* ---- images ------------------------------------------------------------ */

/* an image on `device` with its resident table allocated in `layout`
 * (AOS24: the file's 24-B buckets; PACKED16: 16-B records, a replica of a
 * packed image, so no 24-B table is ever allocated for it) */
static int image_alloc(int device, uint64_t num_sigs, kgx_image **out, int layout = KGX_LAYOUT_AOS24)
{
    if (!out)
        return fail(KGX_EINVAL, "null output");
    if (num_sigs == 0)
        return fail(KGX_EFORMAT, "image with zero buckets");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return fail(KGX_EDEVICE, "no such HIP device " + std::to_string(device));
    if (!is_gfx950(device))
        return fail(KGX_EDEVICE, "device " + std::to_string(device) + " is not gfx950");
    HIP_TRY(hipSetDevice(device));
    kgx_image *img = new kgx_image;
    img->device = device;
    img->num_sigs = num_sigs;
    hipError_t e = layout == KGX_LAYOUT_PACKED16 ? hipMalloc(&img->d_packed, num_sigs * sizeof(packed_bucket))
                                                  : hipMalloc(&img->d_table, num_sigs * sizeof(kgx_sig_kmer));
    if (e != hipSuccess) {
        (void)hipGetLastError();
        delete img;
        return fail(KGX_ENOMEM, "hipMalloc of the image table failed: " +
                                    std::string(hipGetErrorString(e)));
    }
    img->layout = layout;
    *out = img;
    return KGX_OK;
}

/* AOS24 -> PACKED16 on the device; KGX_ERANGE (image unchanged) when some
 * stored bucket's payload does not fit the packed record */
static int image_pack(kgx_image *img)
{
    if (img->layout == KGX_LAYOUT_PACKED16)
        return KGX_OK;
    HIP_TRY(hipSetDevice(img->device));
    packed_bucket *p = nullptr;
    uint32_t *flag = nullptr;
    if (hipMalloc(&p, img->num_sigs * sizeof(packed_bucket)) != hipSuccess) {
        (void)hipGetLastError();
        return fail(KGX_ENOMEM, "no room for the packed table");
    }
    uint32_t bad = 0;
    hipError_t e = hipMalloc(&flag, sizeof(uint32_t));
    if (e == hipSuccess)
        e = hipMemset(flag, 0, sizeof(uint32_t));
    if (e == hipSuccess)
        e = launch_pack(img->d_table, p, img->num_sigs, flag, nullptr);
    if (e == hipSuccess)
        e = hipMemcpy(&bad, flag, sizeof(bad), hipMemcpyDeviceToHost);
    if (flag)
        (void)hipFree(flag);
    if (e != hipSuccess || bad) {
        (void)hipFree(p);
        if (e != hipSuccess)
            return fail(KGX_EDEVICE, std::string("pack: ") + hipGetErrorString(e));
        return fail(KGX_ERANGE, "image payloads do not fit the packed layout");
    }
    (void)hipFree(img->d_table);
    img->d_table = nullptr;
    img->d_packed = p;
    img->layout = KGX_LAYOUT_PACKED16;
    return KGX_OK;
}

static int image_unpack(kgx_image *img)
{
    if (img->layout == KGX_LAYOUT_AOS24)
        return KGX_OK;
    HIP_TRY(hipSetDevice(img->device));
    kgx_sig_kmer *t = nullptr;
    if (hipMalloc(&t, img->num_sigs * sizeof(kgx_sig_kmer)) != hipSuccess) {
        (void)hipGetLastError();
        return fail(KGX_ENOMEM, "no room for the 24-byte table");
    }
    hipError_t e = launch_unpack(img->d_packed, t, img->num_sigs, nullptr);
    if (e == hipSuccess)
        e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(t);
        return fail(KGX_EDEVICE, std::string("unpack: ") + hipGetErrorString(e));
    }
    (void)hipFree(img->d_packed);
    img->d_packed = nullptr;
    img->d_table = t;
    img->layout = KGX_LAYOUT_AOS24;
    return KGX_OK;
}

/* images are packed at load when they fit; otherwise they stay AOS24.
 * KGX_LINE_INDEX=<keys per 64 lines> also builds the line index of every
 * packed image at load (kgx_image_set_line_index; for programs that only
 * see images through the facade or the server) */
static int image_settle(kgx_image *img, kgx_image **out)
{
    int rc = image_pack(img);
    if (rc == KGX_EDEVICE) {
        kgx_image_close(img);
        return rc;
    }
    static const long line_load = [] {
        const char *e = std::getenv("KGX_LINE_INDEX");
        return e ? std::strtol(e, nullptr, 10) : 0L;
    }();
    if (line_load > 0 && img->layout == KGX_LAYOUT_PACKED16 &&
        (rc = kgx_image_set_line_index(img, (uint32_t)std::min(line_load, 255L)))) {
        kgx_image_close(img);
        return rc;
    }
    *out = img;
    return KGX_OK;
}

/* KmerImage::map_image_file validation, kmer_image.cc:128-147 */
static int validate_header(const kgx_image_header &h, uint64_t file_size)
{
    if (file_size != sizeof(kgx_sig_kmer) * h.num_sigs + sizeof(kgx_image_header))
        return fail(KGX_EFORMAT, "Version mismatch: file size does not match");
    if (h.version != 1)
        return fail(KGX_EFORMAT, "Version mismatch: file has " + std::to_string(h.version) +
                                     " code has 1");
    if (h.entry_size != sizeof(kgx_sig_kmer))
        return fail(KGX_EFORMAT, "Version mismatch: entry size " + std::to_string(h.entry_size));
    return KGX_OK;
}

/* A device destination of a file load: `dev` on `device`. */
struct LoadDst {
    char *dev;
    int device;
};

/* file bytes [off, off + total) -> every destination, by `threads` host
 * threads: thread t reads chunks t, t + threads, ... with pread into its own
 * two pinned buffers and copies each chunk up to every destination on that
 * destination's stream, so file reads (page cache or disk) run in parallel and
 * overlap the H2D copies, and a replicated image is read from the file once
 * (each device's copy runs on its own PCIe link).  The reference maps the file
 * with MAP_POPULATE instead (kmer_image.cc:66-77); the bytes are the same. */
static int load_file_range(int fd, uint64_t off, uint64_t total, const std::vector<LoadDst> &dsts, int threads,
                           size_t chunk)
{
    chunk = (size_t)std::max<uint64_t>(1, std::min<uint64_t>(chunk, total)); /* small files: small buffers */
    const uint64_t n_chunks = (total + chunk - 1) / chunk;
    threads = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)threads, n_chunks));
    const size_t D = dsts.size();
    std::atomic<bool> ok(true);
    std::string err;
    std::mutex err_mu;
    auto set_err = [&](const std::string &e) {
        std::lock_guard<std::mutex> g(err_mu);
        if (ok.exchange(false))
            err = e;
    };
    auto worker = [&](int t) {
        void *buf[2] = {nullptr, nullptr};
        std::vector<hipStream_t> st(D, nullptr);
        std::vector<hipEvent_t> ev(2 * D, nullptr); /* ev[k * D + d]: buffer k's copy to dst d */
        bool used[2] = {false, false};
        bool setup = hipSetDevice(dsts[0].device) == hipSuccess && hipHostMalloc(&buf[0], chunk, hipHostMallocPortable) == hipSuccess &&
                     hipHostMalloc(&buf[1], chunk, hipHostMallocPortable) == hipSuccess;
        for (size_t d = 0; setup && d < D; d++) {
            setup = hipSetDevice(dsts[d].device) == hipSuccess &&
                    hipStreamCreateWithFlags(&st[d], hipStreamNonBlocking) == hipSuccess &&
                    hipEventCreateWithFlags(&ev[d], hipEventDisableTiming) == hipSuccess &&
                    hipEventCreateWithFlags(&ev[D + d], hipEventDisableTiming) == hipSuccess;
        }
        if (!setup) {
            set_err("pinned staging allocation failed");
        } else {
            int k = 0;
            for (uint64_t c = (uint64_t)t; c < n_chunks && ok.load(); c += (uint64_t)threads, k ^= 1) {
                const uint64_t at = c * chunk;
                const size_t n = (size_t)std::min<uint64_t>(chunk, total - at);
                bool waited = true;
                for (size_t d = 0; used[k] && d < D; d++)
                    waited = waited && hipEventSynchronize(ev[k * D + d]) == hipSuccess;
                if (!waited) {
                    set_err("staging copy failed");
                    break;
                }
                size_t got = 0;
                while (got < n) {
                    const ssize_t r = pread(fd, static_cast<char *>(buf[k]) + got, n - got, (off_t)(off + at + got));
                    if (r <= 0)
                        break;
                    got += (size_t)r;
                }
                if (got != n) {
                    set_err("short read");
                    break;
                }
                bool copied = true;
                for (size_t d = 0; copied && d < D; d++)
                    copied = hipSetDevice(dsts[d].device) == hipSuccess &&
                             hipMemcpyAsync(dsts[d].dev + at, buf[k], n, hipMemcpyHostToDevice, st[d]) == hipSuccess &&
                             hipEventRecord(ev[k * D + d], st[d]) == hipSuccess;
                if (!copied) {
                    set_err("H2D copy failed");
                    break;
                }
                used[k] = true;
            }
        }
        for (size_t d = 0; d < D; d++)
            if (st[d]) {
                (void)hipSetDevice(dsts[d].device);
                (void)hipStreamSynchronize(st[d]);
            }
        for (auto e : ev)
            if (e)
                (void)hipEventDestroy(e);
        for (int i = 0; i < 2; i++)
            if (buf[i])
                (void)hipHostFree(buf[i]);
        for (size_t d = 0; d < D; d++)
            if (st[d])
                (void)hipStreamDestroy(st[d]);
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++)
        pool.emplace_back(worker, t);
    for (auto &th : pool)
        th.join();
    return ok.load() ? KGX_OK : fail(KGX_EIO, err);
}

/* reader threads of kgx_image_open: KGX_LOAD_THREADS, else one per GiB of
 * table up to 8 (each thread's pinned buffers cost more than they save on
 * small files: 768 MB loads at 8.2 GB/s with 1 thread, 3.3 GB/s with 8;
 * 25.8 GB at 22 GB/s with 8, profiles/r1s_image_load.json) */
static int load_threads(uint64_t bytes)
{
    const char *e = std::getenv("KGX_LOAD_THREADS");
    const int n = e ? std::atoi(e) : (int)std::min<uint64_t>(8, std::max<uint64_t>(1, bytes >> 30));
    return std::max(1, std::min(n, 64));
}

/* <dir>/kmer.table.mem_map: opened, stat'ed and its header validated
 * (kmer_image.cc:128-147); *fd stays open on success */
static int open_image_file(const char *dir, int *fd_out, kgx_image_header *h, std::string *path_out)
{
    const std::string path = std::string(dir) + "/kmer.table.mem_map";
    *path_out = path;
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0)
        return fail(KGX_EIO, "open " + path + ": " + std::strerror(errno));
    struct stat st;
    if (fstat(fd, &st) != 0) {
        ::close(fd);
        return fail(KGX_EIO, "stat " + path + " failed");
    }
    if (pread(fd, h, sizeof(*h), 0) != (ssize_t)sizeof(*h)) {
        ::close(fd);
        return fail(KGX_EFORMAT, "Version mismatch: file size does not match");
    }
    int rc = validate_header(*h, (uint64_t)st.st_size);
    if (rc) {
        ::close(fd);
        return rc;
    }
    *fd_out = fd;
    return KGX_OK;
}

int kgx_image_open(const char *dir, int device, kgx_image **out)
{
    if (!dir || !out)
        return fail(KGX_EINVAL, "null argument");
    return kgx_image_open_replicas(dir, &device, 1, out);
}

int kgx_image_open_replicas(const char *dir, const int *devices, uint32_t n, kgx_image **out)
{
    if (!dir || !out || !devices || n == 0)
        return fail(KGX_EINVAL, "null argument or no devices");
    for (uint32_t i = 0; i < n; i++)
        out[i] = nullptr;
    int fd = -1;
    kgx_image_header h;
    std::string path;
    int rc = open_image_file(dir, &fd, &h, &path);
    if (rc)
        return rc;
    std::vector<kgx_image *> imgs(n, nullptr);
    std::vector<LoadDst> dsts;
    auto close_all = [&]() {
        for (auto *im : imgs)
            kgx_image_close(im);
    };
    for (uint32_t i = 0; i < n; i++) {
        rc = image_alloc(devices[i], h.num_sigs, &imgs[i]);
        if (rc) {
            ::close(fd);
            close_all();
            return rc;
        }
        dsts.push_back({reinterpret_cast<char *>(imgs[i]->d_table), devices[i]});
    }
    rc = load_file_range(fd, sizeof(h), h.num_sigs * sizeof(kgx_sig_kmer), dsts,
                         load_threads(h.num_sigs * sizeof(kgx_sig_kmer)), 32ull << 20);
    ::close(fd);
    if (rc) {
        close_all();
        return fail(rc, "loading " + path + ": " + kgx_last_error());
    }
    /* every replica is packed on its own device at once */
    std::vector<int> rcs(n, KGX_OK);
    std::vector<std::string> errs(n);
    std::vector<std::thread> th;
    for (uint32_t i = 0; i < n; i++)
        th.emplace_back([&, i] {
            kgx_image *settled = nullptr;
            rcs[i] = image_settle(imgs[i], &settled); /* closes the image on failure */
            if (rcs[i])
                errs[i] = kgx_last_error();
            imgs[i] = rcs[i] ? nullptr : settled;
        });
    for (auto &t : th)
        t.join();
    for (uint32_t i = 0; i < n; i++)
        if (rcs[i]) {
            close_all();
            return fail(rcs[i], "replica on device " + std::to_string(devices[i]) + ": " + errs[i]);
        }
    for (uint32_t i = 0; i < n; i++)
        out[i] = imgs[i];
    return KGX_OK;
}

int kgx_image_replicate(const kgx_image *src, int device, kgx_image **out)
{
    if (!src || !out)
        return fail(KGX_EINVAL, "null argument");
    *out = nullptr;
    kgx_image *img = nullptr;
    /* the source's resident layout only (a packed source never costs a 24-B
     * table on the target, not even briefly) */
    int rc = image_alloc(device, src->num_sigs, &img, src->layout);
    if (rc)
        return rc;
    hipError_t e = hipSuccess;
    /* device to device: xGMI between two GPUs (the runtime picks the path),
     * a device-local copy when both are the same GPU */
    e = hipMemcpyPeer(img->layout == KGX_LAYOUT_PACKED16 ? static_cast<void *>(img->d_packed) : img->d_table,
                      device, src->resident(), src->device, src->resident_bytes());
    if (e == hipSuccess && src->d_filter) {
        const uint64_t fbytes = 8ull << src->filter_log2_words;
        e = hipMalloc(&img->d_filter, fbytes);
        if (e == hipSuccess)
            e = hipMemcpyPeer(img->d_filter, device, src->d_filter, src->device, fbytes);
        if (e == hipSuccess)
            img->filter_log2_words = src->filter_log2_words;
    }
    if (e == hipSuccess)
        e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        kgx_image_close(img);
        return fail(KGX_EDEVICE, std::string("replicate: ") + hipGetErrorString(e));
    }
    /* the line index is the caller's choice per replica (kgx_image_set_line_index):
     * it doubles the HBM an image takes, and a device may already hold one */
    *out = img;
    return KGX_OK;
}

int kgx_image_from_memory(const void *file_bytes, uint64_t nbytes, int device, kgx_image **out)
{
    if (!file_bytes || !out || nbytes < sizeof(kgx_image_header))
        return fail(KGX_EINVAL, "bad image buffer");
    kgx_image_header h;
    std::memcpy(&h, file_bytes, sizeof(h));
    int rc = validate_header(h, nbytes);
    if (rc)
        return rc;
    kgx_image *img = nullptr;
    rc = image_alloc(device, h.num_sigs, &img);
    if (rc)
        return rc;
    hipError_t e = hipMemcpy(img->d_table, static_cast<const char *>(file_bytes) + sizeof(h),
                             h.num_sigs * sizeof(kgx_sig_kmer), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        kgx_image_close(img);
        return fail(KGX_EDEVICE, std::string("image upload: ") + hipGetErrorString(e));
    }
    return image_settle(img, out);
}

int kgx_image_build_synthetic(uint64_t n_keys, uint64_t num_sigs, int device, kgx_image **out,
                              uint64_t *n_stored)
{
    if (2 * n_keys >= num_sigs)
        return fail(KGX_EFULL, "Your Kmer hash is half-full (kguts.cc:213-216)");
    kgx_image *img = nullptr;
    int rc = image_alloc(device, num_sigs, &img);
    if (rc)
        return rc;
    unsigned long long *d_count = nullptr;
    if (hipMalloc(&d_count, sizeof(*d_count)) != hipSuccess) {
        kgx_image_close(img);
        return fail(KGX_ENOMEM, "counter allocation failed");
    }
    hipError_t e = launch_synth_image(img->d_table, num_sigs, n_keys, n_keys, true, d_count, nullptr);
    unsigned long long cnt = 0;
    if (e == hipSuccess)
        e = hipMemcpy(&cnt, d_count, sizeof(cnt), hipMemcpyDeviceToHost);
    (void)hipFree(d_count);
    if (e != hipSuccess) {
        kgx_image_close(img);
        return fail(KGX_EDEVICE, std::string("synthetic build: ") + hipGetErrorString(e));
    }
    if (n_stored)
        *n_stored = cnt;
    return image_settle(img, out);
}

int kgx_image_build_synthetic_distinct(uint64_t n_keys, uint64_t n_distinct, uint64_t num_sigs, int device,
                                       kgx_image **out, uint64_t *n_entries)
{
    if (!out)
        return fail(KGX_EINVAL, "null output");
    /* the stream is searched up to 1/8 past n_distinct (a synthetic 8-mer
     * stream repeats keys ~2% of the time at 1e9 of 20^8); owners are 32-bit */
    const uint64_t upper = n_distinct + n_distinct / 8 + 1024;
    if (2 * upper >= num_sigs || upper >= (1ull << 32))
        return fail(KGX_EFULL, "Your Kmer hash is half-full (kguts.cc:213-216)");
    kgx_image *img = nullptr;
    int rc = image_alloc(device, num_sigs, &img);
    if (rc)
        return rc;
    DevBuf d_count, d_hist;
    hipError_t e = d_count.reserve(sizeof(unsigned long long));
    if (e == hipSuccess)
        e = d_hist.reserve(256 * sizeof(unsigned long long));
    unsigned long long cnt = 0;
    if (e == hipSuccess)
        e = launch_synth_image(img->d_table, num_sigs, n_keys, upper, false, d_count.as<unsigned long long>(),
                               nullptr);
    if (e == hipSuccess)
        e = hipMemcpy(&cnt, d_count.p, sizeof(cnt), hipMemcpyDeviceToHost);
    if (e == hipSuccess && cnt < n_distinct) {
        kgx_image_close(img);
        return fail(KGX_ERANGE, "the synthetic stream holds fewer distinct keys than asked for");
    }
    /* radix select of the n_distinct-th smallest owner, a byte per pass */
    uint32_t prefix = 0, mask = 0;
    uint64_t k = n_distinct; /* 1-based rank within the current prefix */
    for (int shift = 24; e == hipSuccess && shift >= 0; shift -= 8) {
        unsigned long long h[256];
        e = launch_owner_hist(img->d_table, num_sigs, prefix, mask, (uint32_t)shift,
                              d_hist.as<unsigned long long>(), nullptr);
        if (e == hipSuccess)
            e = hipMemcpy(h, d_hist.p, sizeof(h), hipMemcpyDeviceToHost);
        if (e != hipSuccess)
            break;
        uint32_t b = 0;
        while (b < 255 && k > h[b])
            k -= h[b++];
        prefix |= b << shift;
        mask |= 255u << shift;
    }
    const uint64_t m = (uint64_t)prefix + 1; /* entries [0, m) hold exactly n_distinct keys */
    if (e == hipSuccess)
        e = launch_synth_image(img->d_table, num_sigs, n_keys, m, true, d_count.as<unsigned long long>(), nullptr);
    if (e == hipSuccess)
        e = hipMemcpy(&cnt, d_count.p, sizeof(cnt), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        kgx_image_close(img);
        return fail(KGX_EDEVICE, std::string("synthetic build: ") + hipGetErrorString(e));
    }
    if (cnt != n_distinct) {
        kgx_image_close(img);
        return fail(KGX_EDEVICE, "synthetic build stored " + std::to_string(cnt) + " keys, not " +
                                     std::to_string(n_distinct));
    }
    if (n_entries)
        *n_entries = m;
    return image_settle(img, out);
}

int kgx_image_build(const uint64_t *keys, const int32_t *function_index, const int32_t *otu_index,
                    const uint16_t *avg_from_end, const float *function_wt, uint64_t n, uint64_t num_sigs,
                    int device, kgx_image **out, uint64_t *n_stored)
{
    if (!out || (n && (!keys || !function_index || !otu_index || !avg_from_end || !function_wt)))
        return fail(KGX_EINVAL, "null argument");
    /* kguts.cc:209-213: every valid key counts (duplicates too) */
    uint64_t valid = 0;
    for (uint64_t i = 0; i < n; i++)
        valid += keys[i] <= MAX_ENCODED;
    if (valid >= num_sigs / 2)
        return fail(KGX_EFULL, "Your Kmer hash is half-full (kguts.cc:209-213)");
    kgx_image *img = nullptr;
    int rc = image_alloc(device, num_sigs, &img);
    if (rc)
        return rc;
    DevBuf d_keys, d_fi, d_otu, d_avg, d_wt, d_count;
    hipError_t e = hipSuccess;
    for (auto rq : {d_keys.reserve(std::max<uint64_t>(n, 1) * 8), d_fi.reserve(std::max<uint64_t>(n, 1) * 4),
                    d_otu.reserve(std::max<uint64_t>(n, 1) * 4), d_avg.reserve(std::max<uint64_t>(n, 1) * 2),
                    d_wt.reserve(std::max<uint64_t>(n, 1) * 4), d_count.reserve(8)})
        if (rq != hipSuccess)
            e = rq;
    if (e == hipSuccess && n) {
        e = hipMemcpy(d_keys.p, keys, n * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(d_fi.p, function_index, n * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(d_otu.p, otu_index, n * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(d_avg.p, avg_from_end, n * 2, hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(d_wt.p, function_wt, n * 4, hipMemcpyHostToDevice);
    }
    unsigned long long cnt = 0;
    if (e == hipSuccess)
        e = launch_entries_image(img->d_table, num_sigs, d_keys.as<uint64_t>(), d_fi.as<int32_t>(),
                                 d_otu.as<int32_t>(), d_avg.as<uint16_t>(), d_wt.as<float>(), n,
                                 d_count.as<unsigned long long>(), nullptr);
    if (e == hipSuccess)
        e = hipMemcpy(&cnt, d_count.p, 8, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        kgx_image_close(img);
        return fail(e == hipErrorOutOfMemory ? KGX_ENOMEM : KGX_EDEVICE,
                    std::string("image build: ") + hipGetErrorString(e));
    }
    if (n_stored)
        *n_stored = cnt;
    return image_settle(img, out);
}

int kgx_image_close(kgx_image *img)
{
    if (!img)
        return KGX_OK;
    svc_shutdown(img);
    (void)hipSetDevice(img->device);
    if (img->d_table)
        (void)hipFree(img->d_table);
    if (img->d_packed)
        (void)hipFree(img->d_packed);
    if (img->d_lines)
        (void)hipFree(img->d_lines);
    if (img->d_filter)
        (void)hipFree(img->d_filter);
    if (img->probe_stream) {
        (void)hipStreamSynchronize(img->probe_stream);
        (void)hipStreamDestroy(img->probe_stream);
    }
    delete img;
    return KGX_OK;
}

uint64_t kgx_image_num_sigs(const kgx_image *img) { return img ? img->num_sigs : 0; }
int kgx_image_device(const kgx_image *img) { return img ? img->device : -1; }
const void *kgx_image_table(const kgx_image *img) { return img ? img->d_table : nullptr; }
int kgx_image_layout(const kgx_image *img) { return img ? img->layout : -1; }

int kgx_image_set_filter(kgx_image *img, int log2_bits)
{
    if (!img || log2_bits < 0 || (log2_bits && (log2_bits < 12 || log2_bits > 40)))
        return fail(KGX_EINVAL, "filter size: 0 (none) or 2^12 .. 2^40 bits");
    /* the device-wide synchronisation below would wait out its instances,
     * and the filter buffer is replaced under any service a call starts */
    const auto hold = svc_shutdown_hold(img);
    HIP_TRY(hipSetDevice(img->device));
    HIP_TRY(hipDeviceSynchronize());
    if (img->d_filter)
        (void)hipFree(img->d_filter);
    img->d_filter = nullptr;
    img->filter_log2_words = 0;
    if (!log2_bits)
        return KGX_OK;
    const uint32_t lw = (uint32_t)log2_bits - 6;
    const uint64_t bytes = 8ull << lw;
    if (hipMalloc(&img->d_filter, bytes) != hipSuccess) {
        (void)hipGetLastError();
        img->d_filter = nullptr;
        return fail(KGX_ENOMEM, "no room for the filter");
    }
    HIP_TRY(hipMemset(img->d_filter, 0, bytes));
    HIP_TRY(launch_filter_build(img->resident(), img->layout, img->num_sigs, img->d_filter, lw, nullptr));
    HIP_TRY(hipDeviceSynchronize());
    img->filter_log2_words = lw;
    return KGX_OK;
}

int kgx_image_set_layout(kgx_image *img, int layout)
{
    if (!img)
        return fail(KGX_EINVAL, "null image");
    /* its workgroups hold the resident table's address: no call starts a
     * service until the table it would use is the new one */
    const auto hold = svc_shutdown_hold(img);
    if (layout == KGX_LAYOUT_PACKED16)
        return image_pack(img);
    if (layout == KGX_LAYOUT_AOS24) {
        if (img->d_lines) { /* the line index holds PACKED16 records */
            HIP_TRY(hipSetDevice(img->device));
            HIP_TRY(hipDeviceSynchronize());
            (void)hipFree(img->d_lines);
            img->d_lines = nullptr;
            img->n_lines = 0;
        }
        return image_unpack(img);
    }
    return fail(KGX_EINVAL, "unknown layout " + std::to_string(layout));
}

int kgx_image_set_line_index(kgx_image *img, uint32_t keys_per_64_lines)
{
    if (!img)
        return fail(KGX_EINVAL, "null image");
    if (keys_per_64_lines > 255)
        return fail(KGX_EINVAL, "line index load: 0 (none) or 1 .. 255 keys per 64 lines");
    /* the service's workgroups hold the probe table's address */
    const auto hold = svc_shutdown_hold(img);
    HIP_TRY(hipSetDevice(img->device));
    HIP_TRY(hipDeviceSynchronize());
    if (img->d_lines)
        (void)hipFree(img->d_lines);
    img->d_lines = nullptr;
    img->n_lines = 0;
    if (!keys_per_64_lines)
        return KGX_OK;
    if (img->layout != KGX_LAYOUT_PACKED16)
        return fail(KGX_EINVAL, "a line index needs a PACKED16 image");
    unsigned long long *d_count = nullptr;
    uint32_t *d_over = nullptr;
    HIP_TRY(hipMalloc(&d_count, 16));
    d_over = reinterpret_cast<uint32_t *>(d_count + 1);
    hipError_t e = hipMemset(d_count, 0, 16);
    if (e == hipSuccess)
        e = launch_count_keys(img->d_packed, img->num_sigs, d_count, nullptr);
    unsigned long long n_keys = 0;
    if (e == hipSuccess)
        e = hipMemcpy(&n_keys, d_count, 8, hipMemcpyDeviceToHost);
    /* lines: n_keys * 64 / load, odd and prime to 5 (keys are base-20 codes) */
    uint64_t n_lines = std::max<uint64_t>(1, (uint64_t)(((unsigned __int128)n_keys * 64 + keys_per_64_lines - 1) /
                                                        keys_per_64_lines));
    while (n_lines % 2 == 0 || n_lines % 5 == 0)
        n_lines++;
    packed_bucket *lines = nullptr;
    if (e == hipSuccess && (4 * n_lines >= (1ull << 40) || hipMalloc(&lines, 4 * n_lines * sizeof(packed_bucket)) != hipSuccess)) {
        (void)hipGetLastError();
        (void)hipFree(d_count);
        return fail(KGX_ENOMEM, "no room for the line index (" + std::to_string(4 * n_lines * 16) + " B)");
    }
    uint32_t over = 0;
    if (e == hipSuccess)
        e = launch_lines_build(img->d_packed, img->num_sigs, lines, n_lines, d_over, nullptr);
    if (e == hipSuccess)
        e = hipMemcpy(&over, d_over, 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_count);
    if (e != hipSuccess || over) {
        if (lines)
            (void)hipFree(lines);
        return fail(KGX_EDEVICE, e != hipSuccess ? std::string("line index: ") + hipGetErrorString(e)
                                                 : std::string("line index: a record found no bucket"));
    }
    img->d_lines = lines;
    img->n_lines = n_lines;
    img->lines_load = keys_per_64_lines;
    return KGX_OK;
}

uint64_t kgx_image_line_count(const kgx_image *img) { return img ? img->n_lines : 0; }

/* buckets [first, first + count) in the file's format into host memory */
static int image_read(const kgx_image *img, uint64_t first, uint64_t count, kgx_sig_kmer *dst)
{
    HIP_TRY(hipSetDevice(img->device));
    if (img->layout == KGX_LAYOUT_AOS24) {
        HIP_TRY(hipMemcpy(dst, img->d_table + first, count * sizeof(kgx_sig_kmer), hipMemcpyDeviceToHost));
        return KGX_OK;
    }
    /* PACKED16: unpack slices on the device, then copy them out */
    const uint64_t slice = 1ull << 24; /* buckets (384 MiB of output) */
    kgx_sig_kmer *tmp = nullptr;
    HIP_TRY(hipMalloc(&tmp, std::max<uint64_t>(1, std::min(slice, count)) * sizeof(kgx_sig_kmer)));
    hipError_t e = hipSuccess;
    for (uint64_t b = 0; b < count && e == hipSuccess; b += slice) {
        const uint64_t m = std::min(slice, count - b);
        e = launch_unpack(img->d_packed + first + b, tmp, m, nullptr);
        if (e == hipSuccess)
            e = hipMemcpy(dst + b, tmp, m * sizeof(kgx_sig_kmer), hipMemcpyDeviceToHost);
    }
    (void)hipFree(tmp);
    if (e != hipSuccess)
        return fail(KGX_EDEVICE, std::string("download: ") + hipGetErrorString(e));
    return KGX_OK;
}

int kgx_image_download(const kgx_image *img, void *dst, uint64_t nbytes)
{
    if (!img || !dst || nbytes != img->num_sigs * sizeof(kgx_sig_kmer))
        return fail(KGX_EINVAL, "bad download buffer");
    return image_read(img, 0, img->num_sigs, static_cast<kgx_sig_kmer *>(dst));
}

int kgx_image_save(const kgx_image *img, const char *dir)
{
    if (!img || !dir)
        return fail(KGX_EINVAL, "null argument");
    const std::string path = std::string(dir) + "/kmer.table.mem_map";
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f)
        return fail(KGX_EIO, "could not open " + path + " for writing: " + std::strerror(errno));
    const kgx_image_header h{img->num_sigs, sizeof(kgx_sig_kmer), 1};
    bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
    const uint64_t chunk = 1ull << 25; /* buckets per write (768 MiB) */
    std::vector<kgx_sig_kmer> buf(std::min(chunk, std::max<uint64_t>(img->num_sigs, 1)));
    for (uint64_t b = 0; ok && b < img->num_sigs; b += chunk) {
        const uint64_t m = std::min(chunk, img->num_sigs - b);
        int rc = image_read(img, b, m, buf.data());
        if (rc) {
            std::fclose(f);
            return rc;
        }
        ok = std::fwrite(buf.data(), sizeof(kgx_sig_kmer), m, f) == m;
    }
    if (std::fclose(f) != 0)
        ok = false;
    return ok ? KGX_OK : fail(KGX_EIO, "short write to " + path);
}

/* ---- contexts ------------------------------------------------------------ */

int kgx_ctx_create(kgx_image *img, kgx_ctx **out)
{
    if (!img || !out)
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(img->device));
    kgx_ctx *c = new kgx_ctx;
    c->img = img;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(KGX_EDEVICE, std::string("stream: ") + hipGetErrorString(e));
    }
    c->own_stream = true;
    /* KGX_SMALL_BATCH: the default of option "small_batch" for new contexts */
    if (const char *sb = std::getenv("KGX_SMALL_BATCH"))
        c->small_batch = std::min<int64_t>(1 << 24, std::max<int64_t>(0, std::atoll(sb)));
    e = hipEventCreateWithFlags(&c->probe_done, hipEventDisableTiming);
    if (e != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return fail(KGX_EDEVICE, std::string("event: ") + hipGetErrorString(e));
    }
    *out = c;
    return KGX_OK;
}

int kgx_ctx_destroy(kgx_ctx *c)
{
    if (!c)
        return KGX_OK;
    (void)hipSetDevice(c->img->device);
    if (c->twin)
        kgx_ctx_destroy(c->twin);
    (void)hipStreamSynchronize(c->stream);
    for (DevBuf *b : {&c->residues, &c->offsets, &c->wbase, &c->tile_seq, &c->hit_mask,
                      &c->hits, &c->calls, &c->hit_count, &c->call_count, &c->dense_hoff,
                      &c->dense_coff, &c->dense_hits, &c->dense_calls, &c->plan_ws, &c->ranges})
        b->release();
    {
        std::lock_guard<std::mutex> lock(c->img->probe_mu);
        if (c->img->last_probe == c->probe_done)
            c->img->last_probe = nullptr;
    }
    (void)hipEventDestroy(c->probe_done);
    if (c->probe_ready)
        (void)hipEventDestroy(c->probe_ready);
    if (c->score_gate)
        (void)hipEventDestroy(c->score_gate);
    c->pool.reset();
    c->stage_pool.reset();
    for (hipEvent_t e : c->chunk_done)
        (void)hipEventDestroy(e);
    for (hipEvent_t e : c->chunk_counts)
        (void)hipEventDestroy(e);
    for (hipEvent_t e : c->chunk_gathered)
        (void)hipEventDestroy(e);
    for (hipEvent_t e : c->chunk_h2d)
        (void)hipEventDestroy(e);
    for (hipEvent_t e : c->prof_ev)
        (void)hipEventDestroy(e);
    for (hipEvent_t e : c->prof_done)
        (void)hipEventDestroy(e);
    if (c->copy_stream) {
        (void)hipStreamSynchronize(c->copy_stream);
        (void)hipStreamDestroy(c->copy_stream);
    }
    if (c->up_stream) {
        (void)hipStreamSynchronize(c->up_stream);
        (void)hipStreamDestroy(c->up_stream);
    }
    if (c->own_stream)
        (void)hipStreamDestroy(c->stream);
    delete c;
    return KGX_OK;
}

void *kgx_ctx_stream(kgx_ctx *c) { return c ? (void *)c->stream : nullptr; }

int kgx_ctx_set_stream(kgx_ctx *c, void *stream)
{
    if (!c)
        return fail(KGX_EINVAL, "null ctx");
    if (stream) {
        if (c->own_stream)
            (void)hipStreamDestroy(c->stream);
        c->stream = (hipStream_t)stream;
        c->own_stream = false;
    } else if (!c->own_stream) {
        HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->own_stream = true;
    }
    return KGX_OK;
}

int kgx_ctx_set_option(kgx_ctx *c, const char *name, int64_t value)
{
    if (!c || !name)
        return fail(KGX_EINVAL, "null argument");
    const std::string n = name;
    if (n == "microbench_ilp") {
        if (value != 1 && value != 2 && value != 4 && value != 8 && value != 16)
            return fail(KGX_EINVAL, "microbench_ilp must be 1, 2, 4, 8 or 16");
        c->microbench_ilp = (int)value;
        return KGX_OK;
    }
    if (n == "microbench_wgs") {
        if (value < 1 || value > 32)
            return fail(KGX_EINVAL, "microbench_wgs must be 1..32");
        c->microbench_wgs = (int)value;
        return KGX_OK;
    }
    if (n == "microbench_span") {
        if (value < 0)
            return fail(KGX_EINVAL, "microbench_span must be >= 0");
        c->microbench_span = (uint64_t)value;
        return KGX_OK;
    }
    if (n == "probe_filter") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "probe_filter must be 0 or 1");
        c->probe_filter = (int)value;
        return KGX_OK;
    }
    if (n == "probe_variant") {
        if (value < PROBE_AUTO || value > PROBE_LINE8)
            return fail(KGX_EINVAL, "probe_variant must be -1, 0, 1, 2 or 3");
        c->probe_variant = (int)value;
        return KGX_OK;
    }
    if (n == "plan_fused") {
        if (value < 0 || value > 2)
            return fail(KGX_EINVAL, "plan_fused must be 0, 1 or 2");
        c->plan_fused = (int)value;
        return KGX_OK;
    }
    if (n == "probe_nt") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "probe_nt must be 0 or 1");
        c->probe_nt = (int)value;
        return KGX_OK;
    }
    if (n == "line_index") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "line_index must be 0 or 1");
        c->use_line_index = (int)value;
        return KGX_OK;
    }
    if (n == "probe_serialize") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "probe_serialize must be 0 or 1");
        c->probe_serialize = (int)value;
        return KGX_OK;
    }
    if (n == "host_copy_blocks") {
        if (value < 1 || value > 4096)
            return fail(KGX_EINVAL, "host_copy_blocks must be 1..4096");
        c->host_copy_blocks = (int)value;
        return KGX_OK;
    }
    if (n == "host_copy") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_copy must be 0 or 1");
        c->host_copy = (int)value;
        return KGX_OK;
    }
    if (n == "host_hits16") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_hits16 must be 0 or 1");
        c->host_hits16 = (int)value;
        return KGX_OK;
    }
    if (n == "stage_threads") {
        if (value < 1 || value > 64)
            return fail(KGX_EINVAL, "stage_threads must be 1..64");
        c->stage_threads = (int)value;
        return KGX_OK;
    }
    if (n == "host_score_variant") {
        if (value < -1 || value > 2)
            return fail(KGX_EINVAL, "host_score_variant must be -1 (the context's score_variant) or 0..2");
        c->host_score_variant = (int)value;
        return KGX_OK;
    }
    if (n == "host_upload_stream") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_upload_stream must be 0 or 1");
        c->host_upload_stream = (int)value;
        return KGX_OK;
    }
    if (n == "host_stream_dma") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_stream_dma must be 0 or 1");
        c->host_stream_dma = (int)value;
        return KGX_OK;
    }
    if (n == "pinned_input") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "pinned_input must be 0 or 1");
        c->pinned_input = (int)value;
        return KGX_OK;
    }
    if (n == "host_stage_all") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_stage_all must be 0 or 1");
        c->host_stage_all = (int)value;
        return KGX_OK;
    }
    if (n == "host_h2d_first") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_h2d_first must be 0 or 1");
        c->host_h2d_first = (int)value;
        return KGX_OK;
    }
    if (n == "host_rec12") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_rec12 must be 0 or 1");
        c->host_rec12 = (int)value;
        return KGX_OK;
    }
    if (n == "host_nt") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_nt must be 0 or 1");
        c->host_nt = (int)value;
        return KGX_OK;
    }
    if (n == "host_taper") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_taper must be 0 or 1");
        c->host_taper = (int)value;
        return KGX_OK;
    }
    if (n == "host_stream") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_stream must be 0 or 1");
        c->host_stream_chunks = (int)value;
        return KGX_OK;
    }
    if (n == "counts_first") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "counts_first must be 0 or 1");
        c->counts_first = (int)value;
        return KGX_OK;
    }
    if (n == "host_threads") {
        if (value < 1 || value > 64)
            return fail(KGX_EINVAL, "host_threads must be 1..64");
        c->host_threads = (int)value;
        return KGX_OK;
    }
    if (n == "small_batch") {
        if (value < 0 || value > (1 << 24))
            return fail(KGX_EINVAL, "small_batch must be 0..16777216 residues");
        c->small_batch = value;
        return KGX_OK;
    }
    if (n == "probe_stream") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "probe_stream must be 0 or 1");
        c->probe_stream = (int)value;
        return KGX_OK;
    }
    if (n == "probe_persist") {
        if (value < 0 || value > 32)
            return fail(KGX_EINVAL, "probe_persist must be 0..32 workgroups per CU");
        c->probe_persist = (int)value;
        return KGX_OK;
    }
    if (n == "small_wave") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "small_wave must be 0 or 1");
        c->small_wave = (int)value;
        return KGX_OK;
    }
    if (n == "host_profile") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "host_profile must be 0 or 1");
        c->host_profile = (int)value;
        return KGX_OK;
    }
    if (n == "host_chunks") {
        if (value < 1 || value > 64)
            return fail(KGX_EINVAL, "host_chunks must be 1..64");
        c->host_chunks = (int)value;
        return KGX_OK;
    }
    if (n == "fq_count") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "fq_count must be 0 or 1");
        c->fq_count = (int)value;
        return KGX_OK;
    }
    if (n == "fq_residues") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "fq_residues must be 0 or 1");
        c->fq_residues = (int)value;
        return KGX_OK;
    }
    if (n == "score_variant") {
        if (value < 0 || value > 2)
            return fail(KGX_EINVAL, "score_variant must be 0, 1 or 2");
        c->score_variant = (int)value;
        return KGX_OK;
    }
    if (n == "probe_lds_kb") {
        if (value < 0 || value > 160)
            return fail(KGX_EINVAL, "probe_lds_kb must be 0..160");
        c->probe_lds_kb = (int)value;
        return KGX_OK;
    }
    if (n == "fused_inline") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "fused_inline must be 0 or 1");
        c->fused_inline = (int)value;
        return KGX_OK;
    }
    if (n == "small_fused") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "small_fused must be 0 or 1");
        c->small_fused = (int)value;
        return KGX_OK;
    }
    if (n == "small_wave_tiles") {
        if (value < 1 || value > 256)
            return fail(KGX_EINVAL, "small_wave_tiles must be 1..256");
        c->small_wave_tiles = (int)value;
        return KGX_OK;
    }
    if (n == "score_wave_tiles") {
        if (value < 1 || value > 256)
            return fail(KGX_EINVAL, "score_wave_tiles must be 1..256");
        c->score_wave_tiles = (int)value;
        return KGX_OK;
    }
    if (n == "fq_fused") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "fq_fused must be 0 or 1");
        c->fq_fused = (int)value;
        return KGX_OK;
    }
    if (n == "fq_plan") {
        if (value != 0 && value != 1)
            return fail(KGX_EINVAL, "fq_plan must be 0 or 1");
        c->fq_plan = (int)value;
        return KGX_OK;
    }
    if (n == "fq_probe_j") {
        if (value < 0 || value > 4)
            return fail(KGX_EINVAL, "fq_probe_j must be 0 (= probe_j), 1, 2, 3 or 4");
        c->fq_probe_j = (int)value;
        return KGX_OK;
    }
    if (n == "probe_j") {
        if (!probe_j_supported((int)value))
            return fail(KGX_EINVAL, "probe_j must be 1, 2, 3, 4, 5 or 8");
        c->probe_j = (int)value;
        return KGX_OK;
    }
    return fail(KGX_EINVAL, "unknown option " + n);
}

int kgx_ctx_check(kgx_ctx *c)
{
    if (!c)
        return fail(KGX_EINVAL, "null ctx");
    HIP_TRY(hipSetDevice(c->img->device));
    if (!c->plan_status.p)
        return KGX_OK; /* nothing planned yet */
    HIP_TRY(c->h_plan_status.resize(1));
    HIP_TRY(hipMemcpyAsync(c->h_plan_status.data(), c->plan_status.p, sizeof(uint32_t), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->h_plan_status[0])
        return fail(KGX_EINVAL, "batch offsets not monotone or spanning more than n_residues bytes "
                                "(the batch was processed as empty)");
    return KGX_OK;
}

int kgx_ctx_synchronize(kgx_ctx *c)
{
    if (!c)
        return fail(KGX_EINVAL, "null ctx");
    HIP_TRY(hipStreamSynchronize(c->stream));
    return KGX_OK;
}

/* ---- stages ------------------------------------------------------------- */

int kgx_stage_plan(kgx_ctx *c, const uint64_t *d_off, uint32_t n_seq, uint64_t n_residues)
{
    if (!c || (!d_off && n_seq))
        return fail(KGX_EINVAL, "null argument");
    if (n_residues > (1ull << 40))
        return fail(KGX_ERANGE, "batch too large");
    HIP_TRY(hipSetDevice(c->img->device));
    int rc = kgx::plan_reserve(c, d_off, n_seq, n_residues);
    if (rc)
        return rc;
    if (c->plan_fused == 2 && n_seq <= (1u << 18)) {
        HIP_TRY(launch_plan_one(d_off, n_seq, n_residues, c->wbase.as<uint64_t>(), c->tile_seq.as<uint32_t>(),
                                c->tile_windows, c->max_tiles, c->plan_status.as<uint32_t>(), c->stream));
        return KGX_OK;
    }
    if (c->plan_fused == 1) {
        /* new states start at zero (every launch leaves them so); a grown
         * buffer may come back at the old address, so its capacity says */
        const size_t had = c->plan_look.cap;
        HIP_TRY(c->plan_look.reserve(plan_look_bytes(n_seq)));
        if (c->plan_look.cap != had)
            HIP_TRY(hipMemsetAsync(c->plan_look.p, 0, c->plan_look.cap, c->stream));
        HIP_TRY(launch_plan_fused(d_off, n_seq, n_residues, c->wbase.as<uint64_t>(), c->tile_seq.as<uint32_t>(),
                                  c->tile_windows, c->max_tiles, c->plan_look.p, c->plan_status.as<uint32_t>(),
                                  c->stream));
        return KGX_OK;
    }
    HIP_TRY(c->plan_ws.reserve(plan_workspace_bytes(n_seq)));
    HIP_TRY(launch_plan(d_off, n_seq, n_residues, c->wbase.as<uint64_t>(), c->tile_seq.as<uint32_t>(),
                        c->tile_windows, c->plan_ws.p, c->plan_status.as<uint32_t>(), c->stream));
    return KGX_OK;
}

}  // extern "C"

namespace kgx {

/* the plan's buffers and bookkeeping (everything of kgx_stage_plan but the
 * plan kernels; the small-batch path writes the plan from the host) */
int plan_reserve(kgx_ctx *c, const uint64_t *d_off, uint32_t n_seq, uint64_t n_residues)
{
    /* bounds: windows <= residues, so tiles <= residues / tile + 1 */
    const uint32_t tile_windows = 64u * (uint32_t)c->probe_j;
    const uint64_t max_tiles = n_residues / tile_windows + 1;
    const uint64_t cap_win = std::max<uint64_t>(n_residues, 1);
    HIP_TRY(c->wbase.reserve((n_seq + 1) * sizeof(uint64_t)));
    HIP_TRY(c->tile_seq.reserve(max_tiles * sizeof(uint32_t)));
    HIP_TRY(c->hit_mask.reserve((cap_win / 64 + 2) * sizeof(uint64_t)));
    /* HIT_PACKED16: one 16-B record per slot; HIT_PLANES: hot plane, then cold plane */
    const bool packed_hits = c->img->layout == KGX_LAYOUT_PACKED16;
    HIP_TRY(c->hits.reserve(cap_win * (packed_hits ? 1 : 2) * sizeof(uint4)));
    HIP_TRY(c->calls.reserve(cap_win * sizeof(kgx_call)));
    HIP_TRY(c->ranges.reserve(cap_win * 2 * sizeof(uint32_t)));
    HIP_TRY(c->hit_count.reserve((n_seq + 1) * sizeof(uint32_t)));
    HIP_TRY(c->call_count.reserve((n_seq + 1) * sizeof(uint32_t)));
    HIP_TRY(c->plan_status.reserve(4 * sizeof(uint32_t))); /* [0] bad offsets, [1] longest sequence (windows) */
    c->n_seq = n_seq;
    c->n_residues = n_residues;
    c->max_tiles = max_tiles;
    c->tile_windows = tile_windows;
    c->hit_slots = cap_win;
    c->d_off = d_off;
    c->counts_enqueued = 0;
    c->have_hits = false;
    c->have_best = false;
    c->have_otus = false;
    return KGX_OK;
}

}  // namespace kgx

namespace {

/* option probe_persist: the line probe's grid capped at that many
 * workgroups per CU (0 = uncapped) */
uint32_t probe_max_blocks(const kgx_ctx *c)
{
    if (!c->probe_persist)
        return 0;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->img->device) != hipSuccess || cus <= 0)
        cus = 256;
    return (uint32_t)c->probe_persist * (uint32_t)cus;
}

/* one probe launch on c's stream; with probe_serialize it waits for the
 * image's previous probe, whichever context issued it */
template <class Launch>
int probe_chained(kgx_ctx *c, Launch launch)
{
    HIP_TRY(hipSetDevice(c->img->device));
    if (c->img->num_sigs >= (1ull << 40))
        return fail(KGX_ERANGE, "image too large");
    kgx_image *img = c->img;
    std::unique_lock<std::mutex> lock(img->probe_mu, std::defer_lock);
    if (c->probe_serialize && c->probe_stream) {
        /* option probe_stream: every chained probe of the image on one stream
         * (one hardware queue), entered when this context's inputs are ready
         * and left back to this context's stream */
        lock.lock();
        if (!img->probe_stream)
            HIP_TRY(hipStreamCreateWithFlags(&img->probe_stream, hipStreamNonBlocking));
        if (!c->probe_ready)
            HIP_TRY(hipEventCreateWithFlags(&c->probe_ready, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(c->probe_ready, c->stream));
        HIP_TRY(hipStreamWaitEvent(img->probe_stream, c->probe_ready, 0));
        hipStream_t own = c->stream;
        c->stream = img->probe_stream; /* the launch reads c->stream */
        const hipError_t le = launch();
        c->stream = own;
        HIP_TRY(le);
        HIP_TRY(hipEventRecord(c->probe_done, img->probe_stream));
        HIP_TRY(hipStreamWaitEvent(c->stream, c->probe_done, 0));
        img->last_probe = c->probe_done;
    } else {
        if (c->probe_serialize) {
            lock.lock();
            if (img->last_probe && img->last_probe != c->probe_done)
                HIP_TRY(hipStreamWaitEvent(c->stream, img->last_probe, 0));
        }
        HIP_TRY(launch());
        if (c->probe_serialize) {
            HIP_TRY(hipEventRecord(c->probe_done, c->stream));
            img->last_probe = c->probe_done;
        }
    }
    /* every PACKED16 probe stores the matching record itself */
    c->hit_format = c->img->layout == KGX_LAYOUT_PACKED16 ? HIT_PACKED16 : HIT_PLANES;
    c->have_hits = true;
    return KGX_OK;
}

}  // namespace

namespace kgx {

bool probe_takes_dna(const kgx_ctx *c)
{
    return c->img->layout == KGX_LAYOUT_PACKED16 && !(c->probe_filter && c->img->d_filter) &&
           (c->probe_variant == PROBE_AUTO || c->probe_variant == PROBE_LINE) && c->probe_j >= 1 && c->probe_j <= 4;
}

int stage_probe_dna(kgx_ctx *c, const uint8_t *bases, uint64_t n_bases, const uint64_t *anchors,
                    const uint64_t *d_off)
{
    if ((!anchors || !bases) && c->n_seq)
        return fail(KGX_EINVAL, "fq probe: anchors or bases missing");
    if (d_off != c->d_off)
        return fail(KGX_EINVAL, "fq probe: offsets differ from the plan");
    if (!probe_takes_dna(c) || (int)(c->tile_windows / 64) != c->probe_j)
        return fail(KGX_EINVAL, "fq probe: fragments without residues need the line probe on a PACKED16 image "
                                "(set fq_residues 1 for other probes)");
    return probe_chained(c, [&] {
        return launch_probe_dna(bases, n_bases, anchors, c->wbase.as<uint64_t>(), c->tile_seq.as<uint32_t>(),
                                c->n_seq, c->max_tiles, ctx_probe_table(c), ctx_probe_buckets(c),
                                c->hits.as<uint4>(), c->hit_mask.as<uint64_t>(), (int)(c->tile_windows / 64),
                                probe_max_blocks(c), c->stream, ctx_home_shift(c));
    });
}

}  // namespace kgx

extern "C" {

int kgx_stage_probe(kgx_ctx *c, const uint8_t *d_res, const uint64_t *d_off)
{
    if (!c || (!d_res && c->n_residues) || d_off != c->d_off)
        return fail(KGX_EINVAL, "probe: residues missing or offsets differ from the plan");
    return probe_chained(c, [&] {
        return launch_probe(d_res, c->n_residues, d_off, c->wbase.as<uint64_t>(), c->tile_seq.as<uint32_t>(),
                            c->n_seq, c->max_tiles, ctx_probe_table(c), c->img->layout, ctx_probe_buckets(c),
                            c->probe_filter ? c->img->d_filter : nullptr, c->img->filter_log2_words,
                            c->hits.as<uint4>(), c->hits.as<uint4>() + c->hit_slots, c->hit_mask.as<uint64_t>(),
                            (int)(c->tile_windows / 64), c->probe_variant, (uint32_t)c->probe_lds_kb,
                            probe_max_blocks(c), c->stream, ctx_home_shift(c), (uint32_t)c->probe_nt);
    });
}



int kgx_stage_score(kgx_ctx *c, const kgx_params *params, uint32_t want)
{
    if (!c)
        return fail(KGX_EINVAL, "null ctx");
    kgx_params p;
    if (params)
        p = *params;
    else
        kgx_params_default(&p);
    HIP_TRY(hipSetDevice(c->img->device));
    const bool best = (want & KGX_WANT_BEST) != 0;
    HIP_TRY(launch_score(c->n_seq, c->n_residues, c->wbase.as<uint64_t>(), c->tile_seq.as<uint32_t>(), c->max_tiles,
                         c->hit_mask.as<uint64_t>(), c->tile_windows, c->hits.as<uint4>(), c->calls.as<kgx_call>(),
                         c->ranges.p, c->hit_count.as<uint32_t>(), c->call_count.as<uint32_t>(), p,
                         want | (best ? KGX_WANT_CALLS : 0u), c->hit_format, c->score_variant,
                         (uint32_t)c->score_wave_tiles, c->plan_status.as<uint32_t>(), c->stream));
    c->have_best = false;
    c->have_otus = false;
    if (want & KGX_WANT_OTU) {
        HIP_TRY(c->otu_ws.reserve(std::max<uint64_t>(c->hit_slots, 1) * sizeof(int32_t)));
        HIP_TRY(c->otus.reserve(std::max<uint64_t>(c->hit_slots, 1) * sizeof(kgx_otu)));
        HIP_TRY(c->otu_count.reserve(std::max<uint64_t>(c->n_seq, 1) * sizeof(uint32_t)));
        HIP_TRY(launch_otus(c->n_seq, c->wbase.as<uint64_t>(), c->hit_mask.as<uint64_t>(), c->tile_windows,
                            c->hits.as<uint4>(), c->hits.as<uint4>() + c->hit_slots, c->otu_ws.as<int32_t>(),
                            c->otus.as<kgx_otu>(), c->otu_count.as<uint32_t>(), c->hit_format, c->stream));
        c->have_otus = true;
    }
    if (best) {
        HIP_TRY(c->best.reserve(std::max<uint64_t>(c->n_seq, 1) * sizeof(kgx_best_call)));
        HIP_TRY(c->best_ws.reserve(c->hit_slots * sizeof(kgx_call)));
        if (!c->defer_best)
            HIP_TRY(launch_best_calls(c->n_seq, c->calls.as<kgx_call>(), c->wbase.as<uint64_t>(),
                                      c->call_count.as<uint32_t>(), c->best_ws.as<kgx_call>(),
                                      c->best.as<kgx_best_call>(), c->stream));
        c->have_best = true;
    }
    return KGX_OK;
}

int kgx_find_best_calls(kgx_ctx *c, const kgx_call *calls, const uint64_t *call_offsets, uint32_t n_seq,
                        kgx_best_call *out)
{
    if (!c || (n_seq && (!call_offsets || !out)))
        return fail(KGX_EINVAL, "null argument");
    if (n_seq == 0)
        return KGX_OK;
    const uint64_t c0 = call_offsets[0], n = call_offsets[n_seq] - c0;
    if (n && !calls)
        return fail(KGX_EINVAL, "null calls");
    std::vector<uint64_t> start(n_seq);
    std::vector<uint32_t> count(n_seq);
    for (uint32_t s = 0; s < n_seq; s++) {
        if (call_offsets[s + 1] < call_offsets[s])
            return fail(KGX_EINVAL, "call_offsets not monotone");
        start[s] = call_offsets[s] - c0;
        count[s] = (uint32_t)(call_offsets[s + 1] - call_offsets[s]);
    }
    HIP_TRY(hipSetDevice(c->img->device));
    HIP_TRY(c->bc_calls.reserve(std::max<uint64_t>(n, 1) * sizeof(kgx_call)));
    HIP_TRY(c->best_ws.reserve(std::max<uint64_t>(n, 1) * sizeof(kgx_call)));
    HIP_TRY(c->bc_start.reserve(n_seq * sizeof(uint64_t)));
    HIP_TRY(c->bc_count.reserve(n_seq * sizeof(uint32_t)));
    HIP_TRY(c->best.reserve(n_seq * sizeof(kgx_best_call)));
    c->have_best = false; /* best[] now belongs to this call, not to the plan */
    if (n)
        HIP_TRY(hipMemcpyAsync(c->bc_calls.p, calls + c0, n * sizeof(kgx_call), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->bc_start.p, start.data(), n_seq * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->bc_count.p, count.data(), n_seq * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(launch_best_calls(n_seq, c->bc_calls.as<kgx_call>(), c->bc_start.as<uint64_t>(),
                              c->bc_count.as<uint32_t>(), c->best_ws.as<kgx_call>(), c->best.as<kgx_best_call>(),
                              c->stream));
    HIP_TRY(hipMemcpyAsync(out, c->best.p, n_seq * sizeof(kgx_best_call), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return KGX_OK;
}

int kgx_device_result_get(kgx_ctx *c, kgx_device_result *out)
{
    if (!c || !out)
        return fail(KGX_EINVAL, "null argument");
    out->n_seq = c->n_seq;
    out->tile_windows = c->tile_windows;
    out->window_base = c->wbase.as<uint64_t>();
    out->hit_mask = c->hit_mask.as<uint64_t>();
    out->hit_count = c->hit_count.as<uint32_t>();
    out->call_count = c->call_count.as<uint32_t>();
    out->hits_hot = c->hits.as<uint32_t>();
    out->hits_cold = c->hit_format == HIT_PLANES ? c->hits.as<uint32_t>() + 4 * c->hit_slots : nullptr;
    out->hit_format = c->hit_format;
    out->otu_count = c->have_otus ? c->otu_count.as<uint32_t>() : nullptr;
    out->otus = c->have_otus ? c->otus.as<kgx_otu>() : nullptr;
    out->calls = c->calls.as<kgx_call>();
    out->best = c->have_best ? c->best.as<kgx_best_call>() : nullptr;
    return KGX_OK;
}

int kgx_run_device(kgx_ctx *c, const kgx_params *params, const uint8_t *d_res, const uint64_t *d_off,
                   uint32_t n_seq, uint64_t n_residues, uint32_t want, kgx_device_result *out)
{
    int rc = kgx_stage_plan(c, d_off, n_seq, n_residues);
    if (rc)
        return rc;
    if ((rc = kgx_stage_probe(c, d_res, d_off)))
        return rc;
    if (c->score_stream) {
        /* the score on its own stream behind the probe (kgx_pool_lookup) */
        if (!c->score_gate)
            HIP_TRY(hipEventCreateWithFlags(&c->score_gate, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(c->score_gate, c->stream));
        HIP_TRY(hipStreamWaitEvent(c->score_stream, c->score_gate, 0));
        hipStream_t own = c->stream;
        c->stream = c->score_stream;
        rc = kgx_stage_score(c, params, want);
        c->stream = own;
        if (rc)
            return rc;
    } else if ((rc = kgx_stage_score(c, params, want))) {
        return rc;
    }
    return out ? kgx_device_result_get(c, out) : KGX_OK;
}

int kgx_fq_run_device(kgx_ctx *c, const kgx_params *params, const kgx_fragments *fr, uint32_t want,
                      kgx_device_result *out)
{
    if (!c || !fr)
        return fail(KGX_EINVAL, "null argument");
    if (fr->residues || fr->n_fragments == 0)
        return kgx_run_device(c, params, fr->residues, fr->offsets, fr->n_fragments, fr->n_residues, want, out);
    /* the DNA probe's own tile (option fq_probe_j): its encode reads 24
     * bases and 32 table entries per window, and one slice per wave keeps
     * more waves' line requests in flight (C4 probe 4.0-4.3 vs 4.4-4.9 ms per
     * 1M reads at J = 1 vs 2, profiles/r3e_fq_probe_j_sweep.json).  The plan,
     * probe and score of the pass use it; the result carries its tile size. */
    HIP_TRY(hipSetDevice(c->img->device));
    const int keep_j = c->probe_j;
    if (c->fq_probe_j)
        c->probe_j = c->fq_probe_j;
    /* this context's own fragments (>= 11 residues each) are planned by one
     * elementwise kernel instead of launch_plan's reduce / scan / scan */
    const bool own = c->fq_plan && fr->offsets == c->fq_off.as<uint64_t>();
    int rc = own ? kgx::plan_reserve(c, fr->offsets, fr->n_fragments, fr->n_residues)
                 : kgx_stage_plan(c, fr->offsets, fr->n_fragments, fr->n_residues);
    if (!rc && own) {
        /* one longest-fragment word per 256-fragment workgroup */
        hipError_t e = c->plan_ws.reserve(((size_t)fr->n_fragments / 256 + 2) * sizeof(uint32_t));
        if (e == hipSuccess)
            e = launch_fq_plan(fr->offsets, fr->n_fragments, c->wbase.as<uint64_t>(), c->tile_seq.as<uint32_t>(),
                               c->tile_windows, c->plan_status.as<uint32_t>(), c->plan_ws.as<uint32_t>(), c->stream);
        if (e != hipSuccess)
            rc = fail(KGX_EDEVICE, std::string("fq plan: ") + hipGetErrorString(e));
    }
    if (!rc)
        rc = stage_probe_dna(c, fr->bases, fr->n_bases, fr->anchors, fr->offsets);
    c->probe_j = keep_j;
    if (rc)
        return rc;
    if ((rc = kgx_stage_score(c, params, want)))
        return rc;
    return out ? kgx_device_result_get(c, out) : KGX_OK;
}

/* ---- host-buffer batch ---------------------------------------------------- */

namespace {

/* a sequence is cut at its first NUL (strlen bound of gather_hits,
 * kguts.cc:792): the NUL's predecessor and everything after become 'X', which
 * kills exactly the windows the reference never visits */
void cut_at_nul(char *b, uint64_t len)
{
    const void *z = len ? std::memchr(b, 0, len) : nullptr;
    if (z) {
        const uint64_t slen = (uint64_t)((const char *)z - b);
        for (uint64_t i = slen ? slen - 1 : 0; i < len; i++)
            b[i] = 'X';
    }
}

/* the n + 1 chunk-relative offsets of sequences [s0, s1) */
void stage_offsets_into(uint64_t *off, const uint64_t *seq_offsets, uint32_t s0, uint32_t s1)
{
    const uint32_t n = s1 - s0;
    const uint64_t r0 = n ? seq_offsets[s0] : 0;
    for (uint32_t i = 0; i <= n; i++)
        off[i] = n ? seq_offsets[s0 + i] - r0 : 0;
}

/* sequences [s0, s1) of a host batch -> pinned staging at dst (residues) and
 * off (the n + 1 chunk-relative offsets); host work only, large ranges copied
 * and NUL-scanned in parts on the stage pool sp */
void stage_copy_into(char *dst, uint64_t *off, const char *residues, const uint64_t *seq_offsets, uint32_t s0,
                     uint32_t s1, HostPool *sp)
{
    const uint32_t n = s1 - s0;
    const uint64_t r0 = n ? seq_offsets[s0] : 0;
    const uint64_t n_res = n ? seq_offsets[s1] - r0 : 0;
    bool has_nul = false;
    if (sp && n_res >= (1u << 20)) {
        const unsigned P = sp->size();
        std::atomic<bool> nul{false};
        const char *src = residues + r0;
        for (unsigned p = 0; p < P; p++) {
            const uint64_t a = n_res * p / P, b = n_res * (p + 1) / P;
            sp->submit([dst, src, a, b, &nul]() -> int {
                std::memcpy(dst + a, src + a, b - a);
                if (std::memchr(dst + a, 0, b - a))
                    nul.store(true, std::memory_order_relaxed);
                return KGX_OK;
            });
        }
        (void)sp->wait();
        has_nul = nul.load();
    } else if (n_res) {
        std::memcpy(dst, residues + r0, n_res);
        /* one scan of the whole range first: NUL bytes are rare */
        has_nul = std::memchr(dst, 0, n_res) != nullptr;
    }
    if (has_nul)
        for (uint32_t s = s0; s < s1; s++)
            cut_at_nul(dst + (seq_offsets[s] - r0), seq_offsets[s + 1] - seq_offsets[s]);
    for (uint32_t i = 0; i <= n; i++)
        off[i] = n ? seq_offsets[s0 + i] - r0 : 0;
}

/* sequences [s0, s1) of a host batch -> x's pinned staging */
int stage_host_copy(kgx_ctx *x, const char *residues, const uint64_t *seq_offsets, uint32_t s0, uint32_t s1,
                    HostPool *sp = nullptr)
{
    const uint32_t n = s1 - s0;
    HIP_TRY(x->h_res.resize(n ? seq_offsets[s1] - seq_offsets[s0] : 0));
    HIP_TRY(x->h_off_stage.resize(n + 1));
    stage_copy_into(x->h_res.data(), x->h_off_stage.data(), residues, seq_offsets, s0, s1, sp);
    return KGX_OK;
}

/* x's staged sequences -> HBM (async on x's stream) */
int stage_upload(kgx_ctx *x)
{
    const uint64_t n_res = x->h_res.size(), n1 = x->h_off_stage.size();
    HIP_TRY(x->residues.reserve(n_res + 16));
    HIP_TRY(x->offsets.reserve(n1 * sizeof(uint64_t)));
    HIP_TRY(hipMemcpyAsync(x->offsets.p, x->h_off_stage.data(), n1 * sizeof(uint64_t), hipMemcpyHostToDevice,
                           x->stream));
    if (n_res)
        HIP_TRY(hipMemcpyAsync(x->residues.p, x->h_res.data(), n_res, hipMemcpyHostToDevice, x->stream));
    return KGX_OK;
}

int stage_host_seqs(kgx_ctx *x, const char *residues, const uint64_t *seq_offsets, uint32_t s0, uint32_t s1)
{
    int rc = stage_host_copy(x, residues, seq_offsets, s0, s1);
    return rc ? rc : stage_upload(x);
}

/* one staged chunk on x: H2D, plan/probe/score, counts + window total -> host */
int enqueue_chunk(kgx_ctx *x, const kgx_params *params, uint32_t want, hipEvent_t counts_done)
{
    int rc = stage_upload(x);
    if (rc)
        return rc;
    const uint32_t n = (uint32_t)x->h_off_stage.size() - 1;
    const uint64_t n_res = x->h_res.size();
    if ((rc = kgx_run_device(x, params, x->residues.as<uint8_t>(), x->offsets.as<uint64_t>(), n, n_res, want,
                             nullptr)))
        return rc;
    HIP_TRY(x->h_hcount.resize(n + 1));
    HIP_TRY(x->h_ccount.resize(n + 1));
    HIP_TRY(x->h_ocount.resize(n + 1));
    HIP_TRY(x->h_nwin.resize(1));
    if (n) {
        HIP_TRY(hipMemcpyAsync(x->h_hcount.data(), x->hit_count.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                               x->stream));
        HIP_TRY(hipMemcpyAsync(x->h_ccount.data(), x->call_count.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                               x->stream));
        if (want & KGX_WANT_OTU)
            HIP_TRY(hipMemcpyAsync(x->h_ocount.data(), x->otu_count.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   x->stream));
    }
    HIP_TRY(hipMemcpyAsync(x->h_nwin.data(), x->wbase.as<uint64_t>() + n, sizeof(uint64_t),
                           hipMemcpyDeviceToHost, x->stream));
    HIP_TRY(hipEventRecord(counts_done, x->stream));
    return KGX_OK;
}

void fill_result(kgx_ctx *c, uint32_t n_seq, bool need_hits, bool want_best, uint64_t nwin, kgx_result *out)
{
    out->best = want_best ? c->h_best.data() : nullptr;
    out->n_seq = n_seq;
    out->hit_offsets = c->h_hoff.data();
    out->hits = need_hits ? c->h_hits.data() : nullptr;
    out->call_offsets = c->h_coff.data();
    out->calls = c->h_calls.data();
    out->otu_offsets = c->h_ooff.data();
    out->otus = c->h_otus.data();
    out->n_windows = nwin;
}

/* residue byte -> code, to_amino_acid_off (kguts.cc:273-339): the 20
 * standard upper-case residues in alphabetical order, anything else 20 */
struct ResidueCodes {
    uint8_t code[256];
    ResidueCodes()
    {
        std::memset(code, 20, sizeof(code));
        const char *aa = "ACDEFGHIKLMNPQRSTVWY";
        for (int i = 0; i < 20; i++)
            code[(uint8_t)aa[i]] = (uint8_t)i;
    }
};
const ResidueCodes kResidueCodes;

/* the 8-mer key of the window at p (encoded_kmer, kguts.cc:438-455) */
inline uint64_t window_key(const uint8_t *p)
{
    const uint8_t *t = kResidueCodes.code;
    const uint32_t ka = ((t[p[0]] * 20u + t[p[1]]) * 20u + t[p[2]]) * 20u + t[p[3]];
    const uint32_t kb = ((t[p[4]] * 20u + t[p[5]]) * 20u + t[p[6]]) * 20u + t[p[7]];
    return (uint64_t)ka * 160000u + kb;
}

}  // namespace

extern "C++" {
namespace kgx {

/* Sequences [a, b) of a compact chunk: table records (dense, CSR order) +
 * the chunk's hit mask -> kgx_hit, position = the hit's mask bit minus the
 * sequence's first window (what gather_kernel computes on the device).
 * 3-word records: the 12-byte form without the key (gather_kernel's hits12),
 * the key re-encoded from the window's residues; 4 words: the 16-byte table
 * records. */

template <bool R12>
static int expand_chunk_t(const kgx_hit_chunk &ch, const uint64_t *hoff, const char *residues,
                          const uint64_t *seq_offsets, uint32_t a, uint32_t b, kgx_hit *out, uint64_t out_base,
                          uint32_t seq_base, bool nt)
{
    const uint64_t *mask = ch.mask;
    for (uint32_t s = a; s < b; s++) {
        uint64_t j = hoff[s];
        const uint64_t j1 = hoff[s + 1];
        if (j == j1)
            continue;
        const uint64_t w0 = ch.window_start[s - ch.seq_begin], w1 = w0 + windows_of(seq_offsets[s + 1] - seq_offsets[s]);
        if (w1 == w0)
            return fail(KGX_EDEVICE, "compact hits: hits for a sequence without windows (" + std::to_string(s) + ")");
        const uint8_t *seq = reinterpret_cast<const uint8_t *>(residues + seq_offsets[s]);
        for (uint64_t g = w0 >> 6; g <= (w1 - 1) >> 6; g++) {
            uint64_t bits = mask[g];
            if (g == w0 >> 6)
                bits &= ~0ull << (w0 & 63);
            if (g == (w1 - 1) >> 6 && (w1 & 63))
                bits &= ~(~0ull << (w1 & 63));
            if (j + (uint64_t)__builtin_popcountll(bits) > j1)
                return fail(KGX_EDEVICE, "compact hits: more mask bits than hits for sequence " + std::to_string(s));
            for (; bits; bits &= bits - 1, j++) {
                const uint32_t pos = (uint32_t)(64 * g + (uint64_t)__builtin_ctzll(bits) - w0);
                const uint32_t *r = ch.records + (R12 ? 3 : 4) * (j - ch.hit_begin);
                packed_bucket pb;
                uint32_t flags;
                if (R12) {
                    pb.lo = window_key(seq + pos) | (uint64_t)r[2] << 35;
                    pb.hi = (uint64_t)r[1] << 32 | r[0];
                    flags = (r[1] >> 28) & 7u;
                } else {
                    pb.lo = (uint64_t)r[1] << 32 | r[0];
                    pb.hi = (uint64_t)r[3] << 32 | r[2];
                    flags = (r[3] >> 28) & 7u;
                }
                const kgx_sig_kmer e = unpack_bucket(pb);
                kgx_hit o;
                o.which_kmer = e.which_kmer;
                o.otu_index = e.otu_index;
                o.avg_from_end = e.avg_from_end;
                o.flags = (uint16_t)flags;
                o.function_index = e.function_index;
                o.function_wt = e.function_wt;
                o.pos = pos;
                o.seq = s + seq_base;
                kgx_hit *dst = out + (j - out_base);
                if (nt) {
                    /* streaming stores: the 32-B records are written once and
                     * not read back here (no read-for-ownership of the lines) */
                    typedef long long v2i __attribute__((vector_size(16)));
                    v2i q[2];
                    std::memcpy(q, &o, sizeof(o));
                    __builtin_nontemporal_store(q[0], reinterpret_cast<v2i *>(dst));
                    __builtin_nontemporal_store(q[1], reinterpret_cast<v2i *>(dst) + 1);
                } else {
                    *dst = o;
                }
            }
        }
        if (j != j1)
            return fail(KGX_EDEVICE, "compact hits: mask and hit count disagree for sequence " + std::to_string(s));
    }
    if (nt)
        __builtin_ia32_sfence(); /* the streaming stores are visible before the task reports done */
    return KGX_OK;
}

int expand_chunk(const kgx_hit_chunk &ch, const uint64_t *hoff, const char *residues, const uint64_t *seq_offsets,
                 uint32_t a, uint32_t b, kgx_hit *out, uint64_t out_base, uint32_t seq_base, bool nt)
{
    if (ch.record_words == 3)
        return expand_chunk_t<true>(ch, hoff, residues, seq_offsets, a, b, out, out_base, seq_base, nt);
    if (ch.record_words == 4)
        return expand_chunk_t<false>(ch, hoff, residues, seq_offsets, a, b, out, out_base, seq_base, nt);
    return fail(KGX_EINVAL, "compact hits: record_words must be 3 or 4");
}

}  // namespace kgx
}  // extern "C++"

extern "C++" {
namespace kgx {

/* kgx_device_batch_collect's first round trip, enqueued: the plan status,
 * window total and per-sequence counts (and, when nothing needs gathering --
 * the /lookup shape, hits staying on the device -- the best calls) by device
 * stores into the mapped pinned arrays, not by DMA: copies from every stream
 * share the DMA engine in order, so a few KB of counts queued behind other
 * contexts' MB uploads (r5m).  A pool enqueues these right behind each
 * shard's pass, so they do not wait in a shared hardware queue behind a later
 * shard's work (r5s). */
int collect_counts_enqueue(kgx_ctx *c, uint32_t want)
{
    const bool want_calls = (want & KGX_WANT_CALLS) != 0;
    const bool want_otu = (want & KGX_WANT_OTU) != 0;
    const bool need_hits = (want & KGX_WANT_HITS) != 0;
    const bool want_best = (want & KGX_WANT_BEST) != 0;
    const uint32_t n_seq = c->n_seq;
    HIP_TRY(hipSetDevice(c->img->device));
    HIP_TRY(c->h_hcount.resize(n_seq + 1));
    HIP_TRY(c->h_ccount.resize(n_seq + 1));
    HIP_TRY(c->h_ocount.resize(n_seq + 1));
    HIP_TRY(c->h_plan_status.resize(1));
    HIP_TRY(c->h_nwin.resize(1));
    c->h_plan_status[0] = 0;
    CopySpans sp; /* one launch for all of them */
    auto d2h = [&](auto &vec, const void *src, size_t bytes) -> hipError_t {
        void *d = nullptr;
        const hipError_t e = vec.device_ptr(0, &d);
        if (e == hipSuccess)
            sp.add(d, src, bytes);
        return e;
    };
    if (c->plan_status.p)
        HIP_TRY(d2h(c->h_plan_status, c->plan_status.p, sizeof(uint32_t)));
    HIP_TRY(d2h(c->h_nwin, c->wbase.as<uint64_t>() + n_seq, sizeof(uint64_t)));
    if (n_seq) {
        HIP_TRY(d2h(c->h_hcount, c->hit_count.p, n_seq * sizeof(uint32_t)));
        HIP_TRY(d2h(c->h_ccount, c->call_count.p, n_seq * sizeof(uint32_t)));
        if (want_otu)
            HIP_TRY(d2h(c->h_ocount, c->otu_count.p, n_seq * sizeof(uint32_t)));
    }
    if (want_best && n_seq && !need_hits && !want_calls && !want_otu) {
        HIP_TRY(c->h_best.resize(n_seq));
        HIP_TRY(d2h(c->h_best, c->best.p, n_seq * sizeof(kgx_best_call)));
    }
    HIP_TRY(launch_copy_spans(sp, 64, c->stream));
    c->counts_enqueued = want + 1;
    return KGX_OK;
}

/* One pass over a whole host batch, split so that a pool can enqueue its
 * shards in order from one thread and collect them on several: the staging
 * (or, for residues in the caller's pinned memory, nothing) and the upload by
 * pull kernels -- on `up` with `up_done` recorded, which the context's stream
 * waits for, when given, else on the context's stream -- then the device pass
 * (plan, probe, score).  A caller-pinned batch is NUL-scanned on the device. */
int one_pass_enqueue(kgx_ctx *c, const kgx_params *params, const char *residues, const uint64_t *seq_offsets,
                     uint32_t n_seq, uint32_t want, hipStream_t up, hipEvent_t up_done, HostPool *stage)
{
    const uint64_t r0 = n_seq ? seq_offsets[0] : 0, n_res = n_seq ? seq_offsets[n_seq] - r0 : 0;
    /* the residues to copy: the caller's pinned buffer, or our staging */
    const void *src = residues + r0;
    const bool pin = c->pinned_input && host_pinned_range(residues + r0, n_res);
    c->one_pass_pinned = pin;
    if (pin) {
        HIP_TRY(c->h_off_stage.resize(n_seq + 1));
        stage_offsets_into(c->h_off_stage.data(), seq_offsets, 0, n_seq);
        c->pinned_batches++;
    } else {
        HostPool *sp = stage;
        if (!sp && c->stage_threads > 1 && n_res >= (1u << 20)) {
            if (!c->stage_pool || c->stage_pool->size() != (unsigned)c->stage_threads)
                c->stage_pool.reset(new HostPool((unsigned)c->stage_threads));
            sp = c->stage_pool.get();
        }
        if (int rc = stage_host_copy(c, residues, seq_offsets, 0, n_seq, sp))
            return rc;
        src = c->h_res.data();
    }
    /* up by DMA, the small copy first (the DMA engine serves every stream in
     * order).  With `up` the copies go on that stream and the context's
     * stream waits for an event: a pool enqueues its shards' uploads on one
     * such stream and their passes in shard order, so a hardware queue shared
     * by two shards' streams never holds a shard's kernels behind a later
     * shard's upload (r5o: per-shard threads uploading on their own streams
     * at once did).  Uploads by kernels reading the mapped memory instead
     * measured worse: the device's PCIe reads held up the other shards'
     * kernels (r5q/r5r: a 10-us plan kernel took 140 us beside them). */
    HIP_TRY(c->residues.reserve(n_res + 16));
    HIP_TRY(c->offsets.reserve((n_seq + 1) * sizeof(uint64_t)));
    hipStream_t us = up ? up : c->stream;
    HIP_TRY(hipMemcpyAsync(c->offsets.p, c->h_off_stage.data(), (n_seq + 1) * sizeof(uint64_t),
                           hipMemcpyHostToDevice, us));
    if (n_res)
        HIP_TRY(hipMemcpyAsync(c->residues.p, src, n_res, hipMemcpyHostToDevice, us));
    if (up) {
        HIP_TRY(hipEventRecord(up_done, up));
        HIP_TRY(hipStreamWaitEvent(c->stream, up_done, 0));
    }
    if (pin) {
        HIP_TRY(c->h_nul.resize(1));
        c->h_nul[0] = 0;
        void *dn = nullptr;
        HIP_TRY(c->h_nul.device_ptr(0, &dn));
        HIP_TRY(launch_nul_scan(c->residues.as<uint8_t>(), 0, n_res, static_cast<uint32_t *>(dn), c->stream));
    }
    /* on the wave scorer, the host knows whether any sequence needs the lane
     * machine's long-sequence pass (score_long): usually none does */
    const int variant = c->score_variant;
    if (c->score_variant == SCORE_WAVE) {
        uint64_t longest = 0;
        for (uint32_t s = 0; s < n_seq; s++)
            longest = std::max(longest, seq_offsets[s + 1] - seq_offsets[s]);
        if (windows_of(longest) <= (uint64_t)RUN_CAP)
            c->score_variant = SCORE_WAVE_ONLY;
    }
    const int rc = kgx_run_device(c, params, c->residues.as<uint8_t>(), c->offsets.as<uint64_t>(), n_seq, n_res,
                                  want, nullptr);
    c->score_variant = variant;
    return rc;
}

/* the enqueued pass's results (kgx_device_batch_collect); a caller-pinned
 * batch whose scan found a NUL runs again, staged and cut at the NUL */
int one_pass_collect(kgx_ctx *c, const kgx_params *params, const char *residues, const uint64_t *seq_offsets,
                     uint32_t n_seq, uint32_t want, kgx_result *out)
{
    int rc = kgx_device_batch_collect(c, want, out);
    if (!rc && c->one_pass_pinned && __atomic_load_n(&c->h_nul[0], __ATOMIC_ACQUIRE)) {
        c->nul_reruns++;
        c->pinned_input = 0;
        rc = one_pass_enqueue(c, params, residues, seq_offsets, n_seq, want, nullptr, nullptr);
        if (!rc)
            rc = kgx_device_batch_collect(c, want, out);
        c->pinned_input = 1;
    }
    return rc;
}

}  // namespace kgx
}  // extern "C++"

namespace {

/* the context's own expansion (into h_hits, CSR numbering): R12 records of
 * hit j at h_hits12 + 3 (j + rec_delta), else h_hits16[j + rec_delta]; the
 * chunk's mask from h_mask + mbase */
int expand_hits(bool R12, kgx_ctx *c, const char *residues, const uint64_t *seq_offsets, uint32_t a, uint32_t b,
                uint64_t mbase, int64_t rec_delta)
{
    kgx_hit_chunk ch{};
    ch.seq_begin = 0;
    ch.record_words = R12 ? 3 : 4;
    ch.hit_begin = 0;
    ch.records = R12 ? c->h_hits12.data() + 3 * rec_delta
                     : reinterpret_cast<const uint32_t *>(c->h_hits16.data() + rec_delta);
    ch.mask = c->h_mask.data() + mbase;
    ch.window_start = c->h_wstart.data();
    return expand_chunk(ch, c->h_hoff.data(), residues, seq_offsets, a, b, c->h_hits.data(), 0, 0, c->host_nt != 0);
}


/* Streamed host batch (compact records, PACKED16 images): no host round
 * trip inside a chunk.  Each chunk runs on its context's stream as
 *   H2D -> plan/probe/score -> count scan (device CSR offsets) -> gather
 *   into dense buffers (+ mask, counts, best calls)
 * and its bulk device-to-host copy runs on the copy stream, sized on the
 * device (the scanned totals) into host regions whose room the host set from
 * the chunk's window count and the hit / call / OTU rates seen so far.  The
 * host enqueues every chunk up front (each context's staging buffer is
 * reused once its H2D is done), then, chunk by chunk as the copies land,
 * builds the CSR offsets from the counts, moves calls / OTUs into place and
 * hands the records to the expansion threads.  A chunk whose results did not
 * fit its region makes the call return STREAM_OVERFLOW after raising the rates;
 * the caller reruns the batch on the exact (host round trip) path. */
constexpr int STREAM_OVERFLOW = 1; /* internal: a region overflowed, rerun exact */
constexpr int STREAM_NUL = 2;      /* internal: the caller's pinned residues hold a NUL, rerun staged */

int process_batch_streamed(kgx_ctx *c, const kgx_params *params, const char *residues, const uint64_t *seq_offsets,
                           uint32_t n_seq, uint32_t want, uint32_t K, const std::vector<uint32_t> &cut,
                           kgx_result *out)
{
    kgx_ctx *t = c->twin;
    kgx_ctx *xs[2] = {c, t};
    const bool want_calls = (want & KGX_WANT_CALLS) != 0;
    const bool want_otu = (want & KGX_WANT_OTU) != 0;
    const bool want_best = (want & KGX_WANT_BEST) != 0;
    const bool timing = std::getenv("KGX_TIMING") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto T0 = now();

    /* per-chunk windows, regions and offsets */
    std::vector<uint64_t> win(K, 0), cap_h(K), cap_c(K), cap_o(K), rb_h(K + 1, 0), rb_c(K + 1, 0), rb_o(K + 1, 0),
        mb(K + 1, 0);
    c->h_wstart.resize(n_seq);
    for (uint32_t k = 0; k < K; k++) {
        uint64_t w = 0;
        for (uint32_t s = cut[k]; s < cut[k + 1]; s++) {
            c->h_wstart[s] = w;
            w += windows_of(seq_offsets[s + 1] - seq_offsets[s]);
        }
        win[k] = w;
        /* region starts stay 16-B aligned: multiples of 4 records */
        auto room = [w](double rate, uint64_t extra) {
            return (std::min<uint64_t>(w, (uint64_t)(rate * (double)w) + extra) + 3) & ~3ull;
        };
        cap_h[k] = room(c->rate_hits, 256);
        cap_c[k] = want_calls ? room(c->rate_calls, 64) : 0;
        cap_o[k] = want_otu ? room(c->rate_otus, 64) : 0;
        rb_h[k + 1] = rb_h[k] + cap_h[k];
        rb_c[k + 1] = rb_c[k] + cap_c[k];
        rb_o[k + 1] = rb_o[k] + cap_o[k];
        mb[k + 1] = mb[k] + (((w + 63) / 64 + 1) & ~1ull); /* 16-B aligned mask regions */
    }
    /* pinned host regions: resized before any copy or expansion is in flight */
    const bool r12 = c->host_rec12 != 0;
    if (r12)
        HIP_TRY(c->h_hits12.resize(3 * rb_h[K]));
    else
        HIP_TRY(c->h_hits16.resize(rb_h[K]));
    HIP_TRY(c->h_mask.resize(mb[K]));
    HIP_TRY(c->h_calls_region.resize(rb_c[K]));
    HIP_TRY(c->h_otus_region.resize(rb_o[K]));
    HIP_TRY(c->h_counts.resize(3 * (uint64_t)n_seq));
    const bool expand = !c->compact_out;
    if (expand)
        HIP_TRY(c->h_hits.resize(rb_h[K])); /* room for every region's records; trimmed below */
    /* host_profile: timing events per chunk (4 on the contexts' streams, 1 on the copy stream) */
    const bool prof = c->host_profile != 0;
    if (prof) {
        auto grow = [](std::vector<hipEvent_t> &v, size_t n) -> hipError_t {
            while (v.size() < n) {
                hipEvent_t e;
                hipError_t err = hipEventCreate(&e);
                if (err != hipSuccess)
                    return err;
                v.push_back(e);
            }
            return hipSuccess;
        };
        HIP_TRY(grow(c->prof_ev, 4 * (size_t)K));
        HIP_TRY(grow(c->prof_done, K));
    }
    double stage_ms = 0;
    std::atomic<uint64_t> expand_ns{0};
    c->compact_segs.clear();
    HIP_TRY(c->h_best.resize(want_best ? n_seq : 0));
    c->h_hoff.assign(n_seq + 1, 0);
    c->h_coff.assign(n_seq + 1, 0);
    c->h_ooff.assign(n_seq + 1, 0);

    /* device buffers of both contexts at the largest chunk's size up front:
     * no reallocation while earlier chunks still read them */
    uint64_t max_res = 1, max_n = 1;
    for (uint32_t k = 0; k < K; k++) {
        max_res = std::max(max_res, seq_offsets[cut[k + 1]] - seq_offsets[cut[k]]);
        max_n = std::max<uint64_t>(max_n, cut[k + 1] - cut[k]);
    }
    for (kgx_ctx *x : xs) {
        HIP_TRY(x->residues.reserve(max_res + 16));
        HIP_TRY(x->offsets.reserve((max_n + 1) * sizeof(uint64_t)));
        HIP_TRY(x->dense_hoff.reserve((max_n + 1) * sizeof(uint64_t)));
        HIP_TRY(x->dense_coff.reserve((max_n + 1) * sizeof(uint64_t)));
        HIP_TRY(x->dense_ooff.reserve((max_n + 1) * sizeof(uint64_t)));
        HIP_TRY(x->cscan_ws.reserve(count_scan_workspace_bytes((uint32_t)max_n)));
        HIP_TRY(x->dense_hits.reserve(max_res * 16));
        if (want_calls)
            HIP_TRY(x->dense_calls.reserve(max_res * sizeof(kgx_call)));
        if (want_otu)
            HIP_TRY(x->dense_otus.reserve(max_res * sizeof(kgx_otu)));
        HIP_TRY(x->dense_mask.reserve((max_res / 64 + 2) * sizeof(uint64_t)));
        HIP_TRY(x->dense_counts.reserve(3 * max_n * sizeof(uint32_t)));
        if (want_best)
            HIP_TRY(x->dense_best.reserve(max_n * sizeof(kgx_best_call)));
    }

    hipStream_t cs = c->copy_stream;
    const int cb = c->host_copy_blocks;
    auto mapped = [](auto &v, uint64_t at, void **d) -> hipError_t { return v.device_ptr(at, d); };
    /* host_upload_stream: each chunk's regions of up_res (256-B aligned, 16
     * bytes of slack for the probe's 16-B residue loads) and up_off */
    const bool up = c->host_upload_stream != 0;
    std::vector<uint64_t> res_at(K + 1, 0), off_at(K + 1, 0);
    for (uint32_t k = 0; k < K; k++) {
        res_at[k + 1] = res_at[k] + ((seq_offsets[cut[k + 1]] - seq_offsets[cut[k]] + 16 + 255) & ~255ull);
        off_at[k + 1] = off_at[k] + ((cut[k + 1] - cut[k] + 1 + 1) & ~1ull);
    }
    if (up) {
        HIP_TRY(c->up_res.reserve(std::max<uint64_t>(res_at[K], 256)));
        HIP_TRY(c->up_off.reserve(std::max<uint64_t>(off_at[K], 2) * sizeof(uint64_t)));
    }
    /* host_stage_all: every chunk staged into a pinned region of its own (the
     * same res_at / off_at layout), so no staging waits for the H2D of the
     * chunk two before to free its context's staging buffer */
    const bool sall = c->host_stage_all != 0;
    if (sall) {
        HIP_TRY(c->h_res_all.resize(std::max<uint64_t>(res_at[K], 256)));
        HIP_TRY(c->h_off_all.resize(std::max<uint64_t>(off_at[K], 2)));
    }
    /* caller-pinned residues: no staging copy, a device NUL scan instead */
    const uint64_t all_res = n_seq ? seq_offsets[n_seq] - seq_offsets[0] : 0;
    const bool pin = c->pinned_input && host_pinned_range(residues + (n_seq ? seq_offsets[0] : 0), all_res);
    uint32_t *d_nul = nullptr;
    if (pin) {
        HIP_TRY(c->h_nul.resize(1));
        c->h_nul[0] = 0;
        void *dn = nullptr;
        HIP_TRY(c->h_nul.device_ptr(0, &dn));
        d_nul = static_cast<uint32_t *>(dn);
        c->pinned_batches++;
    }
    auto staged_res = [&](kgx_ctx *x, uint32_t k) -> const char * {
        if (pin)
            return residues + seq_offsets[cut[k]];
        return sall ? c->h_res_all.data() + res_at[k] : x->h_res.data();
    };
    auto staged_off = [&](kgx_ctx *x, uint32_t k) -> const uint64_t * {
        return sall ? c->h_off_all.data() + off_at[k] : x->h_off_stage.data();
    };

    /* enqueue chunk k on x: everything up to its bulk copy */
    auto enqueue = [&](kgx_ctx *x, uint32_t k) -> int {
        const uint32_t s0 = cut[k], n = cut[k + 1] - cut[k];
        const uint64_t n_res = n ? seq_offsets[cut[k + 1]] - seq_offsets[s0] : 0;
        const char *hres = staged_res(x, k);
        const uint64_t *hoff = staged_off(x, k);
        hipStream_t us = up ? c->up_stream : x->stream;
        if (prof)
            HIP_TRY(hipEventRecord(c->prof_ev[4 * k], us));
        const uint8_t *d_res = x->residues.as<uint8_t>();
        const uint64_t *d_off = x->offsets.as<uint64_t>();
        int rc = KGX_OK;
        if (up) {
            uint8_t *rd = c->up_res.as<uint8_t>() + res_at[k];
            uint64_t *od = c->up_off.as<uint64_t>() + off_at[k];
            HIP_TRY(hipMemcpyAsync(od, hoff, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, us));
            if (n_res)
                HIP_TRY(hipMemcpyAsync(rd, hres, n_res, hipMemcpyHostToDevice, us));
            d_res = rd;
            d_off = od;
        } else {
            /* reserved for the largest chunk above: no reallocation here */
            HIP_TRY(x->residues.reserve(n_res + 16));
            HIP_TRY(x->offsets.reserve((n + 1) * sizeof(uint64_t)));
            HIP_TRY(hipMemcpyAsync(x->offsets.p, hoff, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, us));
            if (n_res)
                HIP_TRY(hipMemcpyAsync(x->residues.p, hres, n_res, hipMemcpyHostToDevice, us));
        }
        HIP_TRY(hipEventRecord(c->chunk_h2d[k], us));
        if (pin)
            HIP_TRY(launch_nul_scan(d_res, 0, n_res, d_nul, us));
        if (prof)
            HIP_TRY(hipEventRecord(c->prof_ev[4 * k + 1], us));
        if (up)
            HIP_TRY(hipStreamWaitEvent(x->stream, c->chunk_h2d[k], 0));
        if ((rc = kgx_run_device(x, params, d_res, d_off, n, n_res, want, nullptr)))
            return rc;
        if (prof)
            HIP_TRY(hipEventRecord(c->prof_ev[4 * k + 2], x->stream));
        const uint64_t rn = std::max<uint64_t>(n_res, 1); /* dense buffers: at most one record per residue */
        HIP_TRY(x->dense_hoff.reserve((n + 1) * sizeof(uint64_t)));
        HIP_TRY(x->dense_coff.reserve((n + 1) * sizeof(uint64_t)));
        HIP_TRY(x->dense_ooff.reserve((n + 1) * sizeof(uint64_t)));
        HIP_TRY(x->cscan_ws.reserve(count_scan_workspace_bytes(n)));
        /* x's dense buffers still feed chunk k-2's bulk copy, and so do its
         * scanned totals (dense_hoff/coff/ooff + n, read by the counted copies
         * when they run): nothing of chunk k touches them before that is done */
        if (k >= 2)
            HIP_TRY(hipStreamWaitEvent(x->stream, c->chunk_done[k - 2], 0));
        HIP_TRY(launch_count_scan(n, x->hit_count.as<uint32_t>(), want_calls ? x->call_count.as<uint32_t>() : nullptr,
                                  want_otu ? x->otu_count.as<uint32_t>() : nullptr, x->dense_hoff.as<uint64_t>(),
                                  x->dense_coff.as<uint64_t>(), x->dense_ooff.as<uint64_t>(), x->cscan_ws.p,
                                  x->stream));
        HIP_TRY(x->dense_hits.reserve(rn * 16));
        if (want_calls)
            HIP_TRY(x->dense_calls.reserve(rn * sizeof(kgx_call)));
        if (want_otu)
            HIP_TRY(x->dense_otus.reserve(rn * sizeof(kgx_otu)));
        HIP_TRY(launch_gather(n, x->wbase.as<uint64_t>(), x->hit_mask.as<uint64_t>(), x->tile_windows,
                              x->call_count.as<uint32_t>(), x->hits.as<uint4>(), x->hits.as<uint4>() + x->hit_slots,
                              x->calls.as<kgx_call>(), x->dense_hoff.as<uint64_t>(), x->dense_coff.as<uint64_t>(),
                              nullptr, want_calls ? x->dense_calls.as<kgx_call>() : nullptr, s0, x->hit_format,
                              x->otu_count.as<uint32_t>(), x->otus.as<kgx_otu>(), x->dense_ooff.as<uint64_t>(),
                              want_otu ? x->dense_otus.as<kgx_otu>() : nullptr, x->stream,
                              r12 ? nullptr : x->dense_hits.as<uint4>(), r12 ? x->dense_hits.as<uint32_t>() : nullptr));
        /* what chunk k+2's kernels overwrite: mask, counts, best calls */
        const uint64_t nwords = (win[k] + 63) / 64;
        if (nwords) {
            HIP_TRY(x->dense_mask.reserve(nwords * sizeof(uint64_t)));
            HIP_TRY(launch_copy_to_host(x->dense_mask.p, x->hit_mask.p, nwords * sizeof(uint64_t), 256, x->stream));
        }
        if (n) {
            HIP_TRY(x->dense_counts.reserve(3 * (uint64_t)n * sizeof(uint32_t)));
            uint32_t *dc = x->dense_counts.as<uint32_t>();
            HIP_TRY(launch_copy_to_host(dc, x->hit_count.p, n * sizeof(uint32_t), 64, x->stream));
            if (want_calls)
                HIP_TRY(launch_copy_to_host(dc + n, x->call_count.p, n * sizeof(uint32_t), 64, x->stream));
            if (want_otu)
                HIP_TRY(launch_copy_to_host(dc + 2 * (uint64_t)n, x->otu_count.p, n * sizeof(uint32_t), 64, x->stream));
        }
        if (want_best && n) {
            HIP_TRY(x->dense_best.reserve(n * sizeof(kgx_best_call)));
            HIP_TRY(hipMemcpyAsync(x->dense_best.p, x->best.p, n * sizeof(kgx_best_call), hipMemcpyDeviceToDevice,
                                   x->stream));
        }
        HIP_TRY(hipEventRecord(c->chunk_gathered[k], x->stream));
        if (prof)
            HIP_TRY(hipEventRecord(c->prof_ev[4 * k + 3], x->stream));
        return KGX_OK;
    };

    /* chunk k's bulk copy, on the copy stream, issued once chunk k+1 is
     * enqueued: with option host_h2d_first it also waits for chunk k+1's
     * residues to be on the device.  A chunk's H2D beside a running D2H of
     * device stores crawled (r4c: 5 MB in 0.36 ms against 0.10 alone -- its
     * read requests queue behind the posted writes upstream), and the next
     * chunk's kernels waited for it; the D2H loses nothing by starting the
     * H2D's ~0.1 ms later. */
    auto copy_out = [&](kgx_ctx *x, uint32_t k) -> int {
        const uint32_t s0 = cut[k], n = cut[k + 1] - cut[k];
        const uint64_t nwords = (win[k] + 63) / 64;
        HIP_TRY(hipStreamWaitEvent(cs, c->chunk_gathered[k], 0));
        if (c->host_h2d_first && k + 1 < K)
            HIP_TRY(hipStreamWaitEvent(cs, c->chunk_h2d[k + 1], 0));
        void *d = nullptr;
        if (c->host_stream_dma) {
            /* DMA engines, sized on the host: every region copied whole */
            auto dma = [&](void *dst, const void *src, uint64_t bytes) -> hipError_t {
                return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, cs) : hipSuccess;
            };
            const uint32_t planes = want_otu ? 3 : want_calls ? 2 : 1;
            HIP_TRY(dma(c->h_counts.data() + 3 * (uint64_t)s0, x->dense_counts.p, planes * (uint64_t)n * sizeof(uint32_t)));
            if (r12)
                HIP_TRY(dma(c->h_hits12.data() + 3 * rb_h[k], x->dense_hits.p, cap_h[k] * 12));
            else
                HIP_TRY(dma(c->h_hits16.data() + rb_h[k], x->dense_hits.p, cap_h[k] * 16));
            HIP_TRY(dma(c->h_mask.data() + mb[k], x->dense_mask.p, nwords * sizeof(uint64_t)));
            if (want_calls)
                HIP_TRY(dma(c->h_calls_region.data() + rb_c[k], x->dense_calls.p, cap_c[k] * sizeof(kgx_call)));
            if (want_otu)
                HIP_TRY(dma(c->h_otus_region.data() + rb_o[k], x->dense_otus.p, cap_o[k] * sizeof(kgx_otu)));
            if (want_best)
                HIP_TRY(dma(c->h_best.data() + s0, x->dense_best.p, n * sizeof(kgx_best_call)));
            HIP_TRY(hipEventRecord(c->chunk_done[k], cs));
            if (prof)
                HIP_TRY(hipEventRecord(c->prof_done[k], cs));
            return KGX_OK;
        }
        if (n) {
            const uint32_t planes = want_otu ? 3 : want_calls ? 2 : 1;
            HIP_TRY(mapped(c->h_counts, 3 * (uint64_t)s0, &d));
            HIP_TRY(launch_copy_to_host(d, x->dense_counts.p, planes * (uint64_t)n * sizeof(uint32_t), cb, cs));
        }
        if (r12)
            HIP_TRY(mapped(c->h_hits12, 3 * rb_h[k], &d));
        else
            HIP_TRY(mapped(c->h_hits16, rb_h[k], &d));
        HIP_TRY(launch_copy_counted(d, x->dense_hits.p, x->dense_hoff.as<uint64_t>() + n, cap_h[k], r12 ? 12 : 16,
                                    cb, cs));
        if (nwords) {
            HIP_TRY(mapped(c->h_mask, mb[k], &d));
            HIP_TRY(launch_copy_to_host(d, x->dense_mask.p, nwords * sizeof(uint64_t), cb, cs));
        }
        if (want_calls && cap_c[k]) {
            HIP_TRY(mapped(c->h_calls_region, rb_c[k], &d));
            HIP_TRY(launch_copy_counted(d, x->dense_calls.p, x->dense_coff.as<uint64_t>() + n, cap_c[k],
                                        sizeof(kgx_call), cb, cs));
        }
        if (want_otu && cap_o[k]) {
            HIP_TRY(mapped(c->h_otus_region, rb_o[k], &d));
            HIP_TRY(launch_copy_counted(d, x->dense_otus.p, x->dense_ooff.as<uint64_t>() + n, cap_o[k],
                                        sizeof(kgx_otu), cb, cs));
        }
        if (want_best && n) {
            HIP_TRY(mapped(c->h_best, s0, &d));
            HIP_TRY(launch_copy_to_host(d, x->dense_best.p, n * sizeof(kgx_best_call), cb, cs));
        }
        HIP_TRY(hipEventRecord(c->chunk_done[k], cs));
        if (prof)
            HIP_TRY(hipEventRecord(c->prof_done[k], cs));
        return KGX_OK;
    };

    /* chunk k's results on the host -> CSR offsets, calls / OTUs in place,
     * expansion tasks; false in *fits when a region overflowed */
    uint64_t hbase = 0, cbase = 0, obase = 0, nwin = 0;
    double max_rh = 0, max_rc = 0, max_ro = 0;
    bool fits = true;
    auto collect = [&](uint32_t k) -> int {
        HIP_TRY(hipEventSynchronize(c->chunk_done[k]));
        const uint32_t s0 = cut[k], n = cut[k + 1] - cut[k];
        const uint32_t *hc = c->h_counts.data() + 3 * (uint64_t)s0, *cc = hc + n, *oc = hc + 2 * (uint64_t)n;
        uint64_t nh = 0, nc = 0, no = 0;
        for (uint32_t i = 0; i < n; i++) {
            nh += hc[i];
            nc += want_calls ? cc[i] : 0;
            no += want_otu ? oc[i] : 0;
            c->h_hoff[s0 + i + 1] = hbase + nh;
            c->h_coff[s0 + i + 1] = cbase + nc;
            c->h_ooff[s0 + i + 1] = obase + no;
        }
        nwin += win[k];
        if (win[k]) {
            max_rh = std::max(max_rh, (double)nh / (double)win[k]);
            max_rc = std::max(max_rc, (double)nc / (double)win[k]);
            max_ro = std::max(max_ro, (double)no / (double)win[k]);
        }
        if (nh > cap_h[k] || nc > cap_c[k] || no > cap_o[k])
            fits = false;
        if (fits) {
            if (nc)
                std::memmove(c->h_calls_region.data() + cbase, c->h_calls_region.data() + rb_c[k],
                             nc * sizeof(kgx_call));
            if (no)
                std::memmove(c->h_otus_region.data() + obase, c->h_otus_region.data() + rb_o[k],
                             no * sizeof(kgx_otu));
            if (nh && !expand) {
                /* compact results: the records stay where they landed */
                c->compact_segs.push_back({s0, s0 + n, r12 ? 3u : 4u, hbase, rb_h[k], mb[k]});
            } else if (nh) {
                const int64_t delta = (int64_t)rb_h[k] - (int64_t)hbase;
                const uint32_t P = c->pool->size();
                uint32_t a = s0;
                for (uint32_t p = 1; p <= P && a < s0 + n; p++) {
                    uint32_t b = s0 + n;
                    if (p < P) {
                        const uint64_t target = hbase + nh * p / P;
                        b = (uint32_t)(std::lower_bound(c->h_hoff.begin() + a, c->h_hoff.begin() + s0 + n, target) -
                                       c->h_hoff.begin());
                        b = std::max(b, a + 1);
                    }
                    const uint64_t m0 = mb[k];
                    c->pool->submit([c, r12, residues, seq_offsets, a, b, m0, delta, k, timing, now, ms,
                                     &expand_ns]() -> int {
                        const auto q0 = now();
                        const int erc = expand_hits(r12, c, residues, seq_offsets, a, b, m0, delta);
                        expand_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(now() - q0).count();
                        if (timing)
                            std::fprintf(stderr, "[kgx] streamed chunk %u expand [%u,%u): %.3f ms\n", k, a, b,
                                         ms(q0, now()));
                        return erc;
                    });
                    a = b;
                }
            }
        }
        hbase += nh;
        cbase += nc;
        obase += no;
        return KGX_OK;
    };

    if (c->stage_threads > 1 && (!c->stage_pool || c->stage_pool->size() != (unsigned)c->stage_threads))
        c->stage_pool.reset(new HostPool((unsigned)c->stage_threads));
    HostPool *sp = c->stage_threads > 1 ? c->stage_pool.get() : nullptr;
    int rc = KGX_OK;
    uint32_t next = 0; /* next chunk to collect */
    /* KGX_TIMING: the host's own clock per chunk (ms from T0): staging
     * entered / staged / enqueued, and each collect's end */
    std::vector<double> ht;
    for (uint32_t k = 0; k < K && !rc; k++) {
        kgx_ctx *x = xs[k & 1];
        if (k >= 2 && !sall)
            HIP_TRY(hipEventSynchronize(c->chunk_h2d[k - 2])); /* x's staging buffer is free */
        const auto ts = now();
        if (pin && sall)
            stage_offsets_into(c->h_off_all.data() + off_at[k], seq_offsets, cut[k], cut[k + 1]);
        else if (pin) {
            if (x->h_off_stage.resize(cut[k + 1] - cut[k] + 1) != hipSuccess)
                rc = fail(KGX_ENOMEM, "pinned staging");
            else
                stage_offsets_into(x->h_off_stage.data(), seq_offsets, cut[k], cut[k + 1]);
        } else if (sall)
            stage_copy_into(c->h_res_all.data() + res_at[k], c->h_off_all.data() + off_at[k], residues, seq_offsets,
                            cut[k], cut[k + 1], sp);
        else
            rc = stage_host_copy(x, residues, seq_offsets, cut[k], cut[k + 1], sp);
        const auto te = now();
        stage_ms += ms(ts, te);
        if (rc || (rc = enqueue(x, k)))
            break;
        if (k >= 1 && (rc = copy_out(xs[(k - 1) & 1], k - 1)))
            break;
        if (timing)
            ht.insert(ht.end(), {(double)k, ms(T0, ts), ms(T0, te), ms(T0, now())});
        /* collect what has landed meanwhile */
        while (!rc && next < k && hipEventQuery(c->chunk_done[next]) == hipSuccess) {
            rc = collect(next++);
            if (timing)
                ht.insert(ht.end(), {-1.0 - (double)(next - 1), ms(T0, now()), 0.0, 0.0});
        }
    }
    if (!rc && K)
        rc = copy_out(xs[(K - 1) & 1], K - 1);
    while (!rc && next < K) {
        rc = collect(next++);
        if (timing)
            ht.insert(ht.end(), {-1.0 - (double)(next - 1), ms(T0, now()), 0.0, 0.0});
    }
    for (size_t i = 0; timing && i + 3 < ht.size(); i += 4) {
        if (ht[i] >= 0)
            std::fprintf(stderr, "[kgx] host chunk %d: stage %.3f-%.3f, enqueued %.3f ms\n", (int)ht[i], ht[i + 1],
                         ht[i + 2], ht[i + 3]);
        else
            std::fprintf(stderr, "[kgx] host collect %d done %.3f ms\n", (int)(-ht[i] - 1), ht[i + 1]);
    }
    /* drain everything, whatever happened above */
    const hipError_t e0 = hipStreamSynchronize(xs[0]->stream), e1 = hipStreamSynchronize(xs[1]->stream);
    hipError_t e2 = hipStreamSynchronize(cs);
    if (c->up_stream) { /* an upload issued before a failed enqueue may still read the staging memory */
        const hipError_t e3 = hipStreamSynchronize(c->up_stream);
        if (e2 == hipSuccess)
            e2 = e3;
    }
    const int prc = c->pool->wait();
    if (rc)
        return rc;
    HIP_TRY(e0);
    HIP_TRY(e1);
    HIP_TRY(e2);
    if (prc)
        return prc;
    if (pin && __atomic_load_n(&c->h_nul[0], __ATOMIC_ACQUIRE))
        return STREAM_NUL;
    /* the rates the next batch's regions are sized by */
    c->rate_hits = std::max(0.02, max_rh * 1.25);
    c->rate_calls = std::max(0.01, max_rc * 1.25);
    c->rate_otus = std::max(0.01, max_ro * 1.25);
    if (!fits)
        return STREAM_OVERFLOW;
    if (expand)
        HIP_TRY(c->h_hits.resize(hbase));
    c->have_hits = false;
    t->have_hits = false;
    if (timing)
        std::fprintf(stderr, "[kgx] streamed batch: %u chunks, %.3f ms\n", K, ms(T0, now()));
    if (prof) {
        kgx_host_profile &P = c->last_profile;
        P = kgx_host_profile{};
        P.chunks = K;
        P.streamed = 1;
        P.wall_ms = ms(T0, now());
        P.stage_ms = stage_ms;
        P.expand_ms = (double)expand_ns.load() * 1e-6;
        P.h2d_bytes = seq_offsets[n_seq] - seq_offsets[0] + (uint64_t)(n_seq + K) * sizeof(uint64_t);
        for (uint32_t k = 0; k < K; k++) {
            float a = 0, b = 0, g = 0, d = 0;
            HIP_TRY(hipEventElapsedTime(&a, c->prof_ev[4 * k], c->prof_ev[4 * k + 1]));
            HIP_TRY(hipEventElapsedTime(&b, c->prof_ev[4 * k + 1], c->prof_ev[4 * k + 2]));
            HIP_TRY(hipEventElapsedTime(&g, c->prof_ev[4 * k + 2], c->prof_ev[4 * k + 3]));
            HIP_TRY(hipEventElapsedTime(&d, c->prof_ev[4 * k + 3], c->prof_done[k]));
            P.h2d_ms += a;
            P.device_ms += b;
            P.gather_ms += g;
            P.d2h_ms += d;
            if (timing) { /* the device's clock, from chunk 0's first event */
                float t0 = 0;
                HIP_TRY(hipEventElapsedTime(&t0, c->prof_ev[0], c->prof_ev[4 * k]));
                std::fprintf(stderr, "[kgx] device chunk %u: h2d %.3f, kernels %.3f, gather %.3f, d2h %.3f, done %.3f ms\n",
                             k, t0, t0 + a, t0 + a + b, t0 + a + b + g, t0 + a + b + g + d);
            }
        }
        const uint64_t recb = r12 ? 12 : 16;
        P.d2h_bytes = hbase * recb + cbase * sizeof(kgx_call) +
                      obase * sizeof(kgx_otu) + mb[K] * sizeof(uint64_t) + 3ull * n_seq * sizeof(uint32_t) +
                      (want_best ? (uint64_t)n_seq * sizeof(kgx_best_call) : 0);
    }
    out->best = want_best ? c->h_best.data() : nullptr;
    out->n_seq = n_seq;
    out->hit_offsets = c->h_hoff.data();
    out->hits = expand ? c->h_hits.data() : nullptr;
    out->call_offsets = c->h_coff.data();
    out->calls = c->h_calls_region.data();
    out->otu_offsets = c->h_ooff.data();
    out->otus = c->h_otus_region.data();
    out->n_windows = nwin;
    return KGX_OK;
}

/* A stream for the host path's bulk copies / uploads.  The runtime spreads a
 * process's streams over a few hardware queues (4 by default), each a FIFO
 * that blocks behind an event wait at its head, so the copy stream's waits
 * held up other streams' work queued behind them.  The copy stream is made at
 * the device's lowest priority: the runtime keeps a queue pool per priority,
 * so it shares a queue only with other copy streams.  (Round 4's full-CU-mask
 * stream got a queue of its own but faulted inside rocprofv3's finalisation
 * when a process exited with it alive, r5c; it is gone.)  KGX_OWN_QUEUES=0:
 * a plain stream. */
hipError_t own_queue_stream(int device, hipStream_t *s)
{
    (void)device;
    const char *e = std::getenv("KGX_OWN_QUEUES");
    if (!e || std::atoi(e) != 0) {
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && least != greatest &&
            hipStreamCreateWithPriority(s, hipStreamNonBlocking, least) == hipSuccess)
            return hipSuccess;
        (void)hipGetLastError();
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

/* The host batch in K residue-balanced chunks of whole sequences, alternating
 * between c and its twin context: while chunk k's hits are gathered and
 * copied to the host on one stream, chunk k+1 is staged, copied up, probed
 * and scored on the other.  The D2H of the hit records is the bulk of the
 * PCIe traffic, so the rest hides behind it.  Results are identical to the
 * one-pass path (per-sequence work never spans chunks). */
int process_batch_chunked(kgx_ctx *c, const kgx_params *params, const char *residues,
                          const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want, uint32_t K,
                          kgx_result *out)
{
    if (!c->twin) {
        int rc = kgx_ctx_create(c->img, &c->twin);
        if (rc)
            return rc;
    }
    kgx_ctx *t = c->twin;
    t->probe_variant = c->probe_variant;
    t->probe_j = c->probe_j;
    t->probe_filter = c->probe_filter;
    t->probe_serialize = c->probe_serialize;
    t->score_variant = c->score_variant;
    t->score_wave_tiles = c->score_wave_tiles;
    kgx_ctx *xs[2] = {c, t};
    if (!c->copy_stream)
        HIP_TRY(own_queue_stream(c->img->device, &c->copy_stream));
    /* the upload stream only when asked for: each own-queue stream holds a
     * hardware queue of the process's few */
    if (c->host_upload_stream && !c->up_stream)
        HIP_TRY(own_queue_stream(c->img->device, &c->up_stream));
    for (auto *ev : {&c->chunk_counts, &c->chunk_gathered, &c->chunk_done, &c->chunk_h2d})
        while (ev->size() < K) {
            hipEvent_t e;
            HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            ev->push_back(e);
        }

    const uint64_t r0 = seq_offsets[0], n_res = seq_offsets[n_seq] - r0;
    std::vector<uint32_t> cut(K + 1, 0);
    cut[K] = n_seq;
    /* chunk weights: with host_taper the first and last chunks are half the
     * others (the first one's kernels and the last one's copy + expansion
     * are the parts of the batch nothing overlaps) */
    const bool taper = c->host_taper && K >= 3;
    const double wsum = taper ? (double)K - 1.0 : (double)K;
    for (uint32_t k = 1; k < K; k++) {
        const double before = taper ? 0.5 + (double)(k - 1) : (double)k; /* weight of chunks < k */
        const uint64_t target = r0 + (uint64_t)((double)n_res * before / wsum);
        uint32_t s = (uint32_t)(std::lower_bound(seq_offsets, seq_offsets + n_seq + 1, target) - seq_offsets);
        cut[k] = std::min(std::max(s, cut[k - 1]), n_seq);
    }
    cut.erase(std::unique(cut.begin(), cut.end()), cut.end()); /* no empty chunks */
    K = (uint32_t)cut.size() - 1;
    const bool want_calls = (want & KGX_WANT_CALLS) != 0;
    const bool want_otu = (want & KGX_WANT_OTU) != 0;
    const bool need_hits = (want & KGX_WANT_HITS) != 0;
    const bool want_best = (want & KGX_WANT_BEST) != 0;
    c->h_hoff.assign(n_seq + 1, 0);
    c->h_coff.assign(n_seq + 1, 0);
    c->h_ooff.assign(n_seq + 1, 0);
    uint64_t hbase = 0, cbase = 0, obase = 0, nwin = 0;
    HIP_TRY(c->h_hits.resize(0));
    HIP_TRY(c->h_calls.resize(0));
    HIP_TRY(c->h_otus.resize(0));
    HIP_TRY(c->h_best.resize(want_best ? n_seq : 0));
    /* compact D2H: records + mask, expanded on the host pool */
    const bool compact = c->host_hits16 && need_hits && c->img->layout == KGX_LAYOUT_PACKED16;
    uint64_t mbase = 0;
    struct PoolDrain { /* no expansion outlives this call, whatever path returns */
        HostPool *p = nullptr;
        ~PoolDrain()
        {
            if (p)
                (void)p->wait();
        }
    } drain;
    while (c->chunk_counts.size() < K) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->chunk_counts.push_back(e);
    }
    if (compact) {
        if (!c->pool || c->pool->size() != (unsigned)c->host_threads)
            c->pool.reset(new HostPool((unsigned)c->host_threads));
        drain.p = c->pool.get();
        HIP_TRY(c->h_hits16.resize(0));
        HIP_TRY(c->h_mask.resize(0));
        if (c->host_stream_chunks) {
            /* option host_score_variant: the scorer for the chunks (a chunk's
             * 17k sequences keep the lane scorer's long chains latency-bound;
             * the wave scorer is 1-3% faster per batch here, r4b) */
            const int sv_c = c->score_variant, sv_t = t->score_variant;
            if (c->host_score_variant >= 0)
                c->score_variant = t->score_variant = c->host_score_variant;
            const int src = process_batch_streamed(c, params, residues, seq_offsets, n_seq, want, K, cut, out);
            c->score_variant = sv_c;
            t->score_variant = sv_t;
            if (src != STREAM_OVERFLOW && src != STREAM_NUL)
                return src;
            /* a region overflowed (the rates are raised), or the caller's
             * pinned residues hold a NUL: this batch runs exact, staged */
            if (src == STREAM_NUL)
                c->nul_reruns++;
            c->h_hoff.assign(n_seq + 1, 0);
            c->h_coff.assign(n_seq + 1, 0);
            c->h_ooff.assign(n_seq + 1, 0);
            HIP_TRY(c->h_hits16.resize(0));
            HIP_TRY(c->h_mask.resize(0));
            HIP_TRY(c->h_hits.resize(0));
            HIP_TRY(c->h_best.resize(want_best ? n_seq : 0));
            c->compact_segs.clear();
            c->stream_fallbacks++;
        }
        c->h_wstart.resize(n_seq);
        for (uint32_t k = 0; k < K; k++) {
            uint64_t w = 0;
            for (uint32_t s = cut[k]; s < cut[k + 1]; s++) {
                c->h_wstart[s] = w;
                w += windows_of(seq_offsets[s + 1] - seq_offsets[s]);
            }
        }
    }

    hipStream_t cs = c->copy_stream;

    /* device bytes -> the pinned result array at element `at`, on the copy
     * stream: device stores into the mapped memory (host_copy 1) or a DMA
     * copy */
    auto copy_out = [&](auto &dst, uint64_t at, const void *src, uint64_t n) -> int {
        if (!n)
            return KGX_OK;
        const uint64_t bytes = n * sizeof(dst[0]);
        if (c->host_copy) {
            void *d = nullptr;
            HIP_TRY(dst.device_ptr(at, &d));
            HIP_TRY(launch_copy_to_host(d, src, bytes, c->host_copy_blocks, cs));
        } else {
            HIP_TRY(hipMemcpyAsync(dst.data() + at, src, bytes, hipMemcpyDeviceToHost, cs));
        }
        return KGX_OK;
    };

    /* Schedule.  Each chunk runs H2D -> plan/probe/score -> counts D2H on its
     * context's stream (contexts alternate), then, once the host has turned
     * the counts into offsets, a gather into that context's dense buffers;
     * the bulk device-to-host copy of those buffers runs on a separate copy
     * stream, so chunk k+2's kernels on the same context are not held behind
     * chunk k's bulk copy (only chunk k+2's gather waits for it).
     * Device-to-host bytes cross PCIe in order, so chunk k+1's counts must
     * leave before chunk k's bulk (option counts_first): otherwise they queue
     * behind it and the host learns chunk k+1's sizes only once the link has
     * gone idle.  Chunks are staged and enqueued as soon as their context's
     * staging buffer is free, and host threads expand chunk k's compact
     * records while later chunks stream. */
    if (c->stage_threads > 1 && (!c->stage_pool || c->stage_pool->size() != (unsigned)c->stage_threads))
        c->stage_pool.reset(new HostPool((unsigned)c->stage_threads));
    HostPool *sp = c->stage_threads > 1 ? c->stage_pool.get() : nullptr;
    int rc = KGX_OK;
    for (uint32_t k = 0; k < std::min<uint32_t>(K, 2) && !rc; k++)
        if (!(rc = stage_host_copy(xs[k], residues, seq_offsets, cut[k], cut[k + 1], sp)))
            rc = enqueue_chunk(xs[k], params, want, c->chunk_counts[k]);
    const bool timing = std::getenv("KGX_TIMING") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    for (uint32_t k = 0; k < K && !rc; k++) {
        kgx_ctx *x = xs[k & 1];
        const auto t0 = now();
        HIP_TRY(hipEventSynchronize(c->chunk_counts[k])); /* chunk k's counts are on the host */
        const auto t1 = now();
        const uint32_t s0 = cut[k], n = cut[k + 1] - cut[k];
        HIP_TRY(x->h_dense_hoff.resize(n + 1));
        HIP_TRY(x->h_dense_coff.resize(n + 1));
        HIP_TRY(x->h_dense_ooff.resize(n + 1));
        uint64_t nh = 0, nc = 0, no = 0;
        for (uint32_t i = 0; i < n; i++) {
            x->h_dense_hoff[i] = nh;
            x->h_dense_coff[i] = nc;
            x->h_dense_ooff[i] = no;
            nh += x->h_hcount[i];
            nc += want_calls ? x->h_ccount[i] : 0;
            no += want_otu ? x->h_ocount[i] : 0;
            c->h_hoff[s0 + i + 1] = hbase + nh;
            c->h_coff[s0 + i + 1] = cbase + nc;
            c->h_ooff[s0 + i + 1] = obase + no;
        }
        x->h_dense_hoff[n] = nh;
        x->h_dense_coff[n] = nc;
        x->h_dense_ooff[n] = no;
        nwin += x->h_nwin[0];
        const uint64_t nh_all = nh; /* hit offsets count every hit; records only when wanted */
        if (!need_hits)
            nh = 0;
        const uint64_t hrec = need_hits ? hbase : 0; /* where this chunk's records go */
        const uint64_t nwords = compact && nh ? (x->h_nwin[0] + 63) / 64 : 0;
        if (hrec + nh > c->h_hits.cap || cbase + nc > c->h_calls.cap || obase + no > c->h_otus.cap ||
            (compact && (hrec + nh > c->h_hits16.cap || mbase + nwords > c->h_mask.cap))) {
            /* growth moves the pinned arrays: no copy into them may be in
             * flight, and no expansion may be reading or writing them */
            HIP_TRY(hipStreamSynchronize(cs));
            if (compact && (rc = c->pool->wait()))
                break;
        }
        if (compact) {
            HIP_TRY(c->h_hits16.resize(hrec + nh));
            HIP_TRY(c->h_mask.resize(mbase + nwords));
        }
        if (!(compact && c->compact_out))
            HIP_TRY(c->h_hits.resize(hrec + nh));
        HIP_TRY(c->h_calls.resize(cbase + nc));
        HIP_TRY(c->h_otus.resize(obase + no));
        /* x's dense buffers still feed chunk k-2's bulk copy */
        if (k >= 2)
            HIP_TRY(hipStreamWaitEvent(x->stream, c->chunk_done[k - 2], 0));
        if (nh || nc || no) {
            HIP_TRY(x->dense_hoff.reserve((n + 1) * sizeof(uint64_t)));
            HIP_TRY(x->dense_coff.reserve((n + 1) * sizeof(uint64_t)));
            HIP_TRY(x->dense_ooff.reserve((n + 1) * sizeof(uint64_t)));
            HIP_TRY(x->dense_hits.reserve(std::max<uint64_t>(nh, 1) * sizeof(kgx_hit)));
            HIP_TRY(x->dense_calls.reserve(std::max<uint64_t>(nc, 1) * sizeof(kgx_call)));
            HIP_TRY(x->dense_otus.reserve(std::max<uint64_t>(no, 1) * sizeof(kgx_otu)));
            HIP_TRY(hipMemcpyAsync(x->dense_hoff.p, x->h_dense_hoff.data(), (n + 1) * sizeof(uint64_t),
                                   hipMemcpyHostToDevice, x->stream));
            HIP_TRY(hipMemcpyAsync(x->dense_coff.p, x->h_dense_coff.data(), (n + 1) * sizeof(uint64_t),
                                   hipMemcpyHostToDevice, x->stream));
            HIP_TRY(hipMemcpyAsync(x->dense_ooff.p, x->h_dense_ooff.data(), (n + 1) * sizeof(uint64_t),
                                   hipMemcpyHostToDevice, x->stream));
            HIP_TRY(launch_gather(n, x->wbase.as<uint64_t>(), x->hit_mask.as<uint64_t>(), x->tile_windows,
                                  x->call_count.as<uint32_t>(), x->hits.as<uint4>(),
                                  x->hits.as<uint4>() + x->hit_slots, x->calls.as<kgx_call>(),
                                  x->dense_hoff.as<uint64_t>(), x->dense_coff.as<uint64_t>(),
                                  nh && !compact ? x->dense_hits.as<kgx_hit>() : nullptr,
                                  nc ? x->dense_calls.as<kgx_call>() : nullptr, s0, x->hit_format,
                                  x->otu_count.as<uint32_t>(), x->otus.as<kgx_otu>(), x->dense_ooff.as<uint64_t>(),
                                  no ? x->dense_otus.as<kgx_otu>() : nullptr, x->stream,
                                  nh && compact ? x->dense_hits.as<uint4>() : nullptr));
        }
        /* the mask and best calls too: chunk k+2's kernels overwrite them */
        if (nwords) {
            HIP_TRY(x->dense_mask.reserve(nwords * sizeof(uint64_t)));
            HIP_TRY(launch_copy_to_host(x->dense_mask.p, x->hit_mask.p, nwords * sizeof(uint64_t), 256,
                                        x->stream));
        }
        if (want_best && n) {
            HIP_TRY(x->dense_best.reserve(n * sizeof(kgx_best_call)));
            HIP_TRY(hipMemcpyAsync(x->dense_best.p, x->best.p, n * sizeof(kgx_best_call),
                                   hipMemcpyDeviceToDevice, x->stream));
        }
        HIP_TRY(hipEventRecord(c->chunk_gathered[k], x->stream));
        HIP_TRY(hipStreamWaitEvent(cs, c->chunk_gathered[k], 0));
        if (k + 1 < K && c->counts_first)
            HIP_TRY(hipStreamWaitEvent(cs, c->chunk_counts[k + 1], 0));
        if (compact) {
            if ((rc = copy_out(c->h_hits16, hrec, x->dense_hits.p, nh)) ||
                (rc = copy_out(c->h_mask, mbase, x->dense_mask.p, nwords)))
                break;
        } else if ((rc = copy_out(c->h_hits, hrec, x->dense_hits.p, nh))) {
            break;
        }
        if ((rc = copy_out(c->h_calls, cbase, x->dense_calls.p, nc)) ||
            (rc = copy_out(c->h_otus, obase, x->dense_otus.p, no)) ||
            (want_best && (rc = copy_out(c->h_best, s0, x->dense_best.p, n))))
            break;
        HIP_TRY(hipEventRecord(c->chunk_done[k], cs));
        if (compact && nh && c->compact_out) {
            /* compact results: the records stay where they land */
            c->compact_segs.push_back({s0, s0 + n, 4u, hbase, hrec, mbase});
        } else if (compact && nh) {
            /* host threads expand this chunk once its bytes have landed, in
             * hit-balanced sequence ranges, while the next chunks stream */
            hipEvent_t ev = c->chunk_done[k];
            const uint32_t P = c->pool->size();
            uint32_t a = s0;
            for (uint32_t p = 1; p <= P && a < s0 + n; p++) {
                uint32_t b = s0 + n;
                if (p < P) {
                    const uint64_t target = c->h_hoff[s0] + (c->h_hoff[s0 + n] - c->h_hoff[s0]) * p / P;
                    b = (uint32_t)(std::lower_bound(c->h_hoff.begin() + a, c->h_hoff.begin() + s0 + n, target) -
                                   c->h_hoff.begin());
                    b = std::max(b, a + 1);
                }
                const uint64_t mb = mbase;
                c->pool->submit([c, ev, residues, seq_offsets, a, b, mb, k, timing, now, ms]() -> int {
                    const auto q0 = now();
                    const hipError_t e = hipEventSynchronize(ev);
                    if (e != hipSuccess)
                        return fail(KGX_EDEVICE, std::string("chunk event: ") + hipGetErrorString(e));
                    const auto q1 = now();
                    const int erc = expand_hits(false, c, residues, seq_offsets, a, b, mb, 0);
                    if (timing)
                        std::fprintf(stderr, "[kgx] chunk %u expand [%u,%u): wait %.3f ms, expand %.3f ms\n", k, a,
                                     b, ms(q0, q1), ms(q1, now()));
                    return erc;
                });
                a = b;
            }
        }
        mbase += nwords;
        hbase += nh_all;
        cbase += nc;
        obase += no;
        const auto t2 = now();
        /* chunk k+2 -> x (its H2D of chunk k finished before chunk k's counts
         * arrived), enqueued at once */
        if (k + 2 < K && !(rc = stage_host_copy(x, residues, seq_offsets, cut[k + 2], cut[k + 3], sp)))
            rc = enqueue_chunk(x, params, want, c->chunk_counts[k + 2]);
        if (timing)
            std::fprintf(stderr, "[kgx] chunk %u: wait counts %.3f ms, enqueue %.3f ms, stage+enqueue k+2 %.3f ms\n",
                         k, ms(t0, t1), ms(t1, t2), ms(t2, now()));
    }
    /* drain both streams, whatever happened above */
    const hipError_t e0 = hipStreamSynchronize(xs[0]->stream), e1 = hipStreamSynchronize(xs[1]->stream);
    const hipError_t e2 = hipStreamSynchronize(cs);
    const int prc = compact ? c->pool->wait() : KGX_OK;
    if (rc)
        return rc;
    if (prc)
        return prc;
    HIP_TRY(e0);
    HIP_TRY(e1);
    HIP_TRY(e2);
    /* the batch's device results are split over two contexts */
    c->have_hits = false;
    t->have_hits = false;
    fill_result(c, n_seq, need_hits, (want & KGX_WANT_BEST) != 0, nwin, out);
    return KGX_OK;
}

inline uint64_t round16(uint64_t bytes) { return (bytes + 15) & ~15ull; }

/* whether a host batch can take the one-launch path (kgx_fused.hip) */
bool fused_eligible(const kgx_ctx *c, const kgx_params &p, const uint64_t *seq_offsets, uint32_t n_seq,
                    uint32_t want)
{
    if (!c->small_fused || c->img->layout != KGX_LAYOUT_PACKED16 || !c->img->d_packed || n_seq == 0 ||
        n_seq > FUSED_MAX_SEQ || want == 0 || (want & ~(KGX_WANT_HITS | KGX_WANT_CALLS)) || p.order_constraint != 0 ||
        p.min_hits < 1)
        return false;
    for (uint32_t s = 0; s < n_seq; s++)
        if (windows_of(seq_offsets[s + 1] - seq_offsets[s]) > FUSED_MAX_WINDOWS)
            return false;
    return true;
}

/* A small host batch in ONE launch: one workgroup per sequence reads its
 * residues from the pinned staging, probes, compacts, scores and stores its
 * kgx_hit / kgx_call records into per-sequence regions of mapped memory
 * (from the sequence's first window), then its count and a completion
 * token; the host polls the tokens and packs the regions into the CSR
 * result.  The device keeps no batch (kgx_kmap_add_hits needs another path:
 * the option is for per-sequence callers, e.g. the facade's process_aa_seq). */
int process_batch_fused(kgx_ctx *c, const kgx_params &p, const char *residues, const uint64_t *seq_offsets,
                        uint32_t n_seq, uint32_t want, kgx_result *out)
{
    int rc = stage_host_copy(c, residues, seq_offsets, 0, n_seq);
    if (rc)
        return rc;
    const uint64_t *off = c->h_off_stage.data();
    HIP_TRY(c->h_fwb.resize(n_seq + 1));
    uint64_t W = 0, longest = 0;
    for (uint32_t s = 0; s < n_seq; s++) {
        c->h_fwb[s] = W;
        const uint64_t w = windows_of(off[s + 1] - off[s]);
        W += w;
        longest = std::max(longest, w);
    }
    c->h_fwb[n_seq] = W;
    const bool need_hits = (want & KGX_WANT_HITS) != 0, want_calls = (want & KGX_WANT_CALLS) != 0;
    HIP_TRY(c->h_fhits.resize(std::max<uint64_t>(W, 1)));
    HIP_TRY(c->h_fcalls.resize(std::max<uint64_t>(W, 1)));
    HIP_TRY(c->h_fcounts.resize(2 * (uint64_t)n_seq));
    HIP_TRY(c->h_fdone.resize(n_seq));
    HIP_TRY(c->h_res.resize(std::max<uint64_t>(c->h_res.size(), 1)));
    void *d_res = nullptr, *d_off = nullptr, *d_wb = nullptr, *d_hits = nullptr, *d_calls = nullptr,
         *d_counts = nullptr, *d_done = nullptr;
    HIP_TRY(c->h_res.device_ptr(0, &d_res));
    HIP_TRY(c->h_off_stage.device_ptr(0, &d_off));
    HIP_TRY(c->h_fwb.device_ptr(0, &d_wb));
    HIP_TRY(c->h_fhits.device_ptr(0, &d_hits));
    HIP_TRY(c->h_fcalls.device_ptr(0, &d_calls));
    HIP_TRY(c->h_fcounts.device_ptr(0, &d_counts));
    HIP_TRY(c->h_fdone.device_ptr(0, &d_done));
    const uint32_t token = ++c->small_token ? c->small_token : ++c->small_token;
    /* KGX_FUSED_DEBUG: wall-clock stamps of the first workgroup's phases, to stderr */
    static const bool debug = std::getenv("KGX_FUSED_DEBUG") != nullptr;
    void *d_dbg = nullptr;
    if (debug) {
        HIP_TRY(c->h_fdbg.resize(16));
        std::memset(c->h_fdbg.data(), 0, 16 * sizeof(uint64_t));
        HIP_TRY(c->h_fdbg.device_ptr(0, &d_dbg));
    }
    HIP_TRY(launch_fused_small(static_cast<const uint8_t *>(d_res), static_cast<const uint64_t *>(d_off),
                               static_cast<const uint64_t *>(d_wb), n_seq, want, ctx_probe_table(c),
                               ctx_probe_buckets(c), p,
                               static_cast<kgx_hit *>(d_hits), static_cast<kgx_call *>(d_calls),
                               static_cast<uint32_t *>(d_counts), static_cast<uint32_t *>(d_done), token,
                               (uint32_t)longest, static_cast<uint64_t *>(d_dbg), c->h_off_stage.data(),
                               c->h_fwb.data(), reinterpret_cast<const uint8_t *>(c->h_res.data()),
                               c->fused_inline && n_seq <= FUSED_INLINE_SEQ && off[n_seq] <= FUSED_INLINE_RES
                                   ? (uint32_t)std::max<uint64_t>(off[n_seq], 1)
                                   : 0u,
                               c->stream, ctx_home_shift(c)));
    /* every sequence's token (stored after its results, behind a
     * system-scope fence); a fault or a lost store still ends the wait */
    const volatile uint32_t *done = c->h_fdone.data();
    for (uint32_t s = 0; s < n_seq; s++)
        for (uint32_t spin = 1; done[s] != token; spin++) {
            if ((spin & 255u) == 0) {
                const hipError_t q = hipStreamQuery(c->stream);
                if (q == hipSuccess) {
                    std::atomic_thread_fence(std::memory_order_acquire);
                    if (done[s] != token)
                        return fail(KGX_EDEVICE, "fused batch: sequence " + std::to_string(s) +
                                                     " ended without its completion token");
                    break;
                }
                if (q != hipErrorNotReady)
                    HIP_TRY(q);
            }
#if defined(__x86_64__)
            __builtin_ia32_pause();
#endif
        }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (debug) {
        const uint64_t *d = c->h_fdbg.data();
        std::fprintf(stderr, "[kgx] fused n=%u: load %llu, probe %llu, compact %llu, store+score %llu, fence %llu ticks\n",
                     n_seq, (unsigned long long)(d[1] - d[0]), (unsigned long long)(d[2] - d[1]),
                     (unsigned long long)(d[3] - d[2]), (unsigned long long)(d[4] - d[3]),
                     (unsigned long long)(d[5] - d[4]));
    }
    /* the regions -> the CSR result */
    const uint32_t *cnt = c->h_fcounts.data();
    c->h_hoff.assign(n_seq + 1, 0);
    c->h_coff.assign(n_seq + 1, 0);
    c->h_ooff.assign(n_seq + 1, 0);
    for (uint32_t s = 0; s < n_seq; s++) {
        const uint64_t w = c->h_fwb[s + 1] - c->h_fwb[s];
        if (cnt[s] > w || cnt[n_seq + s] > w)
            return fail(KGX_EDEVICE, "fused batch: more records than windows");
        c->h_hoff[s + 1] = c->h_hoff[s] + cnt[s];
        c->h_coff[s + 1] = c->h_coff[s] + (want_calls ? cnt[n_seq + s] : 0u);
    }
    HIP_TRY(c->h_hits.resize(need_hits ? c->h_hoff[n_seq] : 0));
    HIP_TRY(c->h_calls.resize(c->h_coff[n_seq]));
    HIP_TRY(c->h_otus.resize(0));
    for (uint32_t s = 0; s < n_seq; s++) {
        if (need_hits && cnt[s])
            std::memcpy(c->h_hits.data() + c->h_hoff[s], c->h_fhits.data() + c->h_fwb[s], cnt[s] * sizeof(kgx_hit));
        if (want_calls && cnt[n_seq + s])
            std::memcpy(c->h_calls.data() + c->h_coff[s], c->h_fcalls.data() + c->h_fwb[s],
                        cnt[n_seq + s] * sizeof(kgx_call));
    }
    c->have_hits = false; /* nothing of the batch stays on the device */
    c->have_best = false;
    c->have_otus = false;
    fill_result(c, n_seq, need_hits, false, W, out);
    return KGX_OK;
}

/* A small host batch (process_aa_seq's one sequence, a request's few) in one
 * host wait: the host writes the plan (window bases, tile owners, longest
 * sequence) beside the staged residues and offsets in one pinned blob, one
 * kernel pulls the blob into the plan's buffers, the probe and scorer run as
 * for any batch, and one workgroup scans the counts into the CSR offsets, which
 * the gather uses to store the records straight into mapped result arrays
 * sized for the worst case (every window a hit).  Same kernels, same records
 * as kgx_run_device + kgx_device_batch_collect. */
int process_batch_small(kgx_ctx *c, const kgx_params *params, const char *residues, const uint64_t *seq_offsets,
                        uint32_t n_seq, uint32_t want, kgx_result *out, kgx_kmap *roll_map = nullptr,
                        int roll_mode = 0)
{
    PhaseTimer tm(c); /* KGX_TIMING: phase times (each mark waits for the stream) */
    int rc = stage_host_copy(c, residues, seq_offsets, 0, n_seq);
    if (rc)
        return rc;
    tm.mark("s.stage");
    const uint64_t n_res = c->h_res.size();
    const uint64_t *off = c->h_off_stage.data();
    HIP_TRY(c->residues.reserve(round16(n_res + 16)));
    HIP_TRY(c->offsets.reserve(round16((n_seq + 1) * sizeof(uint64_t))));
    if ((rc = plan_reserve(c, c->offsets.as<uint64_t>(), n_seq, n_res)))
        return rc;
    HIP_TRY(c->wbase.reserve(round16((n_seq + 1) * sizeof(uint64_t))));
    HIP_TRY(c->tile_seq.reserve(round16(c->max_tiles * sizeof(uint32_t))));
    /* the blob: offsets | window bases | tile owners | status | residues */
    const uint64_t b_off = round16((n_seq + 1) * sizeof(uint64_t)), b_wb = b_off,
                   b_tile = round16(c->max_tiles * sizeof(uint32_t)), b_st = 16, b_res = round16(n_res);
    /* the residues stay in the pinned staging (h_res): the upload reads them
     * from there, no second host copy */
    const uint64_t words = (b_off + b_wb + b_tile + b_st) / 16;
    HIP_TRY(c->h_small.resize(words));
    HIP_TRY(c->h_res.resize(b_res ? b_res : 16)); /* 16-B words: the upload's last one may run past n_res */
    char *blob = reinterpret_cast<char *>(c->h_small.data());
    uint64_t *h_off = reinterpret_cast<uint64_t *>(blob);
    uint64_t *h_wb = reinterpret_cast<uint64_t *>(blob + b_off);
    uint32_t *h_tile = reinterpret_cast<uint32_t *>(blob + b_off + b_wb);
    uint32_t *h_st = reinterpret_cast<uint32_t *>(blob + b_off + b_wb + b_tile);
    std::memcpy(h_off, off, (n_seq + 1) * sizeof(uint64_t));
    /* plan_reduce / plan_scan on the host: window bases, the sequence owning
     * each tile's first window, the longest sequence */
    const uint64_t T = c->tile_windows;
    uint64_t wb = 0;
    uint32_t longest = 0;
    for (uint32_t s = 0; s < n_seq; s++) {
        const uint64_t w = windows_of(off[s + 1] - off[s]);
        h_wb[s] = wb;
        for (uint64_t t = (wb + T - 1) / T; t * T < wb + w; t++)
            h_tile[t] = s;
        wb += w;
        longest = (uint32_t)std::max<uint64_t>(longest, std::min<uint64_t>(w, 0xFFFFFFFFull));
    }
    h_wb[n_seq] = wb;
    for (uint64_t t = (wb + T - 1) / T; t < c->max_tiles; t++)
        h_tile[t] = n_seq ? n_seq - 1 : 0; /* tiles past the last window (never probed) */
    h_st[0] = 0;
    h_st[1] = longest;
    h_st[2] = h_st[3] = 0;
    void *d_blob = nullptr, *d_res = nullptr;
    HIP_TRY(c->h_small.device_ptr(0, &d_blob));
    HIP_TRY(c->h_res.device_ptr(0, &d_res));
    const uint4 *src = static_cast<const uint4 *>(d_blob);
    SmallPieces pc;
    const uint64_t sizes[SMALL_PIECES] = {b_off, b_wb, b_tile, b_st, b_res};
    void *dsts[SMALL_PIECES] = {c->offsets.p, c->wbase.p, c->tile_seq.p, c->plan_status.p, c->residues.p};
    uint64_t at = 0;
    for (int p = 0; p < SMALL_PIECES; p++) {
        pc.dst[p] = static_cast<uint4 *>(dsts[p]);
        /* the last piece (residues) from the staging, the others from the blob */
        pc.src[p] = p == SMALL_PIECES - 1 ? static_cast<const uint4 *>(d_res) : src + at;
        at += sizes[p] / 16;
        pc.end16[p] = at;
    }
    tm.mark("s.plan");
    HIP_TRY(launch_small_upload(pc, c->stream));
    tm.mark("s.upload");
    /* a small probe neither waits for nor holds back the image's other probes:
     * chaining it (probe_serialize, for probes that fill the chip) would make
     * the pool's per-sequence calls run one at a time across worker threads */
    const int serialize = c->probe_serialize;
    c->probe_serialize = 0;
    rc = kgx_stage_probe(c, c->residues.as<uint8_t>(), c->offsets.as<uint64_t>());
    c->probe_serialize = serialize;
    if (rc)
        return rc;
    tm.mark("s.probe");
    /* the scorer: with few sequences the lane machine's one-lane chain per
     * sequence is the whole stage's latency (31 us for one 300-aa protein);
     * the wave scorer spreads each sequence's hits over a wave (option
     * small_wave; the lane machine still takes order_constraint 1) */
    const int variant = c->score_variant, wave_tiles = c->score_wave_tiles;
    if (c->small_wave && variant == SCORE_HYBRID) /* the host plan knows the longest sequence */
        c->score_variant = longest <= (uint32_t)RUN_CAP ? SCORE_WAVE_ONLY : SCORE_WAVE;
    /* a wave walks the sequences that start in its tiles one after another:
     * few tiles per wave (option small_wave_tiles) put a coalesced batch's
     * sequences on different waves, scored at once */
    c->score_wave_tiles = c->small_wave_tiles;
    /* past SMALL_GATHER_SEQ sequences the collect decides the best calls */
    const bool collect_best = (want & KGX_WANT_BEST) && n_seq > SMALL_GATHER_SEQ && n_seq <= SMALL_COLLECT_BEST_SEQ;
    c->defer_best = collect_best;
    rc = kgx_stage_score(c, params, want);
    c->defer_best = false;
    c->score_variant = variant;
    c->score_wave_tiles = wave_tiles;
    tm.mark("s.score");
    if (rc)
        return rc;
    /* results: worst-case mapped arrays, offsets and totals in mapped memory */
    const bool want_calls = (want & KGX_WANT_CALLS) != 0, want_otu = (want & KGX_WANT_OTU) != 0,
               need_hits = (want & KGX_WANT_HITS) != 0, want_best = (want & KGX_WANT_BEST) != 0;
    const uint64_t cap = std::max<uint64_t>(wb, 1);
    HIP_TRY(c->dense_hoff.reserve((n_seq + 1) * sizeof(uint64_t)));
    HIP_TRY(c->dense_coff.reserve((n_seq + 1) * sizeof(uint64_t)));
    HIP_TRY(c->dense_ooff.reserve((n_seq + 1) * sizeof(uint64_t)));
    HIP_TRY(c->h_dense_hoff.resize(n_seq + 1));
    HIP_TRY(c->h_dense_coff.resize(n_seq + 1));
    HIP_TRY(c->h_dense_ooff.resize(n_seq + 1));
    HIP_TRY(c->h_plan_status.resize(1));
    HIP_TRY(c->h_nwin.resize(1));
    HIP_TRY(c->h_hits.resize(need_hits ? cap : 0));
    HIP_TRY(c->h_calls.resize(want_calls ? cap : 0));
    HIP_TRY(c->h_otus.resize(want_otu ? cap : 0));
    HIP_TRY(c->h_best.resize(want_best ? n_seq : 0));
    void *m_hoff, *m_coff, *m_ooff, *m_st, *m_nwin, *mh = nullptr, *mc = nullptr, *mo = nullptr, *mb = nullptr;
    HIP_TRY(c->h_dense_hoff.device_ptr(0, &m_hoff));
    HIP_TRY(c->h_dense_coff.device_ptr(0, &m_coff));
    HIP_TRY(c->h_dense_ooff.device_ptr(0, &m_ooff));
    HIP_TRY(c->h_plan_status.device_ptr(0, &m_st));
    HIP_TRY(c->h_nwin.device_ptr(0, &m_nwin));
    if (need_hits)
        HIP_TRY(c->h_hits.device_ptr(0, &mh));
    if (want_calls)
        HIP_TRY(c->h_calls.device_ptr(0, &mc));
    if (want_otu)
        HIP_TRY(c->h_otus.device_ptr(0, &mo));
    if (want_best && n_seq)
        HIP_TRY(c->h_best.device_ptr(0, &mb));
    /* the fused gather stores a fresh token last; the host polls it (a stream
     * sync costs several us more than the kernel's own end) */
    const bool fused = n_seq <= SMALL_GATHER_SEQ;
    const uint32_t token = ++c->small_token ? c->small_token : ++c->small_token;
    void *m_done = nullptr;
    if (fused) {
        HIP_TRY(c->h_done.resize(1));
        c->h_done[0] = 0;
        HIP_TRY(c->h_done.device_ptr(0, &m_done));
        if (!c->small_blocks_done.p) { /* the gather's workgroup counter, zero between launches */
            HIP_TRY(c->small_blocks_done.reserve(sizeof(uint32_t)));
            HIP_TRY(hipMemsetAsync(c->small_blocks_done.p, 0, sizeof(uint32_t), c->stream));
        }
    }
    if (fused) { /* scan + gather in one workgroup */
        HIP_TRY(launch_small_gather(n_seq, c->wbase.as<uint64_t>(), c->hit_mask.as<uint64_t>(), c->tile_windows,
                                    c->hit_count.as<uint32_t>(), c->call_count.as<uint32_t>(), c->hits.as<uint4>(),
                                    c->hits.as<uint4>() + c->hit_slots, c->calls.as<kgx_call>(),
                                    c->otu_count.as<uint32_t>(), c->otus.as<kgx_otu>(), static_cast<kgx_hit *>(mh),
                                    static_cast<kgx_call *>(mc), static_cast<kgx_otu *>(mo),
                                    static_cast<uint64_t *>(m_hoff), static_cast<uint64_t *>(m_coff),
                                    static_cast<uint64_t *>(m_ooff), c->plan_status.as<uint32_t>(),
                                    want_best ? c->best.as<kgx_best_call>() : nullptr,
                                    static_cast<kgx_best_call *>(mb), static_cast<uint32_t *>(m_st),
                                    static_cast<uint64_t *>(m_nwin), static_cast<uint32_t *>(m_done), token,
                                    c->small_blocks_done.as<uint32_t>(), c->hit_format, c->stream));
    } else if (collect_best) {
        HIP_TRY(launch_small_collect_best(
            n_seq, c->hit_count.as<uint32_t>(), want_calls ? c->call_count.as<uint32_t>() : nullptr,
            want_otu ? c->otu_count.as<uint32_t>() : nullptr, c->dense_hoff.as<uint64_t>(),
            c->dense_coff.as<uint64_t>(), c->dense_ooff.as<uint64_t>(), static_cast<uint64_t *>(m_hoff),
            static_cast<uint64_t *>(m_coff), static_cast<uint64_t *>(m_ooff), c->plan_status.as<uint32_t>(),
            c->wbase.as<uint64_t>(), c->calls.as<kgx_call>(), c->call_count.as<uint32_t>(),
            c->best_ws.as<kgx_call>(), c->best.as<kgx_best_call>(), static_cast<kgx_best_call *>(mb),
            static_cast<uint32_t *>(m_st), static_cast<uint64_t *>(m_nwin), c->stream));
    } else {
        HIP_TRY(launch_small_collect(n_seq, c->hit_count.as<uint32_t>(),
                                     want_calls ? c->call_count.as<uint32_t>() : nullptr, want_otu ? c->otu_count.as<uint32_t>() : nullptr, c->dense_hoff.as<uint64_t>(),
                                     c->dense_coff.as<uint64_t>(), c->dense_ooff.as<uint64_t>(),
                                     static_cast<uint64_t *>(m_hoff), static_cast<uint64_t *>(m_coff),
                                     static_cast<uint64_t *>(m_ooff), c->plan_status.as<uint32_t>(),
                                     c->wbase.as<uint64_t>(), want_best ? c->best.as<kgx_best_call>() : nullptr,
                                     static_cast<kgx_best_call *>(mb), static_cast<uint32_t *>(m_st),
                                     static_cast<uint64_t *>(m_nwin), c->stream));
    }
    if (!fused && (mh || mc || mo)) /* a counts-and-best-calls batch (/lookup's) gathers nothing */
        HIP_TRY(launch_gather(n_seq, c->wbase.as<uint64_t>(), c->hit_mask.as<uint64_t>(), c->tile_windows,
                              c->call_count.as<uint32_t>(), c->hits.as<uint4>(),
                              c->hits.as<uint4>() + c->hit_slots, c->calls.as<kgx_call>(),
                              c->dense_hoff.as<uint64_t>(), c->dense_coff.as<uint64_t>(),
                              static_cast<kgx_hit *>(mh), static_cast<kgx_call *>(mc), 0u, c->hit_format,
                              c->otu_count.as<uint32_t>(), c->otus.as<kgx_otu>(), c->dense_ooff.as<uint64_t>(),
                              static_cast<kgx_otu *>(mo), c->stream));
    /* kgx_lookup: the rollup queued behind the pass, one host wait for both */
    if (roll_map) {
        if ((rc = rollup_enqueue(roll_map, c, roll_mode)))
            return rc;
        HIP_TRY(host_wait(c->stream));
    }
    if (fused) {
        const volatile uint32_t *done = c->h_done.data();
        HIP_TRY(host_wait_word(done, token, c->stream));
        std::atomic_thread_fence(std::memory_order_acquire);
        /* the stream drained without the gather's last store: its results
         * are not there (an early exit or a lost store), never hand them out */
        if (*done != token)
            return fail(KGX_EDEVICE, "small batch: the gather ended without its completion token");
    } else {
        HIP_TRY(host_wait(c->stream));
    }
    if (c->h_plan_status[0])
        return fail(KGX_EINVAL, "small batch: plan status raised");
    c->h_hoff.assign(c->h_dense_hoff.data(), c->h_dense_hoff.data() + n_seq + 1);
    c->h_coff.assign(c->h_dense_coff.data(), c->h_dense_coff.data() + n_seq + 1);
    c->h_ooff.assign(c->h_dense_ooff.data(), c->h_dense_ooff.data() + n_seq + 1);
    const uint64_t nh = c->h_hoff[n_seq], nc = c->h_coff[n_seq], no = c->h_ooff[n_seq];
    if ((need_hits && nh > cap) || (want_calls && nc > cap) || (want_otu && no > cap))
        return fail(KGX_EDEVICE, "small batch: more records than windows");
    HIP_TRY(c->h_hits.resize(need_hits ? nh : 0));
    HIP_TRY(c->h_calls.resize(nc));
    HIP_TRY(c->h_otus.resize(no));
    tm.mark("s.gather");
    fill_result(c, n_seq, need_hits, want_best, c->h_nwin[0], out);
    return KGX_OK;
}

/* One pass over the whole host batch (its results stay on the device for
 * kgx_kmap_rollup / kgx_kmap_add_hits / kgx_matrix_add_hits).  Residues in
 * the caller's pinned memory go up by DMA straight from there (option
 * "pinned_input"; a NUL among them reruns the batch staged, cut at the NUL);
 * others are staged into pinned memory on the stage pool's threads. */
int process_batch_one_pass(kgx_ctx *c, const kgx_params *params, const char *residues, const uint64_t *seq_offsets,
                           uint32_t n_seq, uint32_t want, kgx_result *out)
{
    PhaseTimer tm(c);
    int rc = one_pass_enqueue(c, params, residues, seq_offsets, n_seq, want, nullptr, nullptr);
    if (rc)
        return rc;
    tm.mark("enqueue");
    rc = one_pass_collect(c, params, residues, seq_offsets, n_seq, want, out);
    tm.mark("collect");
    return rc;
}

}  // namespace

int kgx_process_batch(kgx_ctx *c, const kgx_params *params, const char *residues,
                      const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want, kgx_result *out)
{
    if (!c || !out || (!seq_offsets && n_seq))
        return fail(KGX_EINVAL, "null argument");
    const uint64_t r0 = n_seq ? seq_offsets[0] : 0;
    const uint64_t n_res = n_seq ? seq_offsets[n_seq] - r0 : 0;
    for (uint32_t s = 0; s < n_seq; s++)
        if (seq_offsets[s + 1] < seq_offsets[s])
            return fail(KGX_EINVAL, "seq_offsets not monotone");
    if (n_res && !residues)
        return fail(KGX_EINVAL, "null residues");
    HIP_TRY(hipSetDevice(c->img->device));
    /* chunks of at least 2M residues, only when there is something to copy back */
    const uint64_t k_res = std::max<uint64_t>(1, n_res >> 21);
    const uint32_t K = (uint32_t)std::min<uint64_t>({(uint64_t)c->host_chunks, k_res, (uint64_t)n_seq});
    if (K >= 2 && (want & (KGX_WANT_HITS | KGX_WANT_CALLS | KGX_WANT_OTU | KGX_WANT_BEST)))
        return process_batch_chunked(c, params, residues, seq_offsets, n_seq, want, K, out);
    if (n_seq && n_res <= (uint64_t)c->small_batch && n_seq <= (1u << 16)) {
        kgx_params p;
        if (params)
            p = *params;
        else
            kgx_params_default(&p);
        if (fused_eligible(c, p, seq_offsets, n_seq, want)) {
            c->fused_batches++;
            return process_batch_fused(c, p, residues, seq_offsets, n_seq, want, out);
        }
        c->small_batches++;
        return process_batch_small(c, params, residues, seq_offsets, n_seq, want, out);
    }
    return process_batch_one_pass(c, params, residues, seq_offsets, n_seq, want, out);
}

extern "C++" {
namespace kgx {

/* kgx_lookup over a batch kgx_process_batch would take down the small-batch
 * path: that path with the rollup queued behind the pass and one host wait
 * for both (*taken = true); other batches are left to the caller */
int lookup_small(kgx_ctx *c, kgx_kmap *m, int mode, const kgx_params *params, const char *residues,
                 const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want, kgx_result *out, bool *taken)
{
    *taken = false;
    const uint64_t n_res = n_seq ? seq_offsets[n_seq] - seq_offsets[0] : 0;
    if (!n_seq || n_res > (uint64_t)c->small_batch || n_seq > (1u << 16) || (n_res && !residues))
        return KGX_OK;
    const uint64_t k_res = std::max<uint64_t>(1, n_res >> 21);
    if (std::min<uint64_t>({(uint64_t)c->host_chunks, k_res, (uint64_t)n_seq}) >= 2)
        return KGX_OK;
    kgx_params p;
    if (params)
        p = *params;
    else
        kgx_params_default(&p);
    if (fused_eligible(c, p, seq_offsets, n_seq, want))
        return KGX_OK; /* the fused kernel keeps nothing on the device to roll up */
    HIP_TRY(hipSetDevice(c->img->device));
    *taken = true;
    c->small_batches++;
    return process_batch_small(c, params, residues, seq_offsets, n_seq, want, out, m, mode);
}

}  // namespace kgx
}  // extern "C++"

int kgx_process_batch_compact(kgx_ctx *c, const kgx_params *params, const char *residues,
                              const uint64_t *seq_offsets, uint32_t n_seq, uint32_t want, kgx_compact_result *out)
{
    if (!c || !out)
        return fail(KGX_EINVAL, "null argument");
    c->compact_segs.clear();
    c->compact_chunks.clear();
    c->compact_out = 1;
    const int rc = kgx_process_batch(c, params, residues, seq_offsets, n_seq, want, &out->r);
    c->compact_out = 0;
    out->n_chunks = 0;
    out->chunks = nullptr;
    if (rc) {
        c->compact_segs.clear();
        return rc;
    }
    if (!c->compact_segs.empty()) {
        /* the pinned arrays no longer move: offsets -> pointers */
        for (const auto &g : c->compact_segs) {
            kgx_hit_chunk ch{};
            ch.seq_begin = g.s0;
            ch.seq_end = g.s1;
            ch.record_words = g.words;
            ch.hit_begin = g.hit_begin;
            ch.records = g.words == 3 ? c->h_hits12.data() + 3 * g.rec_at
                                      : reinterpret_cast<const uint32_t *>(c->h_hits16.data() + g.rec_at);
            ch.mask = c->h_mask.data() + g.mask_at;
            ch.window_start = c->h_wstart.data() + g.s0;
            c->compact_chunks.push_back(ch);
        }
        out->r.hits = nullptr;
        out->n_chunks = (uint32_t)c->compact_chunks.size();
        out->chunks = c->compact_chunks.data();
    }
    return KGX_OK;
}

int kgx_compact_expand(const kgx_compact_result *r, const char *residues, const uint64_t *seq_offsets,
                       uint32_t s_begin, uint32_t s_end, uint32_t seq_base, kgx_hit *out)
{
    return compact_expand(r, residues, seq_offsets, s_begin, s_end, seq_base, out, false);
}

}  // extern "C"

int kgx::compact_expand(const kgx_compact_result *r, const char *residues, const uint64_t *seq_offsets,
                        uint32_t s_begin, uint32_t s_end, uint32_t seq_base, kgx_hit *out, bool nt)
{
    if (!r || s_begin > s_end || s_end > r->r.n_seq || !r->r.hit_offsets)
        return fail(KGX_EINVAL, "bad compact range");
    const uint64_t *hoff = r->r.hit_offsets;
    const uint64_t j0 = hoff[s_begin], j1 = hoff[s_end];
    if (j0 == j1)
        return KGX_OK;
    if (!out)
        return fail(KGX_EINVAL, "null output");
    if (r->n_chunks == 0) {
        if (!r->r.hits)
            return fail(KGX_EINVAL, "the result holds no hits (want without KGX_WANT_HITS)");
        std::memcpy(out, r->r.hits + j0, (j1 - j0) * sizeof(kgx_hit));
        if (seq_base)
            for (uint64_t j = 0; j < j1 - j0; j++)
                out[j].seq += seq_base;
        return KGX_OK;
    }
    if (!residues || !seq_offsets)
        return fail(KGX_EINVAL, "compact hits need the batch's residues and offsets");
    /* the chunks are in sequence order: the first one that ends past s_begin */
    const kgx_hit_chunk *ch = r->chunks, *end = r->chunks + r->n_chunks;
    ch = std::upper_bound(ch, end, s_begin, [](uint32_t s, const kgx_hit_chunk &x) { return s < x.seq_end; });
    uint32_t s = s_begin;
    for (; ch != end && s < s_end; ch++) {
        if (ch->seq_begin > s) {
            /* sequences between chunks have no hits (a chunk without hits has no records) */
            for (; s < std::min(ch->seq_begin, s_end); s++)
                if (hoff[s + 1] != hoff[s])
                    return fail(KGX_EINVAL, "compact hits: a sequence with hits outside every chunk");
            if (s >= s_end)
                break;
        }
        const uint32_t b = std::min(ch->seq_end, s_end);
        const int rc = expand_chunk(*ch, hoff, residues, seq_offsets, s, b, out, j0, seq_base, nt);
        if (rc)
            return rc;
        s = b;
    }
    for (; s < s_end; s++)
        if (hoff[s + 1] != hoff[s])
            return fail(KGX_EINVAL, "compact hits: a sequence with hits outside every chunk");
    return KGX_OK;
}

extern "C" {

int kgx_ctx_stat(kgx_ctx *c, const char *name, int64_t *value)
{
    if (!c || !name || !value)
        return fail(KGX_EINVAL, "null argument");
    const std::string n = name;
    if (n == "fused_batches")
        *value = (int64_t)c->fused_batches;
    else if (n == "small_batches")
        *value = (int64_t)c->small_batches;
    else if (n == "stream_fallbacks")
        *value = (int64_t)c->stream_fallbacks;
    else if (n == "pinned_batches")
        *value = (int64_t)c->pinned_batches;
    else if (n == "nul_reruns")
        *value = (int64_t)c->nul_reruns;
    else
        return fail(KGX_EINVAL, "unknown statistic " + n);
    return KGX_OK;
}

int kgx_ctx_host_profile(kgx_ctx *c, kgx_host_profile *out)
{
    if (!c || !out)
        return fail(KGX_EINVAL, "null argument");
    *out = c->last_profile;
    return KGX_OK;
}

/* the current device batch's results -> host CSR (gather on the device, OTU
 * tallies on the host) */
int kgx_device_batch_collect(kgx_ctx *c, uint32_t want, kgx_result *out)
{
    if (!c || !out)
        return fail(KGX_EINVAL, "null argument");
    if (!c->have_hits)
        return fail(KGX_EINVAL, "no device batch to collect");
    const bool want_calls = (want & KGX_WANT_CALLS) != 0;
    const bool want_otu = (want & KGX_WANT_OTU) != 0;
    const bool need_hits = (want & KGX_WANT_HITS) != 0;
    const bool want_best = (want & KGX_WANT_BEST) != 0;
    if (want_otu && !c->have_otus)
        return fail(KGX_EINVAL, "no device OTU tallies (score with KGX_WANT_OTU)");
    if (want_best && !c->have_best)
        return fail(KGX_EINVAL, "no device best calls (score with KGX_WANT_BEST)");
    HIP_TRY(hipSetDevice(c->img->device));
    PhaseTimer tm(c);
    const uint32_t n_seq = c->n_seq;
    /* counts -> dense CSR offsets on the host, gather on the device.  The
     * plan's status word (bad device offsets: an error, not an empty result)
     * and the window total come back with the counts, in one round trip
     * (collect_counts_enqueue, unless already enqueued). */
    const bool best_now = want_best && n_seq && !need_hits && !want_calls && !want_otu;
    if (c->counts_enqueued != want + 1) {
        if (int rc = kgx::collect_counts_enqueue(c, want))
            return rc;
    }
    c->counts_enqueued = 0;
    HIP_TRY(host_wait(c->stream));
    if (c->h_plan_status[0])
        return fail(KGX_EINVAL, "batch offsets not monotone or spanning more than n_residues bytes "
                                "(the batch was processed as empty)");
    c->h_hoff.assign(n_seq + 1, 0);
    c->h_coff.assign(n_seq + 1, 0);
    c->h_ooff.assign(n_seq + 1, 0);
    for (uint32_t s = 0; s < n_seq; s++) {
        c->h_hoff[s + 1] = c->h_hoff[s] + c->h_hcount[s];
        c->h_coff[s + 1] = c->h_coff[s] + (want_calls ? c->h_ccount[s] : 0);
        c->h_ooff[s + 1] = c->h_ooff[s] + (want_otu ? c->h_ocount[s] : 0);
    }
    tm.mark(" counts");
    const uint64_t nh = c->h_hoff[n_seq], nc = c->h_coff[n_seq], no = c->h_ooff[n_seq];
    HIP_TRY(c->h_hits.resize(need_hits ? nh : 0));
    HIP_TRY(c->h_calls.resize(nc));
    HIP_TRY(c->h_otus.resize(no));
    /* small results: the gather stores the records straight into the mapped
     * pinned result arrays (no D2H copies to queue behind it) */
    const bool mapped = (need_hits ? nh : 0) + nc + no <= (1u << 16);
    if ((need_hits && nh) || nc || no) {
        HIP_TRY(c->dense_hoff.reserve((n_seq + 1) * sizeof(uint64_t)));
        HIP_TRY(c->dense_coff.reserve((n_seq + 1) * sizeof(uint64_t)));
        HIP_TRY(c->dense_ooff.reserve((n_seq + 1) * sizeof(uint64_t)));
        HIP_TRY(c->dense_hits.reserve(std::max<uint64_t>(nh, 1) * sizeof(kgx_hit)));
        HIP_TRY(c->dense_calls.reserve(std::max<uint64_t>(nc, 1) * sizeof(kgx_call)));
        HIP_TRY(c->dense_otus.reserve(std::max<uint64_t>(no, 1) * sizeof(kgx_otu)));
        HIP_TRY(hipMemcpyAsync(c->dense_hoff.p, c->h_hoff.data(), (n_seq + 1) * sizeof(uint64_t),
                               hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(c->dense_coff.p, c->h_coff.data(), (n_seq + 1) * sizeof(uint64_t),
                               hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(c->dense_ooff.p, c->h_ooff.data(), (n_seq + 1) * sizeof(uint64_t),
                               hipMemcpyHostToDevice, c->stream));
        void *mh = nullptr, *mc = nullptr, *mo = nullptr;
        if (mapped) {
            if (need_hits && nh)
                HIP_TRY(c->h_hits.device_ptr(0, &mh));
            if (nc)
                HIP_TRY(c->h_calls.device_ptr(0, &mc));
            if (no)
                HIP_TRY(c->h_otus.device_ptr(0, &mo));
        }
        kgx_hit *gh = need_hits && nh ? (mapped ? static_cast<kgx_hit *>(mh) : c->dense_hits.as<kgx_hit>()) : nullptr;
        kgx_call *gc = want_calls ? (mapped && nc ? static_cast<kgx_call *>(mc) : c->dense_calls.as<kgx_call>())
                                  : nullptr;
        kgx_otu *go = no ? (mapped ? static_cast<kgx_otu *>(mo) : c->dense_otus.as<kgx_otu>()) : nullptr;
        HIP_TRY(launch_gather(n_seq, c->wbase.as<uint64_t>(), c->hit_mask.as<uint64_t>(), c->tile_windows,
                              c->call_count.as<uint32_t>(), c->hits.as<uint4>(),
                              c->hits.as<uint4>() + c->hit_slots,
                              c->calls.as<kgx_call>(), c->dense_hoff.as<uint64_t>(),
                              c->dense_coff.as<uint64_t>(), gh, gc, 0u, c->hit_format,
                              c->otu_count.as<uint32_t>(), c->otus.as<kgx_otu>(), c->dense_ooff.as<uint64_t>(),
                              go, c->stream));
        if (!mapped) {
            if (need_hits && nh)
                HIP_TRY(hipMemcpyAsync(c->h_hits.data(), c->dense_hits.p, nh * sizeof(kgx_hit),
                                       hipMemcpyDeviceToHost, c->stream));
            if (nc)
                HIP_TRY(hipMemcpyAsync(c->h_calls.data(), c->dense_calls.p, nc * sizeof(kgx_call),
                                       hipMemcpyDeviceToHost, c->stream));
            if (no)
                HIP_TRY(hipMemcpyAsync(c->h_otus.data(), c->dense_otus.p, no * sizeof(kgx_otu),
                                       hipMemcpyDeviceToHost, c->stream));
        }
    }
    if (want_best && n_seq && !best_now) {
        HIP_TRY(c->h_best.resize(n_seq));
        HIP_TRY(hipMemcpyAsync(c->h_best.data(), c->best.p, n_seq * sizeof(kgx_best_call), hipMemcpyDeviceToHost,
                               c->stream));
    }
    if (!best_now)
        HIP_TRY(host_wait(c->stream));
    tm.mark(" gather+d2h");
    fill_result(c, n_seq, need_hits, want_best, c->h_nwin[0], out);
    return KGX_OK;
}

/* ---- synthetic queries / memory helpers ----------------------------------- */

int kgx_synth_queries(kgx_ctx *c, uint64_t image_n_keys, uint32_t n_seq, uint32_t length,
                      uint32_t x_permille, uint64_t q0, uint8_t *d_res, uint64_t *d_off)
{
    if (!c || !d_res || !d_off)
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(c->img->device));
    HIP_TRY(launch_synth_queries(image_n_keys, n_seq, length, x_permille, q0, d_res, d_off,
                                 c->stream));
    return KGX_OK;
}

int kgx_microbench_random_read(kgx_ctx *c, uint64_t n_reads, int mode, float *ms, uint64_t *reads)
{
    if (!c || !ms || mode < 0 || mode > 5)
        return fail(KGX_EINVAL, "bad argument");
    HIP_TRY(hipSetDevice(c->img->device));
    const uint64_t threads = 256ull * 256 * (uint64_t)c->microbench_wgs; /* workgroups of 256 per CU */
    const int ilp = c->microbench_ilp;
    const uint32_t rounds = (uint32_t)std::max<uint64_t>(1, n_reads / (threads * (uint64_t)ilp));
    HIP_TRY(c->plan_ws.reserve(threads * sizeof(uint64_t)));
    hipEvent_t a, b;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    HIP_TRY(hipEventRecord(a, c->stream));
    const uint64_t span = c->microbench_span ? std::min(c->microbench_span, c->img->resident_bytes())
                                             : c->img->resident_bytes();
    HIP_TRY(launch_random_read(c->img->resident(), span, threads, rounds, mode, ilp,
                               c->plan_ws.as<uint64_t>(), c->stream));
    HIP_TRY(hipEventRecord(b, c->stream));
    HIP_TRY(hipEventSynchronize(b));
    HIP_TRY(hipEventElapsedTime(ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (reads)
        *reads = threads * rounds * (uint64_t)ilp / (mode == 4 ? 4 : mode == 5 ? 8 : 1);
    return KGX_OK;
}

int kgx_event_create(void **event)
{
    if (!event)
        return fail(KGX_EINVAL, "null event");
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    *event = (void *)e;
    return KGX_OK;
}

int kgx_event_destroy(void *event)
{
    if (event)
        HIP_TRY(hipEventDestroy((hipEvent_t)event));
    return KGX_OK;
}

int kgx_event_record(void *event, kgx_ctx *c)
{
    if (!event || !c)
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipEventRecord((hipEvent_t)event, c->stream));
    return KGX_OK;
}

int kgx_event_elapsed_ms(void *start, void *end, float *ms)
{
    if (!start || !end || !ms)
        return fail(KGX_EINVAL, "null argument");
    HIP_TRY(hipEventSynchronize((hipEvent_t)end));
    HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end));
    return KGX_OK;
}

int kgx_device_alloc(int device, uint64_t nbytes, void **out)
{
    if (!out)
        return fail(KGX_EINVAL, "null output");
    HIP_TRY(hipSetDevice(device));
    hipError_t e = hipMalloc(out, std::max<uint64_t>(nbytes, 1));
    if (e != hipSuccess)
        return fail(KGX_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return KGX_OK;
}

int kgx_device_free(void *p)
{
    if (p)
        HIP_TRY(hipFree(p));
    return KGX_OK;
}

int kgx_host_alloc(uint64_t nbytes, void **out)
{
    if (!out)
        return fail(KGX_EINVAL, "null output");
    *out = nullptr;
    /* portable: usable by every device's copies (the pool's replicas) */
    hipError_t e = hipHostMalloc(out, std::max<uint64_t>(nbytes, 1), hipHostMallocPortable);
    if (e != hipSuccess) {
        *out = nullptr;
        return fail(KGX_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    }
    return KGX_OK;
}

int kgx_host_free(void *p)
{
    if (p)
        HIP_TRY(hipHostFree(p));
    return KGX_OK;
}

int kgx_memcpy_h2d(void *dst, const void *src, uint64_t n)
{
    HIP_TRY(hipMemcpy(dst, src, n, hipMemcpyHostToDevice));
    return KGX_OK;
}

int kgx_memcpy_d2h(void *dst, const void *src, uint64_t n)
{
    HIP_TRY(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost));
    return KGX_OK;
}

}  /* extern "C" */
