/*
 * kgx_server.cpp -- the kser request server over the HIP engine.
 *
 *   kgx_server [options] listen-port kmer-data-dir
 *
 * Options follow kser.cc:52-75 where they apply to the request path:
 *   --listen-port-file F      write the bound port here (port 0 = any free port)
 *   --n-kmer-threads N        KmerGuts workers (one GPU context each)
 *   --kmer-version V, --families-version V       reported by GET /version
 *   --families-genus-mapping F, --families-file F, --families-nr F [F ...]
 *                             the family DB (family mode = --families-file given)
 *   --bind ADDR               listen address (default 0.0.0.0, as kserver.cc:144-152)
 *   --device N                GPU (default $KGX_DEVICE or 0)
 *   --devices LIST            several GPUs, e.g. 0-7 or 0,2,5 (a device may
 *                             repeat): one image replica each (the file is
 *                             read once and copied to every device), workers
 *                             spread over them (worker w on LIST[w % n]; at
 *                             least one per device), a large /query's pieces
 *                             and concurrent requests dealt to the least busy
 *                             device first (kgx_dispatch.h)
 *   --synthetic-image K:S     benchmark hook: a synthetic image of K keys in S
 *                             buckets built in HBM (kmer-data-dir still holds
 *                             function.index / otu.index)
 *   --max-header-kb N         request line + headers cap (default 64 KiB;
 *                             past it: 431 and the connection is closed)
 *   --max-body-mb N           Content-length cap (default 4096; past it: 413)
 *   --max-mappings N          /mapping/<key> keys that may be created (default
 *                             1024; a new key past it: 503)
 *
 * The listener is unauthenticated and GET /quit stops it, as in the
 * reference: bind it to a trusted interface (--bind 127.0.0.1) when the port
 * is reachable from untrusted peers.
 *
 * One connection = one request, as in krequest2.cc: the request line and
 * headers are read, then Content-length bytes of body, the router builds the
 * response, the connection is closed.  Each connection runs on its own
 * thread (at most 256 open at once); the router's KmerGuts pool bounds how
 * many run on the GPU at once.
 * GET /quit stops the listener after its response.
 */
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cerrno>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "kgx_handlers.h"

using namespace kgx;

namespace {

std::atomic<bool> g_stop{false};
int g_listen_fd = -1;
std::atomic<int> g_active{0}; /* connection threads still running */
constexpr int kMaxConnections = 256; /* accept waits while this many are open */

bool write_all(int fd, const char *p, size_t n)
{
    while (n > 0) {
        ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
        if (w < 0 && errno == EINTR)
            continue;
        if (w <= 0)
            return false;
        p += w;
        n -= (size_t)w;
    }
    return true;
}

/* request size limits (options --max-header-kb, --max-body-mb) */
size_t g_max_header_bytes = 64 << 10;
uint64_t g_max_body_bytes = 4ull << 30;
constexpr size_t TOO_LONG = std::string::npos - 1;

/* reads bytes into buf until it holds "\n" at or after `from`; returns the
 * position of that '\n', npos at EOF/error, TOO_LONG once the request line
 * and headers exceed g_max_header_bytes without one */
size_t read_line(int fd, std::string &buf, size_t from)
{
    for (;;) {
        size_t nl = buf.find('\n', from);
        if (nl != std::string::npos)
            return nl > g_max_header_bytes ? TOO_LONG : nl;
        if (buf.size() > g_max_header_bytes)
            return TOO_LONG;
        char tmp[65536];
        ssize_t r = ::recv(fd, tmp, sizeof tmp, 0);
        if (r < 0 && errno == EINTR)
            continue;
        if (r <= 0)
            return std::string::npos;
        buf.append(tmp, (size_t)r);
    }
}

uint64_t clock_ns()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

void serve_connection(KmerRequestRouter &router, int fd)
{
    const uint64_t t_recv = clock_ns(); /* stage clocks: recv from the accept */
    std::string buf;
    HttpRequest req;
    auto refuse = [&](int code, const char *status) {
        const std::string resp = KmerRequestRouter::respond("1.1", code, status, std::string(status) + "\n");
        write_all(fd, resp.data(), resp.size());
        ::shutdown(fd, SHUT_WR);
        ::close(fd);
    };
    size_t nl = read_line(fd, buf, 0);
    if (nl == TOO_LONG)
        return refuse(431, "Request Header Fields Too Large");
    if (nl == std::string::npos) {
        ::close(fd);
        return;
    }
    std::string line = buf.substr(0, nl);
    size_t cr = line.find('\r');
    if (cr != std::string::npos)
        line.erase(cr);
    size_t pos = nl + 1;
    if (!parse_request_line(line, req)) {
        std::cerr << "Invalid request '" << line << "'\n";
        ::close(fd);
        return;
    }
    for (;;) { /* headers up to the empty line */
        nl = read_line(fd, buf, pos);
        if (nl == TOO_LONG)
            return refuse(431, "Request Header Fields Too Large");
        if (nl == std::string::npos) {
            ::close(fd);
            return;
        }
        line = buf.substr(pos, nl - pos);
        pos = nl + 1;
        cr = line.find('\r');
        if (cr != std::string::npos)
            line.erase(cr);
        if (line.empty())
            break;
        parse_header_line(line, req);
    }
    auto ex = req.headers.find("expect"); /* krequest2.cc:262-270 */
    if (ex != req.headers.end() && ex->second == "100-continue") {
        const std::string cont = "HTTP/" + req.http_version + " 100 Continue\n\n";
        write_all(fd, cont.data(), cont.size());
    }
    auto cl = req.headers.find("content-length");
    if (req.method == "POST" && cl != req.headers.end()) {
        size_t len = 0;
        try {
            len = std::stoul(cl->second);
        } catch (...) {
            len = 0;
        }
        if (len > g_max_body_bytes)
            return refuse(413, "Payload Too Large");
        /* the body straight into place: one copy out of the socket, not two */
        const size_t have = std::min(len, buf.size() - pos);
        req.body.resize(len);
        std::memcpy(&req.body[0], buf.data() + pos, have);
        size_t got = have;
        while (got < len) {
            ssize_t r = ::recv(fd, &req.body[got], len - got, 0);
            if (r < 0 && errno == EINTR)
                continue;
            if (r <= 0)
                break;
            got += (size_t)r;
        }
        req.body.resize(got);
    }
    bool quit = false;
    StageStats &st = stage_stats();
    const uint64_t t_handle = clock_ns();
    const std::string resp = router.handle(req, &quit);
    const uint64_t t_send = clock_ns();
    write_all(fd, resp.data(), resp.size());
    ::shutdown(fd, SHUT_WR);
    ::close(fd);
    if (req.path != "/server_stats") {
        const uint64_t t_end = clock_ns();
        st.requests++;
        st.bytes_in += req.body.size();
        st.bytes_out += resp.size();
        st.recv_ns += t_handle - t_recv;
        st.handle_ns += t_send - t_handle;
        st.send_ns += t_end - t_send;
    }
    if (quit) {
        std::cerr << "stopping io service\n";
        g_stop = true;
        ::shutdown(g_listen_fd, SHUT_RDWR);
    }
}

void on_signal(int)
{
    g_stop = true;
    if (g_listen_fd >= 0)
        ::shutdown(g_listen_fd, SHUT_RDWR);
}

/* "0-7", "0,2,5", "0,0" -> device list; empty on a syntax error */
std::vector<int> parse_devices(const std::string &spec)
{
    std::vector<int> out;
    size_t a = 0;
    while (a <= spec.size()) {
        size_t b = spec.find(',', a);
        if (b == std::string::npos)
            b = spec.size();
        const std::string part = spec.substr(a, b - a);
        const size_t dash = part.find('-');
        char *end = nullptr;
        if (part.empty())
            return {};
        if (dash == std::string::npos) {
            long v = std::strtol(part.c_str(), &end, 10);
            if (*end || v < 0)
                return {};
            out.push_back((int)v);
        } else {
            if (dash == 0 || dash + 1 == part.size())
                return {};
            long lo = std::strtol(part.substr(0, dash).c_str(), &end, 10);
            if (*end)
                return {};
            long hi = std::strtol(part.substr(dash + 1).c_str(), &end, 10);
            if (*end || lo < 0 || hi < lo || hi - lo > 255)
                return {};
            for (long v = lo; v <= hi; v++)
                out.push_back((int)v);
        }
        a = b + 1;
    }
    return out;
}

int usage(const char *argv0)
{
    std::fprintf(stderr,
                 "Usage: %s [options] listen-port kmer-data-dir\n"
                 "  --listen-port-file F  --n-kmer-threads N  --kmer-version V  --families-version V\n"
                 "  --families-genus-mapping F  --families-file F  --families-nr F [F ...]\n"
                 "  --bind ADDR  --device N  --devices LIST  --synthetic-image KEYS:BUCKETS\n"
                 "  --max-header-kb N  --max-body-mb N  --max-mappings N\n",
                 argv0);
    return 2;
}

} // namespace

int main(int argc, char **argv)
{
    KmerRequestRouter::Options opt;
    /* the workers wait for their device work asleep (polling every 20 us),
     * not spinning: a server runs in a CPU share, and with 16 workers the
     * spinning took it from the socket and text threads (r8: the 16-CPU
     * cgroup throttled in 96% of its periods).  KGX_HOST_WAIT overrides. */
    if (!std::getenv("KGX_HOST_WAIT"))
        kgx_set_host_wait(KGX_WAIT_SLEEP, 20);
    const char *dev = std::getenv("KGX_DEVICE");
    opt.device = dev ? std::atoi(dev) : 0;
    std::string port_file = "/dev/null", bind_addr = "0.0.0.0";
    std::vector<std::string> positional;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto value = [&](std::string &dst) {
            if (i + 1 >= argc)
                return false;
            dst = argv[++i];
            return true;
        };
        std::string v;
        if (a == "-h" || a == "--help")
            return usage(argv[0]);
        else if (a == "--listen-port-file") {
            if (!value(port_file))
                return usage(argv[0]);
        } else if (a == "--n-kmer-threads") {
            if (!value(v))
                return usage(argv[0]);
            opt.n_kmer_threads = std::atoi(v.c_str());
        } else if (a == "--kmer-version") {
            if (!value(opt.kmer_version))
                return usage(argv[0]);
        } else if (a == "--families-version") {
            if (!value(opt.families_version))
                return usage(argv[0]);
        } else if (a == "--families-genus-mapping") {
            if (!value(opt.genus_mapping))
                return usage(argv[0]);
        } else if (a == "--families-file") {
            if (!value(opt.families_file))
                return usage(argv[0]);
        } else if (a == "--families-nr") { /* multitoken (kser.cc:65) */
            while (i + 1 < argc && argv[i + 1][0] != '-')
                opt.families_nr.push_back(argv[++i]);
        } else if (a == "--max-header-kb" || a == "--max-body-mb" || a == "--max-mappings") {
            if (!value(v))
                return usage(argv[0]);
            const long long x = std::atoll(v.c_str());
            if (x < 1)
                return usage(argv[0]);
            if (a == "--max-header-kb")
                g_max_header_bytes = (size_t)x << 10;
            else if (a == "--max-body-mb")
                g_max_body_bytes = (uint64_t)x << 20;
            else
                opt.max_mappings = (size_t)x;
        } else if (a == "--bind") {
            if (!value(bind_addr))
                return usage(argv[0]);
        } else if (a == "--device") {
            if (!value(v))
                return usage(argv[0]);
            opt.device = std::atoi(v.c_str());
        } else if (a == "--devices") {
            if (!value(v) || (opt.devices = parse_devices(v)).empty()) {
                std::fprintf(stderr, "bad --devices list\n");
                return usage(argv[0]);
            }
        } else if (a == "--synthetic-image") {
            size_t colon;
            if (!value(v) || (colon = v.find(':')) == std::string::npos)
                return usage(argv[0]);
            opt.synthetic_keys = std::strtoull(v.c_str(), nullptr, 10);
            opt.synthetic_sigs = std::strtoull(v.c_str() + colon + 1, nullptr, 10);
        } else if (!a.empty() && a[0] == '-') {
            std::fprintf(stderr, "unknown option %s\n", a.c_str());
            return usage(argv[0]);
        } else
            positional.push_back(a);
    }
    if (positional.size() != 2)
        return usage(argv[0]);
    opt.kmer_data_dir = positional[1];
    const int port = std::atoi(positional[0].c_str());

    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_port = htons((uint16_t)port);
    if (::inet_pton(AF_INET, bind_addr.c_str(), &addr.sin_addr) != 1) {
        std::fprintf(stderr, "bad --bind address %s\n", bind_addr.c_str());
        return 2;
    }
    if (::bind(fd, (sockaddr *)&addr, sizeof addr) < 0 || ::listen(fd, 128) < 0) {
        std::fprintf(stderr, "cannot listen on %s:%d: %s\n", bind_addr.c_str(), port, std::strerror(errno));
        return 1;
    }
    socklen_t alen = sizeof addr;
    ::getsockname(fd, (sockaddr *)&addr, &alen);
    g_listen_fd = fd;

    std::unique_ptr<KmerRequestRouter> router;
    try {
        router.reset(new KmerRequestRouter(opt));
    } catch (const std::exception &e) {
        std::fprintf(stderr, "kgx_server: %s\n", e.what());
        return 1;
    }
    { /* the port file is written once the data are loaded, as kserver.cc */
        std::ofstream pf(port_file);
        pf << ntohs(addr.sin_port) << "\n";
    }
    {
        std::ostringstream ws;
        for (int d : router->worker_devices())
            ws << " " << d;
        std::cerr << "workers on devices" << ws.str() << "\n";
    }
    std::cerr << "Listening on port " << ntohs(addr.sin_port) << "\n";
    std::signal(SIGINT, on_signal);
    std::signal(SIGTERM, on_signal);

    while (!g_stop) {
        while (g_active >= kMaxConnections && !g_stop)
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        int c = ::accept(fd, nullptr, nullptr);
        if (c < 0) {
            if (errno == EINTR && !g_stop)
                continue;
            break;
        }
        g_active++;
        std::thread([&router, c] {
            serve_connection(*router, c);
            g_active--;
        }).detach();
    }
    while (g_active > 0) /* let running requests finish before the router goes */
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    ::close(fd);
    return 0;
}
