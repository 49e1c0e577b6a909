/*
 * load_gen -- a native HTTP load generator for kgx_server, run as its own
 * process (tools/bench_server.py starts it), so the clients' cost is not the
 * server's Python neighbour.  C client threads each loop: connect to
 * 127.0.0.1:PORT, send "POST PATH" with the next body (one connection per
 * request, as krequest2.cc serves them), read the response to EOF, check it
 * starts with "HTTP/1.1 200".  Bodies are the request bodies of BODIES.bin.
 *
 *   load_gen PORT PATH BODIES.bin CLIENTS SECONDS
 *
 * BODIES.bin: uint64 n, then per body: uint64 residues, uint64 bytes, bytes.
 * Prints one JSON line: requests, residues/s, latency median / p99 (ms).
 */
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cerrno>
#include <cstring>
#include <fstream>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

using clk = std::chrono::steady_clock;

struct Body {
    uint64_t residues;
    std::string bytes;
};

static bool post(int port, const std::string &head, const std::string &body, std::string &resp)
{
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0)
        return false;
    const int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (::connect(fd, reinterpret_cast<sockaddr *>(&a), sizeof a) != 0) {
        ::close(fd);
        return false;
    }
    auto send_all = [fd](const char *p, size_t n) {
        while (n) {
            const ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
            if (w <= 0)
                return false;
            p += w;
            n -= (size_t)w;
        }
        return true;
    };
    bool ok = send_all(head.data(), head.size()) && send_all(body.data(), body.size());
    resp.clear();
    char buf[1 << 16];
    while (ok) {
        const ssize_t r = ::recv(fd, buf, sizeof buf, 0);
        if (r <= 0)
            break;
        resp.append(buf, (size_t)r);
    }
    ::close(fd);
    return ok && resp.compare(0, 12, "HTTP/1.1 200") == 0;
}

int main(int argc, char **argv)
{
    if (argc < 6) {
        std::fprintf(stderr, "usage: load_gen PORT PATH BODIES.bin CLIENTS SECONDS\n");
        return 2;
    }
    const int port = std::atoi(argv[1]);
    const std::string path = argv[2];
    const int C = std::atoi(argv[4]);
    const double seconds = std::atof(argv[5]);
    std::ifstream in(argv[3], std::ios::binary);
    uint64_t n = 0;
    in.read(reinterpret_cast<char *>(&n), 8);
    std::vector<Body> bodies(n);
    for (auto &b : bodies) {
        uint64_t len = 0;
        in.read(reinterpret_cast<char *>(&b.residues), 8);
        in.read(reinterpret_cast<char *>(&len), 8);
        b.bytes.resize(len);
        in.read(&b.bytes[0], (std::streamsize)len);
    }
    if (!in || n == 0) {
        std::fprintf(stderr, "load_gen: bad bodies file\n");
        return 2;
    }
    std::vector<std::string> heads(n);
    for (uint64_t i = 0; i < n; i++)
        heads[i] = "POST " + path + " HTTP/1.1\r\nContent-Length: " + std::to_string(bodies[i].bytes.size()) + "\r\n\r\n";
    std::atomic<uint64_t> next{0}, residues{0}, failures{0};
    std::mutex mu;
    std::string first_failure;
    std::vector<double> lat;
    const auto t0 = clk::now();
    const auto stop = t0 + std::chrono::duration<double>(seconds);
    std::vector<std::thread> ws;
    for (int c = 0; c < C; c++)
        ws.emplace_back([&] {
            std::string resp;
            std::vector<double> my;
            while (clk::now() < stop) {
                const uint64_t i = next++ % n;
                const auto q0 = clk::now();
                if (!post(port, heads[i], bodies[i].bytes, resp)) {
                    if (failures++ == 0) {
                        std::lock_guard<std::mutex> g(mu);
                        first_failure = resp.empty() ? "no response (errno " + std::to_string(errno) + ")"
                                                     : resp.substr(0, std::min<size_t>(resp.find('\r'), 80));
                    }
                    continue;
                }
                my.push_back(std::chrono::duration<double, std::milli>(clk::now() - q0).count());
                residues += bodies[i].residues;
            }
            std::lock_guard<std::mutex> g(mu);
            lat.insert(lat.end(), my.begin(), my.end());
        });
    for (auto &w : ws)
        w.join();
    const double wall = std::chrono::duration<double>(clk::now() - t0).count();
    std::sort(lat.begin(), lat.end());
    auto pct = [&](double p) { return lat.empty() ? 0.0 : lat[std::min(lat.size() - 1, (size_t)(p / 100.0 * lat.size()))]; };
    std::printf("{\"clients\": %d, \"requests\": %zu, \"failures\": %llu, \"residues_per_s\": %.5g, "
                "\"ms_median\": %.3f, \"ms_p99\": %.3f, \"wall_s\": %.3f, \"first_failure\": \"%s\"}\n",
                C, lat.size(), (unsigned long long)failures.load(), (double)residues.load() / wall, pct(50), pct(99),
                wall, first_failure.c_str());
    return failures.load() ? 1 : 0;
}
