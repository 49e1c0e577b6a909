/*
 * fasta_check.cpp -- kgx::parse_fasta_body (line-at-a-time fast path with the
 * byte-at-a-time fallback) against FastaParser's state machine run byte by
 * byte (fasta_parser.h:45-133) on random bodies: well-formed ones (the fast
 * path) and noisy ones ('\r', blanks, '*', '>' in odd places, digits, empty
 * lines, missing final newline).  Prints "ok N" and the parse rates.
 * TEST INFRASTRUCTURE ONLY; CPU, no GPU.
 *
 *   fasta_check N
 */
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

#include "kgx_handlers.h"

using namespace kgx;

static work_list_t machine(const std::string &body)
{
    work_list_t w;
    FastaParser p;
    p.set_callback([&w](const std::string &id, const std::string &seq) {
        w.emplace_back(id, seq);
        return 0;
    });
    p.set_error_callback([](const std::string &, int, const std::string) { return true; });
    for (char c : body)
        p.parse_char(c);
    p.parse_complete();
    return w;
}

static std::string well_formed(std::mt19937_64 &rng, int n_rec)
{
    static const char *aa = "ACDEFGHIKLMNPQRSTVWYXBZacdefg";
    std::string b;
    for (int r = 0; r < n_rec; r++) {
        b += ">id" + std::to_string(rng() % 100000);
        if (rng() % 3 == 0)
            b += (rng() % 2 ? " " : "\t") + std::string("some defline x=1");
        b += "\n";
        int lines = (int)(rng() % 4);
        for (int l = 0; l < lines; l++) {
            int len = (int)(rng() % 90);
            for (int i = 0; i < len; i++)
                b += (i > 0 || l == 0) && rng() % 50 == 0 ? '*' : aa[rng() % 29];
            if (rng() % 8 == 0)
                b += "\n"; /* a blank line */
            b += "\n";
        }
    }
    if (!b.empty() && rng() % 4 == 0)
        b.pop_back(); /* no final newline */
    return b;
}

static std::string noisy(std::mt19937_64 &rng)
{
    std::string b = well_formed(rng, 1 + (int)(rng() % 5));
    /* also the bytes next to the letter ranges and high bytes, for the
     * 16-byte validation: '@' '[' '`' '{' 0x80 0xC1 0xFA */
    static const char extra[] = ">\n\r *\t9-.xA@[`{\x80\xc1\xfa";
    int k = 1 + (int)(rng() % 3);
    for (int i = 0; i < k; i++) {
        size_t at = b.empty() ? 0 : rng() % (b.size() + 1);
        b.insert(b.begin() + at, extra[rng() % (sizeof(extra) - 1)]);
    }
    if (rng() % 10 == 0)
        b = b.substr(1); /* not starting with '>' */
    return b;
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
    std::mt19937_64 rng(0x5EEDFA57);
    for (int t = 0; t < n; t++) {
        const std::string b = t % 2 ? noisy(rng) : well_formed(rng, (int)(rng() % 12));
        const work_list_t want = machine(b);
        const work_list_t got = parse_fasta_body(b.data(), b.size());
        if (got != want) {
            std::printf("MISMATCH case %d (%zu vs %zu records)\n", t, got.size(), want.size());
            std::fwrite(b.data(), 1, b.size(), stdout);
            return 1;
        }
        if (flat_of(want).res != parse_fasta_body_flat(b.data(), b.size()).res ||
            flat_of(want).ids != parse_fasta_body_flat(b.data(), b.size()).ids ||
            flat_of(want).off != parse_fasta_body_flat(b.data(), b.size()).off) {
            std::printf("FLAT MISMATCH case %d\n", t);
            return 1;
        }
    }
    /* pieces cut by split_fasta_body, each parsed line by line, concatenate
     * to the whole-body parse whenever every piece parses */
    int split_used = 0;
    for (int t = 0; t < n; t++) {
        std::string b = t % 3 ? well_formed(rng, 1 + (int)(rng() % 40)) : noisy(rng);
        if (t % 7 == 0)
            b += ">hdr_only\n>next\nACDE\n"; /* a header right before '>' */
        const size_t pieces = 2 + rng() % 6;
        auto cuts = split_fasta_body(b.data(), b.size(), pieces);
        if (cuts.empty())
            continue;
        if (cuts.front().first != 0 || cuts.back().second != b.size()) {
            std::printf("BAD CUTS case %d\n", t);
            return 1;
        }
        work_list_t joined;
        FastaFlat joined_flat;
        bool ok = true;
        for (auto &c : cuts) {
            if (c.second <= c.first || b[c.first] != '>') {
                std::printf("BAD PIECE case %d\n", t);
                return 1;
            }
            ok = ok && parse_fasta_piece(b.data() + c.first, c.second - c.first, joined);
            FastaFlat piece;
            if (ok && !parse_fasta_piece_flat(b.data() + c.first, c.second - c.first, piece)) {
                std::printf("FLAT PIECE REFUSED case %d\n", t);
                return 1;
            }
            for (size_t i = 0; ok && i < piece.size(); i++)
                joined_flat.add(piece.ids.data() + piece.id_off[i], piece.id_off[i + 1] - piece.id_off[i],
                                piece.res.data() + piece.off[i], piece.off[i + 1] - piece.off[i]);
        }
        if (!ok)
            continue;
        split_used++;
        const FastaFlat want_flat = flat_of(machine(b));
        if (joined_flat.res != want_flat.res || joined_flat.ids != want_flat.ids || joined_flat.off != want_flat.off ||
            joined_flat.id_off != want_flat.id_off) {
            std::printf("SPLIT FLAT MISMATCH case %d\n", t);
            return 1;
        }
        if (joined != machine(b)) {
            std::printf("SPLIT MISMATCH case %d\n", t);
            std::fwrite(b.data(), 1, b.size(), stdout);
            return 1;
        }
    }
    if (split_used < n / 20) {
        std::printf("split path too rarely taken (%d)\n", split_used);
        return 1;
    }
    /* rates on a 30 MB body of 300-aa proteins (the C2 request shape) */
    std::string big;
    for (int r = 0; r < 100000; r++) {
        big += ">q" + std::to_string(r) + "\n";
        for (int i = 0; i < 300; i++)
            big += "ACDEFGHIKLMNPQRSTVWY"[rng() % 20];
        big += "\n";
    }
    auto t0 = std::chrono::steady_clock::now();
    const work_list_t a = parse_fasta_body(big.data(), big.size());
    auto t1 = std::chrono::steady_clock::now();
    const work_list_t m = machine(big);
    auto t2 = std::chrono::steady_clock::now();
    if (a != m || a.size() != 100000) {
        std::printf("MISMATCH on the big body\n");
        return 1;
    }
    std::printf("ok %d lines_MBps=%.0f machine_MBps=%.0f\n", n,
                big.size() / 1e6 / std::chrono::duration<double>(t1 - t0).count(),
                big.size() / 1e6 / std::chrono::duration<double>(t2 - t1).count());
    return 0;
}
