/* grow_to (kgx_score_map.h) against the request map it stands in for: over
 * random requests of sequences with 0..300 distinct ids each, a map cleared
 * per sequence (the reference's seq_score_) and, for every sequence, a fresh
 * map grown to the most ids any earlier sequence held iterate that
 * sequence's ids in the same order.  Prints "ok N" or the first mismatch.
 * Built and run by tests/test_score_map.py with the host compiler. */
#include <cstdio>
#include <random>
#include <unordered_map>
#include <vector>

#include "kgx_score_map.h"

struct Acc {
    unsigned hit_count = 0, hit_total = 0;
    float weighted_total = 0;
};

int main()
{
    std::mt19937_64 rng(11);
    long checked = 0;
    for (int req = 0; req < 300; req++) {
        std::unordered_map<unsigned, Acc> serial;
        size_t most = 0;
        const int n_seq = 1 + (int)(rng() % 60);
        for (int s = 0; s < n_seq; s++) {
            /* mostly few rows, now and then many (the bucket array grows) */
            const size_t rows = rng() % 8 == 0 ? rng() % 300 : rng() % 6;
            std::vector<unsigned> ids;
            while (ids.size() < rows) {
                const unsigned id = (unsigned)(rng() % 100000);
                bool dup = false;
                for (unsigned x : ids)
                    dup |= x == id;
                if (!dup)
                    ids.push_back(id);
            }
            std::unordered_map<unsigned, Acc> fresh;
            kgx::grow_to(fresh, most);
            if (!serial.empty())
                serial.clear();
            for (unsigned id : ids) {
                serial[id].hit_count = 1;
                fresh[id].hit_count = 1;
            }
            if (serial.bucket_count() != fresh.bucket_count()) {
                std::printf("bucket count %zu vs %zu (request %d, sequence %d, most %zu)\n", serial.bucket_count(),
                            fresh.bucket_count(), req, s, most);
                return 1;
            }
            auto a = serial.begin();
            for (auto b = fresh.begin(); b != fresh.end(); ++a, ++b)
                if (a->first != b->first) {
                    std::printf("order differs (request %d, sequence %d)\n", req, s);
                    return 1;
                }
            most = std::max(most, rows);
            checked++;
        }
    }
    std::printf("ok %ld\n", checked);
    return 0;
}
