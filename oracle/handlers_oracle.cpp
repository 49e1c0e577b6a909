/*
 * handlers_oracle.cpp -- TEST INFRASTRUCTURE ONLY (never linked into the
 * product).  CPU restatement of the request-handler arithmetic that sits on
 * the hit stream, with the same standard containers the reference uses so
 * iteration and tie orders match:
 *
 *   oracle_kmap_*   KmerPegMapping::add_mapping (kmer.cc:173-210: append,
 *                   duplicates kept) and add_fam_mapping / fam_map_insert
 *                   (kmer.cc:212-256: std::find, push_back if absent)
 *   oracle_matrix_* MatrixRequest (matrix_request.cc:83-95 per-sequence loop,
 *                   on_hit 130-163, process_results 165-190; state
 *                   matrix_request.h:25-26)
 */
#include <cstdint>
#include <cstring>
#include <map>
#include <unordered_map>
#include <algorithm>
#include <utility>
#include <vector>

namespace {

struct Kmap {
    int mode = 0; /* 0 append (kmer_to_id_), 1 set (kmer_to_family_id_) */
    std::unordered_map<uint64_t, std::vector<uint32_t>> m;
    void add(uint64_t kmer, uint32_t id)
    {
        auto &v = m[kmer];
        if (mode == 1 && std::find(v.begin(), v.end(), id) != v.end())
            return; /* fam_map_insert, kmer.cc:214-227 */
        v.push_back(id);
    }
};

struct Matrix {
    std::map<uint32_t, size_t> matrix_proteins;                         /* matrix_request.h:25 */
    std::map<std::pair<uint32_t, uint32_t>, unsigned long> distance;    /* matrix_request.h:26 */
};

}  // namespace

extern "C" {

void *oracle_kmap_new(int mode)
{
    Kmap *k = new Kmap;
    k->mode = mode;
    return k;
}

void oracle_kmap_free(void *p) { delete static_cast<Kmap *>(p); }

void oracle_kmap_add(void *p, const uint64_t *kmers, const uint32_t *ids, uint64_t n)
{
    Kmap *k = static_cast<Kmap *>(p);
    for (uint64_t i = 0; i < n; i++)
        k->add(kmers[i], ids[i]);
}

/* number of ids of `kmer`; copies up to cap of them into ids */
uint64_t oracle_kmap_lookup(void *p, uint64_t kmer, uint32_t *ids, uint64_t cap)
{
    Kmap *k = static_cast<Kmap *>(p);
    auto it = k->m.find(kmer);
    if (it == k->m.end())
        return 0;
    const auto &v = it->second;
    for (uint64_t i = 0; i < v.size() && i < cap; i++)
        ids[i] = v[i];
    return v.size();
}

uint64_t oracle_kmap_num_kmers(void *p) { return static_cast<Kmap *>(p)->m.size(); }

void *oracle_matrix_new(void) { return new Matrix; }
void oracle_matrix_free(void *p) { delete static_cast<Matrix *>(p); }

/* One batch of a /matrix request: sequence s has id seq_ids[s], length
 * seq_lens[s] and hits hit_kmers[hit_off[s] .. hit_off[s+1]) in position order. */
void oracle_matrix_add(void *px, void *pk, const uint32_t *seq_ids, const uint64_t *seq_lens,
                       uint64_t n_seq, const uint64_t *hit_off, const uint64_t *hit_kmers)
{
    Matrix *x = static_cast<Matrix *>(px);
    Kmap *k = static_cast<Kmap *>(pk);
    for (uint64_t s = 0; s < n_seq; s++) {
        const uint32_t id = seq_ids[s];
        x->matrix_proteins[id] = seq_lens[s]; /* matrix_request.cc:91 */
        for (uint64_t h = hit_off[s]; h < hit_off[s + 1]; h++) {
            auto ki = k->m.find(hit_kmers[h]);
            if (ki == k->m.end())
                continue; /* "no mapping for" on stderr, matrix_request.cc:159 */
            for (uint32_t eid : ki->second)
                if (eid != id && x->matrix_proteins.find(eid) != x->matrix_proteins.end())
                    x->distance[std::make_pair(id, eid)]++;
        }
    }
}

/* distance_ in map order with process_results' score (matrix_request.cc:
 * 179-186); returns the number of pairs, fills the arrays when non-null */
uint64_t oracle_matrix_pairs(void *px, uint32_t *id1, uint32_t *id2, uint64_t *count, float *score)
{
    Matrix *x = static_cast<Matrix *>(px);
    uint64_t i = 0;
    for (auto it = x->distance.begin(); it != x->distance.end(); ++it, ++i) {
        if (!id1)
            continue;
        const uint32_t e1 = it->first.first, e2 = it->first.second;
        id1[i] = e1;
        id2[i] = e2;
        count[i] = it->second;
        const size_t l1 = x->matrix_proteins[e1], l2 = x->matrix_proteins[e2];
        score[i] = (float)it->second / ((float)(l1 + l2));
    }
    return x->distance.size();
}

}  /* extern "C" */
