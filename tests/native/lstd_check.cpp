/*
 * Host-side check of kgx_lstd.h (the ordering rules the device kernels use)
 * against libstdc++ itself and the oracle:
 *   lstd_sort        vs std::sort                (pairs with tied keys, tagged)
 *   lstd_heap_sort   vs std::partial_sort(first, last, last)
 *   otu_finalize     vs std::map + std::sort(less_second) (kguts.h:196-218)
 *   best_call_decide vs the oracle's find_best_call (kguts.cc:1008-1199)
 * Test infrastructure, run on the CPU by tests/test_lstd_native.py:
 *   lstd_check [cases]   prints "ok <cases>" or the first mismatch (exit 1)
 */
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "kgx_lstd.h"

extern "C" int oracle_find_best_call(const kgx_call *calls, uint64_t n, const char *const *names, int n_names,
                                     int32_t *function_index, char *fn_buf, uint64_t fn_cap, float *out3,
                                     int *offset_set);

static bool same_f(float a, float b) { return std::memcmp(&a, &b, 4) == 0; }

static int fail(const char *what, long c)
{
    std::printf("MISMATCH %s in case %ld\n", what, c);
    return 1;
}

/* a host emulation of lstd_sort_wave64 (kgx_fused.hip), one "lane" per
 * element of a partition range: the partition by stop ranks (the t-th
 * left stop swaps with the t-th right stop while L_t < R_t, cut =
 * min(L_{P+1}, R_P)) and the final insertion sort as a stable sort by
 * counting.  Checks the formulation the device replays against std::sort. */
template <class T, class C> static void stops_sort(T *a, int n, C comp)
{
    struct Part {
        int f, l, depth;
    };
    if (n > 16) {
        std::vector<Part> st{{0, n, 2 * (31 - __builtin_clz((unsigned)n))}};
        while (!st.empty()) {
            Part p = st.back();
            st.pop_back();
            int f = p.f, l = p.l, depth = p.depth;
            while (l - f > 16) {
                if (depth == 0) {
                    kgx::lstd_heap_sort(a + f, l - f, comp);
                    break;
                }
                --depth;
                const int mid = f + (l - f) / 2;
                const T x = a[f + 1], y = a[mid], z = a[l - 1];
                int pick;
                if (comp(x, y))
                    pick = comp(y, z) ? mid : (comp(x, z) ? l - 1 : f + 1);
                else
                    pick = comp(x, z) ? f + 1 : (comp(y, z) ? l - 1 : mid);
                std::swap(a[f], a[pick]);
                const T pivot = a[f];
                const int len = l - f - 1;
                std::vector<T> v(a + f + 1, a + l), bl(len), br(len);
                std::vector<int> lf(len), rf(len), lb(len), ra(len);
                for (int k = 0; k < len; k++) {
                    lf[k] = !comp(v[k], pivot);
                    rf[k] = !comp(pivot, v[k]);
                }
                for (int k = 0, c = 0; k < len; k++) {
                    lb[k] = c;
                    c += lf[k];
                }
                for (int k = len - 1, c = 0; k >= 0; k--) {
                    ra[k] = c;
                    c += rf[k];
                }
                int P = 0;
                for (int k = 0; k < len; k++) {
                    if (lf[k] && lb[k] + 1 <= ra[k]) {
                        bl[lb[k]] = v[k];
                        P++;
                    }
                    if (rf[k] && ra[k] + 1 <= lb[k])
                        br[ra[k]] = v[k];
                }
                int lcut = 1 << 30, rcut = 1 << 30;
                for (int k = 0; k < len; k++) {
                    const bool swl = lf[k] && lb[k] + 1 <= ra[k], swr = rf[k] && ra[k] + 1 <= lb[k];
                    a[f + 1 + k] = swl ? br[lb[k]] : swr ? bl[ra[k]] : v[k];
                    if (lf[k] && lb[k] + 1 == P + 1 && lcut == (1 << 30))
                        lcut = f + 1 + k;
                    if (P > 0 && rf[k] && ra[k] + 1 == P && rcut == (1 << 30))
                        rcut = f + 1 + k;
                }
                const int cut = std::min(lcut, rcut);
                st.push_back({cut, l, depth});
                l = cut;
            }
        }
    }
    std::vector<T> out(n);
    for (int i = 0; i < n; i++) {
        int pos = 0;
        for (int j = 0; j < n; j++)
            pos += comp(a[j], a[i]) || (j < i && !comp(a[i], a[j]));
        out[pos] = a[i];
    }
    std::copy(out.begin(), out.end(), a);
}

int main(int argc, char **argv)
{
    const long cases = argc > 1 ? std::atol(argv[1]) : 20000;
    std::mt19937_64 rng(0x5EED0006);
    auto uni = [&](long lo, long hi) { return (long)(lo + (long)(rng() % (uint64_t)(hi - lo + 1))); };

    for (long c = 0; c < cases; c++) {
        /* 1. std::sort with less_second on tagged pairs: ties expose the order */
        const long n = c % 10 == 0 ? uni(17, 2000) : uni(0, 40);
        const long keys = uni(1, 12);
        std::vector<kgx_otu> a(n), b;
        for (long i = 0; i < n; i++)
            a[i] = kgx_otu{(int32_t)i, (int32_t)uni(0, keys)};
        b = a;
        auto less_second = [](const kgx_otu &l, const kgx_otu &r) { return r.count < l.count; };
        std::sort(a.begin(), a.end(), less_second);
        kgx::lstd_sort(b.data(), (int64_t)b.size(), less_second);
        for (long i = 0; i < n; i++)
            if (a[i].otu_index != b[i].otu_index || a[i].count != b[i].count)
                return fail("lstd_sort", c);
        /* 1b. the wave replay's formulation, up to 64 elements (many ties) */
        {
            const long n2 = c % 4 ? uni(17, 64) : uni(0, 16);
            std::vector<kgx_otu> w(n2), ws;
            for (long i = 0; i < n2; i++)
                w[i] = kgx_otu{(int32_t)i, (int32_t)uni(0, c % 3 ? keys : 2)};
            ws = w;
            std::sort(ws.begin(), ws.end(), less_second);
            stops_sort(w.data(), (int)n2, less_second);
            for (long i = 0; i < n2; i++)
                if (w[i].otu_index != ws[i].otu_index || w[i].count != ws[i].count)
                    return fail("stops_sort (lstd_sort_wave64's formulation)", c);
        }

        /* 2. partial_sort(first, last, last) = the depth-limit fallback */
        std::vector<kgx_otu> p(n), q;
        for (long i = 0; i < n; i++)
            p[i] = kgx_otu{(int32_t)i, (int32_t)uni(0, keys)};
        q = p;
        std::partial_sort(p.begin(), p.end(), p.end(), less_second);
        kgx::lstd_heap_sort(q.data(), (int64_t)q.size(), less_second);
        for (long i = 0; i < n; i++)
            if (p[i].otu_index != q[i].otu_index)
                return fail("lstd_heap_sort", c);

        /* 3. KmerOtuStats: otu_map then finalize() */
        const long nh = uni(0, c % 7 == 0 ? 3000 : 150);
        const long n_otu = uni(1, c % 3 == 0 ? 400 : 30);
        std::vector<int32_t> v(nh);
        std::map<int, int> m;
        for (long i = 0; i < nh; i++) {
            v[i] = (int32_t)uni(-1, n_otu);
            m[v[i]]++;
        }
        std::vector<std::pair<int, int>> ref(m.begin(), m.end());
        std::sort(ref.begin(), ref.end(),
                  [](const std::pair<int, int> &l, const std::pair<int, int> &r) { return r.second < l.second; });
        std::vector<kgx_otu> o(nh + 1);
        const int64_t k = kgx::otu_finalize(v.data(), (int64_t)v.size(), o.data());
        if (k != (int64_t)ref.size())
            return fail("otu_finalize size", c);
        for (int64_t i = 0; i < k; i++)
            if (o[i].otu_index != ref[i].first || o[i].count != ref[i].second)
                return fail("otu_finalize order", c);

        /* 4. find_best_call: branches, ties, unknown / negative indices */
        static const char *names[] = {"zeta kinase", "alpha protein", "Beta", "alpha protein", "", "gyrase B",
                                      "gyrase A"};
        const long ncall = c % 11 == 0 ? uni(0, 60) : uni(0, 9);
        std::vector<kgx_call> calls(ncall), ws(ncall + 1);
        static const float wsets[3][4] = {{1.0f, 2.0f, 3.0f, 1.0f}, {0.1f, 0.7f, 1.3f, 2.9f}, {0.25f, 4.5f, 0.5f, 8.0f}};
        for (long i = 0; i < ncall; i++) {
            calls[i].start = (uint32_t)(10 * i);
            calls[i].end = (uint32_t)(10 * i + 7);
            calls[i].count = (int32_t)uni(1, 12);
            calls[i].function_index = (uint32_t)(int32_t)(c % 5 == 0 ? uni(-1, 8) : uni(0, 3));
            calls[i].weighted_hits = wsets[c % 3][uni(0, 3)] * (float)uni(1, 3);
        }
        const kgx_best_call d = kgx::best_call_decide(calls.data(), (uint32_t)ncall, ws.data());
        int32_t fi = 0;
        char fn[256];
        float out3[3] = {0, 0, -12345.0f};
        int off_set = 0;
        oracle_find_best_call(calls.data(), (uint64_t)ncall, names, 7, &fi, fn, sizeof(fn), out3, &off_set);
        auto name = [&](int i) { return std::string(i >= 0 && i < 7 ? names[i] : "INVALID_OFFSET"); };
        std::string dfn;
        if (d.kind == 1)
            dfn = name(d.fi0);
        else if (d.kind == 2) {
            std::string f1 = name(d.fi0), f2 = name(d.fi1);
            if (f2 > f1)
                std::swap(f1, f2);
            dfn = f1 + " ?? " + f2;
        }
        const int dfi = d.kind == 1 ? d.fi0 : -1;
        if (dfi != fi || dfn != fn || !same_f(d.score, out3[0]) || !same_f(d.weighted_score, out3[1]) ||
            (d.kind != 0) != (off_set != 0) || (off_set && !same_f(d.score_offset, out3[2])))
            return fail("best_call_decide", c);
    }
    std::printf("ok %ld\n", cases);
    return 0;
}
