"""Parity of the device k-mer -> id tables (kmer_to_id_ / kmer_to_family_id_)
and /matrix pair counting with the CPU oracle (oracle/handlers_oracle.cpp)."""
import numpy as np
import pytest

from close_kmers_amd import synth
from helpers import pack, synthetic_table

pytestmark = pytest.mark.gpu


def _lists_equal(dev_kmap, orc_kmap, kmers):
    off, ids = dev_kmap.lookup(kmers)
    for i, k in enumerate(kmers):
        got = ids[int(off[i]):int(off[i + 1])]
        want = orc_kmap.lookup(int(k))
        assert np.array_equal(got, want), (i, int(k), got[:10], want[:10])


@pytest.mark.parametrize("mode", [0, 1])
def test_kmap_add_matches_oracle(gpu, oracle_lib, mode):
    rng = np.random.default_rng(11 + mode)
    pool = rng.integers(0, 20 ** 8, 700, dtype=np.uint64)
    dev = gpu.Kmap(0, mode)
    orc = oracle_lib.Kmap(mode)
    with dev:
        for n in (3000, 1, 2500, 0, 4000):
            k = pool[rng.integers(0, len(pool), n)]
            v = rng.integers(0, 60, n).astype(np.uint32)
            dev.add(k, v)
            orc.add(k, v)
            assert dev.num_kmers == orc.num_kmers
        absent = rng.integers(0, 20 ** 8, 50, dtype=np.uint64)
        _lists_equal(dev, orc, np.concatenate([pool, absent]))
        if mode == 1:
            off, ids = dev.lookup(pool)
            for i in range(len(pool)):
                lst = ids[int(off[i]):int(off[i + 1])]
                assert len(set(lst.tolist())) == len(lst)


def _family_proteins(spec, rng, n_fam, per_fam, sub=0.06):
    """Members of n_fam families: image source proteins with substitutions."""
    src = synth.ALPHA[synth.source_residue_codes(np.arange(n_fam))].reshape(n_fam, -1)
    seqs = []
    for f in range(n_fam):
        for _ in range(per_fam):
            s = src[f].copy()
            m = rng.random(len(s)) < sub
            s[m] = synth.ALPHA[rng.integers(0, 20, int(m.sum()))]
            cut = int(rng.integers(200, len(s) + 1))
            seqs.append(bytes(s[:cut]))
    return seqs


@pytest.fixture(scope="module", params=["packed", "aos"])
def table_world(gpu, request):
    """Both resident layouts: their probes store different hit records
    (HIT_PACKED16 / HIT_PLANES), which the table kernels read."""
    spec, table = synthetic_table(60000)
    img = gpu.Image.from_table(table)
    if request.param == "aos":
        img.set_layout(gpu.Image.AOS24)
    assert img.layout == (gpu.Image.AOS24 if request.param == "aos" else gpu.Image.PACKED16)
    ctx = gpu.Context(img)
    yield spec, table, img, ctx
    ctx.close()
    img.close()


def _oracle_hit_kmers(oracle_lib, table, seqs):
    res, off = pack([("s", s) for s in seqs])
    r = oracle_lib.process_batch(table, res, off, want=1)
    return r.hit_offsets, r.hits["which_kmer"], res, off


@pytest.mark.parametrize("mode", [0, 1])
def test_kmap_add_hits_matches_oracle(table_world, gpu, oracle_lib, mode):
    spec, table, img, ctx = table_world
    rng = np.random.default_rng(5)
    seqs = _family_proteins(spec, rng, 12, 5)
    hoff, hk, res, off = _oracle_hit_kmers(oracle_lib, table, seqs)
    ids = rng.permutation(1000)[:len(seqs)].astype(np.uint32)
    orc = oracle_lib.Kmap(mode)
    with gpu.Kmap(0, mode) as dev:
        for lo, hi in ((0, 25), (25, len(seqs))):  # two /add requests
            ctx.process_batch(res[int(off[lo]):int(off[hi])], off[lo:hi + 1] - off[lo], want=1)
            dev.add_hits(ctx, ids[lo:hi])
            for s in range(lo, hi):
                k = hk[int(hoff[s]):int(hoff[s + 1])]
                orc.add(k, np.full(len(k), ids[s], np.uint32))
        assert dev.num_kmers == orc.num_kmers
        _lists_equal(dev, orc, np.unique(hk))


def test_matrix_matches_oracle(table_world, gpu, oracle_lib):
    spec, table, img, ctx = table_world
    rng = np.random.default_rng(9)
    seqs = _family_proteins(spec, rng, 10, 6)
    n = len(seqs)
    ids = (np.arange(n) * 7 + 3).astype(np.uint32)
    hoff, hk, res, off = _oracle_hit_kmers(oracle_lib, table, seqs)
    lens = np.diff(off).astype(np.uint64)
    orc_map = oracle_lib.Kmap(0)
    with gpu.Kmap(0, 0) as dev_map:
        # /add of the first 50 proteins
        ctx.process_batch(res[:int(off[50])], off[:51], want=1)
        dev_map.add_hits(ctx, ids[:50])
        for s in range(50):
            k = hk[int(hoff[s]):int(hoff[s + 1])]
            orc_map.add(k, np.full(len(k), ids[s], np.uint32))
        # /matrix over a shuffled request with repeated and never-added ids, two chunks
        order = rng.permutation(n)
        order = np.concatenate([order, order[:5]])
        req_ids = ids[order].copy()
        req_ids[3] = 999999  # an id /add never saw
        orc_mx = oracle_lib.Matrix()
        with gpu.Matrix(dev_map) as mx:
            for lo, hi in ((0, 31), (31, len(order))):
                sel = order[lo:hi]
                r2, o2 = pack([("s", seqs[i]) for i in sel])
                ctx.process_batch(r2, o2, want=1)
                mx.add_hits(ctx, req_ids[lo:hi])
                sub_off = np.concatenate([[0], np.cumsum([int(hoff[i + 1] - hoff[i]) for i in sel])])
                sub_k = np.concatenate([hk[int(hoff[i]):int(hoff[i + 1])] for i in sel])
                orc_mx.add(orc_map, req_ids[lo:hi], lens[sel], sub_off.astype(np.uint64), sub_k)
            got = mx.pairs()
        id1, id2, cnt, score = orc_mx.pairs()
        assert len(id1) > 100
        assert np.array_equal(got["id1"], id1)
        assert np.array_equal(got["id2"], id2)
        assert np.array_equal(got["count"], cnt)


def _on_hit_rollup(hit_kmers, orc_kmap, family):
    """LookupRequest::on_hit (lookup_request.cc:446-482) over one sequence's
    hits in position order: {id: [hit_count, hit_total, weighted_total]} in
    first-touch order (a dict keeps insertion order), f32 sums hit by hit."""
    d = {}
    for k in hit_kmers:
        lst = orc_kmap.lookup(int(k))
        if len(lst) == 0:
            continue
        w = np.float32(1.0) / np.float32(len(lst))
        for i in lst.tolist():
            e = d.setdefault(i, [0, 0, np.float32(0.0)])
            e[0] += 1
            if family:
                e[1] += 1
                e[2] = np.float32(e[2] + w)
    return d


@pytest.mark.parametrize("mode", [0, 1])
def test_kmap_rollup_matches_on_hit(table_world, gpu, oracle_lib, mode):
    """Device rollups (kgx_kmap_rollup) == on_hit replayed over the oracle's
    hits and lists: k-mers mapping to 1-9 ids out of a small pool (tied
    weighted totals), repeated ids in peg lists, unmapped hits, empty and
    hit-free sequences, ids with a high bit."""
    spec, table, img, ctx = table_world
    rng = np.random.default_rng(31 + mode)
    seqs = _family_proteins(spec, rng, 14, 4) + [b"", b"ACDEFGH", bytes(synth.ALPHA[rng.integers(0, 20, 400)])]
    order = rng.permutation(len(seqs))
    seqs = [seqs[i] for i in order]
    hoff, hk, res, off = _oracle_hit_kmers(oracle_lib, table, seqs)
    uk = np.unique(hk)
    mapped = uk[rng.random(len(uk)) < 0.8]
    pool = np.array([3, 7, 11, 12, 40, 41, 1000, 77777, (1 << 31) + 5], np.uint32)
    kms, ids = [], []
    for k in mapped:
        n = int(rng.integers(1, 10))
        sel = pool[rng.integers(0, len(pool), n)]
        kms.append(np.full(n, k, np.uint64))
        ids.append(sel)
    kms, ids = np.concatenate(kms), np.concatenate(ids)
    orc = oracle_lib.Kmap(1 if mode == 1 else 0)
    orc.add(kms, ids)
    family = mode == gpu.ROLLUP_FAMILY
    with gpu.Kmap(0, 1 if family else 0) as dev:
        dev.add(kms, ids)
        for want in (0, 1, 3):
            ctx.process_batch(res, off, want=want)
            roff, rows = dev.rollup(ctx, mode)
            assert len(roff) == len(seqs) + 1
            n_tied = 0
            for s in range(len(seqs)):
                exp = _on_hit_rollup(hk[int(hoff[s]):int(hoff[s + 1])], orc, family)
                got = rows[int(roff[s]):int(roff[s + 1])]
                assert got["id"].tolist() == list(exp.keys()), s
                assert got["hit_count"].tolist() == [v[0] for v in exp.values()], s
                assert got["hit_total"].tolist() == [v[1] for v in exp.values()], s
                wexp = np.array([v[2] for v in exp.values()], np.float32)
                assert np.array_equal(got["weighted_total"].view(np.uint32), wexp.view(np.uint32)), s
                n_tied += len(wexp) - len(np.unique(wexp))
            if family:
                assert n_tied > 0  # the pool makes equal weighted totals within a sequence
    # an empty mapping: every sequence without rows
    with gpu.Kmap(0, 1) as empty:
        roff, rows = empty.rollup(ctx, gpu.ROLLUP_FAMILY)
        assert len(rows) == 0 and not roff.any()


def test_kmap_rollup_many_ids_and_resizing(table_world, gpu, oracle_lib):
    """Sequences with hundreds to thousands of distinct ids (more than one LDS
    table pass holds: the id-class path) and a context whose batches grow and
    shrink between rollups (a rollup sized by the previous event count, then
    one too small for its batch, which runs again at the true size)."""
    spec, table, img, ctx = table_world
    rng = np.random.default_rng(77)
    fam = _family_proteins(spec, rng, 8, 2)
    long_seqs = [b"".join(fam[i:i + 4]) for i in range(0, 8, 4)]  # ~1,100-1,200 aa
    seqs = fam + long_seqs
    hoff, hk, res, off = _oracle_hit_kmers(oracle_lib, table, seqs)
    uk = np.unique(hk)
    kms, ids = [], []
    for k in uk:
        n = int(rng.integers(1, 10))
        kms.append(np.full(n, k, np.uint64))
        ids.append(rng.integers(0, 50000, n).astype(np.uint32))
    kms, ids = np.concatenate(kms), np.concatenate(ids)
    orc = oracle_lib.Kmap(1)
    orc.add(kms, ids)

    def check(lo, hi):
        sub_res = res[int(off[lo]):int(off[hi])]
        ctx.process_batch(sub_res, off[lo:hi + 1] - off[lo], want=0)
        roff, rows = dev.rollup(ctx, gpu.ROLLUP_FAMILY)
        most = 0
        for s in range(lo, hi):
            exp = _on_hit_rollup(hk[int(hoff[s]):int(hoff[s + 1])], orc, True)
            got = rows[int(roff[s - lo]):int(roff[s - lo + 1])]
            assert got["id"].tolist() == list(exp.keys()), s
            assert got["hit_count"].tolist() == [v[0] for v in exp.values()], s
            wexp = np.array([v[2] for v in exp.values()], np.float32)
            assert np.array_equal(got["weighted_total"].view(np.uint32), wexp.view(np.uint32)), s
            most = max(most, len(exp))
        return most

    with gpu.Kmap(0, 1) as dev:
        dev.add(kms, ids)
        assert check(0, 2) > 0              # small: the next rollup's size
        assert check(0, len(seqs)) > 400    # too small a size: run again; class path
        assert check(0, len(seqs)) > 400    # sized by the last count
        check(3, 5)                         # smaller again
