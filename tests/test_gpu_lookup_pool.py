"""The /lookup handler's GPU side for a whole host batch over a pool
(kgx_pool_lookup: LookupRequest::process_work + on_hit,
lookup_request.cc:153-210,446-482) and caller-pinned residues (context
option "pinned_input": no staging copy, a device NUL scan, a staged rerun on
a NUL -- the strlen bound of kguts.cc:792).

Rows are checked against one context's pass + kgx_kmap_rollup, and a slice
against on_hit replayed over the oracle's hits (the same restatement
test_gpu_tables.py uses)."""
import numpy as np
import pytest

from close_kmers_amd import abi, synth
from helpers import synthetic_table
from test_gpu_tables import _on_hit_rollup

pytestmark = pytest.mark.gpu


def family_pairs(spec, n_fam, rng):
    """family i = the k-mers of source protein i; a fifth of the k-mers in a
    second family too (weights 1/2, ties)"""
    codes = synth.source_residue_codes(np.arange(n_fam))
    keys = synth.encode_windows(codes, synth.SRC_WIN).reshape(-1)
    ids = np.repeat(np.arange(n_fam, dtype=np.uint32), synth.SRC_WIN)
    extra = rng.random(len(keys)) < 0.2
    keys = np.concatenate([keys, keys[extra]])
    ids = np.concatenate([ids, (n_fam + rng.integers(0, 7, int(extra.sum()))).astype(np.uint32)])
    return keys, ids


@pytest.fixture(scope="module")
def world(gpu):
    spec, table = synthetic_table(60000)
    img = abi.Image.from_table(table, device=0)
    yield spec, table, img
    img.close()


def _rows_equal(a_off, a_rows, b_off, b_rows):
    assert np.array_equal(a_off, b_off)
    for f in ("id", "hit_count", "hit_total"):
        assert np.array_equal(a_rows[f], b_rows[f]), f
    assert np.array_equal(a_rows["weighted_total"].view(np.uint32), b_rows["weighted_total"].view(np.uint32))


@pytest.mark.parametrize("n_ctx,pinned", [(1, False), (3, False), (4, True)])
def test_pool_lookup_matches_one_context_and_on_hit(world, oracle_lib, n_ctx, pinned):
    spec, table, img = world
    rng = np.random.default_rng(41 + n_ctx)
    keys, ids = family_pairs(spec, spec.n_src, rng)
    res, off = synth.make_queries(spec, 3000, x_permille=3, q0=n_ctx)
    if pinned:
        pres = abi.pinned_empty(len(res))
        pres[:] = res
        res_in = pres
    else:
        res_in = res
    with abi.Kmap(0, abi.KMAP_SET) as fam, abi.Context(img) as ctx, abi.Pool([img], n_ctx) as pool:
        fam.add(keys, ids)
        got, roff, rows = pool.lookup([fam], res_in, off, want=abi.WANT_BEST | abi.WANT_CALLS)
        one = ctx.process_batch(res, off, want=abi.WANT_BEST | abi.WANT_CALLS)
        woff, wrows = fam.rollup(ctx, abi.ROLLUP_FAMILY)
        _rows_equal(roff, rows, woff, wrows)
        assert np.array_equal(got.hit_offsets, one.hit_offsets)
        assert np.array_equal(got.call_offsets, one.call_offsets)
        assert got.calls.tobytes() == one.calls.tobytes()
        assert got.best.tobytes() == one.best.tobytes()
        assert len(rows) > 1000
        # a slice against on_hit over the oracle's hits, byte for byte
        S = 300
        ref = oracle_lib.process_batch(table, res[:int(off[S])], off[:S + 1], want=1)
        orc = oracle_lib.Kmap(1)
        orc.add(keys, ids)
        hk = ref.hits["which_kmer"]
        for s in range(S):
            exp = _on_hit_rollup(hk[int(ref.hit_offsets[s]):int(ref.hit_offsets[s + 1])], orc, True)
            g = rows[int(roff[s]):int(roff[s + 1])]
            assert g["id"].tolist() == list(exp.keys()), s
            assert g["hit_count"].tolist() == [v[0] for v in exp.values()], s
            assert g["hit_total"].tolist() == [v[1] for v in exp.values()], s
            w = np.array([v[2] for v in exp.values()], np.float32)
            assert np.array_equal(g["weighted_total"].view(np.uint32), w.view(np.uint32)), s


def _compact_bytes(cb, res, off):
    r = cb.result
    return (r.hit_offsets.tobytes(), r.call_offsets.tobytes(), r.calls.tobytes(),
            r.best.tobytes() if r.best is not None else b"", cb.expand().tobytes())


def test_pinned_input_streamed_and_one_pass(world):
    """The streamed host path (>= 4M residues: chunks on two contexts) and the
    one-pass path read pinned residues by DMA, with results identical to the
    staged path; a NUL in the pinned buffer reruns staged, cut at the NUL."""
    spec, table, img = world
    res, off = synth.make_queries(spec, 16000, x_permille=2, q0=7)
    pres = abi.pinned_empty(len(res))
    pres[:] = res
    want = abi.WANT_HITS | abi.WANT_CALLS | abi.WANT_BEST
    with abi.Context(img) as ctx:
        base = _compact_bytes(ctx.process_batch_compact(res, off, want=want), res, off)
        p0 = ctx.stat("pinned_batches")
        assert p0 == 0
        got = _compact_bytes(ctx.process_batch_compact(pres, off, want=want), pres, off)
        assert ctx.stat("pinned_batches") == 1
        assert got == base
        # a NUL inside sequence 5000 (its windows past it vanish) and at a sequence's first byte
        for at in (int(off[5000]) + 100, int(off[9000])):
            res[at] = 0
            pres[at] = 0
        base = _compact_bytes(ctx.process_batch_compact(res, off, want=want), res, off)
        n0 = ctx.stat("nul_reruns")
        got = _compact_bytes(ctx.process_batch_compact(pres, off, want=want), pres, off)
        assert ctx.stat("nul_reruns") == n0 + 1
        assert got == base
        # one pass (host_chunks 1): the same
        ctx.set_option("host_chunks", 1)
        a = ctx.process_batch(res, off, want=want)
        b = ctx.process_batch(pres, off, want=want)
        assert ctx.stat("nul_reruns") == n0 + 2
        assert a.hits.tobytes() == b.hits.tobytes() and a.calls.tobytes() == b.calls.tobytes()
        assert a.best.tobytes() == b.best.tobytes()


def test_pool_lookup_tiny_growing_batches_and_pinned_nul(world):
    """Fewer sequences than shards (empty shards, uneven edge shares), batches
    that grow and shrink between calls on one pool (each context's rollup is
    sized by its previous event count: too small, then large enough), and a
    NUL in pinned input (that shard's pass and rollup run again, staged)."""
    spec, table, img = world
    rng = np.random.default_rng(77)
    keys, ids = family_pairs(spec, spec.n_src, rng)
    res_all, off_all = synth.make_queries(spec, 4000, x_permille=3, q0=11)
    want = abi.WANT_BEST | abi.WANT_CALLS
    with abi.Kmap(0, abi.KMAP_SET) as fam, abi.Context(img) as ctx, abi.Pool([img], 4) as pool:
        fam.add(keys, ids)

        def check(n, res=None):
            off = off_all[:n + 1] - off_all[0]
            base = res_all[:int(off[-1])] if res is None else res
            got, roff, rows = pool.lookup([fam], base, off, want=want)
            if n == 0:
                assert len(rows) == 0 and roff.tolist() == [0]
                return 0
            one = ctx.process_batch(res_all[:int(off[-1])] if res is None else np.array(base), off, want=want)
            woff, wrows = fam.rollup(ctx, abi.ROLLUP_FAMILY)
            _rows_equal(roff, rows, woff, wrows)
            assert np.array_equal(got.call_offsets, one.call_offsets)
            assert got.best.tobytes() == one.best.tobytes()
            return len(rows)

        for n in (0, 1, 3, 5, 2000, 40, 4000, 7):
            check(n)
        # a NUL in pinned residues: the staged rerun cuts that sequence there
        n = 3000
        pres = abi.pinned_empty(int(off_all[n] - off_all[0]))
        pres[:] = res_all[:len(pres)]
        pres[int(off_all[1500]) + 50] = 0
        check(n, pres)


@pytest.mark.parametrize("pinned", [False, True])
def test_ctx_lookup_one_wait_matches_pass_plus_rollup(world, pinned):
    """kgx_lookup (a server worker's /lookup piece: the pass and the rollup
    enqueued together, one host wait) == kgx_process_batch (one pass) +
    kgx_kmap_rollup, for batches growing and shrinking between calls (the
    rollup is sized by the previous one), family and peg mode, pinned or
    pageable residues."""
    spec, table, img = world
    rng = np.random.default_rng(77)
    keys, ids = family_pairs(spec, spec.n_src, rng)
    with abi.Kmap(0, abi.KMAP_SET) as fam, abi.Kmap(0, abi.KMAP_APPEND) as peg, \
            abi.Context(img) as ctx, abi.Context(img) as ref:
        fam.add(keys, ids)
        peg.add(keys, ids)
        ref.set_option("host_chunks", 1)
        for k, n in enumerate((2000, 30, 4000, 1, 700)):
            res, off = synth.make_queries(spec, n, x_permille=3, q0=100 * k)
            if pinned:
                pres = abi.pinned_empty(len(res))
                pres[:] = res
                res = pres
            for kmap, mode in ((fam, abi.ROLLUP_FAMILY), (peg, abi.ROLLUP_PEG)):
                got, g_off, g_rows = ctx.lookup(kmap, res, off, want=abi.WANT_BEST, mode=mode)
                one = ref.process_batch(np.array(res), off, want=abi.WANT_BEST)
                w_off, w_rows = kmap.rollup(ref, mode)
                _rows_equal(g_off, g_rows, w_off, w_rows)
                assert np.array_equal(got.best.view(np.uint8), one.best.view(np.uint8))
                assert len(got.hits) == 0
