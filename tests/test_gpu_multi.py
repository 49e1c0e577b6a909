"""Multi-GPU drop-in on one device: image replicas (one file read fanned out,
device-to-device copies) and a pool that splits one batch into residue-
balanced shards over several contexts.  The split must be invisible: the
concatenated result is byte-identical to one context processing the whole
batch (north_star: query batches split across the GPUs of a node, results
bit-exact).  On a 1-GPU box every replica and context sits on device 0,
which exercises the same code the 8-GPU node runs."""
import ctypes
import os

import numpy as np
import pytest

from close_kmers_amd import image_files, synth
from helpers import pack, synthetic_table

pytestmark = pytest.mark.gpu

ALL = 1 | 2 | 4 | 8  # hits + calls + OTU + best call


def _bytes_equal(a, b):
    for k in ("hit_offsets", "call_offsets", "otu_offsets"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    for k in ("hits", "calls", "otus"):
        assert np.array_equal(getattr(a, k).view(np.uint8), getattr(b, k).view(np.uint8)), k
    assert (a.best is None) == (b.best is None)
    if a.best is not None:
        assert np.array_equal(a.best.view(np.uint8), b.best.view(np.uint8))
    assert a.n_windows == b.n_windows


@pytest.fixture(scope="module")
def world(gpu):
    spec, table = synthetic_table(30000)
    img = gpu.Image.from_table(table)
    yield spec, table, img
    img.close()


def _mixed_batch(spec, n, seed):
    rng = np.random.default_rng(seed)
    res, off = synth.make_queries(spec, n, x_permille=5, q0=seed)
    lens = rng.integers(0, 300, n)
    if n >= 10:
        lens[rng.integers(0, n, n // 10)] = 0  # empty sequences between shards
    return pack([("q", bytes(res[int(off[i]):int(off[i]) + int(lens[i])])) for i in range(n)])


@pytest.mark.parametrize("n_ctx,n_seq", [(8, 2000), (3, 1001), (8, 5), (2, 1), (4, 0)])
def test_pool_split_is_byte_identical_to_one_pass(world, gpu, oracle_lib, n_ctx, n_seq, monkeypatch):
    """n_ctx shards, one per context: on a node each replica is on its own
    device; here every replica is on device 0, so the pool's per-device shard
    limit (KGX_POOL_PER_DEVICE, default 2) is raised to keep n_ctx shards"""
    monkeypatch.setenv("KGX_POOL_PER_DEVICE", str(n_ctx))
    spec, table, img = world
    res, off = _mixed_batch(spec, n_seq, n_ctx * 100 + n_seq)
    with gpu.Context(img) as ctx:
        one = ctx.process_batch(res, off, want=ALL)
    # one replica per context, as on a node (device-to-device copies)
    reps = [img.replicate(0) for _ in range(n_ctx)]
    try:
        with gpu.Pool(reps) as pool:
            assert pool.size == n_ctx
            got = pool.process_batch(res, off, want=ALL)
            _bytes_equal(got, one)
            again = pool.process_batch(res, off, want=ALL)  # reused pool buffers
            _bytes_equal(again, one)
    finally:
        for r in reps:
            r.close()
    if n_seq:
        want = oracle_lib.process_batch(table, res, off)
        assert np.array_equal(one.hit_offsets, want.hit_offsets)
        assert np.array_equal(one.hits["seq"], want.hits["seq"])


def test_pool_shards_run_chunked_contexts(world, gpu):
    """Shards large enough for the host-chunked path (twin contexts) inside
    every pool context; more contexts than images."""
    spec, table, img = world
    res, off = synth.make_queries(spec, 40000, x_permille=5, q0=7)
    with gpu.Context(img) as ctx:
        one = ctx.process_batch(res, off, want=ALL)
    with gpu.Pool([img], n_ctx=3) as pool:
        pool.set_option("host_chunks", 4)
        got = pool.process_batch(res, off, want=ALL)
        _bytes_equal(got, one)
        got = pool.process_batch(res, off, want=1 | 2)
        nof = one.hits.copy()
        nof["flags"] = 0  # hit flags are written only with KGX_WANT_OTU
        assert np.array_equal(got.hits.view(np.uint8), nof.view(np.uint8))


def test_open_replicas_reads_once(world, gpu, oracle_lib, tmp_path):
    spec, table, _ = world
    d = image_files.write_data_dir(str(tmp_path), table, [f"function {i}" for i in range(100000)])
    reps = gpu.Image.open_replicas(d, [0, 0, 0])
    try:
        assert len(reps) == 3 and all(r.device == 0 for r in reps)
        res, off = synth.make_queries(spec, 300, x_permille=5)
        want = oracle_lib.process_batch(table, res, off)
        outs = []
        for r in reps:
            assert r.layout == gpu.Image.PACKED16
            with gpu.Context(r) as ctx:
                outs.append(ctx.process_batch(res, off, want=7))
        for o in outs:
            _bytes_equal(o, outs[0])
        assert np.array_equal(outs[0].hit_offsets, want.hit_offsets)
        assert np.array_equal(outs[0].calls["count"], want.calls["count"])
    finally:
        for r in reps:
            r.close()
    with pytest.raises(gpu.KgxError):
        gpu.Image.open_replicas(str(tmp_path / "missing"), [0, 0])
    with pytest.raises(gpu.KgxError):
        gpu.Image.open_replicas(d, [0, 99])  # no such device: nothing is left open


def test_replicate_keeps_layout_and_filter(world, gpu):
    spec, table, _ = world
    res, off = synth.make_queries(spec, 500, x_permille=5, q0=3)
    with gpu.Image.from_table(table) as aos:
        aos.set_layout(gpu.Image.AOS24)
        with aos.replicate(0) as rep, gpu.Context(aos) as c1, gpu.Context(rep) as c2:
            assert rep.layout == gpu.Image.AOS24
            assert np.array_equal(rep.download().view(np.uint8), table.view(np.uint8))
            _bytes_equal(c1.process_batch(res, off, want=ALL), c2.process_batch(res, off, want=ALL))
    with gpu.Image.from_table(table) as packed:
        packed.set_filter(16)
        with packed.replicate(0) as rep, gpu.Context(packed) as c1, gpu.Context(rep) as c2:
            assert rep.layout == gpu.Image.PACKED16
            _bytes_equal(c1.process_batch(res, off, want=ALL), c2.process_batch(res, off, want=ALL))


def test_bad_device_offsets_are_an_error_not_a_fault(world, gpu):
    """kgx_run_device checks its offsets on the device: a batch
    with decreasing offsets, or spanning more than n_residues, runs as empty
    and is reported; the next good batch on the context is unaffected."""
    spec, table, img = world
    L = gpu.lib()
    n, Ls = 64, 300
    res, off = synth.make_queries(spec, n, x_permille=0)
    d_res, d_off = ctypes.c_void_p(), ctypes.c_void_p()
    gpu.check(L.kgx_device_alloc(0, n * Ls, ctypes.byref(d_res)), "alloc")
    gpu.check(L.kgx_device_alloc(0, (n + 1) * 8, ctypes.byref(d_off)), "alloc")
    params = gpu.default_params()
    try:
        gpu.check(L.kgx_memcpy_h2d(d_res, res.ctypes.data, res.nbytes), "h2d")
        with gpu.Context(img) as ctx:
            def run(o, n_res):
                o = np.ascontiguousarray(o, np.uint64)
                gpu.check(L.kgx_memcpy_h2d(d_off, o.ctypes.data, o.nbytes), "h2d")
                gpu.check(L.kgx_run_device(ctx.handle, ctypes.byref(params), d_res, d_off, n, n_res, 3, None),
                          "run_device")

            good = ctx.process_batch(res, off, want=3)
            bad = off.copy()
            bad[10] = bad[40]  # sequence 10 would end before it starts: not monotone
            run(bad, n * Ls)
            with pytest.raises(gpu.KgxError) as e:
                ctx.check_plan()
            assert e.value.code == -1
            r = gpu.Result()
            assert L.kgx_device_batch_collect(ctx.handle, 3, ctypes.byref(r)) == -1
            run(off, n * Ls - 1)  # one residue more than claimed
            with pytest.raises(gpu.KgxError):
                ctx.check_plan()
            huge = off.copy()
            huge[5:] += np.uint64(1 << 40)  # a wild offset: must not be dereferenced
            run(huge, n * Ls)
            with pytest.raises(gpu.KgxError):
                ctx.check_plan()
            run(off, n * Ls)  # a good batch afterwards
            ctx.check_plan()
            gpu.check(L.kgx_device_batch_collect(ctx.handle, 3, ctypes.byref(r)), "collect")
            b = gpu.BatchResult(r, 3)
            assert np.array_equal(b.hits.view(np.uint8), good.hits.view(np.uint8))
    finally:
        L.kgx_device_free(d_res)
        L.kgx_device_free(d_off)


def _compact_equals(cb, one, res, off):
    """A compact result carries the same offsets / calls / OTUs / best calls,
    and its hits expand to the same kgx_hit bytes, as a whole range, per
    sequence and with a seq_base."""
    for k in ("hit_offsets", "call_offsets", "otu_offsets"):
        assert np.array_equal(getattr(cb.result, k), getattr(one, k)), k
    for k in ("calls", "otus"):
        assert np.array_equal(getattr(cb.result, k).view(np.uint8), getattr(one, k).view(np.uint8)), k
    if one.best is not None:
        assert np.array_equal(cb.result.best.view(np.uint8), one.best.view(np.uint8))
    assert cb.result.n_windows == one.n_windows
    assert np.array_equal(cb.expand().view(np.uint8), one.hits.view(np.uint8))
    n = len(off) - 1
    if n:
        rng = np.random.default_rng(n)
        for _ in range(20):
            a = int(rng.integers(0, n))
            b = int(rng.integers(a, n + 1))
            got = cb.expand(a, b, seq_base=1000)
            want = one.hits[int(one.hit_offsets[a]):int(one.hit_offsets[b])].copy()
            want["seq"] += 1000
            assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


@pytest.mark.parametrize("n_ctx,n_seq", [(8, 2000), (3, 80000), (8, 5), (4, 0)])
def test_pool_compact_result_expands_to_one_pass(world, gpu, n_ctx, n_seq):
    """kgx_pool_process_batch_compact: every shard's chunks renumbered into
    the batch, no hit record copied; expanding them gives one pass's bytes."""
    spec, table, img = world
    res, off = _mixed_batch(spec, n_seq, 7 * n_ctx + n_seq) if n_seq != 80000 else \
        synth.make_queries(spec, n_seq, x_permille=5, q0=11)
    with gpu.Context(img) as ctx:
        one = ctx.process_batch(res, off, want=ALL)
    with gpu.Pool([img], n_ctx=n_ctx) as pool:
        pool.set_option("host_chunks", 3)
        for _ in range(2):
            cb = pool.process_batch_compact(res, off, want=ALL)
            _compact_equals(cb, one, res, off)
        if n_seq == 80000:
            assert cb.n_chunks >= n_ctx and not cb.materialized
            seqs = [(c.seq_begin, c.seq_end) for c in cb.chunks]
            assert seqs == sorted(seqs) and all(a[1] <= b[0] for a, b in zip(seqs, seqs[1:]))
        got = pool.process_batch(res, off, want=ALL)  # expanded once into the concatenation
        _bytes_equal(got, one)
