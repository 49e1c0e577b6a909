"""CPU-side checks of the product library: it builds, loads, exports every
symbol include/kgx.h declares, and its host-only rules (parameter parsing,
find_best_call) agree with the oracle.  No device compute here."""
import json
import os

import numpy as np
import pytest

from helpers import GOLDEN


def test_library_exports_every_header_symbol(kgx):
    L = kgx.lib()
    declared = kgx.header_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    # and the ctypes table covers the whole header
    assert sorted(kgx.SIGNATURES) == declared


def test_device_count_without_gpu_is_safe(kgx):
    assert kgx.device_count() >= 0
    assert b"gfx950" in kgx.lib().kgx_version()


def test_compute_without_device_raises_not_falls_back(kgx):
    if kgx.device_count() > 0:
        pytest.skip("a device is present")
    with pytest.raises(kgx.KgxError) as e:
        kgx.Image.from_table(np.zeros(3769, dtype=kgx.SIG_DTYPE))
    assert e.value.code == -5  # KGX_EDEVICE


def test_params_parse_matches_set_parameters(kgx):
    p = kgx.default_params()
    assert (p.min_hits, p.max_gap, p.order_constraint, p.min_weighted_hits) == (5, 200, 0, 0)
    p = kgx.parse_params({"min_hits": "3", "max_gap": " 120xyz", "order_constraint": "1",
                          "min_weighted_hits": "-4", "other": "9"})
    assert (p.min_hits, p.max_gap, p.order_constraint, p.min_weighted_hits) == (3, 120, 1, -4)
    p = kgx.parse_params({"min_hits": "abc"})  # std::invalid_argument: warning, default kept
    assert p.min_hits == 5
    with pytest.raises(kgx.KgxError):
        kgx.parse_params({"max_gap": "99999999999999"})  # std::out_of_range escapes


def test_find_best_call_scoring_txt(kgx):
    ex = json.load(open(os.path.join(GOLDEN, "scoring_example.json")))
    calls = np.array([(s, e, c, f, np.float32(w)) for s, e, c, f, _, w in ex["calls"]],
                     dtype=kgx.CALL_DTYPE)
    names = ["function %d" % i for i in range(7600)]
    for k, v in ex["functions"].items():
        names[int(k)] = v
    fi, fn, score, wscore, off = kgx.find_best_call(calls, names)
    b = ex["best"]
    assert (fi, fn, score, f"{wscore:g}", off) == (b["function_index"], b["function"], b["score"],
                                                  b["weighted"], b["offset"])


def test_find_best_call_random_vs_oracle(kgx, oracle_lib):
    rng = np.random.default_rng(5)
    names = ["Zeta", "alpha", "Beta", "beta", "gamma ?? x", "", "hypothetical protein", "f7"]
    for trial in range(3000):
        n = int(rng.integers(0, 9))
        calls = np.zeros(n, dtype=kgx.CALL_DTYPE)
        calls["start"] = np.sort(rng.integers(0, 300, n))
        calls["end"] = calls["start"] + rng.integers(7, 60, n)
        calls["count"] = rng.integers(1, 16, n)
        calls["function_index"] = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 11, 4294967295], n)
        # ties in weighted totals are common with small integers
        calls["weighted_hits"] = (rng.integers(1, 12, n) * 0.5 if trial % 2 else
                                  rng.random(n) * 20).astype(np.float32)
        got = kgx.find_best_call(calls, names)
        want = oracle_lib.find_best_call(calls, names)
        assert got[:2] == want[:2] and np.float32(got[2]) == np.float32(want[2]) and \
            np.float32(got[3]) == np.float32(want[3]) and \
            (got[4] is None) == (want[4] is None) and (got[4] is None or np.float32(got[4]) == np.float32(want[4])), \
            (trial, calls, got, want)


def test_shard_cuts_match_balanced_shards(kgx):
    """kgx_shard_cuts (the pool's split, C ABI) == shard.balanced_shards (the
    bench's split): contiguous, residue-balanced, whole sequences."""
    from close_kmers_amd import shard
    rng = np.random.default_rng(11)
    for trial in range(300):
        n = int(rng.integers(0, 60))
        lens = rng.integers(0, 400, n) if trial % 3 else np.full(n, 300)
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum(lens)
        off += np.uint64(rng.integers(0, 50))  # absolute offsets need not start at 0
        for k in (1, 2, 3, 8, 13):
            cuts = kgx.shard_cuts(off, k)
            want = shard.balanced_shards(off, k)
            assert [(int(cuts[i]), int(cuts[i + 1])) for i in range(k)] == want, (trial, k)
    with pytest.raises(kgx.KgxError):
        kgx.shard_cuts(np.zeros(1, np.uint64), 0)


def test_synthetic_stream_cut_for_distinct_keys():
    """synth.ImageSpec's n_entries / entries_for_distinct (host side of
    kgx_image_build_synthetic_distinct): the cut holds exactly the asked
    number of distinct keys and one entry less holds one key fewer."""
    from close_kmers_amd import synth
    spec = synth.ImageSpec(5000, 101533)
    for nd in (4000, 5000, 6500):
        m = spec.entries_for_distinct(nd)
        assert len(synth.ImageSpec(5000, 101533, n_entries=m).unique_entries()[0]) == nd
        assert len(synth.ImageSpec(5000, 101533, n_entries=m - 1).unique_entries()[0]) == nd - 1


def test_pool_map_select_more_than_one_map(kgx):
    """kgx_pool_lookup's map per context (kgx_pool.cpp): with several maps,
    each running context takes the first map on its own device, whatever the
    maps' order; missing maps (-1) are skipped; a device with no map fails."""
    ctx = [0, 0, 1, 1, 2, 2, 3, 3]
    assert kgx.pool_map_select(ctx, [3, 2, 1, 0]).tolist() == [3, 3, 2, 2, 1, 1, 0, 0]
    assert kgx.pool_map_select(ctx, [0, 1, 2, 3]).tolist() == [0, 0, 1, 1, 2, 2, 3, 3]
    # duplicates: the first one on the device wins; unrelated devices are ignored
    assert kgx.pool_map_select([1, 0], [5, 1, -1, 0, 1, 0]).tolist() == [1, 3]
    assert kgx.pool_map_select([], [0]).tolist() == []
    with pytest.raises(kgx.KgxError) as e:
        kgx.pool_map_select([0, 4], [0, 1, 2, 3])
    assert e.value.code == -1 and "device 4" in kgx.last_error()


def test_numa_node_cpus(kgx):
    """kgx_numa_node_cpus (the pool threads' NUMA binding, numa.cc:13-42):
    a node's CPUs are the node's cpulist within this process's affinity."""
    aff = os.sched_getaffinity(0)
    assert kgx.numa_node_cpus(-1) == [] and kgx.numa_node_cpus(100000) == []
    base = "/sys/devices/system/node"
    nodes = sorted(int(d[4:]) for d in os.listdir(base) if d.startswith("node") and d[4:].isdigit()) \
        if os.path.isdir(base) else []
    seen = set()
    for nd in nodes:
        cpus = kgx.numa_node_cpus(nd)
        text = open(f"{base}/node{nd}/cpulist").read().strip()
        listed = set()
        for part in filter(None, text.split(",")):
            a, _, b = part.partition("-")
            listed.update(range(int(a), int(b or a) + 1))
        assert set(cpus) == listed & aff, nd
        assert not (set(cpus) & seen)
        seen.update(cpus)
    if nodes:
        assert seen == aff & set().union(*[set(kgx.numa_node_cpus(nd)) for nd in nodes])


def test_host_wait_modes(kgx):
    """kgx_set_host_wait: the three modes round-trip (poll 0 = 20 us, capped at
    0.1 s), anything else is KGX_EINVAL and leaves the mode alone."""
    import ctypes
    L = kgx.lib()
    us = ctypes.c_uint32()
    mode0 = L.kgx_get_host_wait(ctypes.byref(us))
    us0 = us.value
    try:
        for mode, poll, want in ((kgx.KGX_WAIT_SLEEP, 0, 20), (kgx.KGX_WAIT_SLEEP, 7, 7),
                                 (kgx.KGX_WAIT_SLEEP, 10**6, 100000), (kgx.KGX_WAIT_BLOCK, 5, 5),
                                 (kgx.KGX_WAIT_SPIN, 20, 20)):
            assert L.kgx_set_host_wait(mode, poll) == 0
            assert L.kgx_get_host_wait(ctypes.byref(us)) == mode and us.value == want
        assert L.kgx_set_host_wait(3, 1) == kgx.KGX_EINVAL
        assert L.kgx_get_host_wait(None) == kgx.KGX_WAIT_SPIN
    finally:
        L.kgx_set_host_wait(mode0, us0)


def test_format_g6_matches_printf(kgx):
    """kgx_format_g6 -- how the handlers print floats (operator<< at the
    default precision = printf's %.6g of the value widened to double), with
    its fast paths for integral values below 1e6 and for 1e-4 <= |v| < 1e6 --
    against Python's %-format (C printf semantics) on edge values, ties at
    the sixth digit and 520k random floats."""
    import ctypes
    rng = np.random.default_rng(6)
    vals = [0.0, -0.0, 1.0, -1.0, 999999.0, -999999.0, 1e6, -1e6, 1234567.0, 0.5, 1e-5, 123456.5,
            3.4028235e38, 1.17549435e-38, 1e-45, float("inf"), float("-inf"), 2.0 ** 24, 16777217.0]
    vals += rng.integers(-2_000_000, 2_000_000, 100_000).astype(np.float32).tolist()
    vals += (rng.standard_normal(100_000) * 10.0 ** rng.integers(-8, 9, 100_000)).astype(np.float32).tolist()
    vals += rng.integers(0, 300, 100_000).astype(np.float32).tolist()
    # exact decimal ties at the sixth digit (ties to even) and their neighbours,
    # across the fast path's decades, and values that round up to a power of ten
    ints = rng.integers(100_000, 1_000_000, 20_000)
    for scale in (1.0, 2.0, 4.0, 8.0, 16.0, 0.5):
        vals += ((ints + 0.5) / scale).astype(np.float32).tolist()
    for p in range(-4, 6):
        for x in (9.999995, 9.999994, 9.999996, 1.0000005, 9.9999995):
            vals += [x * 10.0 ** p, -x * 10.0 ** p]
    vals += (rng.random(100_000) * 10.0 ** rng.integers(-5, 7, 100_000)).astype(np.float32).tolist()
    buf = ctypes.create_string_buffer(64)
    L = kgx.lib()
    for v in vals:
        f = float(np.float32(v))
        n = L.kgx_format_g6(f, buf, len(buf))
        want = "%.6g" % f
        assert buf.value.decode() == want and n == len(want), (v, buf.value, want)
