"""oracle.diff_batch -- the full-batch comparator bench.py's parity field and
the full-scale GPU tests use -- on CPU: the oracle's own results recast in
the device's record types compare equal, and a change to any one field of
one hit, call, OTU tally or best call is found in that sequence alone."""
import numpy as np
import pytest

from close_kmers_amd import synth


class _Got:
    pass


def _as_device(abi, r):
    """An oracle BatchResult in the device's record types (kgx_hit, kgx_otu,
    kgx_best_call), as abi.BatchResult holds them."""
    g = _Got()
    g.hit_offsets, g.call_offsets, g.otu_offsets = r.hit_offsets, r.call_offsets, r.otu_offsets
    g.hits = np.zeros(len(r.hits), abi.HIT_DTYPE)
    for f in ("which_kmer", "otu_index", "avg_from_end", "function_index", "function_wt", "pos", "seq"):
        g.hits[f] = r.hits[f]
    g.calls = r.calls.copy()
    g.otus = np.zeros(len(r.otus), abi.OTU_DTYPE)
    g.otus["otu_index"], g.otus["count"] = r.otus[:, 0], r.otus[:, 1]
    g.best = np.zeros(len(r.best), abi.BEST_DTYPE)
    for f in ("kind", "fi0", "fi1", "score", "weighted_score"):
        g.best[f] = r.best[f]
    g.best["score_offset"] = np.where(r.best["offset_set"] != 0, r.best["score_offset"], 0)
    # the device reports the top two functions behind a "no call" as well
    return g


@pytest.fixture(scope="module")
def batch(oracle_lib):
    spec = synth.ImageSpec(30000)
    k, f, o, a, w = spec.unique_entries()
    rng = np.random.default_rng(3)
    f = rng.integers(0, 6, len(k)).astype(np.int32)  # few functions: every best-call branch
    table = oracle_lib.build_table(spec.num_sigs, k, f, o, a, w)
    res, off = synth.make_queries(spec, 400, x_permille=5)
    return oracle_lib.process_batch(table, res, off, want=15, n_threads=4)


def test_diff_batch_equal_and_each_output(kgx, oracle_lib, batch):
    r = batch
    assert len(r.hits) > 10000 and len(r.calls) > 100
    assert set(np.unique(r.best["kind"])) >= {0, 1, 3}
    assert oracle_lib.diff_batch(_as_device(kgx, r), r, 15) == {"hits": [], "calls": [], "otus": [], "best": []}
    h = int(r.hit_offsets[58])  # first hit of sequence 58 (a planted one)
    assert h < r.hit_offsets[59]
    for field, delta in (("pos", 1), ("function_wt", 0.5), ("which_kmer", 1)):
        g = _as_device(kgx, r)
        g.hits[field][h] += delta
        assert oracle_lib.diff_batch(g, r, 15)["hits"] == [58], field
    s = int(np.nonzero(np.diff(r.call_offsets))[0][3])
    g = _as_device(kgx, r)
    g.calls["weighted_hits"][int(r.call_offsets[s])] = np.nextafter(
        g.calls["weighted_hits"][int(r.call_offsets[s])], np.float32(1e9))
    assert oracle_lib.diff_batch(g, r, 15)["calls"] == [s]
    s = int(np.nonzero(np.diff(r.otu_offsets))[0][2])
    g = _as_device(kgx, r)
    g.otus["count"][int(r.otu_offsets[s])] += 1
    assert oracle_lib.diff_batch(g, r, 15)["otus"] == [s]
    called = np.nonzero(r.best["kind"] == 1)[0]
    g = _as_device(kgx, r)
    g.best["fi0"][called[0]] += 1
    g.best["kind"][called[1]] = 3
    assert oracle_lib.diff_batch(g, r, 15)["best"] == sorted(called[:2].tolist())
    # a sequence with one hit too many: found by its count
    g = _as_device(kgx, r)
    g.hit_offsets = r.hit_offsets.copy()
    g.hit_offsets[59:] += 1
    g.hits = np.concatenate([g.hits[:h], g.hits[h:h + 1], g.hits[h:]])
    assert oracle_lib.diff_batch(g, r, 1)["hits"] == [58]
