"""The bench's per-device canary (close_kmers_amd/canary.py): the committed
expected digest is the CPU oracle's (tests/golden/make_canary.py), the
digest's plumbing maps device and oracle records to the same bytes, and (on
a GPU) the device pass reproduces it."""
import os
import sys

import numpy as np
import pytest

from close_kmers_amd import canary

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))


def test_committed_digest_is_the_oracles():
    import make_canary
    got = make_canary.compute()
    want = canary.expected()
    assert got["digest"] == want["digest"]
    assert got["hits"] == want["hits"] and got["calls"] == want["calls"] and want["calls"] > 100


def test_digest_plumbing():
    import oracle
    from close_kmers_amd import abi
    rng = np.random.default_rng(1)
    hits = np.zeros(5, abi.HIT_DTYPE)
    hits["which_kmer"] = rng.integers(0, 20 ** 8, 5, dtype=np.uint64)
    hits["function_wt"] = rng.random(5).astype(np.float32)
    ohits = np.zeros(5, oracle.HIT_DTYPE)
    for f in ("which_kmer", "function_wt"):
        ohits[f] = hits[f]
    calls = np.zeros(2, abi.CALL_DTYPE)
    calls["weighted_hits"] = [1.5, 2.25]
    ocalls = np.zeros(2, oracle.CALL_DTYPE)
    ocalls["weighted_hits"] = calls["weighted_hits"]
    # device kinds 0 (no calls), 1 (called), 2 (ambiguous), 3 (no call)
    dev = np.zeros(4, abi.BEST_DTYPE)
    dev["kind"] = [0, 1, 2, 3]
    dev["fi0"] = [-1, 17, 4, 9]
    dev["fi1"] = [-1, 3, 5, 2]
    dev["score"] = [0, 30, 12, 0]
    dev["weighted_score"] = [0, 41.5, 20.25, 0]
    dev["score_offset"] = [123.0, 30, 2, 1]  # kind 0: whatever the caller had
    orc = np.zeros(4, oracle.BEST_DTYPE)
    orc["function_index"] = [-1, 17, -1, -1]
    orc["score"] = dev["score"]
    orc["weighted_score"] = dev["weighted_score"]
    orc["score_offset"] = [0, 30, 2, 1]
    orc["offset_set"] = [0, 1, 1, 1]
    ho = np.array([0, 2, 5, 5, 5], np.uint64)
    co = np.array([0, 1, 1, 2, 2], np.uint64)
    d1 = canary.digest(ho, hits, co, calls, canary.best_from_device(dev))
    d2 = canary.digest(ho, ohits, co, ocalls, orc)
    assert d1 == d2
    hits["function_wt"][3] = np.nextafter(hits["function_wt"][3], np.float32(2))  # one ulp
    assert canary.digest(ho, hits, co, calls, canary.best_from_device(dev)) != d1


@pytest.mark.gpu
@pytest.mark.parametrize("line_index", [0, 36])
def test_canary_on_device(gpu, line_index):
    from close_kmers_amd import synth
    got = canary.run_on_device(gpu, synth, 0, line_index)
    want = canary.expected()
    assert got["digest"] == want["digest"], got
