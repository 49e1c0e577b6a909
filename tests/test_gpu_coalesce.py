"""The unchanged-handler drop-in under the reference's pool shape: T worker
threads with one KmerGuts each over one shared image (threadpool.cc:18-44),
each calling process_aa_seq once per sequence (lookup_request.cc:153-172).
Concurrent calls are coalesced into shared GPU passes (SeqCoalescer,
csrc/kguts_hip.h); every thread must still get exactly its own sequences'
hit callbacks (position order), calls and OTU stats -- compared with the
oracle per sequence under that thread's parameters (tests/native/
coalesce_check.cpp)."""
import json
import os
import subprocess

import numpy as np
import pytest

from close_kmers_amd import build as kbuild
from close_kmers_amd import image_files, synth
from close_kmers_amd.abi import CALL_DTYPE, HIT_DTYPE
from helpers import random_protein, synthetic_table

pytestmark = pytest.mark.gpu

PARAMS = [(5, 200, 0, 0), (3, 50, 0, 0), (5, 200, 1, 0)]  # coalesce_check.cpp: thread t uses t % 3


def _queries(spec, n, seed):
    """C2-like queries mixed with ragged ones: empty, < 9 aa, X / * / lower
    case, a few long ones."""
    rng = np.random.default_rng(seed)
    res, off = synth.make_queries(spec, n, x_permille=3, q0=seed)
    seqs = [bytes(res[int(off[i]):int(off[i + 1])]) for i in range(n)]
    for i in rng.choice(n, n // 20, replace=False):
        seqs[i] = seqs[i][:int(rng.integers(0, 12))]
    for i in rng.choice(n, 4, replace=False):
        seqs[i] = random_protein(rng, 3000).encode() + seqs[i]
    for i in rng.choice(n, n // 50, replace=False):
        s = bytearray(seqs[i])
        if s:
            s[int(rng.integers(0, len(s)))] = ord(rng.choice(list("X*bz")))
        seqs[i] = bytes(s)
    o = np.zeros(n + 1, np.uint64)
    o[1:] = np.cumsum([len(s) for s in seqs])
    return np.frombuffer(b"".join(seqs), np.uint8).copy(), o


def _parse(path, n):
    data = open(path, "rb").read()
    p, out = 0, []
    for _ in range(n):
        k = int(np.frombuffer(data, np.uint32, 1, p)[0])
        p += 4
        hits = np.frombuffer(data, HIT_DTYPE, k, p).copy()
        p += 32 * k
        k = int(np.frombuffer(data, np.uint32, 1, p)[0])
        p += 4
        calls = np.frombuffer(data, CALL_DTYPE, k, p).copy()
        p += 20 * k
        k = int(np.frombuffer(data, np.uint32, 1, p)[0])
        p += 4
        otus = np.frombuffer(data, np.int32, 2 * k, p).reshape(-1, 2).copy()
        p += 8 * k
        out.append((hits, calls, otus))
    assert p == len(data)
    return out


@pytest.mark.parametrize("threads,coalesce,otu,svc,slots", [(16, 1, 1, 1, 0), (5, 1, 1, 1, 0), (1, 1, 1, 1, 0),
                                                            (16, 0, 1, 1, 0), (16, 1, 0, 1, 0), (16, 1, 0, 0, 0),
                                                            (32, 1, 0, 1, 0), (16, 1, 0, 1, 3), (1, 0, 0, 1, 0)])
def test_threads_calling_process_aa_seq_match_oracle(gpu, oracle_lib, tmp_path, threads, coalesce, otu, svc, slots):
    """otu 1: hit callbacks, calls and OTU stats (the query handler's
    outputs), otu 0: hits + calls (the lookup handler's): with the resident
    call service (svc 1, csrc/kgx_svc.cpp) calls under order_constraint 0 of
    at most 2,056 residues run there, the rest through the coalescer; svc 0 (KGX_SVC=0): the coalescer's one-launch path
    (kgx_fused.hip).  slots 3: most calls find every slot taken (KGX_EBUSY)
    and take the coalescer."""
    spec, table = synthetic_table(30000)
    d = image_files.write_data_dir(str(tmp_path), table, [f"function {i}" for i in range(100000)])
    n = 3000
    res, off = _queries(spec, n, 40 + threads)
    q = tmp_path / "queries.bin"
    q.write_bytes(np.uint64(n).tobytes() + off.tobytes() + res.tobytes())
    outp = tmp_path / "out.bin"
    env = dict(os.environ, KGX_SVC=str(svc))
    r = subprocess.run([kbuild.COALESCE_CHECK, d, str(q), str(threads), str(outp), str(coalesce), str(otu),
                        str(slots)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    stats = json.loads(r.stdout)
    assert stats["calls"] + stats["svc_calls"] == (n if coalesce else 0)
    if coalesce and svc:
        # thread parameter sets 0 and 1, ordinary lengths (3 slots: some)
        assert stats["svc_calls"] > (n // 2 if not slots else 0)
    else:
        assert stats["svc_calls"] == 0
    if coalesce and threads >= 5 and not (svc and not slots):
        assert stats["passes"] < n  # calls did share passes
    got = _parse(outp, n)
    # every sequence against the oracle under its thread's parameter set
    for ps in range(3):
        idx = [i for i in range(n) if (i % threads) % 3 == ps]
        if not idx:
            continue
        sres = np.concatenate([res[int(off[i]):int(off[i + 1])] for i in idx])
        soff = np.zeros(len(idx) + 1, np.uint64)
        soff[1:] = np.cumsum([int(off[i + 1] - off[i]) for i in idx])
        want = oracle_lib.process_batch(table, sres, soff, params=PARAMS[ps], want=7)
        for j, i in enumerate(idx):
            gh, gc, go = got[i]
            h0, h1 = int(want.hit_offsets[j]), int(want.hit_offsets[j + 1])
            wh = want.hits[h0:h1]
            assert len(gh) == len(wh), i
            for f in ("which_kmer", "otu_index", "avg_from_end", "function_index", "pos"):
                assert np.array_equal(gh[f], wh[f]), (i, f)
            assert np.array_equal(gh["function_wt"].view(np.uint32), wh["function_wt"].view(np.uint32)), i
            c0, c1 = int(want.call_offsets[j]), int(want.call_offsets[j + 1])
            wc = want.calls[c0:c1]
            for f in ("start", "end", "count", "function_index"):
                assert np.array_equal(gc[f], wc[f]), (i, f)
            assert np.array_equal(gc["weighted_hits"].view(np.uint32), wc["weighted_hits"].view(np.uint32)), i
            o0, o1 = int(want.otu_offsets[j]), int(want.otu_offsets[j + 1])
            assert np.array_equal(go, want.otus[o0:o1] if otu else want.otus[:0]), i
