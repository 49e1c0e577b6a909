"""BASELINE.json's configs at their full sizes, on the GPU, against the oracle.

  C1  1k x 300 aa vs a 10M-entry image (32,000,011 buckets, the builder's
      sizing rule build_signature_kmers.cc:862-883): every hit, call, OTU
      tally and best call of the batch against the oracle, and the same
      results through the file format (kgx_image_save -> kgx_image_open).
  C3  /matrix over 10,000 proteins after /add of all of them, against the
      1B-entry image: the device pair list (matrix_request.cc:83-190) equals
      the oracle's std::map of pair counts.
  C4  10M x 150 bp FASTQ reads (uniform ACGT, seed 0x5EED0004) against the
      1B-entry image: fragments, hits and calls of every 1000th read against
      the oracle (dna_seq.cc:9-47, fq_process_request.cc:298-365), and the
      sampled reads re-run as their own batch and through the host-buffer
      path give the same bytes (a read's results do not depend on its batch).
C2 (and C5's split) is tests/test_gpu_full_scale.py."""
import ctypes

import numpy as np
import pytest

from close_kmers_amd import synth

pytestmark = pytest.mark.gpu

HIT_FIELDS = ("which_kmer", "otu_index", "avg_from_end", "function_index", "pos", "seq")


def _hits_equal(got, want):
    for f in HIT_FIELDS:
        assert np.array_equal(got[f], want[f]), f
    assert np.array_equal(got["function_wt"].view(np.uint32), want["function_wt"].view(np.uint32))


def _calls_equal(got, want):
    for f in ("start", "end", "count", "function_index"):
        assert np.array_equal(got[f], want[f]), f
    assert np.array_equal(got["weighted_hits"].view(np.uint32), want["weighted_hits"].view(np.uint32))


def test_c1_full_config(gpu, oracle_lib, tmp_path):
    spec = synth.ImageSpec(10 ** 7)
    assert spec.num_sigs == 32000011
    img, m = gpu.Image.synthetic_distinct(spec.n_keys, 10 ** 7, spec.num_sigs)
    try:
        table = img.download()
        assert int((table["which_kmer"] <= 20 ** 8).sum()) == 10 ** 7
        res, off = synth.make_queries(spec, 1000, 300, x_permille=5)
        want = oracle_lib.process_batch(table, res, off, want=7)
        assert len(want.hits) > 50000 and len(want.calls) >= 450
        assert 1.4 < want.probes / want.windows < 1.8  # alpha = 0.3125
        with gpu.Context(img) as ctx:
            got = ctx.process_batch(res, off, want=15)
        assert np.array_equal(got.hit_offsets, want.hit_offsets)
        _hits_equal(got.hits, want.hits)
        assert np.array_equal(got.call_offsets, want.call_offsets)
        _calls_equal(got.calls, want.calls)
        assert np.array_equal(got.otu_offsets, want.otu_offsets)
        assert np.array_equal(got.otus["otu_index"], want.otus[:, 0])
        # find_best_call of every sequence on the device == the oracle's rule
        names = [f"function {i}" for i in range(100000)]
        for s in range(0, 1000, 7):
            c = want.calls[int(want.call_offsets[s]):int(want.call_offsets[s + 1])]
            fi, fn, score, wscore, offset = oracle_lib.find_best_call(c, names)
            b = got.best[s]
            if len(c) == 0:
                assert b["kind"] == 0
                continue
            assert np.float32(b["score"]) == np.float32(score)
            assert np.float32(b["weighted_score"]) == np.float32(wscore)
            assert (b["fi0"] if b["kind"] == 1 else -1) == fi
        # the file format round trip: save, then load as KmerImage does
        d = str(tmp_path)
        img.save(d)
        with gpu.Image.open(d) as img2, gpu.Context(img2) as ctx2:
            again = ctx2.process_batch(res, off, want=15)
        for k in ("hits", "calls", "otus", "best"):
            assert np.array_equal(getattr(again, k).view(np.uint8), getattr(got, k).view(np.uint8)), k
    finally:
        img.close()


@pytest.fixture(scope="module")
def c2_image(gpu):
    """The 1B-entry image (1e9 distinct keys, alpha = 0.281) and a host copy."""
    spec = synth.ImageSpec(10 ** 9)
    img, m = gpu.Image.synthetic_distinct(spec.n_keys, 10 ** 9, spec.num_sigs)
    state = {"table": None}

    def table():
        if state["table"] is None:
            state["table"] = img.download()
        return state["table"]

    yield spec, img, table
    state["table"] = None
    img.close()


def _family_proteins(n_prot, fam_size, rng):
    n_fam = n_prot // fam_size
    src = synth.ALPHA[synth.source_residue_codes(np.arange(n_fam))].reshape(n_fam, -1)
    res = np.repeat(src, fam_size, axis=0)
    sub = rng.random(res.shape) < 0.10
    res[sub] = synth.ALPHA[rng.integers(0, 20, int(sub.sum()))]
    off = np.arange(0, res.size + 1, res.shape[1], dtype=np.uint64)
    return res.reshape(-1).copy(), off


def test_c3_full_matrix(c2_image, gpu, oracle_lib):
    spec, img, table = c2_image
    rng = np.random.default_rng(0x5EED0005)
    res, off = _family_proteins(10000, 10, rng)
    n = len(off) - 1
    ids = np.arange(n, dtype=np.uint32)
    lens = np.diff(off).astype(np.uint64)
    with gpu.Context(img) as ctx, gpu.Kmap(0, gpu.KMAP_APPEND) as kmap:
        ctx.set_option("host_chunks", 1)  # the table kernels read a one-pass batch
        ctx.process_batch(res, off, want=0)  # /add of every protein
        kmap.add_hits(ctx, ids)
        with gpu.Matrix(kmap) as mx:  # then /matrix over the same request
            ctx.process_batch(res, off, want=0)
            mx.add_hits(ctx, ids)
            got = mx.pairs()
    r = oracle_lib.process_batch(table(), res, off, want=1, n_threads=8)
    km = oracle_lib.Kmap(0)
    km.add(r.hits["which_kmer"], np.repeat(ids, np.diff(r.hit_offsets).astype(np.int64)))
    om = oracle_lib.Matrix()
    om.add(km, ids, lens, r.hit_offsets, r.hits["which_kmer"])
    id1, id2, cnt, _ = om.pairs()
    assert len(id1) > 40000
    assert np.array_equal(got["id1"], id1)
    assert np.array_equal(got["id2"], id2)
    assert np.array_equal(got["count"], cnt)


def test_c4_full_fq(c2_image, gpu, oracle_lib):
    spec, img, table = c2_image
    L = gpu.lib()
    n, Lr, chunk = 10_000_000, 150, 1_000_000
    rng = np.random.default_rng(0x5EED0004)
    bases = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n * Lr, dtype=np.uint8)]
    sample = np.arange(0, n, 1000)
    params = gpu.default_params()
    d_bases, d_off = ctypes.c_void_p(), ctypes.c_void_p()
    gpu.check(L.kgx_device_alloc(0, bases.nbytes, ctypes.byref(d_bases)), "alloc")
    off = np.arange(0, chunk * Lr + 1, Lr, dtype=np.uint64)
    gpu.check(L.kgx_device_alloc(0, off.nbytes, ctypes.byref(d_off)), "alloc")
    frags = {}  # read -> [(frame, fragment, hits bytes, calls bytes)]
    totals = {"fragments": 0, "hits": 0}
    try:
        gpu.check(L.kgx_memcpy_h2d(d_bases, bases.ctypes.data, bases.nbytes), "h2d")
        gpu.check(L.kgx_memcpy_h2d(d_off, off.ctypes.data, off.nbytes), "h2d")
        with gpu.Context(img) as ctx:
            for c0 in range(0, n, chunk):
                f = gpu.Fragments()
                gpu.check(L.kgx_fq_fragments_device(ctx.handle, d_bases.value + c0 * Lr, d_off, chunk,
                                                    ctypes.byref(f)), "fq_fragments")
                h = ctx.fragments_to_host(f)
                r = ctx.run_fragments(f, params, want=3)
                totals["fragments"] += f.n_fragments
                totals["hits"] += len(r.hits)
                rd = h["read"].astype(np.int64) + c0
                sel = np.nonzero(rd % 1000 == 0)[0]
                for i in sel:
                    s = bytes(h["residues"][int(h["offsets"][i]):int(h["offsets"][i + 1])]).decode()
                    hh = r.hits[int(r.hit_offsets[i]):int(r.hit_offsets[i + 1])]
                    cc = r.calls[int(r.call_offsets[i]):int(r.call_offsets[i + 1])]
                    frags.setdefault(int(rd[i]), []).append((int(h["frame"][i]), s, hh, cc))
    finally:
        L.kgx_device_free(d_bases)
        L.kgx_device_free(d_off)
    assert totals["fragments"] > 90_000_000 and totals["hits"] > 50_000_000
    # the oracle: fragments of every sampled read, then the lookup of them all
    want_frags = []
    for q in sample:
        dna = bytes(bases[q * Lr:(q + 1) * Lr])
        ofr = oracle_lib.fq_fragments(dna)
        got_fr = [(fr, s) for fr, s, _, _ in frags.get(int(q), [])]
        assert got_fr == ofr, int(q)
        want_frags += ofr
    seqs = [s.encode() for _, s in want_frags]
    o2 = np.zeros(len(seqs) + 1, np.uint64)
    o2[1:] = np.cumsum([len(s) for s in seqs])
    r2 = np.frombuffer(b"".join(seqs), np.uint8).copy()
    want = oracle_lib.process_batch(table(), r2, o2, want=3, n_threads=8)
    got_h = np.concatenate([hh for q in sample for _, _, hh, _ in frags.get(int(q), [])])
    got_c = np.concatenate([cc for q in sample for _, _, _, cc in frags.get(int(q), [])])
    got_h = got_h.copy()
    got_h["seq"] = np.repeat(np.arange(len(seqs), dtype=np.uint32), np.diff(want.hit_offsets).astype(np.int64))
    _hits_equal(got_h, want.hits)
    _calls_equal(got_c, want.calls)
    assert len(want.hits) > 30000
    # the sampled reads as their own batch: the same fragments, and through
    # the host-buffer path the same hits and calls
    sb = np.concatenate([bases[q * Lr:(q + 1) * Lr] for q in sample])
    so = np.arange(0, len(sample) * Lr + 1, Lr, dtype=np.uint64)
    with gpu.Context(img) as ctx:
        f = ctx.fq_fragments(sb, so)
        h = ctx.fragments_to_host(f)
        assert np.array_equal(h["residues"], r2) and np.array_equal(h["offsets"], o2)
        hb = ctx.process_batch(r2, o2, params, want=3)
    _hits_equal(hb.hits, want.hits)
    _calls_equal(hb.calls, want.calls)
