"""The line index (kgx_image_set_line_index): the probes read the PACKED16
records again with line-aligned homes, built from the buckets the reference's
probe reaches first (lookup_hash_entry, kguts.cc:585-602).  Every path that
probes -- batches under every probe variant and tile size, the small fused
batches, the call service, the fq DNA probe -- must give the oracle's answer
over the reference table, including tables with duplicates, stray stop keys,
wrapping chains and no empty bucket at all, and at loads where every line is
full (chains across lines and around the end)."""
import numpy as np
import pytest

from close_kmers_amd import abi, synth
from helpers import DesignedImage, pack, random_protein, synthetic_table
from test_gpu_parity import _chain_table, _decode, assert_same

pytestmark = pytest.mark.gpu

# keys per 64 lines: 36 = the bench's load (9/16 of a key per line), 255 = every
# line full (chains run across lines and around the table's end)
LOADS = (36, 255)


def _batch_from(rng, keys, n=60):
    absent = [int(x) for x in rng.integers(0, 20 ** 8, 400)]
    pool = keys + absent
    recs = []
    for r in range(n):
        pick = [pool[int(i)] for i in rng.integers(0, len(pool), 40)]
        recs.append((f"q{r}", "X".join(_decode(k) for k in pick) + random_protein(rng, 30)))
    return recs


@pytest.mark.parametrize("filt", [0, 12])
@pytest.mark.parametrize("shape", ["wrap", "dups_strays", "full"])
def test_line_index_chain_shapes_all_variants(gpu, oracle_lib, shape, filt):
    """Every probe variant and tile size over the index at both loads; with a
    presence filter (filt: 2^12 bits) too, which sends the probes to the
    filtered per-bucket kernel over the index (home shift 2), the filter
    built from the reference slots; and context option line_index 0 (the
    reference slots while the image keeps its index)."""
    rng = np.random.default_rng({"wrap": 11, "dups_strays": 12, "full": 13}[shape])
    if shape == "wrap":
        table, keys = _chain_table(rng, 1001, 800, tail_frac=0.3)
    elif shape == "dups_strays":
        table, keys = _chain_table(rng, 997, 500, dup_every=3, stray_every=4, tail_frac=0.2)
    else:
        table, keys = _chain_table(rng, 203, 300, tail_frac=0.1)
        assert (table["which_kmer"] <= 20 ** 8).all()
    recs = _batch_from(rng, keys)
    res, off = pack(recs)
    want = oracle_lib.process_batch(table, res, off, params=(2, 200, 0, 0))
    assert int(want.hit_offsets[-1]) > 0
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        if filt:
            img.set_filter(filt)
        for load in LOADS:
            img.set_line_index(load)
            assert img.line_count > 0
            for variant in (-1, 0, 1, 2, 3):
                for probe_j in (1, 2, 3, 4):
                    ctx.set_option("probe_variant", variant)
                    ctx.set_option("probe_j", probe_j)
                    got = ctx.process_batch(res, off, gpu.Params(2, 200, 0, 0))
                    assert_same(got, want, len(recs))
            ctx.set_option("line_index", 0)
            assert_same(ctx.process_batch(res, off, gpu.Params(2, 200, 0, 0)), want, len(recs))
            ctx.set_option("line_index", 1)
        img.set_line_index(0)
        assert img.line_count == 0
        ctx.set_option("probe_variant", -1)
        ctx.set_option("probe_j", 2)
        assert_same(ctx.process_batch(res, off, gpu.Params(2, 200, 0, 0)), want, len(recs))


def test_line_index_stray_stops_and_layout_changes(gpu, oracle_lib):
    """Entries behind a stray stop key are never found by the reference; the
    index leaves them out.  Switching to AOS24 drops the index; packing again
    and rebuilding it gives the same answers."""
    rng = np.random.default_rng(5)
    img_d = DesignedImage()
    recs = []
    for t in range(30):
        s = random_protein(rng, 120)
        img_d.add_windows(s, range(0, 100, 2), fI=t % 4, rng=rng)
        recs.append((f"s{t}", s))
    table = img_d.table()
    occ = np.nonzero(table["which_kmer"] <= 20 ** 8)[0]
    for i in occ[::3]:
        j = (i + 1) % len(table)
        if table["which_kmer"][j] > 20 ** 8:
            table["which_kmer"][j] = 20 ** 8 + 2 + int(i % 1000) * 977
    # and entries placed behind stops: a second copy of some keys after the
    # first stop bucket past their home (the reference never reaches them)
    res, off = pack(recs)
    want = oracle_lib.process_batch(table, res, off)
    with gpu.Image.from_table(table) as im, gpu.Context(im) as ctx:
        for load in LOADS:
            im.set_line_index(load)
            assert_same(ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0)), want, len(recs))
        im.set_layout(gpu.Image.AOS24)
        assert im.line_count == 0
        assert_same(ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0)), want, len(recs))
        im.set_layout(gpu.Image.PACKED16)
        im.set_line_index(36)
        assert_same(ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0)), want, len(recs))
        # the download is still the reference table (stop keys read back as the
        # empty sentinel, as PACKED16 stores them)
        assert np.array_equal(im.download()["which_kmer"], np.minimum(table["which_kmer"], 20 ** 8 + 1))


def test_line_index_entries_behind_stops_are_left_out(gpu, oracle_lib):
    """A key stored only behind a stop bucket (unreachable for the reference)
    must stay a miss with the index."""
    rng = np.random.default_rng(21)
    num_sigs = 4099
    table = np.zeros(num_sigs, abi.SIG_DTYPE)
    table["which_kmer"] = 20 ** 8 + 1
    keys = []
    while len(keys) < 200:
        k = int(rng.integers(0, 20 ** 8))
        h = k % num_sigs
        if table["which_kmer"][h] > 20 ** 8 and table["which_kmer"][(h + 1) % num_sigs] > 20 ** 8 \
                and table["which_kmer"][(h + 2) % num_sigs] > 20 ** 8:
            # home left empty (a stop), the entry one bucket further: unreachable
            table[(h + 1) % num_sigs] = (k, 1, 7, 0, 3, 1.5)
            keys.append(k)
    recs = _batch_from(rng, keys, 20)
    res, off = pack(recs)
    want = oracle_lib.process_batch(table, res, off, params=(1, 200, 0, 0))
    assert int(want.hit_offsets[-1]) == 0  # none of them is found by the reference
    with gpu.Image.from_table(table) as im, gpu.Context(im) as ctx:
        im.set_line_index(36)
        got = ctx.process_batch(res, off, gpu.Params(1, 200, 0, 0))
        assert_same(got, want, len(recs))


@pytest.mark.parametrize("load", LOADS)
def test_line_index_service_small_batches_and_fq(gpu, oracle_lib, load):
    from tests_golden_codons import back_translate, revcomp
    spec, table = synthetic_table(40000)
    rng = np.random.default_rng(9)
    src = synth.ALPHA[synth.source_residue_codes(np.arange(40))].reshape(40, -1)
    seqs = [bytes(src[i % 40][: int(rng.integers(60, 300))]) for i in range(60)]
    prm = gpu.Params(5, 200, 0, 0)
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        img.set_line_index(load)
        # the call service, one sequence at a time
        for k, s in enumerate(seqs[:30]):
            hits, calls = img.svc_call(s, prm)
            r, o = pack([("s", s.decode())])
            w = oracle_lib.process_batch(table, r, o, params=(5, 200, 0, 0))
            assert np.array_equal(hits["which_kmer"], w.hits["which_kmer"]), k
            assert np.array_equal(calls["weighted_hits"].view(np.uint32),
                                  w.calls["weighted_hits"].view(np.uint32)), k
        # small fused batches
        ctx.set_option("small_fused", 1)
        r, o = pack([("s", s.decode()) for s in seqs[:8]])
        assert_same(ctx.process_batch(r, o, prm), oracle_lib.process_batch(table, r, o), 8)
        # fq fragments through the DNA line probe
        reads = []
        for i in range(200):
            p = bytes(src[i % 40][int(rng.integers(0, 200)):][:60]).decode()
            d = back_translate(p, rng)
            reads.append((d if i % 2 else revcomp(d)).encode())
        res, off = pack([("r", x) for x in reads])
        h = ctx.fragments_to_host(ctx.fq_fragments(res, off))
        ctx.set_option("fq_residues", 0)
        f = ctx.fq_fragments(res, off)
        got = ctx.run_fragments(f, prm, want=3)
    want = oracle_lib.process_batch(table, h["residues"], h["offsets"], want=3)
    assert np.array_equal(got.hit_offsets, want.hit_offsets)
    assert np.array_equal(got.hits["which_kmer"], want.hits["which_kmer"])
    assert np.array_equal(got.calls["weighted_hits"].view(np.uint32), want.calls["weighted_hits"].view(np.uint32))
    assert len(want.calls) > 20


@pytest.mark.parametrize("probe", ["thread", "quad"])
def test_svc_probe_modes_chain_shapes(gpu, oracle_lib, monkeypatch, probe):
    """The call service's two probe loops (KGX_SVC_PROBE: a thread's own
    four 16-B loads per line, or quads reading a window's line together) over
    tables that wrap, hold duplicates and stray stop keys, or have no empty
    bucket, over the reference slots and the line index: every call is the
    oracle's."""
    monkeypatch.setenv("KGX_SVC_PROBE", probe)
    rng = np.random.default_rng(31)
    prm = gpu.Params(2, 200, 0, 0)
    for shape in ("wrap", "dups_strays", "full"):
        if shape == "wrap":
            table, keys = _chain_table(rng, 1001, 800, tail_frac=0.3)
        elif shape == "dups_strays":
            table, keys = _chain_table(rng, 997, 500, dup_every=3, stray_every=4, tail_frac=0.2)
        else:
            table, keys = _chain_table(rng, 203, 300, tail_frac=0.1)
        recs = _batch_from(rng, keys, 12)
        with gpu.Image.from_table(table) as img:
            for load in (0,) + LOADS:
                img.set_line_index(load)
                for name, s in recs:
                    hits, calls = img.svc_call(s.encode(), prm)
                    r, o = pack([(name, s)])
                    w = oracle_lib.process_batch(table, r, o, params=(2, 200, 0, 0))
                    for f in ("which_kmer", "pos", "function_index", "otu_index"):
                        assert np.array_equal(hits[f], w.hits[f]), (shape, load, name, f)
                    assert np.array_equal(hits["function_wt"].view(np.uint32), w.hits["function_wt"].view(np.uint32))
                    for f in ("start", "end", "count", "function_index"):
                        assert np.array_equal(calls[f], w.calls[f]), (shape, load, name, f)
                    assert np.array_equal(calls["weighted_hits"].view(np.uint32),
                                          w.calls["weighted_hits"].view(np.uint32)), (shape, load, name)
