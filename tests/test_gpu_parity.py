"""Parity of the HIP path (through the C ABI / the KmerGuts facade driver)
with the CPU oracle: bit-exact hits, calls, OTU tallies and handler text."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from close_kmers_amd import build as kbuild
from close_kmers_amd import image_files, synth
from close_kmers_amd.abi import SIG_DTYPE
from helpers import ALPHA, GOLDEN, DesignedImage, pack, random_protein, synthetic_table

pytestmark = pytest.mark.gpu

HIT_FIELDS = ["which_kmer", "otu_index", "avg_from_end", "function_index", "function_wt", "pos", "seq"]
PARAM_SETS = [(5, 200, 0, 0), (3, 200, 0, 0), (5, 50, 0, 0), (5, 200, 1, 0), (5, 200, 0, 20),
              (2, 1000, 0, 0), (7, 10, 1, 3), (5, -1, 0, 0), (1, 200, 0, 0)]


def eq_fields(a, b, fields=HIT_FIELDS):
    if len(a) != len(b):
        return False
    for f in fields:
        x, y = a[f], b[f]
        if x.dtype.kind == "f":
            x, y = x.view(np.uint32), y.view(np.uint32)
        if not np.array_equal(x, y):
            return False
    return True


def assert_same(got, want, n_seq):
    """got: abi.BatchResult, want: oracle.BatchResult."""
    assert np.array_equal(got.hit_offsets, want.hit_offsets)
    for f in HIT_FIELDS:
        wf = want.hits[f]
        gf = got.hits[f]
        if f == "function_wt":
            assert np.array_equal(gf.view(np.uint32), wf.view(np.uint32)), f
        else:
            assert np.array_equal(gf, wf), f
    assert np.array_equal(got.call_offsets, want.call_offsets)
    for f in ["start", "end", "count", "function_index"]:
        assert np.array_equal(got.calls[f], want.calls[f]), f
    assert np.array_equal(got.calls["weighted_hits"].view(np.uint32),
                          want.calls["weighted_hits"].view(np.uint32))
    assert np.array_equal(got.otu_offsets, want.otu_offsets)
    assert np.array_equal(got.otus["otu_index"], want.otus[:, 0])
    assert np.array_equal(got.otus["count"], want.otus[:, 1])


# ---------------------------------------------------------------------------
# golden handler text through the C++ facade (kgx_query)

def _golden_cases():
    for ds in ("scoring", "edge", "cap", "matrix", "fq", "lookup"):
        d = os.path.join(GOLDEN, ds)
        for f in sorted(os.listdir(d)):
            if f.startswith("expected_") and f.endswith(".txt"):
                yield ds, f


@pytest.mark.parametrize("ds,fname", list(_golden_cases()))
def test_facade_text_matches_golden(gpu, ds, fname):
    from test_oracle_golden import case_params, parse_case
    mode, pname = parse_case(fname)
    d = os.path.join(GOLDEN, ds)
    args = [kbuild.QUERY, os.path.join(d, "data"), os.path.join(d, "input.fasta"), mode]
    args += [f"{k}={v}" for k, v in case_params(ds, pname).items()]
    r = subprocess.run(args, capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout == open(os.path.join(d, fname), "rb").read()


# ---------------------------------------------------------------------------
# random synthetic batches through kgx_process_batch

@pytest.fixture(scope="module")
def small_world(gpu):
    spec, table = synthetic_table(30000)
    img = gpu.Image.from_table(table)
    ctx = gpu.Context(img)
    yield spec, table, img, ctx
    ctx.close()
    img.close()


@pytest.mark.parametrize("params", PARAM_SETS)
@pytest.mark.parametrize("small_batch", [1 << 21, 0])
def test_random_batch_matches_oracle(small_world, oracle_lib, gpu, params, small_batch):
    """400 proteins: the one-wait small path (default) and the one-pass path."""
    spec, table, img, ctx = small_world
    res, off = synth.make_queries(spec, 400, x_permille=5)
    want = oracle_lib.process_batch(table, res, off, params=params)
    ctx.set_option("small_batch", small_batch)
    try:
        got = ctx.process_batch(res, off, gpu.Params(*params))
    finally:
        ctx.set_option("small_batch", 1 << 21)
    assert_same(got, want, 400)
    lens = np.diff(off).astype(np.int64)
    assert got.n_windows == int(np.maximum(lens - 8, 0).sum())
    assert got.n_windows >= want.windows


@pytest.fixture(scope="module")
def few_functions_world(gpu, oracle_lib):
    """A table whose k-mers carry 6 functions, so best calls take every
    branch (one function, ambiguous pair, no call)."""
    spec = synth.ImageSpec(30000)
    k, f, o, a, w = spec.unique_entries()
    f = np.random.default_rng(3).integers(0, 6, len(k)).astype(np.int32)
    table = oracle_lib.build_table(spec.num_sigs, k, f, o, a, w)
    img = gpu.Image.from_table(table)
    ctx = gpu.Context(img)
    yield spec, table, img, ctx
    ctx.close()
    img.close()


@pytest.mark.parametrize("n", [200, 257, 1000, 5000, 8192, 8193])
def test_small_batch_best_calls_in_the_collect(few_functions_world, oracle_lib, gpu, n):
    """Small batches of 257..8,192 sequences decide their best calls inside
    the multi-block collect (small_collect_best_kernel: each block sums the
    counts before its range itself) instead of best_call_kernel + the
    one-workgroup collect; below and above that the old kernels.  Every
    sequence's hits, calls, OTU tallies and best calls equal the oracle's at
    want 15, and the offsets and best calls at want BEST and CALLS | BEST."""
    spec, table, img, ctx = few_functions_world
    res, off = synth.make_queries(spec, n, length=200, x_permille=5, q0=n)
    assert int(off[-1]) <= 1 << 21  # the small-batch path
    ref = oracle_lib.process_batch(table, res, off, want=15, n_threads=4)
    for want in (15, gpu.WANT_BEST, gpu.WANT_CALLS | gpu.WANT_BEST):
        got = ctx.process_batch(res, off, want=want)
        assert oracle_lib.diff_batch(got, ref, want) == {k: [] for k in oracle_lib.diff_batch(got, ref, want)}, \
            (n, want)
        assert np.array_equal(got.hit_offsets, ref.hit_offsets), (n, want)
    assert set(np.unique(ref.best["kind"])) >= {0, 1}


@pytest.fixture(scope="module")
def aos_world(small_world, gpu):
    """The same table kept in the file's 24-byte layout."""
    spec, table, _, _ = small_world
    img = gpu.Image.from_table(table)
    img.set_layout(gpu.Image.AOS24)
    ctx = gpu.Context(img)
    yield img, ctx
    ctx.close()
    img.close()


@pytest.mark.parametrize("mode", ["packed_record", "packed_key_first", "aos_bucket", "aos_key_first",
                                  "packed_line", "packed_line8"])
@pytest.mark.parametrize("probe_j", [1, 2, 3, 4, 5, 8])
def test_probe_variants_agree(small_world, aos_world, oracle_lib, gpu, mode, probe_j):
    spec, table, img, ctx = small_world
    assert img.layout == gpu.Image.PACKED16
    if mode.startswith("aos"):
        img, ctx = aos_world
        assert img.layout == gpu.Image.AOS24
    # mixed lengths so tiles straddle many sequence boundaries
    rng = np.random.default_rng(probe_j * 10 + len(mode))
    res, off = synth.make_queries(spec, 300, x_permille=5, q0=1000)
    lens = rng.integers(0, 300, 300)
    recs = [("q", bytes(res[int(off[i]):int(off[i]) + int(lens[i])])) for i in range(300)]
    res, off = pack(recs)
    want = oracle_lib.process_batch(table, res, off)
    variant = {"packed_line": 2, "packed_line8": 3}.get(mode, 1 if mode.endswith("key_first") else 0)
    ctx.set_option("probe_variant", variant)
    ctx.set_option("probe_j", probe_j)
    try:
        got = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0))
    finally:
        ctx.set_option("probe_variant", -1)
        ctx.set_option("probe_j", 2)
    assert_same(got, want, 300)


def _occupied_equal(a, b):
    oa, ob = a[a["which_kmer"] <= 20 ** 8], b[b["which_kmer"] <= 20 ** 8]
    assert np.array_equal(a["which_kmer"] <= 20 ** 8, b["which_kmer"] <= 20 ** 8)
    for fld in ["which_kmer", "otu_index", "avg_from_end", "function_index"]:
        assert np.array_equal(oa[fld], ob[fld]), fld
    assert np.array_equal(oa["function_wt"].view(np.uint32), ob["function_wt"].view(np.uint32))


def test_resident_layout_round_trip(small_world, gpu):
    spec, table, img, ctx = small_world
    assert img.layout == gpu.Image.PACKED16
    d = img.download()
    _occupied_equal(d, table)
    emp = d[d["which_kmer"] > 20 ** 8]
    assert (emp["which_kmer"] == 20 ** 8 + 1).all() and (emp["function_index"] == 0).all()
    assert (d["pad"] == 0).all()
    with gpu.Image.from_table(table) as im2:
        im2.set_layout(gpu.Image.AOS24)
        assert im2.layout == gpu.Image.AOS24
        assert np.array_equal(im2.download().view(np.uint8), table.view(np.uint8))
        im2.set_layout(gpu.Image.PACKED16)
        _occupied_equal(im2.download(), table)


@pytest.mark.parametrize("fi,otu,packs", [
    (-1, -1, True), ((1 << 20) - 2, (1 << 21) - 2, True), (0, 0, True),
    ((1 << 20) - 1, 0, False), (0, (1 << 21) - 1, False), (-2, 0, False), (0, -7, False),
    (2 ** 31 - 1, 2 ** 31 - 1, False)])
def test_payload_ranges_pick_the_layout(gpu, oracle_lib, fi, otu, packs):
    """Boundary payloads: packed when they fit, the 24-byte layout otherwise;
    lookups identical to the oracle either way."""
    rng = np.random.default_rng(abs(fi) % 97 + abs(otu) % 89)
    img = DesignedImage()
    recs = []
    for t in range(20):
        s = random_protein(rng, 200)
        img.add_windows(s, range(10, 60), fI=t % 3, oI=t % 4 - 1, rng=rng, avg=7)
        recs.append((f"s{t}", s))
    img.add(recs[0][1][100:108], fi, otu, 65535, -0.0)  # extreme payload, also hit
    img.add(recs[1][1][100:108], fi, otu, 1, float("inf"))
    table = img.table()
    res, off = pack(recs)
    with gpu.Image.from_table(table) as im, gpu.Context(im) as ctx:
        assert im.layout == (gpu.Image.PACKED16 if packs else gpu.Image.AOS24)
        _occupied_equal(im.download(), table)
        for params in [(5, 200, 0, 0), (1, 200, 0, 0)]:
            want = oracle_lib.process_batch(table, res, off, params=params)
            got = ctx.process_batch(res, off, gpu.Params(*params))
            assert_same(got, want, len(recs))
        if not packs:
            with pytest.raises(Exception):
                im.set_layout(gpu.Image.PACKED16)
            assert im.layout == gpu.Image.AOS24


def test_stray_keys_above_max_stop_probes(gpu, oracle_lib):
    """Any key > 20^8 ends a probe (kguts.cc:592), not just the 20^8+1 sentinel."""
    rng = np.random.default_rng(5)
    img = DesignedImage()
    recs = []
    for t in range(30):
        s = random_protein(rng, 120)
        img.add_windows(s, range(0, 100, 2), fI=t % 4, rng=rng)
        recs.append((f"s{t}", s))
    table = img.table()
    occ = np.nonzero(table["which_kmer"] <= 20 ** 8)[0]
    # overwrite the bucket after every 3rd occupied one with a stray stop key
    for i in occ[::3]:
        j = (i + 1) % len(table)
        if table["which_kmer"][j] > 20 ** 8:
            table["which_kmer"][j] = 20 ** 8 + 2 + int(i % 1000) * 977
    res, off = pack(recs)
    want = oracle_lib.process_batch(table, res, off)
    for layout in ("packed", "aos"):
        with gpu.Image.from_table(table) as im, gpu.Context(im) as ctx:
            if layout == "aos":
                im.set_layout(gpu.Image.AOS24)
            got = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0))
            assert_same(got, want, len(recs))


def _decode(key: int) -> str:
    out = []
    for _ in range(8):
        out.append(ALPHA[key % 20])
        key //= 20
    return "".join(reversed(out))


def _chain_table(rng, num_sigs, n_keys, dup_every=0, stray_every=0, tail_frac=0.0):
    """A hand-placed linear-probe table: keys inserted in order from their home
    slot (key % num_sigs) to the first free bucket, wrapping at the end.
    tail_frac of the keys are drawn with homes in the last 16 buckets, so
    chains cross line boundaries and wrap; every dup_every-th key is stored a
    second time further down its chain with another payload; every
    stray_every-th free bucket after an occupied one gets a stray key > 20^8."""
    table = np.zeros(num_sigs, SIG_DTYPE)
    table["which_kmer"] = 20 ** 8 + 1
    keys = []
    while len(keys) < n_keys:
        k = int(rng.integers(0, 20 ** 8))
        if rng.random() < tail_frac:
            k = k - k % num_sigs + num_sigs - 1 - int(rng.integers(0, 16))
            if k >= 20 ** 8 or k < 0:
                continue
        keys.append(k)
    stored = []
    for n, k in enumerate(keys):
        for copy in range(2 if dup_every and n % dup_every == 0 else 1):
            h = k % num_sigs
            for _ in range(num_sigs):
                if table["which_kmer"][h] > 20 ** 8:
                    break
                h = (h + 1) % num_sigs
            else:
                break  # full
            table[h] = (k, int(rng.integers(-1, 1000)), int(rng.integers(0, 300)), 0,
                        int(rng.integers(0, 5000)), np.float32(rng.random() * 4))
            stored.append(k)
    if stray_every:
        occ = np.nonzero(table["which_kmer"] <= 20 ** 8)[0]
        for i in occ[::stray_every]:
            j = (i + 1) % num_sigs
            if table["which_kmer"][j] > 20 ** 8:
                table["which_kmer"][j] = 20 ** 8 + 2 + int(i) * 31
    return table, keys


@pytest.mark.parametrize("shape", ["wrap", "dups_strays", "full"])
def test_probe_chain_shapes_all_variants(gpu, oracle_lib, shape):
    """Chains that cross 64-B / 128-B lines, wrap past the last bucket of a
    table whose size is not a multiple of the line, meet duplicates (the
    earliest copy wins) and stray stop keys, or never end (a full table with
    absent keys): every probe variant gives the oracle's answer."""
    rng = np.random.default_rng({"wrap": 1, "dups_strays": 2, "full": 3}[shape])
    if shape == "wrap":
        table, keys = _chain_table(rng, 1001, 800, tail_frac=0.3)
    elif shape == "dups_strays":
        table, keys = _chain_table(rng, 997, 500, dup_every=3, stray_every=4, tail_frac=0.2)
    else:
        table, keys = _chain_table(rng, 203, 300, tail_frac=0.1)
        assert (table["which_kmer"] <= 20 ** 8).all()
    absent = [int(x) for x in rng.integers(0, 20 ** 8, 400)]
    pool = keys + absent
    recs = []
    for r in range(60):
        pick = [pool[int(i)] for i in rng.integers(0, len(pool), 40)]
        # runs of present k-mers (calls) separated by X, plus some overlapping windows
        recs.append((f"q{r}", "X".join(_decode(k) for k in pick) + random_protein(rng, 30)))
    res, off = pack(recs)
    want = oracle_lib.process_batch(table, res, off)
    assert int(want.hit_offsets[-1]) > 0
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        assert img.layout == gpu.Image.PACKED16
        for variant in (-1, 0, 1, 2, 3):
            for probe_j in (1, 2, 3, 4):
                ctx.set_option("probe_variant", variant)
                ctx.set_option("probe_j", probe_j)
                got = ctx.process_batch(res, off, gpu.Params(2, 200, 0, 0))
                assert_same(got, oracle_lib.process_batch(table, res, off, params=(2, 200, 0, 0)),
                            len(recs))


def test_ragged_long_and_empty_sequences(small_world, oracle_lib, gpu):
    spec, table, img, ctx = small_world
    rng = np.random.default_rng(9)
    src = synth.ALPHA[synth.source_residue_codes(np.arange(spec.n_src))].reshape(spec.n_src, -1)
    recs = []
    for i in range(120):
        kind = i % 6
        if kind == 0:
            n = int(rng.integers(0, 12))
            s = random_protein(rng, n)
        elif kind == 1:  # long: many planted sources back to back (multi-chunk)
            parts = [bytes(src[int(rng.integers(0, spec.n_src))]).decode() for _ in range(int(rng.integers(2, 40)))]
            s = "".join(parts)
        elif kind == 2:
            s = bytes(src[int(rng.integers(0, spec.n_src))]).decode()[: int(rng.integers(5, 300))]
        elif kind == 3:  # ambiguity sprinkled over a planted sequence
            s = list(bytes(src[int(rng.integers(0, spec.n_src))]).decode())
            for p in rng.integers(0, len(s), 6):
                s[p] = "XxB*u"[int(rng.integers(0, 5))]
            s = "".join(s)
        elif kind == 4:
            s = random_protein(rng, int(rng.integers(300, 3000)))
        else:
            s = bytes(src[int(rng.integers(0, spec.n_src))]).decode().lower()
        recs.append((f"s{i}", s))
    res, off = pack(recs)
    for params in [(5, 200, 0, 0), (3, 20, 1, 0)]:
        want = oracle_lib.process_batch(table, res, off, params=params)
        got = ctx.process_batch(res, off, gpu.Params(*params))
        assert_same(got, want, len(recs))


def test_want_flags_and_unaligned_offsets(small_world, oracle_lib, gpu):
    spec, table, img, ctx = small_world
    res, off = synth.make_queries(spec, 64)
    # a batch that starts mid-buffer (seq_offsets[0] != 0)
    pad = np.frombuffer(b"QQQ", np.uint8)
    res2 = np.concatenate([pad, res])
    off2 = off + np.uint64(3)
    want = oracle_lib.process_batch(table, res, off)
    for w in (1, 2, 4, 3, 5, 6, 7):
        got = ctx.process_batch(res2, off2, gpu.Params(5, 200, 0, 0), want=w)
        assert np.array_equal(got.hit_offsets, want.hit_offsets)
        if w & 1:
            assert np.array_equal(got.hits["pos"], want.hits["pos"])
        if w & 2:
            assert np.array_equal(got.call_offsets, want.call_offsets)
            assert np.array_equal(got.calls["start"], want.calls["start"])
        else:
            assert len(got.calls) == 0
        if w & 4:
            assert np.array_equal(got.otu_offsets, want.otu_offsets)


def test_nul_byte_cuts_the_sequence(small_world, oracle_lib, gpu):
    """gather_hits bounds the walk with strlen() (kguts.cc:792)."""
    spec, table, img, ctx = small_world
    src = synth.ALPHA[synth.source_residue_codes(np.arange(4))]
    recs = []
    for cut in (0, 1, 7, 8, 9, 10, 50, 150, 299):
        s = bytearray(bytes(src[cut % 4]))
        s[cut] = 0
        recs.append(("n", bytes(s)))
    res, off = pack(recs)
    want = oracle_lib.process_batch(table, res, off)
    got = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0))
    assert_same(got, want, len(recs))


def test_hit_flags_reproduce_otu_tallies(small_world, gpu):
    spec, table, img, ctx = small_world
    res, off = synth.make_queries(spec, 200)
    got = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0))
    for s in range(200):
        h = got.hits[got.hit_offsets[s]:got.hit_offsets[s + 1]]
        m = {}
        for o in h["otu_index"][(h["flags"] & 2) != 0]:
            m[int(o)] = m.get(int(o), 0) + 1
        o = got.otus[got.otu_offsets[s]:got.otu_offsets[s + 1]]
        assert dict(zip(o["otu_index"].tolist(), o["count"].tolist())) == m
        c = got.calls[got.call_offsets[s]:got.call_offsets[s + 1]]
        assert int(c["count"].sum()) == int(((h["flags"] & 2) != 0).sum())


# ---------------------------------------------------------------------------
# designed run-rule edge cases at the API level (cap, carries, order constraint)

def test_hit_buffer_cap(gpu, oracle_lib):
    d = os.path.join(GOLDEN, "cap")
    table = image_files.read_image(os.path.join(d, "data"))
    seq = open(os.path.join(d, "input.fasta")).read().split("\n")[1]
    res, off = pack([("capped", seq)])
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        for params in [(5, 200, 0, 0), (5, 200, 1, 0), (2, 200, 0, 0)]:
            want = oracle_lib.process_batch(table, res, off, params=params)
            got = ctx.process_batch(res, off, gpu.Params(*params))
            assert want.calls["count"].max() == 39998 or params[2]
            assert_same(got, want, 1)


def test_pair_switch_chains(gpu, oracle_lib):
    """Alternating same-function pairs: every pair flushes and carries."""
    rng = np.random.default_rng(21)
    img = DesignedImage()
    recs = []
    for t in range(40):
        s = random_protein(rng, 400)
        p = 3
        f = 0
        while p < 380:
            run = int(rng.integers(1, 7))
            img.add_windows(s, range(p, min(p + run, 390)), f % 5, oI=int(rng.integers(-1, 3)), rng=rng)
            p += run + int(rng.integers(0, 30))
            f += int(rng.integers(1, 3))
        recs.append((f"p{t}", s))
    table = img.table()
    res, off = pack(recs)
    with gpu.Image.from_table(table) as im, gpu.Context(im) as ctx:
        for params in PARAM_SETS:
            want = oracle_lib.process_batch(table, res, off, params=params)
            got = ctx.process_batch(res, off, gpu.Params(*params))
            assert_same(got, want, len(recs))


# ---------------------------------------------------------------------------
# image loading and the device-side builders

def test_image_open_validation(gpu, tmp_path):
    L = gpu.lib()
    h = ctypes.c_void_p()
    assert L.kgx_image_open(str(tmp_path / "missing").encode(), 0, ctypes.byref(h)) == -2
    t = np.zeros(3769, dtype=gpu.SIG_DTYPE)
    t["which_kmer"] = 20 ** 8 + 1
    d = tmp_path / "bad"
    image_files.write_data_dir(str(d), t, ["f"], ["o"])
    p = d / "kmer.table.mem_map"
    raw = bytearray(p.read_bytes())
    p.write_bytes(raw[:-1])  # size mismatch
    assert L.kgx_image_open(str(d).encode(), 0, ctypes.byref(h)) == -3
    raw2 = bytearray(raw)
    raw2[16] = 2  # version 2
    p.write_bytes(raw2)
    assert L.kgx_image_open(str(d).encode(), 0, ctypes.byref(h)) == -3
    p.write_bytes(raw)
    assert L.kgx_image_open(str(d).encode(), 0, ctypes.byref(h)) == 0
    L.kgx_image_close(h)


@pytest.mark.parametrize("n_distinct", [39000, 41000])
def test_device_synthetic_distinct_equals_host_build(gpu, oracle_lib, n_distinct):
    """kgx_image_build_synthetic_distinct: the spec's stream cut at the
    smallest entry count holding n_distinct distinct keys (bench.py's 1e9
    distinct keys at C2), the same buckets as the host build of that cut."""
    spec = synth.ImageSpec(40000, 101533)
    m_host = spec.entries_for_distinct(n_distinct)
    img, m = gpu.Image.synthetic_distinct(spec.n_keys, n_distinct, spec.num_sigs)
    with img:
        dev = img.download()
    assert m == m_host
    cut = synth.ImageSpec(40000, 101533, n_entries=m)
    k, f, o, a, w = cut.unique_entries()
    assert len(k) == n_distinct
    occ_d = np.sort(dev[dev["which_kmer"] <= 20 ** 8], order="which_kmer")
    host = oracle_lib.build_table(spec.num_sigs, k, f, o, a, w)
    occ_h = np.sort(host[host["which_kmer"] <= 20 ** 8], order="which_kmer")
    assert np.array_equal(occ_d.view(np.uint8), occ_h.view(np.uint8))


def test_device_synthetic_image_equals_host_build(gpu, oracle_lib):
    spec = synth.ImageSpec(40000)
    img, stored = gpu.Image.synthetic(spec.n_keys, spec.num_sigs)
    with img:
        dev = img.download()
    k, f, o, a, w = spec.unique_entries()
    assert stored == len(k)
    host = oracle_lib.build_table(spec.num_sigs, k, f, o, a, w)
    # same multiset of buckets (placement may differ: parallel insertion)
    occ_d = dev[dev["which_kmer"] <= 20 ** 8]
    occ_h = host[host["which_kmer"] <= 20 ** 8]
    assert len(occ_d) == len(occ_h)
    sd = np.sort(occ_d, order="which_kmer")
    sh = np.sort(occ_h, order="which_kmer")
    for fld in ["which_kmer", "otu_index", "avg_from_end", "pad", "function_index"]:
        assert np.array_equal(sd[fld], sh[fld]), fld
    assert np.array_equal(sd["function_wt"].view(np.uint32), sh["function_wt"].view(np.uint32))
    # empty buckets are zeroed like the reference writer's memset
    emp = dev[dev["which_kmer"] > 20 ** 8]
    assert (emp["which_kmer"] == 20 ** 8 + 1).all() and (emp["function_index"] == 0).all()
    # lookups agree: the oracle over the device-built table == over the host table
    res, off = synth.make_queries(spec, 300, x_permille=3)
    a1 = oracle_lib.process_batch(dev, res, off)
    a2 = oracle_lib.process_batch(host, res, off)
    assert eq_fields(a1.hits, a2.hits)
    assert eq_fields(a1.calls, a2.calls, list(a1.calls.dtype.names))


def _dev_alloc(gpu, nbytes):
    p = ctypes.c_void_p()
    gpu.check(gpu.lib().kgx_device_alloc(0, nbytes, ctypes.byref(p)), "alloc")
    return p.value


@pytest.mark.parametrize("layout", ["packed", "aos"])
def test_device_queries_and_run_device(gpu, oracle_lib, layout):
    spec, table = synthetic_table(30000)
    n, L = 500, 300
    L_ = gpu.lib()
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        if layout == "aos":
            img.set_layout(gpu.Image.AOS24)
        d_res = _dev_alloc(gpu, n * L)
        d_off = _dev_alloc(gpu, (n + 1) * 8)
        try:
            gpu.check(L_.kgx_synth_queries(ctx.handle, spec.n_keys, n, L, 4, 17, d_res, d_off), "synth")
            ctx.synchronize()
            res = np.empty(n * L, np.uint8)
            off = np.empty(n + 1, np.uint64)
            gpu.check(L_.kgx_memcpy_d2h(res.ctypes.data, d_res, res.nbytes), "d2h")
            gpu.check(L_.kgx_memcpy_d2h(off.ctypes.data, d_off, off.nbytes), "d2h")
            hres, hoff = synth.make_queries(spec, n, x_permille=4, q0=17)
            assert np.array_equal(res, hres) and np.array_equal(off, hoff)
            out = gpu.DeviceResult()
            p = gpu.Params(5, 200, 0, 0)
            gpu.check(L_.kgx_run_device(ctx.handle, ctypes.byref(p), d_res, d_off, n, n * L, 7,
                                        ctypes.byref(out)), "run_device")
            ctx.synchronize()
            wb = np.empty(n + 1, np.uint64)
            hc = np.empty(n, np.uint32)
            cc = np.empty(n, np.uint32)
            for arr, ptr in ((wb, out.window_base), (hc, out.hit_count), (cc, out.call_count)):
                gpu.check(L_.kgx_memcpy_d2h(arr.ctypes.data, ptr, arr.nbytes), "d2h")
            hot = np.empty((int(wb[-1]), 4), np.uint32)
            calls = np.empty(int(wb[-1]), gpu.CALL_DTYPE)
            mask = np.empty((int(wb[-1]) + 63) // 64, np.uint64)
            gpu.check(L_.kgx_memcpy_d2h(hot.ctypes.data, out.hits_hot, hot.nbytes), "d2h")
            packed = out.hit_format == gpu.HIT_PACKED16
            assert packed == (img.layout == gpu.Image.PACKED16)
            if packed:
                assert not out.hits_cold
                hits = gpu.hits_from_packed(hot)
            else:
                cold = np.empty((int(wb[-1]), 4), np.uint32)
                gpu.check(L_.kgx_memcpy_d2h(cold.ctypes.data, out.hits_cold, cold.nbytes), "d2h")
                hits = gpu.hits_from_planes(hot, cold)
            gpu.check(L_.kgx_memcpy_d2h(calls.ctypes.data, out.calls, calls.nbytes), "d2h")
            gpu.check(L_.kgx_memcpy_d2h(mask.ctypes.data, out.hit_mask, mask.nbytes), "d2h")
            want = oracle_lib.process_batch(table, hres, hoff)
            assert np.array_equal(np.diff(want.hit_offsets), hc)
            assert np.array_equal(np.diff(want.call_offsets), cc)
            per_seq = gpu.tiled_hits_per_sequence(wb, mask, out.tile_windows, hits, fill_pos=packed)
            assert [len(x) for x in per_seq] == hc.tolist()
            gh = np.concatenate(per_seq)
            gc = np.concatenate([calls[wb[s]:wb[s] + cc[s]] for s in range(n)])
            assert eq_fields(gh, want.hits)
            assert eq_fields(gc, want.calls, list(want.calls.dtype.names))
        finally:
            L_.kgx_device_free(d_res)
            L_.kgx_device_free(d_off)


def test_image_build_from_entries_and_save(gpu, oracle_lib, tmp_path):
    """kgx_image_build (insert_kmer semantics: invalid keys skipped, duplicated
    keys resolved to their first entry) and kgx_image_save (a file KmerImage
    and kgx_image_open load): lookups equal the oracle's sequential build."""
    from close_kmers_amd import image_files
    rng = np.random.default_rng(17)
    img = DesignedImage()
    recs = []
    for t in range(40):
        s = random_protein(rng, 150)
        img.add_windows(s, range(0, 120), t % 6, oI=t % 3, rng=rng)
        recs.append((f"s{t}", s))
    k, f, o, a, w = img.arrays()
    # append duplicates (later entries for existing keys, other payloads), keys
    # above 20^8 (skipped, kguts.cc:203-207) and 20^8 itself (stored: it passes
    # the `> MAX_ENCODED` test although no window encodes to it)
    dup = rng.integers(0, len(k), 300)
    k2 = np.concatenate([k, k[dup], np.array([20 ** 8, 20 ** 8 + 5, 2 ** 63], np.uint64)])
    f2 = np.concatenate([f, (f[dup] + 1) % 6, np.zeros(3, np.int32)])
    o2 = np.concatenate([o, o[dup] + 7, np.zeros(3, np.int32)])
    a2 = np.concatenate([a, a[dup] + 1, np.zeros(3, np.uint16)])
    w2 = np.concatenate([w, w[dup] * 2, np.zeros(3, np.float32)])
    num_sigs = synth.builder_num_sigs(len(k2))
    host = oracle_lib.build_table(num_sigs, k2, f2, o2, a2, w2)  # sequential insert_kmer
    res, off = pack(recs)
    want = oracle_lib.process_batch(host, res, off)
    dev, stored = gpu.Image.build(k2, f2, o2, a2, w2, num_sigs)
    with dev:
        assert stored == len(k) + 1
        with gpu.Context(dev) as ctx:
            assert_same(ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0)), want, len(recs))
        data = str(tmp_path / "img")
        os.makedirs(data)
        dev.save(data)
    table = image_files.read_image(data)
    occ = table[table["which_kmer"] <= 20 ** 8]
    assert len(occ) == len(k) + 1
    got = dict(zip(occ["which_kmer"].tolist(), occ["function_index"].tolist()))
    assert all(got[int(kk)] == int(ff) for kk, ff in zip(k, f))  # first entry's payload
    assert np.array_equal(oracle_lib.process_batch(table, res, off).hits["pos"], want.hits["pos"])
    with gpu.Image.open(data) as reopened, gpu.Context(reopened) as ctx:
        assert_same(ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0)), want, len(recs))
    with pytest.raises(Exception):
        gpu.Image.build(k, f, o, a, w, 2 * len(k))  # half full


@pytest.mark.parametrize("log2_bits", [12, 16, 22])
def test_presence_filter_keeps_results(small_world, oracle_lib, gpu, log2_bits):
    """A probe gated by the presence filter gives the unfiltered results,
    from a tiny saturated filter (every key passes) to a sparse one."""
    spec, table, _, _ = small_world
    res, off = synth.make_queries(spec, 400, x_permille=5, q0=77)
    want = oracle_lib.process_batch(table, res, off)
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        img.set_filter(log2_bits)
        for variant in (-1, 0, 1):
            ctx.set_option("probe_variant", variant)
            assert_same(ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0)), want, 400)
        img.set_layout(gpu.Image.AOS24)  # the filter depends on the keys only
        assert_same(ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0)), want, 400)


def test_chunked_host_batch_matches_oracle(small_world, oracle_lib, gpu):
    """kgx_process_batch in K chunks alternating over two contexts (option
    host_chunks) returns the same CSR as one pass and as the oracle: global
    sequence indices, offsets continued across chunks, NUL cuts, calls/OTU."""
    spec, table, img, ctx = small_world
    res, off = synth.make_queries(spec, 16000, x_permille=3)
    rng = np.random.default_rng(17)
    res = res.copy()
    lens = np.diff(off).astype(np.int64)
    for s in rng.choice(len(lens), 40, replace=False):  # NULs inside some sequences
        res[int(off[s]) + int(rng.integers(0, lens[s]))] = 0
    # a long sequence and some empties, and a batch that starts mid-buffer
    seqs = [res[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    long_seq = np.frombuffer(random_protein(rng, 3_000_000).encode(), np.uint8)
    empty = np.zeros(0, np.uint8)
    seqs = seqs[:8000] + [empty, long_seq, empty] + seqs[8000:]
    lens = np.array([0] + [len(x) for x in seqs], np.uint64)
    off = np.cumsum(lens).astype(np.uint64) + np.uint64(2)
    res = np.concatenate([np.frombuffer(b"MK", np.uint8)] + seqs)
    want = oracle_lib.process_batch(table, res, off)
    best_one_pass = None
    ctx.set_option("host_chunks", 1)  # one pass, 32-B records gathered on the device
    flags_ref = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0), want=7).hits["flags"].copy()
    assert flags_ref.any()
    # (chunks, host_copy, host_hits16, host_threads, host_stream): host_hits16
    # 1 sends the 16-B table records + the hit mask and expands kgx_hit on host
    # threads; host_stream 1 sizes each chunk's copy on the device (no host
    # round trip inside a chunk), 0 the exact round-trip schedule
    for k, hc, h16, nt, hs in ((2, 1, 1, 8, 1), (3, 0, 1, 3, 1), (3, 1, 0, 8, 1), (3, 1, 1, 1, 0), (8, 1, 1, 8, 1),
                               (8, 0, 0, 8, 0), (5, 1, 1, 8, 0), (1, 1, 1, 8, 1)):
        ctx.set_option("host_chunks", k)
        ctx.set_option("host_copy", hc)
        ctx.set_option("host_hits16", h16)
        ctx.set_option("host_threads", nt)
        ctx.set_option("host_stream", hs)
        got = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0))
        assert_same(got, want, len(off) - 1)
        assert np.array_equal(got.hits["seq"], want.hits["seq"])
        gb = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0), want=gpu.WANT_BEST | gpu.WANT_HITS)
        if best_one_pass is None:
            ctx.set_option("host_chunks", 1)
            best_one_pass = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0), want=gpu.WANT_BEST).best
            ctx.set_option("host_chunks", k)
        assert np.array_equal(gb.best, best_one_pass) and eq_fields(gb.hits, want.hits)
        for w in (1, 2):
            g = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0), want=w)
            assert np.array_equal(g.hit_offsets, want.hit_offsets)
            if w == 1:
                assert eq_fields(g.hits, want.hits)
            else:
                assert np.array_equal(g.call_offsets, want.call_offsets)
        # with OTU tallies the hit flags are set: the same bits either way
        g7 = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0), want=7)
        assert eq_fields(g7.hits, want.hits)
        assert np.array_equal(g7.hits["flags"], flags_ref)
    ctx.set_option("host_chunks", 3)
    ctx.set_option("host_copy", 1)
    ctx.set_option("host_hits16", 1)
    ctx.set_option("host_threads", 8)
    ctx.set_option("host_stream", 1)


def test_streamed_host_batch_region_overflow(small_world, oracle_lib, gpu):
    """The streamed schedule sizes each chunk's host regions from the hit /
    call rates of earlier batches.  A hitless batch drives the rates to their
    floor; the next, hit-dense batch overflows its regions and must rerun on
    the exact schedule with identical results (and raise the rates)."""
    spec, table, img, ctx = small_world
    rng = np.random.default_rng(5)
    ctx.set_option("host_chunks", 4)
    ctx.set_option("host_stream", 1)
    noise = np.frombuffer("".join(random_protein(rng, 300) for _ in range(20000)).encode(), np.uint8)
    noff = np.arange(20001, dtype=np.uint64) * np.uint64(300)
    for _ in range(2):
        r0 = ctx.process_batch(noise, noff, gpu.Params(5, 200, 0, 0))
        assert np.array_equal(r0.hit_offsets, oracle_lib.process_batch(table, noise, noff).hit_offsets)
    res, off = synth.make_queries(spec, 16000, x_permille=0)
    want = oracle_lib.process_batch(table, res, off)
    for _ in range(2):  # overflow + exact rerun, then the raised rates fit
        got = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0))
        assert_same(got, want, len(off) - 1)
        assert np.array_equal(got.hits["seq"], want.hits["seq"])
    ctx.set_option("host_chunks", 3)


def test_streamed_host_batch_copy_stream_lag(small_world, oracle_lib, gpu):
    """The streamed schedule with its copy stream far behind the compute: one
    workgroup per bulk copy, many chunks of unequal sizes (so chunk k's scanned
    totals differ from chunk k-2's), hit-dense queries, every want mask.  Chunk
    k reuses chunk k-2's device buffers, including the scanned totals that
    chunk k-2's counted copies read when they run; nothing of chunk k may touch
    them before those copies are done."""
    spec, table, img, ctx = small_world
    res, off = synth.make_queries(spec, 24000, x_permille=0)
    seqs = [res[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    # unequal chunks: runs of long and short sequences
    lens = np.where((np.arange(len(seqs)) // 1500) % 2 == 0, 300, 60)
    seqs = [s[:l] for s, l in zip(seqs, lens)]
    off = np.zeros(len(seqs) + 1, np.uint64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    res = np.concatenate(seqs)
    want = oracle_lib.process_batch(table, res, off)
    try:
        ctx.set_option("host_stream", 1)
        ctx.set_option("host_hits16", 1)
        ctx.set_option("host_copy_blocks", 1)
        # chunk k's D2H behind chunk k+1's H2D, or not; uploads on their own stream, or not;
        # every chunk staged into its own pinned region, or into its context's buffer;
        # chunk copies by device stores (sized on the device) or DMA (whole regions)
        for k, h2d_first, up, sv, sall, dma in ((16, 1, 0, 1, 1, 0), (37, 0, 1, -1, 0, 1), (64, 1, 1, 0, 1, 0),
                                                (9, 1, 0, 1, 0, 1)):
            ctx.set_option("host_chunks", k)
            ctx.set_option("host_h2d_first", h2d_first)
            ctx.set_option("host_upload_stream", up)
            ctx.set_option("host_score_variant", sv)
            ctx.set_option("host_stage_all", sall)
            ctx.set_option("host_stream_dma", dma)
            for _ in range(2):  # the second pass runs with the rates the first one raised
                got = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0), want=7)
                assert_same(got, want, len(off) - 1)
                assert np.array_equal(got.hits["seq"], want.hits["seq"])
            g = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0), want=gpu.WANT_HITS)
            assert eq_fields(g.hits, want.hits)
    finally:
        ctx.set_option("host_copy_blocks", 64)
        ctx.set_option("host_chunks", 3)
        ctx.set_option("host_h2d_first", 1)
        ctx.set_option("host_upload_stream", 0)
        ctx.set_option("host_score_variant", 1)
        ctx.set_option("host_stage_all", 0)
        ctx.set_option("host_stream_dma", 0)


@pytest.mark.parametrize("schedule", ["streamed_rec12", "streamed_rec16", "exact", "small", "aos24",
                                      "one_pass", "overflow"])
def test_compact_results_match_oracle(small_world, aos_world, oracle_lib, gpu, schedule):
    """kgx_process_batch_compact: whatever path a batch takes, the compact
    result carries the oracle's offsets, calls and OTUs, and its hits expand
    (whole batch, any sequence range, seq_base) to the oracle's hits."""
    spec, table, img, ctx = small_world
    n = 60 if schedule == "small" else 16000
    res, off = synth.make_queries(spec, n, x_permille=3, q0=5)
    want = oracle_lib.process_batch(table, res, off)
    opts = {"streamed_rec12": {"host_chunks": 5}, "streamed_rec16": {"host_chunks": 5, "host_rec12": 0},
            "exact": {"host_chunks": 4, "host_stream": 0}, "small": {}, "aos24": {"host_chunks": 3},
            "one_pass": {"host_chunks": 1}, "overflow": {"host_chunks": 4}}[schedule]
    c = aos_world[1] if schedule == "aos24" else ctx
    try:
        for k, v in opts.items():
            c.set_option(k, v)
        if schedule == "overflow":  # a hitless batch drives the region rates to their floor
            rng = np.random.default_rng(8)
            noise = np.frombuffer("".join(random_protein(rng, 300) for _ in range(20000)).encode(), np.uint8)
            c.process_batch_compact(noise, np.arange(20001, dtype=np.uint64) * np.uint64(300))
        cb = c.process_batch_compact(res, off, gpu.Params(5, 200, 0, 0), want=7)
        compact_paths = ("streamed_rec12", "streamed_rec16", "exact", "overflow")
        assert (cb.n_chunks > 0) == (schedule in compact_paths), cb.n_chunks
        if schedule in compact_paths:
            assert {ch.record_words for ch in cb.chunks} == ({4} if schedule in ("exact", "overflow",
                                                                               "streamed_rec16") else {3})
        r = cb.result
        assert np.array_equal(r.hit_offsets, want.hit_offsets)
        assert np.array_equal(r.call_offsets, want.call_offsets)
        for f in ["start", "end", "count", "function_index"]:
            assert np.array_equal(r.calls[f], want.calls[f]), f
        assert np.array_equal(r.calls["weighted_hits"].view(np.uint32), want.calls["weighted_hits"].view(np.uint32))
        assert np.array_equal(r.otus["otu_index"], want.otus[:, 0])
        hits = cb.expand()
        assert eq_fields(hits, want.hits)
        rng = np.random.default_rng(len(schedule))
        for _ in range(10):
            a = int(rng.integers(0, n))
            b = int(rng.integers(a, n + 1))
            part = cb.expand(a, b, seq_base=7)
            sl = want.hits[int(want.hit_offsets[a]):int(want.hit_offsets[b])]
            assert eq_fields(part, sl, [f for f in HIT_FIELDS if f != "seq"])
            assert np.array_equal(part["seq"], sl["seq"] + 7)
    finally:
        for k in opts:
            c.set_option(k, {"host_chunks": 3, "host_rec12": 1, "host_stream": 1}[k])


def test_host_profile_reports_the_streamed_stages(small_world, gpu):
    spec, table, img, ctx = small_world
    res, off = synth.make_queries(spec, 16000, x_permille=0, q0=9)
    ctx.set_option("host_profile", 1)
    ctx.set_option("host_chunks", 4)
    try:
        ctx.process_batch(res, off, want=3)
        p = ctx.host_profile()
        assert p["streamed"] == 1 and p["chunks"] >= 2
        assert p["h2d_ms"] > 0 and p["device_ms"] > 0 and p["d2h_ms"] > 0 and p["expand_ms"] > 0
        assert p["h2d_bytes"] >= res.nbytes and p["d2h_bytes"] > 0 and p["wall_ms"] > 0
        ctx.process_batch_compact(res, off, want=3)
        assert ctx.host_profile()["expand_ms"] == 0
    finally:
        ctx.set_option("host_profile", 0)
        ctx.set_option("host_chunks", 3)


# ---------------------------------------------------------------------------
# find_best_call on the device (KGX_WANT_BEST, kgx_find_best_calls)

def _best_as_reference(b, names):
    """kgx_best_call -> find_best_call's (function_index, function, score,
    weighted_score, score_offset or None), names as function_at_index."""
    def name(i):
        return names[i] if 0 <= i < len(names) else "INVALID_OFFSET"
    kind = int(b["kind"])
    fn, fi = "", -1
    if kind == 1:
        fi, fn = int(b["fi0"]), name(int(b["fi0"]))
    elif kind == 2:
        a, c = name(int(b["fi0"])), name(int(b["fi1"]))
        if c > a:
            a, c = c, a
        fn = a + " ?? " + c
    return (fi, fn, float(b["score"]), float(b["weighted_score"]),
            None if kind == 0 else float(b["score_offset"]))


def _same_decision(got, want):
    f = np.float32
    return (got[0] == want[0] and got[1] == want[1]
            and f(got[2]).view(np.uint32) == f(want[2]).view(np.uint32)
            and f(got[3]).view(np.uint32) == f(want[3]).view(np.uint32)
            and (got[4] is None) == (want[4] is None)
            and (got[4] is None or f(got[4]).view(np.uint32) == f(want[4]).view(np.uint32)))


def test_device_best_call_on_crafted_lists(small_world, oracle_lib, gpu):
    """Call lists built to hit every branch: collapses, F1|F2|F1 joins, weight
    ties (partial_sort's tie order and the element left at index 2), one
    function, ambiguous pairs with and without a clear third, unknown and
    negative function indices, and empty lists."""
    spec, table, img, ctx = small_world
    rng = np.random.default_rng(23)
    names = ["zeta kinase", "alpha protein", "Beta", "alpha protein", "", "gyrase B", "gyrase A"]
    lists = []
    for i in range(30000):
        n = int(rng.integers(0, 9)) if i % 7 else int(rng.integers(0, 40))
        fis = rng.integers(-1, 8, n) if i % 5 == 0 else rng.integers(0, 4, n)
        cnt = rng.integers(1, 13, n)
        wsets = [np.float32([1.0, 2.0, 3.0]), np.float32([0.1, 0.7, 1.3, 2.9]),
                 rng.random(8).astype(np.float32) * 10]
        wt = rng.choice(wsets[i % 3], n)
        c = np.zeros(n, gpu.CALL_DTYPE)
        c["start"] = np.arange(n) * 10
        c["end"] = np.arange(n) * 10 + 7
        c["count"] = cnt
        c["function_index"] = fis.astype(np.int64).astype(np.uint32)
        c["weighted_hits"] = wt
        lists.append(c)
    off = np.zeros(len(lists) + 1, np.uint64)
    off[1:] = np.cumsum([len(c) for c in lists])
    allc = np.concatenate(lists)
    best = ctx.find_best_calls(allc, off)
    bad = []
    for i, c in enumerate(lists):
        want = oracle_lib.find_best_call(c, names)
        if not _same_decision(_best_as_reference(best[i], names), want):
            bad.append((i, c, best[i], want))
    assert not bad, (len(bad), bad[:3])
    assert set(np.unique(best["kind"])) == {0, 1, 2, 3}


def test_device_best_call_on_batches(small_world, oracle_lib, gpu):
    spec, table, img, ctx = small_world
    names = [f"function {i % 977}" for i in range(spec.n_src + 10)]
    res, off = synth.make_queries(spec, 3000, x_permille=5)
    for params in [(5, 200, 0, 0), (2, 50, 0, 0), (3, 200, 1, 0)]:
        got = ctx.process_batch(res, off, gpu.Params(*params), want=gpu.WANT_BEST | gpu.WANT_CALLS)
        want = oracle_lib.process_batch(table, res, off, params=params)
        assert np.array_equal(got.call_offsets, want.call_offsets)
        assert got.best is not None and len(got.best) == len(off) - 1
        for s in range(len(off) - 1):
            c = want.calls[int(want.call_offsets[s]):int(want.call_offsets[s + 1])]
            ref = oracle_lib.find_best_call(c, names)
            assert _same_decision(_best_as_reference(got.best[s], names), ref), s
        # BEST alone (no calls copied back), and in chunks
        only = ctx.process_batch(res, off, gpu.Params(*params), want=gpu.WANT_BEST)
        assert len(only.calls) == 0 and np.array_equal(only.best, got.best)


@pytest.mark.parametrize("otu_range,layout,maxlen", [(60, "packed", 0), (60, "aos", 0), (8, "packed", 0),
                                                     (2000, "packed", 0), (2000, "packed", 36), (5, "aos", 36)])
def test_device_otu_tallies_match_oracle(gpu, oracle_lib, otu_range, layout, maxlen):
    """OTU tallies on the device (otu_kernel): per-sequence otu_map in key
    order, then libstdc++ std::sort by count (less_second, kguts.h:196-218).
    60 OTUs over ~126 planted hits gives >16 distinct OTUs per sequence with
    many tied counts (the introsort path of std::sort), 8 the insertion-sort
    path; the AOS24 layout reads the OTU from the cold plane.  maxlen 36:
    sequences cut to <= 36 aa, so every tally has at most 29 hits -- the
    kernel's single-OTU and LDS-sorted paths."""
    import oracle
    spec = synth.ImageSpec(30000)
    k, f, o, a, w = spec.unique_entries()
    rng = np.random.default_rng(otu_range)
    o = rng.integers(-1, otu_range, len(k)).astype(np.int32)
    table = oracle.build_table(spec.num_sigs, k, f, o, a, w)
    res, off = synth.make_queries(spec, 600, x_permille=3)
    if maxlen:
        cut = [res[int(off[i]):min(int(off[i + 1]), int(off[i]) + maxlen)] for i in range(len(off) - 1)]
        off = np.concatenate([[0], np.cumsum([len(c) for c in cut])]).astype(off.dtype)
        res = np.concatenate(cut)
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        if layout == "aos":
            img.set_layout(gpu.Image.AOS24)
        for params in [(5, 200, 0, 0), (2, 30, 0, 0)]:
            want = oracle_lib.process_batch(table, res, off, params=params)
            for w_ in (4, 7, 6):
                got = ctx.process_batch(res, off, gpu.Params(*params), want=w_)
                assert np.array_equal(got.otu_offsets, want.otu_offsets)
                assert np.array_equal(got.otus["otu_index"], want.otus[:, 0])
                assert np.array_equal(got.otus["count"], want.otus[:, 1])
                if not w_ & 1:
                    assert len(got.hits) == 0
            n_otu = np.diff(want.otu_offsets)
            if otu_range >= 60 and not maxlen:
                assert n_otu.max() > 16  # the introsort path ran


@pytest.mark.parametrize("params", PARAM_SETS)
def test_fused_small_path_matches_oracle(small_world, oracle_lib, gpu, params):
    """small_fused 1 (the facade's per-sequence calls): a small batch runs as
    one launch, one workgroup per sequence (kgx_fused.hip), when its
    parameters, outputs and lengths allow -- else the one-wait path.  Either
    way the oracle's hits and calls, for one sequence, empties, sub-window,
    X / * / lower case / NUL-cut sequences, a mid-buffer start, the
    2,048-window boundary (2,056 aa fused, 2,057 aa not) and 300 sequences."""
    spec, table, img, ctx = small_world
    rng = np.random.default_rng(31)
    res, off = synth.make_queries(spec, 60, x_permille=5, q0=4242)
    seqs = [res[int(off[i]):int(off[i + 1])].copy() for i in range(60)]
    seqs[3][40] = 0  # NUL cut
    seqs[4][17] = ord("x")
    seqs[5][100] = ord("*")
    planted, poff = synth.make_queries(spec, 40, x_permille=0, q0=9000)
    edge = [np.concatenate([planted[int(poff[i]):int(poff[i + 1])] for i in range(2 * k, 2 * k + 7)])[:n]
            for k, n in enumerate((2056, 2057))]
    res2, off2 = synth.make_queries(spec, 300, x_permille=5, q0=6000)
    many = [res2[int(off2[i]):int(off2[i]) + int(k)] for i, k in enumerate(rng.integers(0, 400, 300))]
    batches = [seqs[:1], seqs[1:2] + [np.zeros(0, np.uint8)], [np.zeros(0, np.uint8)] + seqs[2:20],
               [seqs[20][:5], seqs[21][:9], seqs[22][:8]] + seqs[23:60], edge[:1], edge[1:], edge + seqs[:4],
               many, seqs[30:36], [s[:60] for s in seqs[:32]]]
    p = gpu.Params(*params)
    eligible = params[2] == 0 and params[0] >= 1
    ctx.set_option("small_fused", 1)
    try:
        # fused_inline 1: batches of <= 32 sequences and 2,048 residues travel
        # in the kernel arguments; 0: always from mapped memory
        for b, inl in [(b, inl) for inl in (1, 0) for b in batches]:
            ctx.set_option("fused_inline", inl)
            lens = np.array([0] + [len(x) for x in b], np.uint64)
            boff = np.cumsum(lens).astype(np.uint64) + np.uint64(3)
            bres = np.concatenate([np.frombuffer(b"MKV", np.uint8)] + list(b))
            want = oracle_lib.process_batch(table, bres, boff, params=params)
            fits = eligible and all(max(0, len(x) - 8) <= 2048 for x in b)
            for w in (3, 1, 2):
                f0 = ctx.stat("fused_batches")
                got = ctx.process_batch(bres, boff, p, want=w)
                assert ctx.stat("fused_batches") - f0 == (1 if fits else 0), (w, [len(x) for x in b][:5])
                assert got.n_windows == int(np.maximum(lens[1:].astype(np.int64) - 8, 0).sum())
                assert np.array_equal(got.hit_offsets, want.hit_offsets)
                if w & 1:
                    assert eq_fields(got.hits, want.hits)
                    assert not got.hits["flags"].any()
                if w & 2:
                    assert np.array_equal(got.call_offsets, want.call_offsets)
                    for f in ["start", "end", "count", "function_index"]:
                        assert np.array_equal(got.calls[f], want.calls[f]), f
                    assert np.array_equal(got.calls["weighted_hits"].view(np.uint32),
                                          want.calls["weighted_hits"].view(np.uint32))
                else:
                    assert not got.call_offsets.any()
            # OTU / best calls are never fused; the results stay the oracle's
            f0 = ctx.stat("fused_batches")
            assert_same(ctx.process_batch(bres, boff, p, want=7), want, len(b))
            assert ctx.stat("fused_batches") == f0
    finally:
        ctx.set_option("small_fused", 0)
        ctx.set_option("fused_inline", 1)


@pytest.mark.parametrize("params", PARAM_SETS[:4])
def test_small_batch_path_matches_oracle(small_world, aos_world, oracle_lib, gpu, params):
    """Batches of <= small_batch residues (the facade's process_aa_seq) take
    the one-wait path: host plan in the pinned blob, results stored into
    mapped memory.  Same records as the oracle, and the same best calls as the
    ordinary path (small_batch 0), for one sequence, a few with empties,
    sub-window and NUL-cut sequences, a mid-buffer start and one long sequence
    (wave scorer), on both resident layouts, with the small path's wave
    scorer and with the hybrid."""
    spec, table, img, ctx = small_world
    rng = np.random.default_rng(23)
    res, off = synth.make_queries(spec, 60, x_permille=5, q0=777)
    seqs = [res[int(off[i]):int(off[i + 1])].copy() for i in range(60)]
    seqs[3][40] = 0  # NUL cut
    long_seq = np.frombuffer(random_protein(rng, 20_000).encode(), np.uint8)
    # more than SMALL_GATHER_SEQ (256) sequences: scan and gather in separate launches
    res2, off2 = synth.make_queries(spec, 400, x_permille=5, q0=5000)
    many = [res2[int(off2[i]):int(off2[i]) + int(k)] for i, k in enumerate(rng.integers(0, 150, 400))]
    batches = [seqs[:1], seqs[1:2] + [np.zeros(0, np.uint8)], [np.zeros(0, np.uint8)] + seqs[2:20],
               [seqs[20][:5], seqs[21][:9], seqs[22][:8]] + seqs[23:60], [long_seq] + seqs[:3], many]
    p = gpu.Params(*params)
    for layout_ctx, sw in ((ctx, 1), (ctx, 0), (aos_world[1], 1)):
        layout_ctx.set_option("small_wave", sw)  # wave scorer (default) / the hybrid
        for b in batches:
            lens = np.array([0] + [len(x) for x in b], np.uint64)
            boff = np.cumsum(lens).astype(np.uint64) + np.uint64(3)
            bres = np.concatenate([np.frombuffer(b"MKV", np.uint8)] + list(b))
            want = oracle_lib.process_batch(table, bres, boff, params=params)
            layout_ctx.set_option("small_batch", 65536)
            got = layout_ctx.process_batch(bres, boff, p, want=7)
            assert_same(got, want, len(b))
            assert got.n_windows == int(np.maximum(lens[1:].astype(np.int64) - 8, 0).sum())
            small_best = layout_ctx.process_batch(bres, boff, p, want=gpu.WANT_BEST | gpu.WANT_HITS)
            assert eq_fields(small_best.hits, want.hits)
            for w in (1, 2):
                g = layout_ctx.process_batch(bres, boff, p, want=w)
                assert np.array_equal(g.hit_offsets, want.hit_offsets)
                assert np.array_equal(g.call_offsets, want.call_offsets if w == 2 else np.zeros_like(g.call_offsets))
            layout_ctx.set_option("small_batch", 0)
            try:
                ref_best = layout_ctx.process_batch(bres, boff, p, want=gpu.WANT_BEST).best
            finally:
                layout_ctx.set_option("small_batch", 1 << 21)
            assert np.array_equal(small_best.best, ref_best)
        layout_ctx.set_option("small_wave", 1)


@pytest.mark.parametrize("persist", [1, 3])
def test_probe_persist_matches_oracle(small_world, oracle_lib, gpu, persist):
    """probe_persist caps the line probe's grid (waves stride over the tiles:
    a 900k-residue batch gives each wave several tiles); same records as the
    oracle."""
    spec, table, img, ctx = small_world
    res, off = synth.make_queries(spec, 3000, x_permille=5, q0=9000)
    want = oracle_lib.process_batch(table, res, off)
    ctx.set_option("probe_persist", persist)
    try:
        got = ctx.process_batch(res, off, gpu.Params(5, 200, 0, 0))
    finally:
        ctx.set_option("probe_persist", 0)
    assert_same(got, want, 3000)


def test_probe_stream_two_contexts_match_oracle(small_world, oracle_lib, gpu):
    """probe_stream 1: two contexts' chained probes share the image's probe
    stream (entered on an event from each context's stream, left back to it);
    both contexts' alternating batches give the oracle's records."""
    spec, table, img, ctx = small_world
    other = gpu.Context(img)
    try:
        for c in (ctx, other):
            c.set_option("probe_stream", 1)
        for k in range(4):
            res, off = synth.make_queries(spec, 1500, x_permille=5, q0=20000 + 1500 * k)
            got = (ctx, other)[k % 2].process_batch(res, off, gpu.Params(5, 200, 0, 0))
            assert_same(got, oracle_lib.process_batch(table, res, off), 1500)
    finally:
        ctx.set_option("probe_stream", 0)
        other.close()
