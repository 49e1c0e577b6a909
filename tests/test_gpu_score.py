"""The run scorers against each other and the oracle: the lane machine
(score_variant 2), the wave-parallel scorer (1) and the default hybrid (0:
lanes, with sequences over 2,048 windows on the wave scorer): gather_hits /
process_set_of_hits (kguts.cc:734-877) on hit-dense batches built to hit
every rule -- gap breaks, pair switches with carry-over, runs that span many
64-hit chunks, fragments whose hits share a chunk, empty and hitless
sequences, a sequence past the 40,000-hit buffer -- under many parameter
sets.  Calls, hit flags and OTU tallies must be bit-identical."""
import numpy as np
import pytest

from helpers import DesignedImage, pack, random_protein

pytestmark = pytest.mark.gpu

# (min_hits, max_gap, order_constraint, min_weighted_hits)
SCORE_PARAMS = [(5, 200, 0, 0), (0, 200, 0, 0), (1, 3, 0, 0), (2, 0, 0, 0), (3, 10, 0, 2), (5, -1, 0, 0),
                (2, 2147483647, 0, 0), (4, 40, 0, 10), (-1, 5, 0, 0)]


def make_run_world(gpu):
    """Source proteins whose 8-mers carry functions in blocks: stretches of one
    function, alternating pairs (switches) and singletons, random weights
    (some 0 and negative zero) and OTUs."""
    rng = np.random.default_rng(2024)
    img = DesignedImage()
    sources = [random_protein(rng, int(rng.integers(200, 700))) for _ in range(60)]
    for si, src in enumerate(sources):
        p = 0
        while p + 8 <= len(src):
            blk = int(rng.integers(1, 12))
            style = int(rng.integers(0, 4))
            base = int(rng.integers(0, 6))
            for q in range(p, min(p + blk, len(src) - 7)):
                if style == 0:
                    f = base
                elif style == 1:
                    f = base + ((q - p) & 1)
                elif style == 2:
                    f = base + ((q - p) // 2 & 1)
                else:
                    f = int(rng.integers(0, 6))
                w = [0.0, -0.0, 1.0, float(np.float32(rng.random() * 3))][int(rng.integers(0, 4))]
                if rng.random() < 0.15:
                    continue  # a miss inside the stretch
                img.add(src[q:q + 8], f, int(rng.integers(-1, 9)), int(rng.integers(0, 400)), w)
            p += blk
    table = img.table()
    gimg = gpu.Image.from_table(table)
    ctx = gpu.Context(gimg)
    return rng, sources, table, gimg, ctx


@pytest.fixture(scope="module")
def run_world(gpu):
    rng, sources, table, gimg, ctx = make_run_world(gpu)
    yield rng, sources, table, ctx
    ctx.close()
    gimg.close()


def _batch(rng, sources, n):
    recs = []
    for i in range(n):
        kind = i % 9
        src = sources[int(rng.integers(0, len(sources)))]
        if kind == 0:
            s = ""
        elif kind == 1:
            s = random_protein(rng, int(rng.integers(0, 40)))  # hitless (mostly)
        elif kind in (2, 3):  # a short fragment (fq-like)
            a = int(rng.integers(0, len(src) - 20))
            s = src[a:a + int(rng.integers(9, 30))]
        else:  # a long stretch with gaps (X runs) and mutations
            a = int(rng.integers(0, len(src) // 2))
            s = list(src[a:])
            for _ in range(int(rng.integers(0, 6))):
                p = int(rng.integers(0, len(s)))
                s[p:p + int(rng.integers(1, 30))] = ["X"] * int(rng.integers(1, 30))
            s = "".join(s)
            if kind == 8:
                s = s + "".join(sources[int(rng.integers(0, len(sources)))] for _ in range(4))
        recs.append((f"s{i}", s))
    return pack(recs)


def _same(a, b, want):
    assert np.array_equal(a.hit_offsets, b.hit_offsets)
    if want & 1:
        for f in ("which_kmer", "pos", "function_index", "flags"):
            assert np.array_equal(a.hits[f], b.hits[f]), f
    if want & 2:
        assert np.array_equal(a.call_offsets, b.call_offsets)
        for f in ("start", "end", "count", "function_index"):
            assert np.array_equal(a.calls[f], b.calls[f]), f
        assert np.array_equal(a.calls["weighted_hits"].view(np.uint32), b.calls["weighted_hits"].view(np.uint32))
    if want & 4:
        assert np.array_equal(a.otu_offsets, b.otu_offsets)
        assert np.array_equal(a.otus["otu_index"], b.otus["otu_index"])
        assert np.array_equal(a.otus["count"], b.otus["count"])


@pytest.mark.parametrize("params", SCORE_PARAMS)
def test_wave_scorer_matches_lane_scorer(run_world, gpu, params):
    rng, sources, table, ctx = run_world
    res, off = _batch(rng, sources, 3000)
    ctx.set_option("host_chunks", 1)
    n_calls = 0
    for want in (1, 3, 5, 7, 2, 4):
        ctx.set_option("score_variant", 2)
        a = ctx.process_batch(res, off, gpu.Params(*params), want=want)
        ctx.set_option("score_variant", 1)
        b = ctx.process_batch(res, off, gpu.Params(*params), want=want)
        _same(a, b, want)
        if want == 3:
            n_calls = len(b.calls)
    assert n_calls > 20 or params[1] in (0, -1)  # max_gap 0 / -1 (wraps): every hit breaks its run


@pytest.mark.parametrize("params", SCORE_PARAMS[:5])
def test_wave_scorer_matches_oracle(run_world, gpu, oracle_lib, params):
    rng, sources, table, ctx = run_world
    res, off = _batch(rng, sources, 1500)
    ctx.set_option("score_variant", 1)
    got = ctx.process_batch(res, off, gpu.Params(*params), want=7)
    want = oracle_lib.process_batch(table, res, off, params=params)
    assert np.array_equal(got.hit_offsets, want.hit_offsets)
    assert np.array_equal(got.call_offsets, want.call_offsets)
    for f in ("start", "end", "count", "function_index"):
        assert np.array_equal(got.calls[f], want.calls[f]), f
    assert np.array_equal(got.calls["weighted_hits"].view(np.uint32), want.calls["weighted_hits"].view(np.uint32))
    assert np.array_equal(got.otu_offsets, want.otu_offsets)
    assert np.array_equal(got.otus["otu_index"], want.otus[:, 0])
    assert np.array_equal(got.otus["count"], want.otus[:, 1])


def test_scorers_on_long_sequences(run_world, gpu):
    """Sequences past RUN_CAP windows (the lane machine inside every variant),
    between 2,048 and RUN_CAP windows (the hybrid's wave range) and short ones,
    with empties: lane (2), wave (1) and hybrid (0) agree bit for bit."""
    rng, sources, table, ctx = run_world
    def longp(n):
        return "".join(sources[int(rng.integers(0, len(sources)))] for _ in range(n))
    res0, off0 = _batch(rng, sources, 300)
    short = [(f"s{i}", bytes(res0[int(off0[i]):int(off0[i + 1])])) for i in range(300)]
    recs = short[:100] + [("huge", longp(100))] + short[100:150] + [("mid1", longp(8)), ("mid2", longp(40))] \
        + short[150:250] + [("edge", "A" * 2056), ("mid3", longp(70)), ("", "")] + short[250:]
    assert len(recs[100][1]) > 40100
    res, off = pack(recs)
    for params in SCORE_PARAMS[:5]:
        outs = []
        for v in (2, 1, 0):
            ctx.set_option("score_variant", v)
            outs.append(ctx.process_batch(res, off, gpu.Params(*params), want=7))
        _same(outs[0], outs[1], 7)
        _same(outs[0], outs[2], 7)
    ctx.set_option("score_variant", 0)


@pytest.mark.parametrize("params", SCORE_PARAMS[:3])
def test_hybrid_scorer_with_long_sequences_matches_oracle(run_world, gpu, oracle_lib, params):
    rng, sources, table, ctx = run_world
    res0, off0 = _batch(rng, sources, 400)
    recs = [(f"s{i}", bytes(res0[int(off0[i]):int(off0[i + 1])])) for i in range(400)]
    for k in range(3):
        recs.insert(100 * (k + 1), (f"long{k}", "".join(sources[(7 * k + j) % len(sources)] for j in range(12))))
    res, off = pack(recs)
    ctx.set_option("score_variant", 0)
    got = ctx.process_batch(res, off, gpu.Params(*params), want=7)
    want = oracle_lib.process_batch(table, res, off, params=params)
    assert np.array_equal(got.hit_offsets, want.hit_offsets)
    assert np.array_equal(got.call_offsets, want.call_offsets)
    for f in ("start", "end", "count", "function_index"):
        assert np.array_equal(got.calls[f], want.calls[f]), f
    assert np.array_equal(got.calls["weighted_hits"].view(np.uint32), want.calls["weighted_hits"].view(np.uint32))
    assert np.array_equal(got.otus["count"], want.otus[:, 1])
