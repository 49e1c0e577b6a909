"""fq path on the GPU: 6-frame code-11 fragments vs the oracle's
get_possible_proteins + split (dna_seq.cc:9-47), and their lookup."""
import ctypes

import numpy as np
import pytest

from helpers import pack, synthetic_table

pytestmark = pytest.mark.gpu


def _random_reads(rng, n):
    alphabet = np.frombuffer(b"ACGTACGTACGTacgtNnUuRYKMSWBDHVX.-", np.uint8)
    reads = []
    for i in range(n):
        L = int(rng.integers(0, 320)) if i % 7 else int(rng.integers(0, 12))
        if i % 3 == 0:
            b = alphabet[rng.integers(0, len(alphabet), L)]
        else:
            b = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, L)]
        reads.append(bytes(b))
    return reads


def test_fragments_match_oracle(gpu, oracle_lib):
    spec, table = synthetic_table(20000)
    rng = np.random.default_rng(3)
    reads = _random_reads(rng, 700)
    res, off = pack([("r", r) for r in reads])
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        f = ctx.fq_fragments(res, off)
        h = ctx.fragments_to_host(f)
    got = {}
    for i in range(f.n_fragments):
        s = bytes(h["residues"][int(h["offsets"][i]):int(h["offsets"][i + 1])]).decode()
        got.setdefault(int(h["read"][i]), []).append((int(h["frame"][i]), s))
    assert np.all(np.diff(h["read"].astype(np.int64)) >= 0)
    n = 0
    for r, dna in enumerate(reads):
        want = oracle_lib.fq_fragments(dna)
        assert got.get(r, []) == want, r
        n += len(want)
    assert n == f.n_fragments and n > 500


@pytest.mark.parametrize("fq_count,max_len", [(0, 1000), (1, 1000), (1, 257), (1, 200)])
def test_fragments_long_reads_both_count_passes(gpu, oracle_lib, fq_count, max_len):
    """Both count passes (lane-per-read stop scan / wave translation) give
    the emit pass the offsets that reproduce the oracle's fragments: reads of 0-1000 bases (several 64-base blocks
    of the stop scan, the emit's serial path past 194 bases), stop-rich and
    IUPAC-laden, at every start alignment."""
    spec, table = synthetic_table(20000)
    rng = np.random.default_rng(11)
    stoppy = np.frombuffer(b"TAAGTGATAGCTTATCAACGT", np.uint8)
    reads = []
    for i in range(600):
        L = int(rng.integers(0, max_len)) if i % 5 else int(rng.integers(0, 70))
        pool = stoppy if i % 4 == 0 else np.frombuffer(b"ACGTACGTACGTacgtNnUuRYKX", np.uint8)
        reads.append(bytes(pool[rng.integers(0, len(pool), L)]))
    res, off = pack([("r", r) for r in reads])
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        ctx.set_option("fq_count", fq_count)
        f = ctx.fq_fragments(res, off)
        h = ctx.fragments_to_host(f)
    got = {}
    for i in range(f.n_fragments):
        s = bytes(h["residues"][int(h["offsets"][i]):int(h["offsets"][i + 1])]).decode()
        got.setdefault(int(h["read"][i]), []).append((int(h["frame"][i]), s))
    n = 0
    for r, dna in enumerate(reads):
        want = oracle_lib.fq_fragments(dna)
        assert got.get(r, []) == want, (r, len(dna))
        n += len(want)
    assert n == f.n_fragments and n > 1000


def test_fragment_lookup_matches_oracle(gpu, oracle_lib):
    """Fragments fed to the lookup give the oracle's hits and calls."""
    from close_kmers_amd import synth
    spec, table = synthetic_table(40000)
    rng = np.random.default_rng(4)
    # reads that encode planted image proteins (so fragments hit), both strands
    src = synth.ALPHA[synth.source_residue_codes(np.arange(30))].reshape(30, -1)
    from tests_golden_codons import back_translate, revcomp
    reads = []
    for i in range(200):
        p = bytes(src[i % 30][int(rng.integers(0, 200)):][:60]).decode()
        d = back_translate(p, rng)
        reads.append((d if i % 2 else revcomp(d)).encode())
    res, off = pack([("r", r) for r in reads])
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        f = ctx.fq_fragments(res, off)
        h = ctx.fragments_to_host(f)
        got = ctx.run_fragments(f, gpu.Params(5, 200, 0, 0), want=3)
    want = oracle_lib.process_batch(table, h["residues"], h["offsets"], want=3)
    assert np.array_equal(got.hit_offsets, want.hit_offsets)
    assert np.array_equal(got.hits["which_kmer"], want.hits["which_kmer"])
    assert np.array_equal(got.calls["start"], want.calls["start"])
    assert np.array_equal(got.calls["weighted_hits"].view(np.uint32), want.calls["weighted_hits"].view(np.uint32))
    assert len(want.calls) > 50


def test_fq_handler_c_abi_matches_golden(gpu, oracle_lib):
    """kgx_fq_* (in-process handler) on the golden fq data set, in one block
    and in three blocks split mid-record."""
    import os
    from close_kmers_amd import image_files
    from helpers import GOLDEN
    d = os.path.join(GOLDEN, "fq")
    files = {k: os.path.join(d, v) for k, v in
             {"genus": "genus.map", "families": "families.tsv", "nr": "nr.fasta"}.items()}
    want = open(os.path.join(d, "expected_fq_default.txt"), "rb").read()
    fastq = open(os.path.join(d, "input.fasta"), "rb").read()
    table = image_files.read_image(os.path.join(d, "data"))
    with gpu.Image.from_table(table) as img:
        with gpu.FqHandler(img, os.path.join(d, "data"), **files) as fq:
            assert fq.process(fastq, True) == want
        with gpu.FqHandler(img, os.path.join(d, "data"), **files) as fq:
            cuts = [0, len(fastq) // 3 + 7, 2 * len(fastq) // 3 + 3, len(fastq)]
            out = b"".join(fq.process(fastq[a:b], b == len(fastq)) for a, b in zip(cuts, cuts[1:]))
        assert out == want


def test_fq_handler_without_families_matches_oracle(gpu, oracle_lib):
    """No family DB: reads without calls are skipped on the host (fast path);
    the output must still equal the oracle's."""
    import os
    from close_kmers_amd import image_files
    from helpers import GOLDEN
    d = os.path.join(GOLDEN, "fq")
    fastq = open(os.path.join(d, "input.fasta"), "rb").read()
    table = image_files.read_image(os.path.join(d, "data"))
    want = oracle_lib.query_text(os.path.join(d, "data"), os.path.join(d, "input.fasta"), "fq", {})
    assert want.count(b"\n") > 20
    with gpu.Image.from_table(table) as img, gpu.FqHandler(img, os.path.join(d, "data")) as fq:
        assert fq.process(fastq, True) == want


def test_fragments_of_long_and_empty_batches(gpu, oracle_lib):
    """Workgroups whose reads or output overflow the LDS staging take the
    global-memory path; an empty batch yields no fragments."""
    spec, table = synthetic_table(20000)
    rng = np.random.default_rng(8)
    reads = [bytes(np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(n))])
             for n in [5000, 0, 120000, 3, 900] + [150] * 60]
    res, off = pack([("r", r) for r in reads])
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        f = ctx.fq_fragments(res, off)
        h = ctx.fragments_to_host(f)
        empty = ctx.fq_fragments(np.zeros(0, np.uint8), np.zeros(1, np.uint64))
        assert empty.n_fragments == 0 and empty.n_residues == 0
    got = {}
    for i in range(f.n_fragments):
        s = bytes(h["residues"][int(h["offsets"][i]):int(h["offsets"][i + 1])]).decode()
        got.setdefault(int(h["read"][i]), []).append((int(h["frame"][i]), s))
    for r, dna in enumerate(reads):
        assert got.get(r, []) == oracle_lib.fq_fragments(dna), r


_CODE11 = "KNKNTTTTRSRSIIMIQHQHPPPPRRRRLLLLEDEDAAAAGGGGVVVV*Y*YSSSS*CWCLFLF"
_CLS = {c: i for i, c in enumerate("ACGT")} | {"U": 3}


def _translate_anchor(bases: bytes, anchor: int, n: int) -> str:
    """n residues from a fragment anchor: (first base) << 1 | reverse."""
    a, rev = anchor >> 1, anchor & 1
    out = []
    for i in range(n):
        if rev:
            cs = [_CLS.get(chr(bases[a - 3 * i - k]).upper()) for k in range(3)]
            cs = [None if c is None else 3 - c for c in cs]
        else:
            cs = [_CLS.get(chr(bases[a + 3 * i + k]).upper()) for k in range(3)]
        out.append("X" if None in cs else _CODE11[cs[0] * 16 + cs[1] * 4 + cs[2]])
    return "".join(out)


def _anchor_reads(rng):
    reads = _random_reads(rng, 500)
    stoppy = np.frombuffer(b"TAAGTGATAGCTTATCAACGT", np.uint8)
    for i in range(120):  # long reads: several stop-scan blocks, the unstaged path
        L = int(rng.integers(150, 1200))
        pool = stoppy if i % 3 == 0 else np.frombuffer(b"ACGTACGTACGTacgtNnUuRYKX", np.uint8)
        reads.append(bytes(pool[rng.integers(0, len(pool), L)]))
    reads += [bytes(np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 30000)])]
    return reads


@pytest.mark.parametrize("fq_count,fq_fused", [(0, 1), (1, 1), (1, 0)])
def test_fragment_anchors_translate_to_residues(gpu, oracle_lib, fq_count, fq_fused):
    """fq_residues 0: the same fragment records (offsets, read, frame, frame
    counts) as with residues, and each anchor translates to the fragment's
    residues (forward and reverse strand, IUPAC and lower case, long reads)."""
    spec, table = synthetic_table(20000)
    reads = _anchor_reads(np.random.default_rng(21))
    res, off = pack([("r", r) for r in reads])
    bases = bytes(res)
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        ctx.set_option("fq_count", fq_count)
        h1 = ctx.fragments_to_host(ctx.fq_fragments(res, off))
        ctx.set_option("fq_residues", 0)
        ctx.set_option("fq_fused", fq_fused)
        f0 = ctx.fq_fragments(res, off)
        h0 = ctx.fragments_to_host(f0)
    assert h0["residues"] is None and h0["read"] is None and f0.n_bases == len(bases)
    for k in ("offsets", "frame_counts"):
        assert np.array_equal(h0[k], h1[k]), k
    # read and frame of each fragment, from the per-(read, frame) counts
    fc = h0["frame_counts"]
    assert np.array_equal(np.repeat(np.arange(len(fc)) // 6, fc), h1["read"])
    assert np.array_equal(np.repeat(np.tile(np.array([1, 2, 3, -1, -2, -3], np.int8), len(fc) // 6), fc),
                          h1["frame"])
    o = h1["offsets"].astype(np.int64)
    for i in range(f0.n_fragments):
        want = bytes(h1["residues"][o[i]:o[i + 1]]).decode()
        assert _translate_anchor(bases, int(h0["anchors"][i]), len(want)) == want, i
    assert f0.n_fragments > 1000 and (h0["anchors"] & 1).sum() > 100


def test_fused_anchor_pass_equals_four_launches(gpu):
    """fq_fused 1 (count + look-back scan + anchors in one launch) writes the
    same offsets, anchors, per-(read, frame) counts and first fragments as
    the count / scan / tail / anchor launches, over thousands of tiles (the
    look-back walks many 64-tile steps), batch after batch on one context
    (epoch-tagged tile states, a shrinking and a growing batch), with empty
    and short reads (the overflow report: test_fragments_start_finish_ahead_schedule)."""
    spec, table = synthetic_table(20000)
    rng = np.random.default_rng(77)
    lens = rng.integers(0, 300, 200_000)
    lens[rng.choice(len(lens), 2000, replace=False)] = 0
    pool = np.frombuffer(b"ACGTACGTACGTNacgtRY", np.uint8)
    reads = [bytes(pool[rng.integers(0, len(pool), int(L))]) for L in lens]
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        ctx.set_option("fq_residues", 0)
        for n in (200_000, 3_000, 150_000, 1, 0, 200_000):
            res, off = pack([("r", r) for r in reads[:n]])
            out = []
            for fused in (0, 1):
                ctx.set_option("fq_fused", fused)
                f = ctx.fq_fragments(res, off)
                h = ctx.fragments_to_host(f)
                out.append((f.n_fragments, f.n_residues, h["offsets"], h["anchors"], h["frame_counts"]))
            assert out[0][0] == out[1][0] and out[0][1] == out[1][1], n
            for k in (2, 3, 4):
                assert np.array_equal(out[0][k], out[1][k]), (n, k)
            if n > 1000:
                assert out[1][0] > n


@pytest.mark.parametrize("fq_probe_j,fq_plan", [(1, 1), (2, 1), (4, 1), (0, 1), (1, 0)])
def test_fragment_lookup_dna_probe_matches_oracle(gpu, oracle_lib, fq_probe_j, fq_plan):
    """kgx_fq_run_device over anchors (the probe translating codons itself)
    gives the oracle's hits and calls over the translated fragments, and the
    same device results as the residue probe -- at each DNA probe tile
    (fq_probe_j; 0 = the context's probe_j, here 3)."""
    from close_kmers_amd import synth
    from tests_golden_codons import back_translate, revcomp
    spec, table = synthetic_table(40000)
    rng = np.random.default_rng(5)
    src = synth.ALPHA[synth.source_residue_codes(np.arange(30))].reshape(30, -1)
    reads = []
    for i in range(300):
        p = bytes(src[i % 30][int(rng.integers(0, 200)):][:60]).decode()
        d = bytearray(back_translate(p, rng).encode())
        if i % 5 == 0:  # ambiguity codes and lower case inside planted runs
            for j in rng.integers(0, len(d), 3):
                d[j] = b"NnRacgt"[int(rng.integers(0, 7))]
        d = bytes(d).decode()
        reads.append((d if i % 2 else revcomp(d)).encode())
    res, off = pack([("r", r) for r in reads])
    prm = gpu.Params(5, 200, 0, 0)
    with gpu.Image.from_table(table) as img, gpu.Context(img) as ctx:
        h = ctx.fragments_to_host(ctx.fq_fragments(res, off))
        ref = ctx.run_fragments(ctx.fq_fragments(res, off), prm, want=3)
        ctx.set_option("fq_residues", 0)
        ctx.set_option("fq_probe_j", fq_probe_j)
        ctx.set_option("fq_plan", fq_plan)
        if fq_probe_j == 0:
            ctx.set_option("probe_j", 3)
        f = ctx.fq_fragments(res, off)
        assert not f.residues
        got = ctx.run_fragments(f, prm, want=3)
        # the fragment pass wrote the lookup's plan; another batch on the
        # context replaces it, and the same fragments then plan again
        ctx.process_batch(h["residues"][:5000], np.array([0, 2000, 5000], np.uint64), prm)
        again = ctx.run_fragments(f, prm, want=3)
    want = oracle_lib.process_batch(table, h["residues"], h["offsets"], want=3)
    for r in (got, ref, again):
        assert np.array_equal(r.hit_offsets, want.hit_offsets)
        for k in ("which_kmer", "pos", "function_index", "otu_index", "avg_from_end"):
            assert np.array_equal(r.hits[k], want.hits[k]), k
        assert np.array_equal(r.call_offsets, want.call_offsets)
        for k in ("start", "end", "count", "function_index"):
            assert np.array_equal(r.calls[k], want.calls[k]), k
        assert np.array_equal(r.calls["weighted_hits"].view(np.uint32),
                              want.calls["weighted_hits"].view(np.uint32))
    assert len(want.calls) > 50 and len(want.hits) > 2000


_BACK = {"A": "GCT", "C": "TGT", "D": "GAT", "E": "GAA", "F": "TTT", "G": "GGT", "H": "CAT", "I": "ATT",
         "K": "AAA", "L": "CTT", "M": "ATG", "N": "AAT", "P": "CCT", "Q": "CAA", "R": "CGT", "S": "TCT",
         "T": "ACT", "V": "GTT", "W": "TGG", "Y": "TAT"}


def test_fq_handler_parallel_parse_matches_oracle(gpu, oracle_lib, tmp_path, monkeypatch):
    """A 40 MB FASTQ block is parsed by several threads (cut at record starts,
    each cut checked against the sequential parse): the handler's output must
    equal the oracle's, with irregular records at and around the cuts
    (quality lines starting with '@', blank lines, descriptions, non-letters
    and lower case in sequence lines, reads without calls), and equal the
    output of the same text fed as small blocks."""
    from close_kmers_amd import synth
    from helpers import data_dir_for
    spec, table = synthetic_table(30000)
    d = data_dir_for(str(tmp_path), table)
    rng = np.random.default_rng(31)
    src = synth.ALPHA[synth.source_residue_codes(np.arange(spec.n_src))].reshape(spec.n_src, -1)
    recs = []
    for i in range(130000):
        if i % 3:
            p = bytes(src[int(rng.integers(0, spec.n_src))]).decode()
            a = int(rng.integers(0, len(p) - 50))
            seq = "".join(_BACK[c] for c in p[a:a + 50])
        else:
            seq = "".join("ACGT"[x] for x in rng.integers(0, 4, 150))
        qual = "I" * len(seq)
        head = f"r{i}"
        if i % 997 == 0:
            qual = "@" + qual[1:]          # a quality line that looks like a header
        if i % 1009 == 0:
            head += "\tsome description"
        if i % 1013 == 0:
            seq = seq[:40].lower() + "N1-" + seq[40:]
        blank = "\n" if i % 1019 == 0 else ""
        recs.append(f"{blank}@{head}\n{seq}\n+\n{qual}\n")
    fastq = "".join(recs).encode()
    assert len(fastq) > 32 << 20
    path = tmp_path / "reads.fq"
    path.write_bytes(fastq)
    want = oracle_lib.query_text(d, str(path), "fq", {})
    assert want.count(b"\n") > 50000
    with gpu.Image.from_table(table) as img, gpu.FqHandler(img, d) as fq:
        assert fq.process(fastq, True) == want
        # parts of 1 MiB: ~40 parts parsed ahead by the worker threads
        monkeypatch.setenv("KGX_FQ_PART_KB", "1024")
        assert fq.process(fastq, True) == want
        monkeypatch.delenv("KGX_FQ_PART_KB")
    with gpu.Image.from_table(table) as img, gpu.FqHandler(img, d) as fq:
        cuts = [0] + sorted(int(x) for x in rng.integers(1, len(fastq), 12)) + [len(fastq)]
        out = b"".join(fq.process(fastq[a:b], b == len(fastq)) for a, b in zip(cuts, cuts[1:]))
    assert out == want


def test_fq_handler_fooled_cuts_match_oracle(gpu, oracle_lib, tmp_path, monkeypatch):
    """Every quality line starts with '@' and every sequence line with '+'
    (dropped by the parser as a non-letter), so a quality line followed two
    lines on by a '+' line looks like a record start to the cut search: many
    of a block's part boundaries are not record starts, the speculative parse
    of such a part is refused, and the rest of the block is parsed exactly
    from the true state.  The output must still be the oracle's."""
    from close_kmers_amd import synth
    from helpers import data_dir_for
    spec, table = synthetic_table(30000)
    d = data_dir_for(str(tmp_path), table)
    rng = np.random.default_rng(77)
    src = synth.ALPHA[synth.source_residue_codes(np.arange(spec.n_src))].reshape(spec.n_src, -1)
    recs = []
    for i in range(6000):
        p = bytes(src[int(rng.integers(0, spec.n_src))]).decode()
        a = int(rng.integers(0, len(p) - 50))
        seq = "".join(_BACK[c] for c in p[a:a + 50])
        recs.append(f"@q{i}\n+{seq}\n+\n@{'I' * len(seq)}\n")
    fastq = "".join(recs).encode()
    path = tmp_path / "fooled.fq"
    path.write_bytes(fastq)
    want = oracle_lib.query_text(d, str(path), "fq", {})
    assert want.count(b"\n") > 1000
    with gpu.Image.from_table(table) as img, gpu.FqHandler(img, d) as fq:
        for kb in ("16", "40", "100000"):
            monkeypatch.setenv("KGX_FQ_PART_KB", kb)
            assert fq.process(fastq, True) == want, kb


def test_fragments_start_finish_ahead_schedule(gpu):
    """kgx_fq_fragments_device_start / _finish: the same fragments as
    kgx_fq_fragments_device (anchors and residues); chunks sized one ahead on
    two contexts (bench_fq's schedule) give the same hits and calls as chunk
    by chunk; a span bound smaller than the reads' span is an error with
    nothing written past the buffers, and the context stays usable."""
    from close_kmers_amd import abi
    L = abi.lib()
    spec, table = synthetic_table(20000)
    rng = np.random.default_rng(8)
    Lr, n, chunk = 150, 6000, 1500
    bases = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n * Lr, dtype=np.uint8)].copy()
    off = np.arange(0, chunk * Lr + 1, Lr, dtype=np.uint64)
    prm = gpu.Params(5, 200, 0, 0)
    d_b, d_o = ctypes.c_void_p(), ctypes.c_void_p()
    abi.check(L.kgx_device_alloc(0, bases.nbytes, ctypes.byref(d_b)), "alloc")
    abi.check(L.kgx_device_alloc(0, off.nbytes, ctypes.byref(d_o)), "alloc")
    try:
        abi.check(L.kgx_memcpy_h2d(d_b, bases.ctypes.data, bases.nbytes), "h2d")
        abi.check(L.kgx_memcpy_h2d(d_o, off.ctypes.data, off.nbytes), "h2d")
        with gpu.Image.from_table(table) as img, gpu.Context(img) as c0, gpu.Context(img) as c1:
            for fq_res in (1, 0):
                for c in (c0, c1):
                    c.set_option("fq_residues", fq_res)
                # chunk by chunk (kgx_fq_fragments_device)
                want_frag, want_res = [], []
                for k in range(n // chunk):
                    f = abi.Fragments()
                    abi.check(L.kgx_fq_fragments_device(c0.handle, d_b.value + k * chunk * Lr, d_o, chunk,
                                                        ctypes.byref(f)), "frag")
                    want_frag.append(c0.fragments_to_host(f))
                    want_res.append(c0.run_fragments(f, prm))
                # sized one ahead over two contexts
                ctxs = [c0, c1]

                def start(k):
                    abi.check(L.kgx_fq_fragments_device_start(ctxs[k % 2].handle, d_b.value + k * chunk * Lr, d_o,
                                                              chunk, chunk * Lr), "start")

                def finish(k):
                    f = abi.Fragments()
                    abi.check(L.kgx_fq_fragments_finish(ctxs[k % 2].handle, ctypes.byref(f)), "finish")
                    return f
                start(0)
                f = finish(0)
                for k in range(n // chunk):
                    if k + 1 < n // chunk:
                        start(k + 1)
                    h = ctxs[k % 2].fragments_to_host(f)
                    for key, a in want_frag[k].items():
                        assert (a is None and h[key] is None) or np.array_equal(a, h[key]), (fq_res, k, key)
                    got = ctxs[k % 2].run_fragments(f, prm)
                    w = want_res[k]
                    assert np.array_equal(got.hit_offsets, w.hit_offsets)
                    assert np.array_equal(got.hits["which_kmer"], w.hits["which_kmer"])
                    assert np.array_equal(got.call_offsets, w.call_offsets)
                    if k + 1 < n // chunk:
                        f = finish(k + 1)
                assert sum(len(r.hits) for r in want_res) > 0
            # a span bound past which the reads run: an error, then the context still works
            abi.check(L.kgx_fq_fragments_device_start(c0.handle, d_b, d_o, chunk, 600), "start")
            f = abi.Fragments()
            assert L.kgx_fq_fragments_finish(c0.handle, ctypes.byref(f)) == -1
            assert L.kgx_fq_fragments_finish(c0.handle, ctypes.byref(f)) == -1  # nothing pending
            abi.check(L.kgx_fq_fragments_device(c0.handle, d_b, d_o, chunk, ctypes.byref(f)), "frag")
            assert f.n_fragments == len(want_frag[0]["offsets"]) - 1
    finally:
        L.kgx_device_free(d_b)
        L.kgx_device_free(d_o)
