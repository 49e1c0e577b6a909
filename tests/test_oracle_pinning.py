"""Pin the CPU oracle (oracle/kmer_oracle.cpp) before trusting it.

* against the reference's own code that builds here (oracle/_ref/libref.so:
  kmer_encoder.cc, kguts.h KmerOtuStats, fasta_parser.cc, trans_table.cc);
* against the known answers printed in the reference's SCORING.txt.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from helpers import GOLDEN

ALPHA = "ACDEFGHIKLMNPQRSTVWY"


@pytest.fixture(scope="module")
def ref(oracle_lib):
    L = oracle_lib.ref_lib()
    if L is None:
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    return L


def test_encoder_matches_reference_kmer_encoder(oracle_lib, ref):
    rng = np.random.default_rng(1)
    kmers = ["AAAAAAAA", "YYYYYYYY", "ACDEFGHI", "WWWWWWWW"]
    kmers += ["".join(ALPHA[i] for i in rng.integers(0, 20, 8)) for _ in range(3000)]
    # invalid residues -> MAX_ENCODED + 1 in both (encoded_aa_kmer, kmer_encoder.h:212-225)
    kmers += ["AAAXAAAA", "aaaaaaaa", "ACDEFGH*", "BCDEFGHI", "ACDEFGHU"]
    for k in kmers:
        assert oracle_lib.encode8(k) == ref.ref_encode(k.encode()), k
    buf = __import__("ctypes").create_string_buffer(9)
    for k in kmers[:500]:
        key = oracle_lib.encode8(k)
        if key < 20 ** 8:
            ref.ref_decode(key, buf)
            assert buf.value.decode() == oracle_lib.decode8(key) == k


def test_residue_map_matches_reference(ref):
    # every byte but 255, which KmerEncoder leaves uninitialised (kmer_encoder.cc:9)
    for c in range(255):
        want = ALPHA.index(chr(c)) if chr(c) in ALPHA else 20
        assert ref.ref_residue_code(c) == want, c


def test_otu_finalize_matches_reference(ref):
    import ctypes
    rng = np.random.default_rng(7)
    from oracle import lib  # noqa: F401  (oracle's finalize runs inside process_batch)
    for trial in range(200):
        n = int(rng.integers(0, 40))
        otus = rng.integers(-3, 30, n).astype(np.int32)
        counts = rng.integers(1, 6, n).astype(np.int32)
        out = np.zeros(2 * n + 2, np.int32)
        k = ref.ref_otu_finalize(otus.ctypes.data, counts.ctypes.data, n, out.ctypes.data)
        got = [tuple(x) for x in out[:2 * k].reshape(-1, 2)]
        # the same multiset through the oracle's own finalize (std::sort, less_second)
        m = {}
        for o, c in zip(otus, counts):
            m[int(o)] = m.get(int(o), 0) + int(c)
        exp = _oracle_finalize(m)
        assert got == exp, (trial, got, exp)


def _oracle_finalize(m):
    """Run the oracle's OtuStats::finalize via a tiny driver image: one hit per
    OTU count, all in one run of one function."""
    import oracle
    from helpers import DesignedImage, random_protein
    rng = np.random.default_rng(len(m) * 7919 + sum(m.values()))
    total = sum(m.values())
    if total == 0:
        return []
    seq = random_protein(rng, total + 8 + 1)
    img = DesignedImage()
    p = 0
    for o in sorted(m):
        for _ in range(m[o]):
            img.add(seq[p:p + 8], 1, o, 0, 1.0)
            p += 1
    table = img.table()
    res = np.frombuffer(seq.encode(), np.uint8)
    r = oracle.process_batch(table, res, np.array([0, len(seq)], np.uint64), params=(1, 200, 0, 0))
    if len(np.unique(r.hits["pos"])) != total:
        pytest.skip("random filler collided")
    return [tuple(x) for x in r.otus]


def test_fasta_framing_matches_reference_parser(oracle_lib, ref):
    import ctypes
    cases = [
        b">a\nACDE\nFGH\n>b desc here\nKLMN\n\n>c\n\n",
        b">x\r\nAC*D\r\n>y\tdef\nAAAA",
        b"junk\n>a\nAC1DE\n>b\nXX\n",
        b">only_id",
        b"",
        b">a\n*ABC\nDEF\n>b\n",
        b">a\nabc\n  \n>b\nAAA\n",
    ]
    rng = np.random.default_rng(3)
    for _ in range(300):
        parts = []
        for i in range(int(rng.integers(0, 6))):
            parts.append(b">" + f"id{i}".encode() + (b" d" if rng.random() < .3 else b"") + b"\n")
            for _ in range(int(rng.integers(0, 4))):
                parts.append(bytes(rng.choice(list(b"ACDEFGHIKLMNPQRSTVWYxX*\r 1>"), int(rng.integers(0, 30)))) + b"\n")
        cases.append(b"".join(parts))
    for text in cases:
        p = ref.ref_fasta_parse(text, len(text))
        want = ctypes.string_at(p).decode("latin-1")
        ref.ref_free(p)
        assert oracle_lib.fasta_parse(text) == want, text


def test_translate_code11_matches_reference(ref):
    import ctypes
    from oracle import translate11
    rng = np.random.default_rng(11)
    for _ in range(300):
        dna = bytes(rng.choice(list(b"ACGTacgtuUNRY"), int(rng.integers(0, 40))))
        p = ref.ref_translate11(dna, len(dna))
        want = ctypes.string_at(p).decode()
        ref.ref_free(p)
        assert translate11(dna.decode()) == want, dna


def test_find_best_call_scoring_txt_known_answer(oracle_lib):
    """SCORING.txt:15-19 calls -> :84-97 (merged 10-129 = 18, 40.6567; best =
    gyrase, score 28, weighted 62.6252, offset 23)."""
    ex = json.load(open(os.path.join(GOLDEN, "scoring_example.json")))
    calls = np.array([(s, e, c, f, np.float32(w)) for s, e, c, f, _, w in ex["calls"]],
                     dtype=oracle_lib.CALL_DTYPE)
    names = ["function %d" % i for i in range(7600)]
    for k, v in ex["functions"].items():
        names[int(k)] = v
    fi, fn, score, wscore, off = oracle_lib.find_best_call(calls, names)
    best = ex["best"]
    assert (fi, fn, score, f"{wscore:g}", off) == (best["function_index"], best["function"], best["score"],
                                                  best["weighted"], best["offset"])
    # the collapse step's first region (SCORING.txt:84)
    w = np.float32(calls["weighted_hits"][0]) + np.float32(calls["weighted_hits"][1])
    assert f"{np.float32(w):g}" == ex["collapsed_first"][4]


def test_scoring_example_oracle_text_is_reference_text(oracle_lib):
    """The completed SCORING example through the oracle prints the reference's
    four CALL lines (SCORING.txt:16-19) and its best call (:93-97)."""
    ex = json.load(open(os.path.join(GOLDEN, "scoring_example.json")))
    d = os.path.join(GOLDEN, "scoring")
    txt = oracle_lib.query_text(os.path.join(d, "data"), os.path.join(d, "input.fasta"), "query").decode()
    lines = txt.splitlines()
    assert lines[0] == f"PROTEIN-ID\t{ex['protein_id']}\t{ex['length']}"
    assert lines[1:5] == ["CALL\t" + "\t".join(str(x) for x in c) for c in ex["calls"]]
    det = oracle_lib.query_text(os.path.join(d, "data"), os.path.join(d, "input.fasta"),
                                "query_details").decode().splitlines()
    hits = [l.split("\t") for l in det if l.startswith("HIT\t")]
    got = {(int(h[1]), h[2]) for h in hits}
    for pos, kmer, _ in ex["hits"]:
        assert (pos, kmer) in got
