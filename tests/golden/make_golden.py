"""Generate the committed golden fixtures under tests/golden/.

    python tests/golden/make_golden.py

Outputs (all small):
  scoring/   data dir + FASTA for the SCORING.txt worked example.  The 22 HIT
             windows, the protein id / length, the four CALL lines and the
             best call come from the reference (scoring_example.json); the
             residues between them and the hits SCORING.txt elides (the tail
             of the second gyrase run, the topo IV run and the last gyrase
             run) are completed here so that the four CALL lines come out as
             printed.  Expected text = the reference's lines, not the oracle's.
  edge/      data dir + FASTA of edge cases (empty / short / lower-case /
             ambiguous sequences, gap, pair-switch, carry-over, order
             constraint, OTU ties, multi-chunk sequences, invalid function
             indices) and the oracle's expected handler text per mode and
             parameter set.
  cap/       one 40,100-residue sequence whose single run overflows the
             40,000-entry hit buffer (kguts.cc:850-851), plus expected text.
  fq/        FASTQ reads back-translated (code 11, both strands, stops, N,
             lower case) from members of protein families, with a families
             file, a genus map and the NR proteins that fill
             kmer_to_family_id_: the fq request body (fq_process_request.cc:
             298-365) from the oracle.
  lookup/    /lookup (lookup_request.cc:153-482) over proteins against the fq
             data set's image and family DB: family mode with and without
             find_best_match (ambiguous calls, target genus, reps), and the
             peg mode after an /add of the same proteins.
  matrix/    protein families sharing signature k-mers (plus cross-family
             k-mers, repeated ids and unrelated proteins): the /add-then-
             /matrix body (matrix_request.cc:165-190) from the oracle.
The oracle (oracle/_build/oracle_query) produces every expected_*.txt; the
scoring case is additionally checked against the reference's own lines.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import oracle  # noqa: E402
from close_kmers_amd import image_files  # noqa: E402
from helpers import DesignedImage, encode, random_protein, write_fasta  # noqa: E402

MODES = ["query", "query_details", "query_best", "add"]
PARAM_SETS = {
    "default": {},
    "min_hits3": {"min_hits": "3"},
    "max_gap300": {"max_gap": "300"},
    "max_gap50": {"max_gap": "50"},
    "order": {"order_constraint": "1"},
    "min_weighted20": {"min_weighted_hits": "20"},
    "min_hits2": {"min_hits": "2"},
    "bad_int": {"min_hits": "abc", "max_gap": " 120xyz"},
}


def _fill(length: int, known: dict, rng) -> list:
    s = list(random_protein(rng, length))
    for p, ch in known.items():
        s[p] = ch
    return s


# --------------------------------------------------------------------------
def make_scoring(rng) -> None:
    ex = json.load(open(os.path.join(HERE, "scoring_example.json")))
    out = os.path.join(HERE, "scoring")
    fi = {v: int(k) for k, v in ex["functions"].items()}
    other = {}
    for _, _, name in ex["hits"]:
        if name not in fi and name not in other:
            other[name] = 100 + len(other)
    fi.update(other)
    L = ex["length"]
    known = {}
    for pos, kmer, _ in ex["hits"]:
        for j, ch in enumerate(kmer):
            assert known.get(pos + j, ch) == ch, "SCORING.txt HIT windows disagree"
            known[pos + j] = ch
    GY, TP = 7241, 7507
    # completion of the elided hits (see module docstring)
    extra = [(p, GY) for p in list(range(103, 110)) + [122]] + \
            [(p, TP) for p in range(162, 167)] + \
            [(p, GY) for p in list(range(182, 191)) + [209]]
    # weights: every hit of an emitted call weighs 1.0 except the last, which
    # brings the call's f32 sum to the printed value
    targets = {10: "8.7125", 99: "31.9442", 162: "9.1869", 182: "21.9685"}
    runs = {10: [10, 11, 12, 13, 14, 79], 99: list(range(99, 110)) + [122],
            162: list(range(162, 167)), 182: list(range(182, 191)) + [209]}
    weight = {}
    for start, members in runs.items():
        for p in members[:-1]:
            weight[p] = np.float32(1.0)
        weight[members[-1]] = np.float32(float(targets[start]) - (len(members) - 1))
        acc = np.float32(0.0)
        for p in members:
            acc = np.float32(acc + weight[p])
        assert f"{acc:g}" == targets[start], (start, acc)
    for attempt in range(100):
        seq = "".join(_fill(L, known, rng))
        img = DesignedImage()
        for pos, kmer, name in ex["hits"]:
            img.add(kmer, fi[name], oI=pos % 3, avg=L - pos, wt=float(weight.get(pos, np.float32(0.5))))
        for pos, f in extra:
            img.add(seq[pos:pos + 8], f, oI=pos % 3, avg=L - pos, wt=float(weight[pos]))
        table = img.table()
        res = np.frombuffer(seq.encode(), np.uint8)
        r = oracle.process_batch(table, res, np.array([0, L], np.uint64))
        want = sorted([p for p, _, _ in ex["hits"]] + [p for p, _ in extra])
        if list(r.hits["pos"]) == want:
            break
    else:
        raise RuntimeError("could not build a clean SCORING example")
    names = [f"function {i}" for i in range(7600)]
    for name, i in fi.items():
        names[i] = name
    data = os.path.join(out, "data")
    image_files.write_data_dir(data, table, names, ["otu0", "otu1", "otu2"])
    write_fasta(os.path.join(out, "input.fasta"), [(ex["protein_id"], seq)])
    for mode in MODES:
        txt = oracle.query_text(data, os.path.join(out, "input.fasta"), mode)
        open(os.path.join(out, f"expected_{mode}_default.txt"), "wb").write(txt)
    # the reference's own lines must come out of the oracle
    q = open(os.path.join(out, "expected_query_default.txt")).read().splitlines()
    assert q[0] == f"PROTEIN-ID\t{ex['protein_id']}\t{L}", q[0]
    for line, c in zip(q[1:5], ex["calls"]):
        assert line == "CALL\t" + "\t".join(str(x) for x in c), (line, c)
    b = open(os.path.join(out, "expected_add_default.txt")).read().splitlines()
    best = ex["best"]
    assert b[-1] == (f"BEST-CALL\t{ex['protein_id']}\t{best['function']}\t{best['score']}\t"
                     f"{best['weighted']}\t{best['offset']}"), b[-1]


# --------------------------------------------------------------------------
def make_edge(rng) -> None:
    out = os.path.join(HERE, "edge")
    img = DesignedImage()
    recs = []

    def seq_with(name, length, hit_spec, lower=False, edits=None):
        """hit_spec: list of (positions, fI, oI, wt or None)."""
        s = random_protein(rng, length)
        for positions, f, o, w in hit_spec:
            img.add_windows(s, positions, f, oI=o, wt=w, rng=rng)
        s2 = list(s)
        for p, ch in (edits or {}).items():
            s2[p] = ch
        s = "".join(s2)
        recs.append((name, s.lower() if lower else s))
        return s

    recs.append(("len0", ""))
    recs.append(("len1", "A"))
    seq_with("len8", 8, [([0], 1, 0, None)])
    seq_with("len9", 9, [([0], 1, 0, None)])
    seq_with("len10", 10, [([0, 1], 1, 0, None)])
    seq_with("len16", 16, [(range(0, 8), 2, 1, None)])
    base = seq_with("run_basic", 120, [(range(10, 20), 5, 1, None)])
    recs.append(("lower", base.lower()))
    seq_with("gap", 600, [(range(5, 13), 5, 2, None), (range(250, 258), 5, 2, None),
                          (range(320, 326), 6, 2, None)])
    seq_with("pair_switch", 200, [(range(10, 16), 5, 1, None), ([20, 21], 6, 1, None),
                                  (range(30, 37), 5, 3, None), ([50, 51, 52], 7, 4, None),
                                  (range(60, 66), 7, 4, None)])
    seq_with("singles", 160, [([3, 4, 5], 6, 0, None), (range(10, 15), 5, 0, None),
                              ([40], 7, 0, None), ([42], 8, 0, None), ([43], 9, 0, None),
                              ([51], 7, 0, None), ([61], 10, 0, None), ([79], 5, 0, None),
                              ([92, 93], 6, 0, None), (range(99, 110), 5, 0, None)])
    seq_with("ambig", 100, [(range(5, 95), 11, 5, None)], edits={40: "X", 60: "*", 80: "B", 81: "x"})
    seq_with("otu_mix", 150, [(range(10, 20), 8, 3, None), (range(20, 25), 8, 7, None),
                              (range(25, 30), 8, 12, None), (range(30, 35), 8, -1, None),
                              (range(35, 40), 8, 7, None), (range(40, 42), 8, 9, None),
                              (range(60, 70), 12, 3, None), (range(70, 80), 12, 4, None)])
    # order constraint: consistent avg (L - pos) then inconsistent avg
    s = random_protein(rng, 200)
    for p in range(10, 22):
        img.add(s[p:p + 8], 9, 2, 200 - p, 1.25)
    for p in range(30, 38):
        img.add(s[p:p + 8], 9, 2, 5, 1.5)
    for p in range(40, 50):
        img.add(s[p:p + 8], 9, 2, 200 - p + (p % 3) * 10, 0.75)
    recs.append(("order", s))
    seq_with("multichunk", 1300, [(range(300, 341, 2), 10, 6, None), (range(630, 652), 10, 6, None),
                                  (range(655, 662), 13, 6, None), (range(950, 1001, 5), 10, 7, None),
                                  (range(1250, 1285), 14, 8, None)])
    seq_with("invalid_fi", 120, [(range(10, 17), 5000, 0, None), (range(40, 47), -3, 0, None)])
    seq_with("weights", 120, [(range(10, 16), 15, 0, 0.125), (range(40, 52), 16, 0, 3.3)])
    seq_with("ambiguous_best", 300, [(range(10, 18), 20, 0, None), (range(40, 47), 21, 0, None),
                                     (range(80, 85), 22, 0, None), (range(120, 126), 20, 0, None),
                                     (range(160, 164), 23, 1, None), (range(200, 204), 22, 0, None)])
    seq_with("tie_two", 200, [(range(10, 17), 24, 0, 1.0), (range(60, 67), 25, 0, 1.0)])
    # a repeated 8-mer: both occurrences hit the same bucket
    rep = random_protein(rng, 20)
    img.add(rep[0:8], 17, 1, 3, 2.0)
    recs.append(("repeat", rep + random_protein(rng, 30) + rep[0:8] + random_protein(rng, 10)))
    recs.append(("star_first", "*" + base[1:]))
    # merge F1 F2 F1 with weak interior (find_best_call :1063-1086)
    seq_with("merge_f1f2f1", 300, [(range(10, 18), 30, 0, None), ([40, 41], 31, 0, None),
                                    (range(60, 64), 30, 0, None), (range(100, 105), 32, 0, None)])

    table = img.table()
    names = [f"function {i}" for i in range(40)]
    names[5] = "DNA gyrase subunit B (EC 5.99.1.3)"
    names[6] = "DNA topoisomerase IV subunit B (EC 5.99.1.3)"
    names[7] = "hypothetical protein"
    names[20], names[21], names[22] = "Zeta kinase", "alpha kinase", "Beta kinase"
    names[24], names[25] = "tie function B", "tie function A"
    data = os.path.join(out, "data")
    image_files.write_data_dir(data, table, names, [f"otu{i}" for i in range(16)])
    fasta = os.path.join(out, "input.fasta")
    write_fasta(fasta, recs)
    for mode in MODES:
        for pname, params in PARAM_SETS.items():
            txt = oracle.query_text(data, fasta, mode, params)
            open(os.path.join(out, f"expected_{mode}_{pname}.txt"), "wb").write(txt)


# --------------------------------------------------------------------------
def make_cap(rng) -> None:
    """One run longer than MAX_HITS_PER_SEQ - 2 = 39,998 buffered hits, then a
    different function: the frozen buffer's last pair triggers the flush."""
    out = os.path.join(HERE, "cap")
    img = DesignedImage()
    unit = random_protein(rng, 23)  # period 23: 23 distinct cyclic windows
    body = (unit * (40100 // 23 + 2))[:40100]
    for p in range(23):
        img.add(body[p:p + 8], 3, p % 4, 40000 - p, float(np.float32(0.25 + (p % 7) * 0.125)))
    tail_unit = random_protein(rng, 19)
    tail = (tail_unit * 4)[:60]
    for p in range(19):
        img.add(tail[p:p + 8], 4, 9, 7, 1.5)
    seq = body + random_protein(rng, 12) + tail
    table = img.table(num_sigs=3769)
    data = os.path.join(out, "data")
    image_files.write_data_dir(data, table, [f"function {i}" for i in range(8)], ["o"])
    fasta = os.path.join(out, "input.fasta")
    write_fasta(fasta, [("capped", seq)])
    for mode in ["query", "add", "query_best"]:
        txt = oracle.query_text(data, fasta, mode)
        open(os.path.join(out, f"expected_{mode}_default.txt"), "wb").write(txt)


def make_matrix(rng) -> None:
    out = os.path.join(HERE, "matrix")
    img = DesignedImage()
    bases = [random_protein(rng, int(rng.integers(120, 200))) for _ in range(6)]
    for f, b in enumerate(bases):
        img.add_windows(b, range(0, len(b) - 8, 2), f, oI=f % 3 - 1, rng=rng)
    shared = random_protein(rng, 40)  # a motif planted in several families
    img.add_windows(shared, range(0, 32), 7, rng=rng)
    recs = []
    for f, b in enumerate(bases):
        for m in range(5):
            s = list(b)
            for p in rng.integers(0, len(s), int(len(s) * 0.08)):
                s[p] = "ACDEFGHIKLMNPQRSTVWY"[int(rng.integers(0, 20))]
            s = "".join(s)
            if f % 2 == 0 and m < 3:
                at = int(rng.integers(0, len(s) - 40))
                s = s[:at] + shared + s[at + 40:]
            recs.append((f"fig|6666666.{f}.peg.{m}", s))
    recs.append(("fig|6666666.9.peg.1", random_protein(rng, 150)))   # unrelated
    recs.append(("fig|6666666.0.peg.1", bases[0]))                   # repeated id
    recs.append(("fig|6666666.9.peg.2", bases[3][10:90]))            # fragment
    order = rng.permutation(len(recs))
    recs = [recs[i] for i in order]
    table = img.table()
    data = os.path.join(out, "data")
    image_files.write_data_dir(data, table, [f"function {i}" for i in range(8)], ["o0", "o1"])
    fasta = os.path.join(out, "input.fasta")
    write_fasta(fasta, recs)
    txt = oracle.query_text(data, fasta, "matrix")
    assert txt.count(b"\n") > 50
    open(os.path.join(out, "expected_matrix_default.txt"), "wb").write(txt)


CODE11 = ("FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
          "TTTTTTTTTTTTTTTTCCCCCCCCCCCCCCCCAAAAAAAAAAAAAAAAGGGGGGGGGGGGGGGG",
          "TTTTCCCCAAAAGGGGTTTTCCCCAAAAGGGGTTTTCCCCAAAAGGGGTTTTCCCCAAAAGGGG",
          "TCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAGTCAG")


def back_translate(prot: str, rng) -> str:
    codons = {}
    for i, aa in enumerate(CODE11[0]):
        codons.setdefault(aa, []).append(CODE11[1][i] + CODE11[2][i] + CODE11[3][i])
    return "".join(codons[a][int(rng.integers(0, len(codons[a])))] for a in prot)


def revcomp(dna: str) -> str:
    return dna[::-1].translate(str.maketrans("ACGTacgt", "TGCAtgca"))


FQ_FILES = {"genus": "genus.map", "families": "families.tsv", "nr": "nr.fasta"}


def make_fq(rng) -> None:
    out = os.path.join(HERE, "fq")
    data = os.path.join(out, "data")
    img = DesignedImage()
    n_fam = 8
    bases = [random_protein(rng, 160) for _ in range(n_fam)]
    fam_fn = [0, 1, 2, 2, 3, 3, 3, 4]  # families sharing a function share pgf rollups
    for f, b in enumerate(bases):
        img.add_windows(b, range(0, len(b) - 8), fam_fn[f], rng=rng)
    members = []
    for f, b in enumerate(bases):
        for m in range(4):
            s = list(b)
            for p in rng.integers(0, len(s), 6):
                s[p] = "ACDEFGHIKLMNPQRSTVWY"[int(rng.integers(0, 20))]
            members.append((f, m, "".join(s)))
    functions = [f"function {i}" for i in range(6)]
    image_files.write_data_dir(data, img.table(), functions, ["o"])
    genera = ["Escherichia", "Bacillus", "Mycoplasma"]
    with open(os.path.join(out, "genus.map"), "w") as g:
        g.write("Escherichia\t561\nBacillus\t1386\n")  # Mycoplasma left unmapped
    with open(os.path.join(out, "families.tsv"), "w") as fam:
        for f, m, s in members:
            gf = f"GF{f // 2:08d}"              # two local families per global family
            genus = genera[(f + m) % 3]
            local = str(100 + f)
            fam.write(f"{gf}\t2\t2\tfig|{1000 + f}.{m}.peg.{m}\t{len(s)}\t{functions[fam_fn[f]]}\t"
                      f"{local}\t{genus}\t{local}\n")
    write_fasta(os.path.join(out, "nr.fasta"),
                [(f"fig|{1000 + f}.{m}.peg.{m}", s) for f, m, s in members] +
                [("fig|9999.1.peg.1", bases[0])])  # no family: skipped
    recs = []
    for i in range(60):
        f, m, s = members[int(rng.integers(0, len(members)))]
        at = int(rng.integers(0, len(s) - 50))
        prot = s[at:at + 50]
        kind = i % 6
        if kind == 1:  # a stop codon splits the protein
            prot = prot[:20] + "*" + prot[21:]
        dna = back_translate(prot, rng)
        if kind == 2:
            dna = revcomp(dna)
        if kind == 3:
            dna = "AC" + dna[:-2]  # frame 3
        if kind == 4:
            dna = dna.lower()
            dna = dna[:30] + "N" + dna[31:]
        if kind == 5:
            dna = "".join("ACGT"[int(x)] for x in rng.integers(0, 4, 150))  # random read
        recs.append((f"read{i}", dna))
    recs.append(("", "ACGT" * 30))  # an empty id is skipped
    with open(os.path.join(out, "input.fasta"), "w") as fq:  # FASTQ despite the name
        for rid, dna in recs:
            fq.write(f"@{rid} desc\n{dna}\n+\n{'I' * len(dna)}\n")
    args = {k: os.path.join(out, v) for k, v in FQ_FILES.items()}
    txt = oracle.query_text(data, os.path.join(out, "input.fasta"), "fq", args)
    assert txt.count(b"\n") > 20
    open(os.path.join(out, "expected_fq_default.txt"), "wb").write(txt)
    return bases, members


LOOKUP_PARAMS = {
    "fam_best": {"family_mode": "1", "find_best_match": "1"},
    "fam_best_ambig": {"family_mode": "1", "find_best_match": "1", "allow_ambiguous_functions": "1"},
    "fam_best_genus": {"family_mode": "1", "find_best_match": "1", "target_genus": "Escherichia"},
    "fam_list": {"family_mode": "1"},
    "fam_list_reps": {"family_mode": "1", "find_reps": "1", "kmer_hit_threhsold": "1"},
    "peg": {},
    "peg_all": {"kmer_hit_threhsold": "0"},
}


def make_lookup(rng, bases, members) -> None:
    """/lookup over proteins, against the fq data set's image and family DB."""
    out = os.path.join(HERE, "lookup")
    src = os.path.join(HERE, "fq")
    table = image_files.read_image(os.path.join(src, "data"))
    image_files.write_data_dir(os.path.join(out, "data"), table, [f"function {i}" for i in range(6)], ["o"])
    recs = []
    for f, m, s in members[::3]:
        recs.append((f"fig|{1000 + f}.{m}.peg.{m}", s))  # ids the families file knows
    for i in range(6):
        f, m, s = members[int(rng.integers(0, len(members)))]
        t = list(s)
        for p in rng.integers(0, len(t), 25):
            t[p] = "ACDEFGHIKLMNPQRSTVWY"[int(rng.integers(0, 20))]
        recs.append((f"query{i}", "".join(t)))
    recs.append(("chimera", bases[2][:70] + bases[4][70:140]))  # two functions: "F1 ?? F2"
    recs.append(("chimera2", bases[1][:80] + bases[6][80:150]))
    recs.append(("random", random_protein(rng, 120)))
    recs.append(("short", bases[0][:12]))
    fasta = os.path.join(out, "input.fasta")
    write_fasta(fasta, recs)
    files = {k: os.path.join(src, v) for k, v in FQ_FILES.items()}
    for pname, params in LOOKUP_PARAMS.items():
        txt = oracle.query_text(os.path.join(out, "data"), fasta, "lookup", {**params, **files})
        open(os.path.join(out, f"expected_lookup_{pname}.txt"), "wb").write(txt)


def main() -> None:
    oracle.build(ref=False)
    make_scoring(np.random.default_rng(2024_08_07))
    make_edge(np.random.default_rng(12345))
    make_cap(np.random.default_rng(777))
    make_matrix(np.random.default_rng(4242))
    bases, members = make_fq(np.random.default_rng(31337))
    make_lookup(np.random.default_rng(2718), bases, members)
    print("golden fixtures written under", HERE)


if __name__ == "__main__":
    main()
