"""Host-side checks of the fq path (no GPU)."""
import os
import re

from tests_golden_codons import CODE11, back_translate, revcomp

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "close_kmers_amd", "csrc")


def test_device_code11_table_rederived_from_the_reference_table_text():
    """kCode11 in kgx_fq.hip = trans_table.cc:8-15 re-indexed A0 C1 G2 T3."""
    src = open(os.path.join(CSRC, "kgx_fq.hip")).read()
    table = re.search(r'kCode11\[66\] = "([A-Z*]+)"', src).group(1)
    code = {"A": 0, "C": 1, "G": 2, "T": 3}
    want = ["?"] * 64
    for i, aa in enumerate(CODE11[0]):
        want[code[CODE11[1][i]] * 16 + code[CODE11[2][i]] * 4 + code[CODE11[3][i]]] = aa
    assert table == "".join(want) + "X"


def test_oracle_fragments_of_a_worked_read(oracle_lib):
    import numpy as np
    rng = np.random.default_rng(0)
    p1, p2 = "MKTAYIAKQRQISFVKSHFSRQ", "LEERLGLIEVQAPILSRVGDGT"
    dna = back_translate(p1 + "*" + p2, rng)
    frags = oracle_lib.fq_fragments(dna.encode())
    assert (1, p1) in frags and (1, p2) in frags
    rc = oracle_lib.fq_fragments(revcomp(dna).encode())
    assert (-1, p1) in rc and (-1, p2) in rc
    # a base outside ACGTU makes an 'X' codon, which does not split
    bad = dna[:9] + "N" + dna[10:]
    assert any(f == 1 and "X" in s for f, s in oracle_lib.fq_fragments(bad.encode()))
