"""Code-11 back-translation helpers for tests (mirrors tests/golden/make_golden.py)."""
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
