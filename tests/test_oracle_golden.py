"""The oracle reproduces the committed golden handler text (regression of the
checker itself; tests/golden/make_golden.py wrote these files)."""
import os

import pytest

from helpers import GOLDEN


def _cases():
    for ds in ("scoring", "edge", "cap", "matrix", "fq", "lookup"):
        d = os.path.join(GOLDEN, ds)
        for f in sorted(os.listdir(d)):
            if f.startswith("expected_") and f.endswith(".txt"):
                yield ds, f


PARAMS = {
    "default": {}, "min_hits3": {"min_hits": "3"}, "max_gap300": {"max_gap": "300"},
    "max_gap50": {"max_gap": "50"}, "order": {"order_constraint": "1"},
    "min_weighted20": {"min_weighted_hits": "20"}, "min_hits2": {"min_hits": "2"},
    "bad_int": {"min_hits": "abc", "max_gap": " 120xyz"},
    # /lookup request parameters (tests/golden/make_golden.py LOOKUP_PARAMS)
    "fam_best": {"family_mode": "1", "find_best_match": "1"},
    "fam_best_ambig": {"family_mode": "1", "find_best_match": "1", "allow_ambiguous_functions": "1"},
    "fam_best_genus": {"family_mode": "1", "find_best_match": "1", "target_genus": "Escherichia"},
    "fam_list": {"family_mode": "1"},
    "fam_list_reps": {"family_mode": "1", "find_reps": "1", "kmer_hit_threhsold": "1"},
    "peg": {},
    "peg_all": {"kmer_hit_threhsold": "0"},
}


# the fq data set's family DB files (tests/golden/make_golden.py FQ_FILES)
FQ_FILES = {"genus": "genus.map", "families": "families.tsv", "nr": "nr.fasta"}


def case_params(ds, pname):
    p = dict(PARAMS[pname])
    if ds in ("fq", "lookup"):  # the lookup set reads the fq set's family DB
        p.update({k: os.path.join(GOLDEN, "fq", v) for k, v in FQ_FILES.items()})
    return p


def parse_case(fname):
    stem = fname[len("expected_"):-len(".txt")]
    for mode in ("query_details", "query_best", "query", "add", "matrix", "fq", "lookup"):
        if stem.startswith(mode + "_"):
            return mode, stem[len(mode) + 1:]
    raise ValueError(fname)


@pytest.mark.parametrize("ds,fname", list(_cases()))
def test_oracle_matches_golden(oracle_lib, ds, fname):
    mode, pname = parse_case(fname)
    d = os.path.join(GOLDEN, ds)
    got = oracle_lib.query_text(os.path.join(d, "data"), os.path.join(d, "input.fasta"), mode,
                                case_params(ds, pname))
    assert got == open(os.path.join(d, fname), "rb").read()
