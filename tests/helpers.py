"""Shared test helpers: designed images, FASTA writing, synthetic datasets."""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from close_kmers_amd import image_files, synth

ALPHA = "ACDEFGHIKLMNPQRSTVWY"
MAX_ENCODED = 20 ** 8


def encode(kmer: str) -> int:
    v = 0
    for ch in kmer:
        v = v * 20 + ALPHA.index(ch)
    return v


def random_protein(rng: np.random.Generator, n: int) -> str:
    return "".join(ALPHA[i] for i in rng.integers(0, 20, n))


@dataclass
class DesignedImage:
    """Entries keyed by 8-mer; first insertion wins (the builder de-dups)."""
    entries: dict = field(default_factory=dict)  # key -> (fI, oI, avg, wt)
    order: list = field(default_factory=list)

    def add(self, kmer: str, fI: int, oI: int = -1, avg: int = 0, wt: float = 1.0) -> None:
        k = encode(kmer)
        if k not in self.entries:
            self.entries[k] = (fI, oI, avg, np.float32(wt))
            self.order.append(k)

    def add_windows(self, seq: str, positions, fI: int, oI: int = -1, wt=None, avg=None,
                    rng: np.random.Generator | None = None) -> None:
        for p in positions:
            w = wt if wt is not None else float(np.float32(0.1 + 4.9 * rng.random())) if rng is not None else 1.0
            a = avg if avg is not None else max(0, len(seq) - p)
            self.add(seq[p:p + 8], fI, oI, a, w)

    def arrays(self):
        keys = np.array(self.order, dtype=np.uint64)
        fI = np.array([self.entries[k][0] for k in self.order], dtype=np.int32)
        oI = np.array([self.entries[k][1] for k in self.order], dtype=np.int32)
        avg = np.array([self.entries[k][2] for k in self.order], dtype=np.uint16)
        wt = np.array([self.entries[k][3] for k in self.order], dtype=np.float32)
        return keys, fI, oI, avg, wt

    def table(self, num_sigs: int | None = None):
        import oracle
        keys, fI, oI, avg, wt = self.arrays()
        n = num_sigs or synth.builder_num_sigs(max(1, len(keys)))
        return oracle.build_table(n, keys, fI, oI, avg, wt)


def write_fasta(path: str, records) -> None:
    with open(path, "w") as f:
        for rid, seq in records:
            f.write(f">{rid}\n{seq}\n")


def pack(records):
    """(id, seq) list -> residues uint8, offsets uint64."""
    seqs = [s.encode() if isinstance(s, str) else s for _, s in records]
    off = np.zeros(len(seqs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    res = np.frombuffer(b"".join(seqs), dtype=np.uint8) if seqs else np.zeros(0, np.uint8)
    return res.copy(), off


def synthetic_table(n_keys: int, num_sigs: int | None = None):
    import oracle
    spec = synth.ImageSpec(n_keys, num_sigs)
    k, f, o, a, w = spec.unique_entries()
    return spec, oracle.build_table(spec.num_sigs, k, f, o, a, w)


def data_dir_for(tmpdir: str, table, n_functions: int = 100000, otus=None) -> str:
    funcs = [f"function {i}" for i in range(n_functions)]
    return image_files.write_data_dir(tmpdir, table, funcs, otus)


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
