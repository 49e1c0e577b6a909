"""Synthetic signature images and query batches.

The same generators exist as HIP kernels in csrc/kgx_synth.hip (used by
bench.py to build 1B-entry images directly in HBM); these numpy versions make
the identical bytes on the host for the parity tests.  Every random draw is
``rnd(seed, i) = mix64(seed ^ mix64(i))`` with splitmix64's finaliser, so host
and device agree bit for bit.

Image (n_keys entries, num_sigs buckets):
  * ``n_src = (n_keys // 4) // 292`` source proteins of 300 residues; entry
    ``e < n_src*292`` is window ``pos = e % 292`` of source ``s = e // 292``:
    key = its 8-mer, function_index = s % 100000, avg_from_end = 300 - pos;
  * the remaining entries are uniform keys in [0, 20^8) with random
    function_index < 100000 and avg_from_end < 300;
  * otu_index = -1 (as the builder writes, build_signature_kmers.cc:708-709);
  * function_wt = k * 1e-4f, k uniform in [1000, 50000) (non-dyadic f32);
  * duplicate keys: the lowest entry id wins (the builder's de-dup keeps one).
Queries (n_seq x length):
  * even q: planted -- a copy of source protein rnd(Q_SRC, q) % n_src with 10%
    substitutions; odd q: uniform residues; optional X at x_permille.
"""
from __future__ import annotations

import numpy as np

ALPHA = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
MAX_ENCODED = 20 ** 8
EMPTY_KEY = MAX_ENCODED + 1
SRC_LEN = 300
SRC_WIN = SRC_LEN - 8  # windows probed in a 300-aa protein (positions 0..291)

SEED_SRC = 0x5EED0001      # source-protein residues
SEED_KEY = 0x5EED0002      # random keys
SEED_FI = 0x5EED0012       # random function indices
SEED_AVG = 0x5EED0022      # random avg_from_end
SEED_WT = 0x5EED0032       # weights
SEED_Q_SRC = 0x5EED0003    # planted query -> source
SEED_Q_SUB = 0x5EED0013    # substitution draw
SEED_Q_RES = 0x5EED0023    # random residue draw
SEED_Q_X = 0x5EED0033      # ambiguity draw

# build_signature_kmers.cc:862-865 (list order kept: it is not sorted)
BUILDER_PRIMES = [3769, 6337, 12791, 24571, 51043, 101533, 206933, 400187, 821999,
                  2000003, 4000037, 8000009, 16000057, 32000011, 64000031, 128000003,
                  248000009, 508000037, 1073741824, 1400303159, 2147483648, 1190492993,
                  3559786523, 6461346257]

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def builder_num_sigs(n_keys: int) -> int:
    """First listed size p > 3*n_keys (build_signature_kmers.cc:870-883)."""
    for p in BUILDER_PRIMES:
        if p > 3 * n_keys:
            return p
    raise ValueError(f"no table size for {n_keys} keys")


def mix64(x):
    """splitmix64 finaliser over uint64 arrays (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def rnd(seed: int, idx):
    return mix64(np.uint64(seed) ^ mix64(np.asarray(idx, dtype=np.uint64)))


def source_residue_codes(src_ids) -> np.ndarray:
    """(len(src_ids), 300) residue codes 0..19 of the given source proteins."""
    s = np.asarray(src_ids, dtype=np.uint64)[:, None]
    idx = s * np.uint64(SRC_LEN) + np.arange(SRC_LEN, dtype=np.uint64)[None, :]
    return (rnd(SEED_SRC, idx) % np.uint64(20)).astype(np.uint8)


def encode_windows(codes: np.ndarray, n_win: int) -> np.ndarray:
    """Big-endian base-20 codes of windows 0..n_win-1 of each row."""
    key = np.zeros((codes.shape[0], n_win), dtype=np.uint64)
    for j in range(8):
        key = key * np.uint64(20) + codes[:, j:j + n_win].astype(np.uint64)
    return key


class ImageSpec:
    """n_keys fixes the generator (its source proteins); the image holds the
    first n_entries entries of its stream (default n_keys; entries past n_keys
    are random keys) -- kgx_image_build_synthetic_distinct picks n_entries so
    that exactly n_distinct keys are stored."""

    def __init__(self, n_keys: int, num_sigs: int | None = None, n_entries: int | None = None):
        self.n_keys = int(n_keys)
        self.n_entries = int(n_entries) if n_entries is not None else self.n_keys
        self.num_sigs = int(num_sigs) if num_sigs else builder_num_sigs(self.n_keys)
        self.n_src = (self.n_keys // 4) // SRC_WIN
        if 2 * self.n_entries >= self.num_sigs:
            raise ValueError("more keys than a half-full table allows (kguts.cc:213)")

    def entries_for_distinct(self, n_distinct: int) -> int:
        """The smallest n such that entries [0, n) hold n_distinct distinct keys."""
        hi = n_distinct + n_distinct // 8 + 1024
        keys = self.entries(0, hi)[0]
        _, first = np.unique(keys, return_index=True)
        if len(first) < n_distinct:
            raise ValueError("stream too short")
        return int(np.sort(first)[n_distinct - 1]) + 1

    def entries(self, lo: int = 0, hi: int | None = None):
        """Raw entries [lo, hi) before de-duplication: keys, fI, oI, avg, wt."""
        hi = self.n_entries if hi is None else hi
        e = np.arange(lo, hi, dtype=np.uint64)
        keys = np.zeros(hi - lo, dtype=np.uint64)
        fI = np.zeros(hi - lo, dtype=np.int32)
        avg = np.zeros(hi - lo, dtype=np.uint16)
        n_src_e = self.n_src * SRC_WIN
        src_mask = e < np.uint64(n_src_e)
        if src_mask.any():
            es = e[src_mask]
            s = es // np.uint64(SRC_WIN)
            pos = (es % np.uint64(SRC_WIN)).astype(np.int64)
            us, inv = np.unique(s, return_inverse=True)
            codes = source_residue_codes(us)
            win = encode_windows(codes, SRC_WIN)
            keys[src_mask] = win[inv, pos]
            fI[src_mask] = (s % np.uint64(100000)).astype(np.int32)
            avg[src_mask] = (SRC_LEN - pos).astype(np.uint16)
        rm = ~src_mask
        if rm.any():
            er = e[rm]
            keys[rm] = rnd(SEED_KEY, er) % np.uint64(MAX_ENCODED)
            fI[rm] = (rnd(SEED_FI, er) % np.uint64(100000)).astype(np.int32)
            avg[rm] = (rnd(SEED_AVG, er) % np.uint64(SRC_LEN)).astype(np.uint16)
        k = (rnd(SEED_WT, e) % np.uint64(49000) + np.uint64(1000)).astype(np.float32)
        wt = (k * np.float32(1e-4)).astype(np.float32)
        oI = np.full(hi - lo, -1, dtype=np.int32)
        return keys, fI, oI, avg, wt

    def unique_entries(self):
        """Entries with duplicate keys removed (lowest entry id kept), in id order."""
        keys, fI, oI, avg, wt = self.entries()
        _, first = np.unique(keys, return_index=True)
        first.sort()
        return keys[first], fI[first], oI[first], avg[first], wt[first]


def make_queries(spec: ImageSpec | None, n_seq: int, length: int = SRC_LEN,
                 x_permille: int = 0, q0: int = 0):
    """Residue bytes (uint8, concatenated) and offsets (uint64, n_seq+1) for
    queries q0 .. q0+n_seq-1."""
    q = np.arange(q0, q0 + n_seq, dtype=np.uint64)
    i = np.arange(length, dtype=np.uint64)
    idx = q[:, None] * np.uint64(length) + i[None, :]
    rand_codes = (rnd(SEED_Q_RES, idx) % np.uint64(20)).astype(np.uint8)
    codes = rand_codes.copy()
    n_src = spec.n_src if spec is not None else 0
    if n_src > 0 and length <= SRC_LEN:
        planted = (q % np.uint64(2)) == np.uint64(0)
        if planted.any():
            src = rnd(SEED_Q_SRC, q[planted]) % np.uint64(n_src)
            scodes = source_residue_codes(src)[:, :length]
            keep = (rnd(SEED_Q_SUB, idx[planted]) % np.uint64(10)) != np.uint64(0)
            codes[planted] = np.where(keep, scodes, rand_codes[planted])
    res = ALPHA[codes]
    if x_permille > 0:
        xm = (rnd(SEED_Q_X, idx) % np.uint64(1000)) < np.uint64(x_permille)
        res = np.where(xm, np.uint8(ord("X")), res)
    offsets = np.arange(n_seq + 1, dtype=np.uint64) * np.uint64(length)
    return np.ascontiguousarray(res.reshape(-1)), offsets
