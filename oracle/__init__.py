"""ctypes wrapper over the CPU oracle (oracle/kmer_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by close_kmers_amd/.  See kmer_oracle.h for
what the oracle restates and how it is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
REFDIR = os.path.join(HERE, "_ref")
LIB_PATH = os.path.join(BUILD, "liboracle.so")
QUERY_BIN = os.path.join(BUILD, "oracle_query")
REF_LIB_PATH = os.path.join(REFDIR, "libref.so")
REFERENCE_SRC = "/root/reference"

HIT_DTYPE = np.dtype(
    [
        ("which_kmer", "<u8"),
        ("otu_index", "<i4"),
        ("avg_from_end", "<u2"),
        ("reserved", "<u2"),
        ("function_index", "<i4"),
        ("function_wt", "<f4"),
        ("pos", "<u4"),
        ("seq", "<u4"),
    ]
)
assert HIT_DTYPE.itemsize == 32
CALL_DTYPE = np.dtype(
    [
        ("start", "<u4"),
        ("end", "<u4"),
        ("count", "<i4"),
        ("function_index", "<u4"),
        ("weighted_hits", "<f4"),
    ]
)
assert CALL_DTYPE.itemsize == 20
SIG_DTYPE = np.dtype(
    [
        ("which_kmer", "<u8"),
        ("otu_index", "<i4"),
        ("avg_from_end", "<u2"),
        ("pad", "<u2"),
        ("function_index", "<i4"),
        ("function_wt", "<f4"),
    ]
)
assert SIG_DTYPE.itemsize == 24

WANT_HITS, WANT_CALLS, WANT_OTU, WANT_BEST = 1, 2, 4, 8


class _Result(ctypes.Structure):
    _fields_ = [
        ("n_seq", ctypes.c_uint64),
        ("hit_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("hits", ctypes.c_void_p),
        ("call_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("calls", ctypes.c_void_p),
        ("otu_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("otus", ctypes.POINTER(ctypes.c_int32)),
        ("probes", ctypes.c_uint64),
        ("windows", ctypes.c_uint64),
        ("seconds", ctypes.c_double),
        ("best", ctypes.c_void_p),
    ]


# oracle_best: find_best_call per sequence (want WANT_BEST)
# kind / fi0 / fi1: which branch decided (0 no calls, 1 called, 2 ambiguous
# pair, 3 no call) and the function indices behind it (-1 where none)
BEST_DTYPE = np.dtype([("function_index", "<i4"), ("score", "<f4"), ("weighted_score", "<f4"),
                       ("score_offset", "<f4"), ("offset_set", "<i4"), ("kind", "<i4"), ("fi0", "<i4"),
                       ("fi1", "<i4")])


def build(ref: bool | None = None) -> None:
    """Compile the oracle (and, when /root/reference exists, oracle/_ref)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref is None:
        ref = os.path.isdir(REFERENCE_SRC)
    if ref:
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build(ref=False)
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_process_batch.argtypes = [
            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
            ctypes.POINTER(_Result),
        ]
        L.oracle_result_free.argtypes = [ctypes.POINTER(_Result)]
        L.oracle_build_table.argtypes = [ctypes.c_void_p, ctypes.c_uint64] + [ctypes.c_void_p] * 5 + [ctypes.c_uint64]
        L.oracle_build_table.restype = ctypes.c_int64
        L.oracle_find_best_call.argtypes = [
            ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
            ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_uint64,
            ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int),
        ]
        L.oracle_encode8.argtypes = [ctypes.c_char_p]
        L.oracle_encode8.restype = ctypes.c_uint64
        L.oracle_decode8.argtypes = [ctypes.c_uint64, ctypes.c_char_p]
        L.oracle_fasta_parse.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
        L.oracle_fasta_parse.restype = ctypes.c_void_p
        L.oracle_translate11.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
        L.oracle_translate11.restype = ctypes.c_void_p
        L.oracle_free.argtypes = [ctypes.c_void_p]
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        L.oracle_kmap_new.argtypes = [ctypes.c_int]
        L.oracle_kmap_new.restype = vp
        L.oracle_kmap_free.argtypes = [vp]
        L.oracle_kmap_add.argtypes = [vp, vp, vp, u64]
        L.oracle_kmap_lookup.argtypes = [vp, u64, vp, u64]
        L.oracle_kmap_lookup.restype = u64
        L.oracle_kmap_num_kmers.argtypes = [vp]
        L.oracle_kmap_num_kmers.restype = u64
        L.oracle_matrix_new.restype = vp
        L.oracle_matrix_free.argtypes = [vp]
        L.oracle_matrix_add.argtypes = [vp, vp, vp, vp, u64, vp, vp]
        L.oracle_matrix_pairs.argtypes = [vp, vp, vp, vp, vp]
        L.oracle_matrix_pairs.restype = u64
        L.oracle_fq_new.argtypes = [vp, u64, ctypes.POINTER(ctypes.c_char_p), u64, ctypes.c_char_p,
                                    ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_fq_new.restype = vp
        L.oracle_fq_free.argtypes = [vp]
        L.oracle_fq_process.argtypes = [vp, ctypes.c_char_p, u64]
        L.oracle_fq_process.restype = vp
        L.oracle_fq_fragments.argtypes = [ctypes.c_char_p, u64]
        L.oracle_fq_fragments.restype = vp
        _lib = L
    return _lib


def ref_lib():
    """The reference's own encoder / FASTA parser / translator / OTU sort
    (oracle/_ref/libref.so), or None when it was not built."""
    if not os.path.exists(REF_LIB_PATH):
        return None
    L = ctypes.CDLL(REF_LIB_PATH)
    L.ref_encode.argtypes = [ctypes.c_char_p]
    L.ref_encode.restype = ctypes.c_ulonglong
    L.ref_decode.argtypes = [ctypes.c_ulonglong, ctypes.c_char_p]
    L.ref_residue_code.argtypes = [ctypes.c_int]
    L.ref_residue_code.restype = ctypes.c_int
    L.ref_otu_finalize.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    L.ref_otu_finalize.restype = ctypes.c_int
    L.ref_fasta_parse.argtypes = [ctypes.c_char_p, ctypes.c_ulong]
    L.ref_fasta_parse.restype = ctypes.c_void_p
    L.ref_translate11.argtypes = [ctypes.c_char_p, ctypes.c_ulong]
    L.ref_translate11.restype = ctypes.c_void_p
    L.ref_free.argtypes = [ctypes.c_void_p]
    return L


@dataclass
class BatchResult:
    hit_offsets: np.ndarray
    hits: np.ndarray
    call_offsets: np.ndarray
    calls: np.ndarray
    otu_offsets: np.ndarray
    otus: np.ndarray  # (n, 2) int32
    probes: int
    windows: int
    seconds: float
    best: np.ndarray | None = None  # BEST_DTYPE per sequence with WANT_BEST


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    buf = (ctypes.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype).copy()


def process_batch(table: np.ndarray, residues: np.ndarray, offsets: np.ndarray,
                  params=(5, 200, 0, 0), want=WANT_HITS | WANT_CALLS | WANT_OTU,
                  n_threads: int = 1) -> BatchResult:
    """Run the oracle over a residue batch.  table: SIG_DTYPE array (or raw
    bytes of num_sigs*24); residues: uint8; offsets: uint64 (n_seq+1);
    params = (min_hits, max_gap, order_constraint, min_weighted_hits)."""
    L = lib()
    table = np.ascontiguousarray(table)
    num_sigs = table.nbytes // 24
    residues = np.ascontiguousarray(residues, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    p4 = np.asarray(params, dtype=np.int32)
    r = _Result()
    L.oracle_process_batch(table.ctypes.data, num_sigs, p4.ctypes.data,
                           residues.ctypes.data if residues.size else None,
                           offsets.ctypes.data, n, want, n_threads, ctypes.byref(r))
    try:
        ho = np.ctypeslib.as_array(r.hit_offsets, shape=(n + 1,)).copy()
        co = np.ctypeslib.as_array(r.call_offsets, shape=(n + 1,)).copy()
        oo = np.ctypeslib.as_array(r.otu_offsets, shape=(n + 1,)).copy()
        hits = _arr(r.hits, int(ho[-1]), HIT_DTYPE)
        calls = _arr(r.calls, int(co[-1]), CALL_DTYPE)
        otus = _arr(ctypes.cast(r.otus, ctypes.c_void_p).value, 2 * int(oo[-1]), np.int32).reshape(-1, 2)
        best = _arr(r.best, n, BEST_DTYPE) if r.best else None
        return BatchResult(ho, hits, co, calls, oo, otus, r.probes, r.windows, r.seconds, best)
    finally:
        L.oracle_result_free(ctypes.byref(r))


def _bad_seqs(got_off, want_off, rows_equal) -> np.ndarray:
    """Sequences whose rows differ: by count first, else by the rows that do."""
    gc, wc = np.diff(np.asarray(got_off, np.int64)), np.diff(np.asarray(want_off, np.int64))
    if len(gc) != len(wc):
        return np.arange(max(len(gc), len(wc)))
    if (gc != wc).any():
        return np.nonzero(gc != wc)[0]
    bad = np.nonzero(~rows_equal)[0] if rows_equal is not None else np.zeros(0, np.int64)
    return np.unique(np.searchsorted(np.asarray(want_off, np.int64), bad, side="right") - 1)


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def diff_batch(got, want: BatchResult, mask: int) -> dict:
    """Per output the sequences whose device results differ from the
    oracle's, compared as bits: got has the device's hit_offsets / hits
    (kgx_hit), call_offsets / calls, otu_offsets / otus (kgx_otu) and best
    (kgx_best_call) arrays; mask = the WANT_* bits both were run with.
    Returns {"hits": [...], "calls": [...], ...} of differing sequence
    indices (empty lists: equal)."""
    out = {}
    if mask & WANT_HITS:
        gh, wh = got.hits, want.hits
        eq = None
        if len(gh) == len(wh):
            eq = np.ones(len(wh), bool)
            for f in ("which_kmer", "otu_index", "avg_from_end", "function_index", "pos", "seq"):
                eq &= gh[f] == wh[f]
            eq &= _bits(gh["function_wt"]) == _bits(wh["function_wt"])
        out["hits"] = _bad_seqs(got.hit_offsets, want.hit_offsets, eq).tolist()
    if mask & WANT_CALLS:
        gc, wc = got.calls, want.calls
        eq = None
        if len(gc) == len(wc):
            eq = np.ones(len(wc), bool)
            for f in ("start", "end", "count", "function_index"):
                eq &= gc[f] == wc[f]
            eq &= _bits(gc["weighted_hits"]) == _bits(wc["weighted_hits"])
        out["calls"] = _bad_seqs(got.call_offsets, want.call_offsets, eq).tolist()
    if mask & WANT_OTU:
        go, wo = got.otus, want.otus
        eq = None
        if len(go) == len(wo):
            eq = (go["otu_index"] == wo[:, 0]) & (go["count"] == wo[:, 1])
        out["otus"] = _bad_seqs(got.otu_offsets, want.otu_offsets, eq).tolist()
    if mask & WANT_BEST:
        gb, wb = got.best, want.best
        if gb is None or wb is None or len(gb) != len(wb):
            out["best"] = list(range(len(want.hit_offsets) - 1))
        else:
            # kgx_best_call (kind, fi0, fi1, score, weighted_score, score_offset)
            # against find_best_call's outputs and decision (kguts.cc:1008-1199)
            k = gb["kind"]
            eq = (k == wb["kind"]) & (_bits(gb["score"]) == _bits(wb["score"]))
            eq &= _bits(gb["weighted_score"]) == _bits(wb["weighted_score"])
            eq &= (k == 0) | (_bits(gb["score_offset"]) == _bits(wb["score_offset"]))
            eq &= (k == 0) == (wb["offset_set"] == 0)
            eq &= ((k != 1) & (k != 2)) | (gb["fi0"] == wb["fi0"])
            eq &= (k != 2) | (gb["fi1"] == wb["fi1"])
            eq &= np.where(k == 1, gb["fi0"], -1) == wb["function_index"]
            out["best"] = np.nonzero(~eq)[0].tolist()
    return out


def build_table(num_sigs: int, keys, fI, oI, avg, wt) -> np.ndarray:
    """Sequential insert in key order (kguts.cc:202-222); returns SIG_DTYPE table."""
    L = lib()
    t = np.zeros(num_sigs, dtype=SIG_DTYPE)
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    fI = np.ascontiguousarray(fI, dtype=np.int32)
    oI = np.ascontiguousarray(oI, dtype=np.int32)
    avg = np.ascontiguousarray(avg, dtype=np.uint16)
    wt = np.ascontiguousarray(wt, dtype=np.float32)
    n = L.oracle_build_table(t.ctypes.data, num_sigs, keys.ctypes.data, fI.ctypes.data,
                             oI.ctypes.data, avg.ctypes.data, wt.ctypes.data, len(keys))
    if n < 0:
        raise ValueError("table would reach half full (kguts.cc:213-216)")
    return t


def find_best_call(calls: np.ndarray, functions: list[str]):
    """Returns (function_index, function, score, weighted_score, score_offset or None)."""
    L = lib()
    calls = np.ascontiguousarray(calls, dtype=CALL_DTYPE)
    names = (ctypes.c_char_p * max(1, len(functions)))(*[f.encode() for f in functions])
    fi = ctypes.c_int32()
    buf = ctypes.create_string_buffer(1 << 16)
    out3 = (ctypes.c_float * 3)()
    off_set = ctypes.c_int()
    L.oracle_find_best_call(calls.ctypes.data if len(calls) else None, len(calls), names,
                            len(functions), ctypes.byref(fi), buf, len(buf), out3,
                            ctypes.byref(off_set))
    return (fi.value, buf.value.decode(), out3[0], out3[1], out3[2] if off_set.value else None)


def encode8(kmer: str) -> int:
    return lib().oracle_encode8(kmer.encode())


def decode8(key: int) -> str:
    b = ctypes.create_string_buffer(9)
    lib().oracle_decode8(key, b)
    return b.value.decode()


def _take_string(p) -> bytes:
    b = ctypes.string_at(p)
    lib().oracle_free(p)
    return b


def fasta_parse(text: bytes) -> str:
    """FastaParser framing -> "id\tseq\n" lines."""
    return _take_string(lib().oracle_fasta_parse(text, len(text))).decode("latin-1")


def translate11(dna: str) -> str:
    b = dna.encode("latin-1")
    return _take_string(lib().oracle_translate11(b, len(b))).decode("latin-1")


def query_text(data_dir: str, fasta: str, mode: str, params: dict | None = None) -> bytes:
    """Run oracle/_build/oracle_query (handler-surface text)."""
    if not os.path.exists(QUERY_BIN):
        build(ref=False)
    args = [QUERY_BIN, data_dir, fasta, mode] + [f"{k}={v}" for k, v in (params or {}).items()]
    return subprocess.run(args, check=True, capture_output=True).stdout


class Kmap:
    """KmerPegMapping kmer_to_id_ (mode 0, append) / kmer_to_family_id_ (mode 1, set)."""

    def __init__(self, mode: int = 0):
        self.h = lib().oracle_kmap_new(mode)

    def add(self, kmers, ids) -> None:
        k = np.ascontiguousarray(kmers, dtype=np.uint64)
        v = np.ascontiguousarray(ids, dtype=np.uint32)
        lib().oracle_kmap_add(self.h, k.ctypes.data, v.ctypes.data, len(k))

    def lookup(self, kmer: int) -> np.ndarray:
        n = lib().oracle_kmap_lookup(self.h, int(kmer), None, 0)
        out = np.zeros(n, np.uint32)
        if n:
            lib().oracle_kmap_lookup(self.h, int(kmer), out.ctypes.data, n)
        return out

    @property
    def num_kmers(self) -> int:
        return lib().oracle_kmap_num_kmers(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_kmap_free(self.h)
            self.h = None


class Matrix:
    """One /matrix request's state (matrix_request.h:25-26)."""

    def __init__(self):
        self.h = lib().oracle_matrix_new()

    def add(self, kmap: Kmap, seq_ids, seq_lens, hit_off, hit_kmers) -> None:
        ids = np.ascontiguousarray(seq_ids, dtype=np.uint32)
        lens = np.ascontiguousarray(seq_lens, dtype=np.uint64)
        off = np.ascontiguousarray(hit_off, dtype=np.uint64)
        km = np.ascontiguousarray(hit_kmers, dtype=np.uint64)
        lib().oracle_matrix_add(self.h, kmap.h, ids.ctypes.data, lens.ctypes.data, len(ids),
                                off.ctypes.data, km.ctypes.data if len(km) else None)

    def pairs(self):
        """(id1, id2, count, score) arrays in distance_ (std::map) order."""
        n = lib().oracle_matrix_pairs(self.h, None, None, None, None)
        id1, id2 = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        cnt, sc = np.zeros(n, np.uint64), np.zeros(n, np.float32)
        if n:
            lib().oracle_matrix_pairs(self.h, id1.ctypes.data, id2.ctypes.data, cnt.ctypes.data,
                                      sc.ctypes.data)
        return id1, id2, cnt, sc

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_matrix_free(self.h)
            self.h = None


def fq_fragments(dna: bytes) -> list[tuple[int, str]]:
    """(frame, fragment) of the >10-aa fragments of a read, in the order the
    fq handler visits them (get_possible_proteins, dna_seq.cc:9-47)."""
    p = lib().oracle_fq_fragments(dna, len(dna))
    text = _take_string(p).decode()
    out = []
    for line in text.splitlines():
        f, s = line.split(":", 1)
        out.append((int(f), s))
    return out


class FqSession:
    """The fq handler restated (oracle/handlers_oracle.cpp) over a host table."""

    def __init__(self, table: np.ndarray, functions: list[str], genus: str = "", families: str = "",
                 nr: str = ""):
        self.table = np.ascontiguousarray(table)  # referenced, not copied, by the session
        names = (ctypes.c_char_p * max(1, len(functions)))(*[f.encode() for f in functions])
        self.h = lib().oracle_fq_new(self.table.ctypes.data, len(self.table), names, len(functions),
                                     genus.encode(), families.encode(), nr.encode())
        if not self.h:
            raise RuntimeError("oracle_fq_new failed")

    def process(self, fastq: bytes) -> bytes:
        return _take_string(lib().oracle_fq_process(self.h, fastq, len(fastq)))

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_fq_free(self.h)
            self.h = None
