"""ctypes binding of include/kgx.h (the C ABI of libkgx.so).

Everything here calls the HIP engine; there is no CPU fallback.  Loading the
library works without a GPU (symbols only); compute entry points return
KGX_EDEVICE when no gfx950 device is visible, and the wrappers raise.
"""
from __future__ import annotations

import ctypes
import weakref
import os
import re

import numpy as np

from . import build as _build

KGX_OK = 0
ERRORS = {-1: "EINVAL", -2: "EIO", -3: "EFORMAT", -4: "ENOMEM", -5: "EDEVICE", -6: "ERANGE",
          -7: "EFULL", -8: "EBUSY"}
KGX_EBUSY = -8
KGX_EDEVICE = -5
KGX_EINVAL = -1
KGX_WAIT_SPIN, KGX_WAIT_SLEEP, KGX_WAIT_BLOCK = 0, 1, 2
WANT_HITS, WANT_CALLS, WANT_OTU, WANT_BEST = 1, 2, 4, 8
HIT_IN_RUN, HIT_OTU = 1, 2

HIT_DTYPE = np.dtype([("which_kmer", "<u8"), ("otu_index", "<i4"), ("avg_from_end", "<u2"),
                      ("flags", "<u2"), ("function_index", "<i4"), ("function_wt", "<f4"),
                      ("pos", "<u4"), ("seq", "<u4")])
CALL_DTYPE = np.dtype([("start", "<u4"), ("end", "<u4"), ("count", "<i4"),
                       ("function_index", "<u4"), ("weighted_hits", "<f4")])
OTU_DTYPE = np.dtype([("otu_index", "<i4"), ("count", "<i4")])
# kgx_best_call: find_best_call's decision (kind 0 no calls, 1 called, 2 ambiguous pair, 3 no call)
BEST_DTYPE = np.dtype([("kind", "<i4"), ("fi0", "<i4"), ("fi1", "<i4"), ("score", "<f4"),
                       ("weighted_score", "<f4"), ("score_offset", "<f4")])
SIG_DTYPE = np.dtype([("which_kmer", "<u8"), ("otu_index", "<i4"), ("avg_from_end", "<u2"),
                      ("pad", "<u2"), ("function_index", "<i4"), ("function_wt", "<f4")])
assert HIT_DTYPE.itemsize == 32 and CALL_DTYPE.itemsize == 20 and SIG_DTYPE.itemsize == 24


class KgxError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        super().__init__(f"{what}: {ERRORS.get(code, code)} ({last_error()})")


class Params(ctypes.Structure):
    _fields_ = [("min_hits", ctypes.c_int32), ("max_gap", ctypes.c_int32),
                ("order_constraint", ctypes.c_int32), ("min_weighted_hits", ctypes.c_int32)]


class Result(ctypes.Structure):
    _fields_ = [("n_seq", ctypes.c_uint32), ("hit_offsets", ctypes.c_void_p),
                ("hits", ctypes.c_void_p), ("call_offsets", ctypes.c_void_p),
                ("calls", ctypes.c_void_p), ("otu_offsets", ctypes.c_void_p),
                ("otus", ctypes.c_void_p), ("n_windows", ctypes.c_uint64), ("best", ctypes.c_void_p)]


class DeviceResult(ctypes.Structure):
    _fields_ = [("n_seq", ctypes.c_uint32), ("tile_windows", ctypes.c_uint32),
                ("window_base", ctypes.c_void_p), ("hit_mask", ctypes.c_void_p),
                ("hit_count", ctypes.c_void_p), ("call_count", ctypes.c_void_p),
                ("hits_hot", ctypes.c_void_p), ("hits_cold", ctypes.c_void_p),
                ("calls", ctypes.c_void_p), ("best", ctypes.c_void_p), ("hit_format", ctypes.c_uint32),
                ("otu_count", ctypes.c_void_p), ("otus", ctypes.c_void_p)]


HIT_PLANES, HIT_PACKED16 = 0, 1


class RollupResult(ctypes.Structure):
    _fields_ = [("n_seq", ctypes.c_uint32), ("offsets", ctypes.c_void_p), ("rows", ctypes.c_void_p),
                ("n_events", ctypes.c_uint64)]


# kgx_rollup_row: LookupRequest's sequence_accumulated_score_t with its id
ROLLUP_DTYPE = np.dtype([("id", "<u4"), ("hit_count", "<u4"), ("hit_total", "<u4"), ("weighted_total", "<f4")])
ROLLUP_PEG, ROLLUP_FAMILY = 0, 1


class HitChunk(ctypes.Structure):
    _fields_ = [("seq_begin", ctypes.c_uint32), ("seq_end", ctypes.c_uint32), ("record_words", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("hit_begin", ctypes.c_uint64), ("records", ctypes.c_void_p),
                ("mask", ctypes.c_void_p), ("window_start", ctypes.c_void_p)]


class CompactResult(ctypes.Structure):
    _fields_ = [("r", Result), ("n_chunks", ctypes.c_uint32), ("chunks", ctypes.POINTER(HitChunk))]


class HostProfile(ctypes.Structure):
    _fields_ = [("chunks", ctypes.c_uint32), ("streamed", ctypes.c_uint32)] + \
        [(k, ctypes.c_double) for k in ("wall_ms", "stage_ms", "h2d_ms", "device_ms", "gather_ms", "d2h_ms",
                                        "expand_ms")] + [("h2d_bytes", ctypes.c_uint64), ("d2h_bytes", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


def hits_from_planes(hot: np.ndarray, cold: np.ndarray) -> np.ndarray:
    """kgx_hit records from kgx_device_result's two hit planes (uint32 [n, 4]
    each): hot = {avg | flags << 16, function_index, function_wt, pos},
    cold = {which_kmer lo, hi, otu_index, seq}."""
    hot = np.asarray(hot, np.uint32).reshape(-1, 4)
    cold = np.asarray(cold, np.uint32).reshape(-1, 4)
    w = np.empty((len(hot), 8), np.uint32)
    w[:, 0:3] = cold[:, 0:3]
    w[:, 3:7] = hot
    w[:, 7] = cold[:, 3]
    return w.view(HIT_DTYPE).reshape(-1)


class Fragments(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_uint32), ("n_fragments", ctypes.c_uint32),
                ("n_residues", ctypes.c_uint64), ("residues", ctypes.c_void_p),
                ("offsets", ctypes.c_void_p), ("read", ctypes.c_void_p), ("frame", ctypes.c_void_p),
                ("frame_counts", ctypes.c_void_p), ("anchors", ctypes.c_void_p), ("bases", ctypes.c_void_p),
                ("n_bases", ctypes.c_uint64)]


def hits_from_packed(recs: np.ndarray) -> np.ndarray:
    """kgx_hit records (pos and seq 0) from HIT_PACKED16 records (uint32
    [n, 4]: the table's packed record, flags in bits 28-30 of word 3)."""
    r = np.asarray(recs, np.uint32).reshape(-1, 4).astype(np.uint64)
    lo = r[:, 0] | (r[:, 1] << np.uint64(32))
    out = np.zeros(len(r), HIT_DTYPE)
    out["which_kmer"] = lo & np.uint64((1 << 35) - 1)
    out["function_index"] = (((r[:, 1] >> np.uint64(3)) & np.uint64(0xFFFFF)).astype(np.int64) - 1).astype(np.int32)
    otu = ((r[:, 1] >> np.uint64(23)) & np.uint64(0x1FF)) | (((r[:, 3] >> np.uint64(16)) & np.uint64(0xFFF)) << np.uint64(9))
    out["otu_index"] = (otu.astype(np.int64) - 1).astype(np.int32)
    out["function_wt"] = r[:, 2].astype(np.uint32).view(np.float32)
    out["avg_from_end"] = (r[:, 3] & np.uint64(0xFFFF)).astype(np.uint16)
    out["flags"] = ((r[:, 3] >> np.uint64(28)) & np.uint64(7)).astype(np.uint16)
    return out


def tiled_hits_per_sequence(window_base: np.ndarray, hit_mask: np.ndarray, tile_windows: int,
                            hits: np.ndarray, fill_pos: bool = False) -> list[np.ndarray]:
    """Host-side walk of kgx_device_result's tiled hit layout (for tests and
    tools): the hit records of every sequence, in position order.  fill_pos
    sets pos and seq from the hits' mask bits (HIT_PACKED16 stores neither)."""
    J = tile_windows // 64
    pc = np.array([bin(int(x)).count("1") for x in hit_mask], dtype=np.int64)
    out = []
    for s in range(len(window_base) - 1):
        gw0, gw1 = int(window_base[s]), int(window_base[s + 1])
        parts = []
        for g in range(gw0 >> 6, ((gw1 - 1) >> 6) + 1 if gw1 > gw0 else gw0 >> 6):
            t = g // J
            pre = int(pc[t * J:g].sum())
            lo = gw0 & 63 if g == gw0 >> 6 else 0
            hi = ((gw1 - 1) & 63) + 1 if g == (gw1 - 1) >> 6 else 64
            full = int(hit_mask[g])
            sel = full & (((1 << hi) - 1) & ~((1 << lo) - 1))
            start = t * tile_windows + pre + bin(full & ((1 << lo) - 1)).count("1")
            part = hits[start:start + bin(sel).count("1")]
            if fill_pos:
                part = part.copy()
                part["pos"] = [64 * g + b - gw0 for b in range(64) if sel >> b & 1]
                part["seq"] = s
            parts.append(part)
        out.append(np.concatenate(parts) if parts else hits[:0])
    return out


_P = ctypes.c_void_p
_U64, _U32, _I32, _INT, _SZ = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int, ctypes.c_size_t
_CS = ctypes.c_char_p
_PP = ctypes.POINTER(ctypes.c_void_p)

# name -> (restype, argtypes), mirroring include/kgx.h
SIGNATURES = {
    "kgx_version": (_CS, []),
    "kgx_last_error": (_CS, []),
    "kgx_strerror": (_CS, [_INT]),
    "kgx_device_count": (_INT, []),
    "kgx_params_default": (_INT, [ctypes.POINTER(Params)]),
    "kgx_set_host_wait": (_INT, [ctypes.c_int, ctypes.c_uint32]),
    "kgx_get_host_wait": (_INT, [ctypes.POINTER(ctypes.c_uint32)]),
    "kgx_params_parse": (_INT, [ctypes.POINTER(Params), ctypes.POINTER(_CS), ctypes.POINTER(_CS), _SZ]),
    "kgx_image_open": (_INT, [_CS, _INT, _PP]),
    "kgx_image_from_memory": (_INT, [_P, _U64, _INT, _PP]),
    "kgx_image_build_synthetic": (_INT, [_U64, _U64, _INT, _PP, ctypes.POINTER(_U64)]),
    "kgx_image_build_synthetic_distinct": (_INT, [_U64, _U64, _U64, _INT, _PP, ctypes.POINTER(_U64)]),
    "kgx_image_build": (_INT, [_P, _P, _P, _P, _P, _U64, _U64, _INT, _PP, ctypes.POINTER(_U64)]),
    "kgx_image_save": (_INT, [_P, _CS]),
    "kgx_image_close": (_INT, [_P]),
    "kgx_image_num_sigs": (_U64, [_P]),
    "kgx_image_device": (_INT, [_P]),
    "kgx_image_table": (_P, [_P]),
    "kgx_image_layout": (_INT, [_P]),
    "kgx_image_set_layout": (_INT, [_P, _INT]),
    "kgx_image_set_line_index": (_INT, [_P, _U32]),
    "kgx_image_line_count": (_U64, [_P]),
    "kgx_image_set_filter": (_INT, [_P, _INT]),
    "kgx_image_download": (_INT, [_P, _P, _U64]),
    "kgx_ctx_create": (_INT, [_P, _PP]),
    "kgx_ctx_destroy": (_INT, [_P]),
    "kgx_find_best_calls": (_INT, [_P, _P, _P, _U32, _P]),
    "kgx_fq_called_reads": (_INT, [_P, _P, _P]),
    "kgx_ctx_stream": (_P, [_P]),
    "kgx_ctx_set_stream": (_INT, [_P, _P]),
    "kgx_ctx_set_option": (_INT, [_P, _CS, ctypes.c_int64]),
    "kgx_process_batch": (_INT, [_P, ctypes.POINTER(Params), _P, _P, _U32, _U32, ctypes.POINTER(Result)]),
    "kgx_run_device": (_INT, [_P, ctypes.POINTER(Params), _P, _P, _U32, _U64, _U32,
                              ctypes.POINTER(DeviceResult)]),
    "kgx_stage_plan": (_INT, [_P, _P, _U32, _U64]),
    "kgx_stage_probe": (_INT, [_P, _P, _P]),
    "kgx_stage_score": (_INT, [_P, ctypes.POINTER(Params), _U32]),
    "kgx_device_result_get": (_INT, [_P, ctypes.POINTER(DeviceResult)]),
    "kgx_synth_queries": (_INT, [_P, _U64, _U32, _U32, _U32, _U64, _P, _P]),
    "kgx_find_best_call": (_INT, [_P, _SZ, ctypes.POINTER(_CS), _INT, ctypes.POINTER(_I32), _P, _SZ,
                                  ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                  ctypes.POINTER(ctypes.c_float), ctypes.POINTER(_INT)]),
    "kgx_microbench_random_read": (_INT, [_P, _U64, _INT, ctypes.POINTER(ctypes.c_float),
                                          ctypes.POINTER(_U64)]),
    "kgx_device_batch_collect": (_INT, [_P, _U32, ctypes.POINTER(Result)]),
    "kgx_fq_fragments": (_INT, [_P, _P, _P, _U32, ctypes.POINTER(Fragments)]),
    "kgx_fq_upload": (_INT, [_P, _P, _P, _U32]),
    "kgx_fq_fragments_uploaded": (_INT, [_P, ctypes.POINTER(Fragments)]),
    "kgx_fq_fragments_uploaded_start": (_INT, [_P]),
    "kgx_fq_fragments_device": (_INT, [_P, _P, _P, _U32, ctypes.POINTER(Fragments)]),
    "kgx_fq_fragments_device_start": (_INT, [_P, _P, _P, _U32, _U64]),
    "kgx_fq_fragments_finish": (_INT, [_P, ctypes.POINTER(Fragments)]),
    "kgx_fq_run_device": (_INT, [_P, ctypes.POINTER(Params), ctypes.POINTER(Fragments), _U32, _P]),
    "kgx_fq_create": (_INT, [_P, _CS, _CS, _CS, _CS, _PP]),
    "kgx_fq_destroy": (_INT, [_P]),
    "kgx_fq_process": (_INT, [_P, _CS, _U64, _INT, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_U64)]),
    "kgx_kmap_create": (_INT, [_INT, _INT, _PP]),
    "kgx_kmap_destroy": (_INT, [_P]),
    "kgx_kmap_add": (_INT, [_P, _P, _P, _U64]),
    "kgx_kmap_add_hits": (_INT, [_P, _P, _P]),
    "kgx_kmap_num_kmers": (_U64, [_P]),
    "kgx_kmap_num_values": (_U64, [_P]),
    "kgx_kmap_lookup": (_INT, [_P, _P, _U64, _P, _P, _U64]),
    "kgx_kmap_rollup": (_INT, [_P, _P, _INT, ctypes.POINTER(RollupResult)]),
    "kgx_kmap_device": (_INT, [_P]),
    "kgx_lookup": (_INT, [_P, _P, _INT, ctypes.POINTER(Params), _P, _P, _U32, _U32, ctypes.POINTER(Result),
                          ctypes.POINTER(RollupResult)]),
    "kgx_pool_lookup": (_INT, [_P, _PP, _U32, _INT, ctypes.POINTER(Params), _P, _P, _U32, _U32,
                               ctypes.POINTER(Result), ctypes.POINTER(RollupResult)]),
    "kgx_matrix_create": (_INT, [_P, _PP]),
    "kgx_matrix_destroy": (_INT, [_P]),
    "kgx_matrix_add_hits": (_INT, [_P, _P, _P]),
    "kgx_matrix_pairs": (_INT, [_P, _PP, ctypes.POINTER(_U64)]),
    "kgx_event_create": (_INT, [_PP]),
    "kgx_event_destroy": (_INT, [_P]),
    "kgx_event_record": (_INT, [_P, _P]),
    "kgx_event_elapsed_ms": (_INT, [_P, _P, ctypes.POINTER(ctypes.c_float)]),
    "kgx_device_alloc": (_INT, [_INT, _U64, _PP]),
    "kgx_device_free": (_INT, [_P]),
    "kgx_host_alloc": (_INT, [_U64, _PP]),
    "kgx_host_free": (_INT, [_P]),
    "kgx_memcpy_h2d": (_INT, [_P, _P, _U64]),
    "kgx_memcpy_d2h": (_INT, [_P, _P, _U64]),
    "kgx_ctx_synchronize": (_INT, [_P]),
    "kgx_ctx_check": (_INT, [_P]),
    "kgx_image_open_replicas": (_INT, [_CS, ctypes.POINTER(_INT), _U32, _PP]),
    "kgx_image_replicate": (_INT, [_P, _INT, _PP]),
    "kgx_pool_create": (_INT, [_PP, _U32, _U32, _PP]),
    "kgx_pool_destroy": (_INT, [_P]),
    "kgx_pool_size": (_U32, [_P]),
    "kgx_pool_ctx": (_P, [_P, _U32]),
    "kgx_pool_process_batch": (_INT, [_P, ctypes.POINTER(Params), _P, _P, _U32, _U32, ctypes.POINTER(Result)]),
    "kgx_shard_cuts": (_INT, [_P, _U32, _U32, _P]),
    "kgx_pool_numa_node": (_INT, [_P, _U32]),
    "kgx_format_g6": (_SZ, [ctypes.c_float, ctypes.c_char_p, _SZ]),
    "kgx_pool_map_select": (_INT, [_P, _U32, _P, _U32, _P]),
    "kgx_device_numa_node": (_INT, [_INT]),
    "kgx_numa_node_cpus": (_INT, [_INT, _P, _U32]),
    "kgx_device_memory": (_INT, [_INT, ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    "kgx_process_batch_compact": (_INT, [_P, ctypes.POINTER(Params), _P, _P, _U32, _U32,
                                         ctypes.POINTER(CompactResult)]),
    "kgx_pool_process_batch_compact": (_INT, [_P, ctypes.POINTER(Params), _P, _P, _U32, _U32,
                                              ctypes.POINTER(CompactResult)]),
    "kgx_compact_expand": (_INT, [ctypes.POINTER(CompactResult), _P, _P, _U32, _U32, _U32, _P]),
    "kgx_ctx_host_profile": (_INT, [_P, ctypes.POINTER(HostProfile)]),
    "kgx_ctx_stat": (_INT, [_P, _CS, ctypes.POINTER(ctypes.c_int64)]),
    "kgx_svc_call": (_INT, [_P, ctypes.POINTER(Params), _P, _U64, _U32, _P, _U64, ctypes.POINTER(_U64), _P, _U64,
                            ctypes.POINTER(_U64), _P, _U64, ctypes.POINTER(_U64)]),
    "kgx_svc_config": (_INT, [_P, _U32, _U32, _U32]),
    "kgx_svc_stop": (_INT, [_P]),
    "kgx_svc_stat": (_INT, [_P, _CS, ctypes.POINTER(_U64)]),
}


def header_symbols() -> list[str]:
    """Function names declared in include/kgx.h."""
    with open(os.path.join(_build.INCLUDE, "kgx.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(kgx_\w+)\s*\(", text)))


_lib = None


def lib() -> ctypes.CDLL:
    """Load libkgx.so (building it first if it is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(_build.LIB):
            _build.build()
        L = ctypes.CDLL(_build.LIB)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return (lib().kgx_last_error() or b"").decode()


def check(rc: int, what: str) -> None:
    if rc != KGX_OK:
        raise KgxError(rc, what)


def device_count() -> int:
    return lib().kgx_device_count()


def default_params() -> Params:
    p = Params()
    check(lib().kgx_params_default(ctypes.byref(p)), "kgx_params_default")
    return p


def parse_params(values: dict | None) -> Params:
    """set_parameters (kguts.cc:244-268) over a query-string dict."""
    p = Params()
    items = list((values or {}).items())
    names = (_CS * max(1, len(items)))(*[k.encode() for k, _ in items])
    vals = (_CS * max(1, len(items)))(*[str(v).encode() for _, v in items])
    check(lib().kgx_params_parse(ctypes.byref(p), names, vals, len(items)), "kgx_params_parse")
    return p


def _view(ptr: int | None, n: int, dtype, copy: bool = True) -> np.ndarray:
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    buf = (ctypes.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
    a = np.frombuffer(buf, dtype=dtype)
    return a.copy() if copy else a


class Image:
    """A device-resident signature image (KmerImage)."""

    def __init__(self, handle: int):
        self.handle = handle

    @classmethod
    def open(cls, data_dir: str, device: int = 0) -> "Image":
        h = ctypes.c_void_p()
        check(lib().kgx_image_open(data_dir.encode(), device, ctypes.byref(h)), f"kgx_image_open({data_dir})")
        return cls(h.value)

    @classmethod
    def open_replicas(cls, data_dir: str, devices: list[int]) -> list["Image"]:
        """One replica per listed device, the file read once (kgx_image_open_replicas)."""
        n = len(devices)
        devs = (_INT * max(1, n))(*devices)
        hs = (ctypes.c_void_p * max(1, n))()
        check(lib().kgx_image_open_replicas(data_dir.encode(), devs, n, hs), f"kgx_image_open_replicas({data_dir})")
        return [cls(hs[i]) for i in range(n)]

    def replicate(self, device: int) -> "Image":
        """A device-to-device copy of this image on `device` (kgx_image_replicate)."""
        h = ctypes.c_void_p()
        check(lib().kgx_image_replicate(self.handle, device, ctypes.byref(h)), "kgx_image_replicate")
        return Image(h.value)

    @property
    def device(self) -> int:
        return lib().kgx_image_device(self.handle)

    @classmethod
    def from_table(cls, table: np.ndarray, device: int = 0) -> "Image":
        table = np.ascontiguousarray(table)
        hdr = np.array([table.nbytes // 24, 24, 1], dtype=np.int64)
        blob = np.concatenate([hdr.view(np.uint8), table.view(np.uint8).reshape(-1)])
        h = ctypes.c_void_p()
        check(lib().kgx_image_from_memory(blob.ctypes.data, blob.nbytes, device, ctypes.byref(h)),
              "kgx_image_from_memory")
        return cls(h.value)

    @classmethod
    def synthetic(cls, n_keys: int, num_sigs: int, device: int = 0) -> tuple["Image", int]:
        h = ctypes.c_void_p()
        stored = ctypes.c_uint64()
        check(lib().kgx_image_build_synthetic(n_keys, num_sigs, device, ctypes.byref(h),
                                              ctypes.byref(stored)), "kgx_image_build_synthetic")
        return cls(h.value), stored.value

    @classmethod
    def synthetic_distinct(cls, n_keys: int, n_distinct: int, num_sigs: int,
                           device: int = 0) -> tuple["Image", int]:
        """The n_keys spec's stream cut where it holds n_distinct distinct keys;
        returns (image, entries used)."""
        h = ctypes.c_void_p()
        m = ctypes.c_uint64()
        check(lib().kgx_image_build_synthetic_distinct(n_keys, n_distinct, num_sigs, device, ctypes.byref(h),
                                                       ctypes.byref(m)), "kgx_image_build_synthetic_distinct")
        return cls(h.value), m.value

    @classmethod
    def build(cls, keys, function_index, otu_index, avg_from_end, function_wt, num_sigs: int,
              device: int = 0) -> tuple["Image", int]:
        """Device image build from entry arrays (insert_kmer semantics)."""
        k = np.ascontiguousarray(keys, dtype=np.uint64)
        f = np.ascontiguousarray(function_index, dtype=np.int32)
        o = np.ascontiguousarray(otu_index, dtype=np.int32)
        a = np.ascontiguousarray(avg_from_end, dtype=np.uint16)
        w = np.ascontiguousarray(function_wt, dtype=np.float32)
        h, stored = ctypes.c_void_p(), ctypes.c_uint64()
        check(lib().kgx_image_build(k.ctypes.data, f.ctypes.data, o.ctypes.data, a.ctypes.data, w.ctypes.data,
                                    len(k), num_sigs, device, ctypes.byref(h), ctypes.byref(stored)),
              "kgx_image_build")
        return cls(h.value), stored.value

    def set_filter(self, log2_bits: int) -> None:
        check(lib().kgx_image_set_filter(self.handle, log2_bits), "kgx_image_set_filter")

    def save(self, data_dir: str) -> None:
        check(lib().kgx_image_save(self.handle, data_dir.encode()), "kgx_image_save")

    @property
    def num_sigs(self) -> int:
        return lib().kgx_image_num_sigs(self.handle)

    AOS24, PACKED16 = 0, 1

    @property
    def layout(self) -> int:
        return lib().kgx_image_layout(self.handle)

    def set_layout(self, layout: int) -> None:
        check(lib().kgx_image_set_layout(self.handle, layout), "kgx_image_set_layout")

    def set_line_index(self, keys_per_64_lines: int) -> None:
        """kgx_image_set_line_index: probes read a copy of the records with
        line-aligned homes (0 drops it); results are unchanged."""
        check(lib().kgx_image_set_line_index(self.handle, keys_per_64_lines), "kgx_image_set_line_index")

    @property
    def line_count(self) -> int:
        return lib().kgx_image_line_count(self.handle)

    def download(self) -> np.ndarray:
        t = np.empty(self.num_sigs, dtype=SIG_DTYPE)
        check(lib().kgx_image_download(self.handle, t.ctypes.data, t.nbytes), "kgx_image_download")
        return t

    def svc_call(self, seq: bytes, params=None, want: int = WANT_HITS | WANT_CALLS, otus: bool = False):
        """One sequence through the resident call service (kgx_svc_call):
        (hits, calls) arrays, or (hits, calls, otus) with otus=True (want
        then includes WANT_OTU); raises KgxError (code KGX_EBUSY) for a call
        the service does not take."""
        p = params if isinstance(params, Params) else parse_params(params)
        W = max(len(seq) - 8, 0)
        hits = np.empty(max(W, 1), HIT_DTYPE)
        calls = np.empty(max(W, 1), CALL_DTYPE)
        ot = np.empty(max(W, 1), OTU_DTYPE)
        nh, nc, no = _U64(), _U64(), _U64()
        if otus:
            want |= WANT_OTU
        buf = ctypes.create_string_buffer(bytes(seq), max(len(seq), 1))
        check(lib().kgx_svc_call(self.handle, ctypes.byref(p), buf, len(seq), want, hits.ctypes.data, W,
                                 ctypes.byref(nh), calls.ctypes.data, W, ctypes.byref(nc), ot.ctypes.data, W,
                                 ctypes.byref(no)), "kgx_svc_call")
        if otus:
            return hits[:nh.value].copy(), calls[:nc.value].copy(), ot[:no.value].copy()
        return hits[:nh.value].copy(), calls[:nc.value].copy()

    def svc_config(self, slots: int = 32, idle_us: int = 1000, life_us: int = 4000) -> None:
        check(lib().kgx_svc_config(self.handle, slots, idle_us, life_us), "kgx_svc_config")

    def svc_stop(self) -> None:
        check(lib().kgx_svc_stop(self.handle), "kgx_svc_stop")

    def svc_stat(self, name: str) -> int:
        v = _U64()
        check(lib().kgx_svc_stat(self.handle, name.encode(), ctypes.byref(v)), "kgx_svc_stat")
        return v.value

    def close(self) -> None:
        if self.handle:
            lib().kgx_image_close(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class BatchResult:
    """Host CSR results.  copy=False gives views of the context's buffers
    (valid until its next call, as in the C ABI) instead of numpy copies."""

    def __init__(self, r: Result, want: int, copy: bool = True):
        n = r.n_seq
        self.hit_offsets = _view(r.hit_offsets, n + 1, np.uint64, copy)
        self.call_offsets = _view(r.call_offsets, n + 1, np.uint64, copy)
        self.otu_offsets = _view(r.otu_offsets, n + 1, np.uint64, copy)
        self.hits = _view(r.hits, int(self.hit_offsets[-1]) if n + 1 else 0, HIT_DTYPE, copy)
        self.calls = _view(r.calls, int(self.call_offsets[-1]), CALL_DTYPE, copy)
        self.otus = _view(r.otus, int(self.otu_offsets[-1]), OTU_DTYPE, copy)
        self.n_windows = r.n_windows
        self.best = _view(r.best, n, BEST_DTYPE, copy) if r.best else None


class CompactBatch:
    """kgx_compact_result: offsets / calls / OTUs / best as BatchResult views
    (valid until the producer's next call), hits kept as compact records.
    expand() builds kgx_hit records (HIT_DTYPE) for a range of sequences."""

    def __init__(self, cr: CompactResult, residues: np.ndarray, offsets: np.ndarray, want: int):
        self._cr = cr
        self._res = residues  # the batch's buffers: the keys are re-encoded from them
        self._off = offsets
        r = Result()
        ctypes.memmove(ctypes.byref(r), ctypes.byref(cr.r), ctypes.sizeof(Result))
        hits_ptr = r.hits
        r.hits = None
        self.result = BatchResult(r, want, copy=False)
        self.n_chunks = cr.n_chunks
        self.materialized = bool(hits_ptr)
        self.chunks = [cr.chunks[i] for i in range(cr.n_chunks)]

    def expand(self, s_begin: int = 0, s_end: int | None = None, seq_base: int = 0) -> np.ndarray:
        n = len(self.result.hit_offsets) - 1
        s_end = n if s_end is None else s_end
        ho = self.result.hit_offsets
        out = np.empty(int(ho[s_end] - ho[s_begin]) if n >= 0 else 0, HIT_DTYPE)
        check(lib().kgx_compact_expand(ctypes.byref(self._cr), self._res.ctypes.data if self._res.size else None,
                                       self._off.ctypes.data, s_begin, s_end, seq_base,
                                       out.ctypes.data if len(out) else None), "kgx_compact_expand")
        return out


def _batch_args(residues, offsets, params):
    if params is None or isinstance(params, dict):
        params = parse_params(params)
    residues = np.ascontiguousarray(np.frombuffer(bytes(residues), np.uint8)
                                    if isinstance(residues, (bytes, bytearray)) else residues, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    return residues, offsets, params


class Context:
    """One per host thread (like one KmerGuts per pool thread)."""

    def __init__(self, image: Image):
        self.image = image
        h = ctypes.c_void_p()
        check(lib().kgx_ctx_create(image.handle, ctypes.byref(h)), "kgx_ctx_create")
        self.handle = h.value

    def process_batch(self, residues, offsets, params: Params | dict | None = None,
                      want: int = WANT_HITS | WANT_CALLS | WANT_OTU, copy: bool = True) -> BatchResult:
        if params is None or isinstance(params, dict):
            params = parse_params(params)
        residues = np.ascontiguousarray(np.frombuffer(bytes(residues), np.uint8)
                                        if isinstance(residues, (bytes, bytearray)) else residues,
                                        dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        r = Result()
        check(lib().kgx_process_batch(self.handle, ctypes.byref(params),
                                      residues.ctypes.data if residues.size else None,
                                      offsets.ctypes.data, len(offsets) - 1, want, ctypes.byref(r)),
              "kgx_process_batch")
        return BatchResult(r, want, copy)

    def process_batch_compact(self, residues, offsets, params: Params | dict | None = None,
                              want: int = WANT_HITS | WANT_CALLS) -> CompactBatch:
        residues, offsets, params = _batch_args(residues, offsets, params)
        cr = CompactResult()
        check(lib().kgx_process_batch_compact(self.handle, ctypes.byref(params),
                                              residues.ctypes.data if residues.size else None,
                                              offsets.ctypes.data, len(offsets) - 1, want, ctypes.byref(cr)),
              "kgx_process_batch_compact")
        return CompactBatch(cr, residues, offsets, want)

    def lookup(self, kmap: "Kmap", residues, offsets, params: Params | dict | None = None, want: int = WANT_BEST,
               mode: int = 1):
        """kgx_lookup: the pass and the rollup over kmap with one host wait:
        (BatchResult without hits, rollup offsets, rollup rows)."""
        residues, offsets, params = _batch_args(residues, offsets, params)
        r, ru = Result(), RollupResult()
        check(lib().kgx_lookup(self.handle, kmap.handle, mode, ctypes.byref(params),
                               residues.ctypes.data if residues.size else None, offsets.ctypes.data,
                               len(offsets) - 1, want, ctypes.byref(r), ctypes.byref(ru)), "kgx_lookup")
        off = _view(ru.offsets, ru.n_seq + 1, np.uint64)
        return BatchResult(r, want), off, _view(ru.rows, int(off[-1]) if len(off) else 0, ROLLUP_DTYPE)

    def stat(self, name: str) -> int:
        v = ctypes.c_int64()
        check(lib().kgx_ctx_stat(self.handle, name.encode(), ctypes.byref(v)), f"stat({name})")
        return v.value

    def host_profile(self) -> dict:
        p = HostProfile()
        check(lib().kgx_ctx_host_profile(self.handle, ctypes.byref(p)), "kgx_ctx_host_profile")
        return p.as_dict()

    def find_best_calls(self, calls: np.ndarray, call_offsets) -> np.ndarray:
        """find_best_call of every sequence's calls, on the device."""
        calls = np.ascontiguousarray(calls, dtype=CALL_DTYPE)
        off = np.ascontiguousarray(call_offsets, dtype=np.uint64)
        out = np.zeros(len(off) - 1, BEST_DTYPE)
        check(lib().kgx_find_best_calls(self.handle, calls.ctypes.data if calls.size else None,
                                        off.ctypes.data, len(off) - 1, out.ctypes.data),
              "kgx_find_best_calls")
        return out

    def fq_fragments(self, bases, read_offsets) -> Fragments:
        """6-frame code-11 fragments (> 10 aa) of the reads, left on the device."""
        bases = np.ascontiguousarray(np.frombuffer(bytes(bases), np.uint8)
                                     if isinstance(bases, (bytes, bytearray)) else bases, dtype=np.uint8)
        off = np.ascontiguousarray(read_offsets, dtype=np.uint64)
        f = Fragments()
        check(lib().kgx_fq_fragments(self.handle, bases.ctypes.data if bases.size else None,
                                     off.ctypes.data, len(off) - 1, ctypes.byref(f)), "kgx_fq_fragments")
        return f

    def fragments_to_host(self, f: Fragments) -> dict:
        """Host copies of a kgx_fragments (tests / tools)."""
        self.synchronize()
        n, nr = f.n_fragments, f.n_residues
        out = {"residues": np.zeros(nr, np.uint8), "offsets": np.zeros(n + 1, np.uint64),
               "read": np.zeros(n, np.uint32), "frame": np.zeros(n, np.int8)}
        if not f.residues:  # fq_residues 0: anchors into the bases instead
            out["residues"] = out["read"] = out["frame"] = None
            out["anchors"] = np.zeros(n, np.uint64)
        out["frame_counts"] = np.zeros(6 * f.n_reads, np.uint32)
        for k, ptr in (("residues", f.residues), ("offsets", f.offsets), ("read", f.read),
                       ("frame", f.frame), ("anchors", f.anchors), ("frame_counts", f.frame_counts)):
            a = out.get(k)
            if a is not None and a.nbytes:
                check(lib().kgx_memcpy_d2h(a.ctypes.data, ptr, a.nbytes), "d2h")
        return out

    def run_fragments(self, f: Fragments, params: Params | dict | None = None,
                      want: int = WANT_HITS | WANT_CALLS) -> BatchResult:
        """The lookup over device fragments, results collected to the host."""
        if params is None or isinstance(params, dict):
            params = parse_params(params)
        check(lib().kgx_fq_run_device(self.handle, ctypes.byref(params), ctypes.byref(f), want, None),
              "kgx_fq_run_device")
        r = Result()
        check(lib().kgx_device_batch_collect(self.handle, want, ctypes.byref(r)), "collect")
        return BatchResult(r, want)

    @property
    def stream(self) -> int:
        return lib().kgx_ctx_stream(self.handle)

    def set_stream(self, stream: int | None) -> None:
        check(lib().kgx_ctx_set_stream(self.handle, stream), "kgx_ctx_set_stream")

    def set_option(self, name: str, value: int) -> None:
        check(lib().kgx_ctx_set_option(self.handle, name.encode(), value), f"set_option({name})")

    def synchronize(self) -> None:
        check(lib().kgx_ctx_synchronize(self.handle), "kgx_ctx_synchronize")

    def check_plan(self) -> None:
        """kgx_ctx_check: raises when the last plan's offsets were bad."""
        check(lib().kgx_ctx_check(self.handle), "kgx_ctx_check")

    def close(self) -> None:
        if self.handle:
            lib().kgx_ctx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def find_best_call(calls: np.ndarray, functions: list[str]):
    """(function_index, function, score, weighted_score, score_offset|None)."""
    calls = np.ascontiguousarray(calls, dtype=CALL_DTYPE)
    names = (_CS * max(1, len(functions)))(*[f.encode() for f in functions])
    fi = _I32()
    buf = ctypes.create_string_buffer(1 << 16)
    sc, ws, off = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
    off_set = _INT()
    check(lib().kgx_find_best_call(calls.ctypes.data if len(calls) else None, len(calls), names,
                                   len(functions), ctypes.byref(fi), buf, len(buf),
                                   ctypes.byref(sc), ctypes.byref(ws), ctypes.byref(off),
                                   ctypes.byref(off_set)), "kgx_find_best_call")
    return fi.value, buf.value.decode(), sc.value, ws.value, (off.value if off_set.value else None)


KMAP_APPEND, KMAP_SET = 0, 1
PAIR_DTYPE = np.dtype([("id1", np.uint32), ("id2", np.uint32), ("count", np.uint64)])


class Kmap:
    """Device k-mer -> id table: kmer_to_id_ (KMAP_APPEND) or kmer_to_family_id_ (KMAP_SET)."""

    def __init__(self, device: int = 0, mode: int = KMAP_APPEND):
        h = ctypes.c_void_p()
        check(lib().kgx_kmap_create(device, mode, ctypes.byref(h)), "kgx_kmap_create")
        self.handle = h.value

    def add(self, kmers, ids) -> None:
        k = np.ascontiguousarray(kmers, dtype=np.uint64)
        v = np.ascontiguousarray(ids, dtype=np.uint32)
        check(lib().kgx_kmap_add(self.handle, k.ctypes.data, v.ctypes.data, len(k)), "kgx_kmap_add")

    def add_hits(self, ctx: "Context", seq_ids) -> None:
        v = np.ascontiguousarray(seq_ids, dtype=np.uint32)
        check(lib().kgx_kmap_add_hits(self.handle, ctx.handle, v.ctypes.data), "kgx_kmap_add_hits")

    @property
    def num_kmers(self) -> int:
        return lib().kgx_kmap_num_kmers(self.handle)

    @property
    def num_values(self) -> int:
        return lib().kgx_kmap_num_values(self.handle)

    def lookup(self, kmers) -> tuple[np.ndarray, np.ndarray]:
        """(offsets[n+1], ids) CSR of the lists of `kmers`."""
        k = np.ascontiguousarray(kmers, dtype=np.uint64)
        off = np.zeros(len(k) + 1, np.uint64)
        check(lib().kgx_kmap_lookup(self.handle, k.ctypes.data, len(k), off.ctypes.data, None, 0),
              "kgx_kmap_lookup")
        ids = np.zeros(int(off[-1]), np.uint32)
        if len(ids):
            check(lib().kgx_kmap_lookup(self.handle, k.ctypes.data, len(k), off.ctypes.data,
                                        ids.ctypes.data, len(ids)), "kgx_kmap_lookup")
        return off, ids

    def rollup(self, ctx: "Context", mode: int = ROLLUP_FAMILY) -> tuple[np.ndarray, np.ndarray]:
        """kgx_kmap_rollup over ctx's last batch: (offsets [n_seq + 1], rows)."""
        r = RollupResult()
        check(lib().kgx_kmap_rollup(self.handle, ctx.handle, mode, ctypes.byref(r)), "kgx_kmap_rollup")
        off = _view(r.offsets, r.n_seq + 1, np.uint64)
        return off, _view(r.rows, int(off[-1]), ROLLUP_DTYPE)

    def close(self) -> None:
        if self.handle:
            lib().kgx_kmap_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Matrix:
    """One /matrix request (matrix_request.cc:83-190) over a device Kmap."""

    def __init__(self, kmap: Kmap):
        self.kmap = kmap
        h = ctypes.c_void_p()
        check(lib().kgx_matrix_create(kmap.handle, ctypes.byref(h)), "kgx_matrix_create")
        self.handle = h.value

    def add_hits(self, ctx: "Context", seq_ids) -> None:
        v = np.ascontiguousarray(seq_ids, dtype=np.uint32)
        check(lib().kgx_matrix_add_hits(self.handle, ctx.handle, v.ctypes.data), "kgx_matrix_add_hits")

    def pairs(self) -> np.ndarray:
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        check(lib().kgx_matrix_pairs(self.handle, ctypes.byref(p), ctypes.byref(n)), "kgx_matrix_pairs")
        return _view(p.value, n.value, PAIR_DTYPE).copy()

    def close(self) -> None:
        if self.handle:
            lib().kgx_matrix_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class FqHandler:
    """The fq request handler (kgx_fq_*) over an image."""

    def __init__(self, image: Image, data_dir: str, genus: str = "", families: str = "", nr: str = ""):
        h = ctypes.c_void_p()
        check(lib().kgx_fq_create(image.handle, data_dir.encode(), genus.encode(), families.encode(),
                                  nr.encode(), ctypes.byref(h)), "kgx_fq_create")
        self.handle = h.value

    def process(self, fastq: bytes, finished: bool = True) -> bytes:
        t, n = ctypes.c_char_p(), ctypes.c_uint64()
        fastq = bytes(fastq)  # passed by pointer, not copied
        check(lib().kgx_fq_process(self.handle, fastq, len(fastq), int(finished), ctypes.byref(t),
                                   ctypes.byref(n)), "kgx_fq_process")
        return ctypes.string_at(t, n.value) if n.value else b""

    def close(self) -> None:
        if self.handle:
            lib().kgx_fq_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def shard_cuts(offsets, n_shards: int) -> np.ndarray:
    """kgx_shard_cuts: cut points of n_shards residue-balanced contiguous shards."""
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    cuts = np.zeros(n_shards + 1, np.uint32)
    check(lib().kgx_shard_cuts(off.ctypes.data, len(off) - 1, n_shards, cuts.ctypes.data), "kgx_shard_cuts")
    return cuts


def pool_map_select(ctx_devices, map_devices) -> np.ndarray:
    """kgx_pool_map_select: for each context device the index of its map."""
    c = np.ascontiguousarray(ctx_devices, np.int32)
    m = np.ascontiguousarray(map_devices, np.int32)
    out = np.zeros(max(len(c), 1), np.int32)
    check(lib().kgx_pool_map_select(c.ctypes.data, len(c), m.ctypes.data, len(m), out.ctypes.data),
          "kgx_pool_map_select")
    return out[:len(c)]


def numa_node_cpus(node: int) -> list[int]:
    """The CPUs of NUMA node `node` this process may run on (no device needed)."""
    n = lib().kgx_numa_node_cpus(node, None, 0)
    out = np.zeros(max(n, 1), np.uint32)
    n = lib().kgx_numa_node_cpus(node, out.ctypes.data, len(out))
    return out[:n].tolist()


def device_memory(device: int) -> tuple[int, int]:
    """(free, total) HBM bytes of a device."""
    f, t = _U64(), _U64()
    check(lib().kgx_device_memory(device, ctypes.byref(f), ctypes.byref(t)), "kgx_device_memory")
    return f.value, t.value


def pinned_empty(n: int, dtype=np.uint8) -> np.ndarray:
    """An uninitialised array in pinned, device-mapped host memory
    (kgx_host_alloc), freed with the last reference to it.  Residues passed
    in such memory go to the device by DMA with no staging copy (context
    option "pinned_input")."""
    dt = np.dtype(dtype)
    nbytes = max(1, int(n) * dt.itemsize)
    p = ctypes.c_void_p()
    check(lib().kgx_host_alloc(nbytes, ctypes.byref(p)), "kgx_host_alloc")
    buf = (ctypes.c_char * nbytes).from_address(p.value)
    weakref.finalize(buf, lib().kgx_host_free, p.value)
    return np.frombuffer(buf, dtype=dt, count=int(n))


class Pool:
    """Contexts over image replicas; one batch split across them (kgx_pool)."""

    def __init__(self, images: list[Image], n_ctx: int | None = None):
        self.images = images
        n_ctx = len(images) if n_ctx is None else n_ctx
        hs = (ctypes.c_void_p * len(images))(*[im.handle for im in images])
        h = ctypes.c_void_p()
        check(lib().kgx_pool_create(hs, len(images), n_ctx, ctypes.byref(h)), "kgx_pool_create")
        self.handle = h.value

    @property
    def size(self) -> int:
        return lib().kgx_pool_size(self.handle)

    def numa_nodes(self) -> list[int]:
        """The NUMA node each context's host thread is bound to (-1: unbound)."""
        return [lib().kgx_pool_numa_node(self.handle, i) for i in range(self.size)]

    def set_option(self, name: str, value: int) -> None:
        """kgx_ctx_set_option on every context of the pool."""
        for i in range(self.size):
            check(lib().kgx_ctx_set_option(lib().kgx_pool_ctx(self.handle, i), name.encode(), value),
                  f"set_option({name})")

    def process_batch(self, residues, offsets, params: Params | dict | None = None,
                      want: int = WANT_HITS | WANT_CALLS | WANT_OTU, copy: bool = True) -> BatchResult:
        if params is None or isinstance(params, dict):
            params = parse_params(params)
        residues = np.ascontiguousarray(np.frombuffer(bytes(residues), np.uint8)
                                        if isinstance(residues, (bytes, bytearray)) else residues,
                                        dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        r = Result()
        check(lib().kgx_pool_process_batch(self.handle, ctypes.byref(params),
                                           residues.ctypes.data if residues.size else None,
                                           offsets.ctypes.data, len(offsets) - 1, want, ctypes.byref(r)),
              "kgx_pool_process_batch")
        return BatchResult(r, want, copy)

    def process_batch_compact(self, residues, offsets, params: Params | dict | None = None,
                              want: int = WANT_HITS | WANT_CALLS) -> CompactBatch:
        residues, offsets, params = _batch_args(residues, offsets, params)
        cr = CompactResult()
        check(lib().kgx_pool_process_batch_compact(self.handle, ctypes.byref(params),
                                                   residues.ctypes.data if residues.size else None,
                                                   offsets.ctypes.data, len(offsets) - 1, want, ctypes.byref(cr)),
              "kgx_pool_process_batch_compact")
        return CompactBatch(cr, residues, offsets, want)

    def lookup(self, maps: list, residues, offsets, params: Params | dict | None = None,
               want: int = WANT_BEST, mode: int = ROLLUP_FAMILY, copy: bool = True):
        """kgx_pool_lookup: (BatchResult without hits, rollup offsets, rollup rows)."""
        residues, offsets, params = _batch_args(residues, offsets, params)
        hs = (ctypes.c_void_p * len(maps))(*[m.handle for m in maps])
        r, ru = Result(), RollupResult()
        check(lib().kgx_pool_lookup(self.handle, hs, len(maps), mode, ctypes.byref(params),
                                    residues.ctypes.data if residues.size else None, offsets.ctypes.data,
                                    len(offsets) - 1, want, ctypes.byref(r), ctypes.byref(ru)), "kgx_pool_lookup")
        off = _view(ru.offsets, ru.n_seq + 1, np.uint64, copy)
        return BatchResult(r, want, copy), off, _view(ru.rows, int(off[-1]) if len(off) else 0, ROLLUP_DTYPE, copy)

    def close(self) -> None:
        if self.handle:
            lib().kgx_pool_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
