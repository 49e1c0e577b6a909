"""The bench's per-device self-check (a "canary" pass).

Every rank of a bench run builds the same small signature image on its own
device (CANARY_KEYS entries of the synthetic generator, built in HBM by
kgx_image_build_synthetic), runs one fixed batch of CANARY_SEQ proteins
through the host-buffer boundary (kgx_process_batch: hits, calls and the
device find_best_call -- what lookup_request's find_best_match step consumes,
lookup_request.cc:166-210), and digests the result.  The expected digest was
computed once by the CPU oracle over the same image and batch
(tests/golden/make_canary.py -> tests/golden/canary/digest.json), so a device
whose results differ from the reference path by one bit fails the run, on
any rank, without the oracle travelling with the bench.

The digest is SHA-256 over a canonical byte layout of the CSR result, so the
GPU's kgx_result and the oracle's BatchResult digest identically.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

CANARY_KEYS = 10_000_000  # BASELINE.json configs[0]'s 10M-entry image
CANARY_SEQ = 1000         # ... and its 1k x 300-aa batch
CANARY_LEN = 300
CANARY_X_PERMILLE = 5     # some ambiguous residues: the skip path runs too
CANARY_Q0 = 7_000_000     # queries past the bench's own stream
CANARY_WANT = 11          # KGX_WANT_HITS | KGX_WANT_CALLS | KGX_WANT_BEST
DIGEST_JSON = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                           "tests", "golden", "canary", "digest.json")

_HIT = np.dtype([("which_kmer", "<u8"), ("pos", "<u4"), ("function_index", "<i4"), ("otu_index", "<i4"),
                 ("avg_from_end", "<u4"), ("function_wt", "<u4")])
_CALL = np.dtype([("start", "<u4"), ("end", "<u4"), ("count", "<i4"), ("function_index", "<u4"),
                  ("weighted_hits", "<u4")])
_BEST = np.dtype([("function_index", "<i4"), ("score", "<u4"), ("weighted_score", "<u4"),
                  ("score_offset", "<u4"), ("offset_set", "<i4")])


def _f32_bits(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def digest(hit_offsets, hits, call_offsets, calls, best) -> str:
    """hits / calls: structured arrays with the kgx_hit / kgx_call field names;
    best: structured array with function_index, score, weighted_score,
    score_offset, offset_set (offset_set 0: score_offset left untouched,
    digested as 0)."""
    h = np.zeros(len(hits), _HIT)
    for f in ("which_kmer", "pos", "function_index", "otu_index", "avg_from_end"):
        h[f] = hits[f]
    h["function_wt"] = _f32_bits(hits["function_wt"])
    c = np.zeros(len(calls), _CALL)
    for f in ("start", "end", "count", "function_index"):
        c[f] = calls[f]
    c["weighted_hits"] = _f32_bits(calls["weighted_hits"])
    b = np.zeros(len(best), _BEST)
    b["function_index"] = best["function_index"]
    b["score"] = _f32_bits(best["score"])
    b["weighted_score"] = _f32_bits(best["weighted_score"])
    b["offset_set"] = best["offset_set"]
    b["score_offset"] = np.where(np.asarray(best["offset_set"]) != 0, _f32_bits(best["score_offset"]), 0)
    m = hashlib.sha256()
    for part in (np.ascontiguousarray(hit_offsets, np.uint64), h, np.ascontiguousarray(call_offsets, np.uint64),
                 c, b):
        m.update(part.tobytes())
    return m.hexdigest()


def best_from_device(best) -> np.ndarray:
    """kgx_best_call records -> the digest's best fields: kind 1 (called)
    names fi0, every other kind no function; kind 0 (no calls) leaves
    score_offset untouched (kguts.cc:1015-1018)."""
    out = np.zeros(len(best), [("function_index", "<i4"), ("score", "<f4"), ("weighted_score", "<f4"),
                               ("score_offset", "<f4"), ("offset_set", "<i4")])
    out["function_index"] = np.where(best["kind"] == 1, best["fi0"], -1)
    out["score"] = best["score"]
    out["weighted_score"] = best["weighted_score"]
    out["score_offset"] = best["score_offset"]
    out["offset_set"] = (best["kind"] != 0).astype(np.int32)
    return out


def verdict(recs: list, expected_digest: str, distinct_devices: bool) -> tuple:
    """The whole job's verdict over every rank's canary record (rank order):
    (ok, reason).  Every digest must be the oracle's; with distinct_devices
    (one rank per GPU, no KGX_BENCH_DEVICE override) no two ranks may share a
    device."""
    bad = [r["rank"] for r in recs if r["digest"] != expected_digest]
    if bad:
        return False, f"rank(s) {bad}: the canary digest differs from the CPU oracle's"
    devs = [r["device"] for r in recs]
    if distinct_devices and len(set(devs)) != len(devs):
        return False, f"ranks share a device: {devs}"
    return True, "ok"


def expected() -> dict:
    with open(DIGEST_JSON) as f:
        return json.load(f)


def run_on_device(abi, synth, device: int, line_index: int = 0) -> dict:
    """The canary pass on `device` through the C ABI: {"digest", "hits",
    "calls", "device", "line_index"}.  `line_index` > 0 builds the image's
    line index at that load first (as bench.py does for its timed image), so
    the canary probes through the same path the timed steps use."""
    spec = synth.ImageSpec(CANARY_KEYS)
    img, _ = abi.Image.synthetic(spec.n_keys, spec.num_sigs, device=device)
    try:
        if line_index and img.layout == abi.Image.PACKED16:
            img.set_line_index(line_index)
        else:
            line_index = 0
        res, off = synth.make_queries(spec, CANARY_SEQ, length=CANARY_LEN, x_permille=CANARY_X_PERMILLE,
                                      q0=CANARY_Q0)
        with abi.Context(img) as ctx:
            r = ctx.process_batch(res, off, abi.default_params(), want=CANARY_WANT)
            dg = digest(r.hit_offsets, r.hits, r.call_offsets, r.calls, best_from_device(r.best))
            return {"device": device, "digest": dg, "hits": int(r.hit_offsets[-1]), "calls": int(r.call_offsets[-1]),
                    "line_index": int(line_index)}
    finally:
        img.close()
