"""close_kmers_amd -- MI355X-native k-mer encode -> hash-probe -> hit-score.

The hot path of close_kmers' KmerGuts::process_aa_seq (kguts.cc:783-908) as
hand-written gfx950 HIP kernels behind a C ABI (include/kgx.h, libkgx.so),
with a KmerGuts-compatible C++ facade (csrc/kguts_hip.h) and this thin Python
binding for tests and benchmarks.  There is no CPU fallback: without the
library or a gfx950 device the entry points raise.

Submodules load on first use, so `import close_kmers_amd.shard` (the rank
launcher bench.py runs before any GPU call) pulls in nothing of the ABI.
"""
import importlib

_SUBMODULES = ("abi", "image_files", "synth", "shard", "build")
_ABI_NAMES = ("CALL_DTYPE", "HIT_DTYPE", "OTU_DTYPE", "SIG_DTYPE", "WANT_CALLS", "WANT_HITS", "WANT_OTU",
              "Context", "Image", "KgxError", "device_count", "find_best_call", "parse_params")

__all__ = ["abi", "synth", "image_files", "shard", *_ABI_NAMES]


def __getattr__(name):
    if name in _SUBMODULES:
        return importlib.import_module(f".{name}", __name__)
    if name in _ABI_NAMES:
        return getattr(importlib.import_module(".abi", __name__), name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
