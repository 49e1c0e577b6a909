"""close_kmers_amd -- MI355X-native k-mer encode -> hash-probe -> hit-score.

The hot path of close_kmers' KmerGuts::process_aa_seq (kguts.cc:783-908) as
hand-written gfx950 HIP kernels behind a C ABI (include/kgx.h, libkgx.so),
with a KmerGuts-compatible C++ facade (csrc/kguts_hip.h) and this thin Python
binding for tests and benchmarks.  There is no CPU fallback: without the
library or a gfx950 device the entry points raise.
"""
from . import abi, image_files, synth  # noqa: F401
from .abi import (CALL_DTYPE, HIT_DTYPE, OTU_DTYPE, SIG_DTYPE, WANT_CALLS, WANT_HITS,  # noqa: F401
                  WANT_OTU, Context, Image, KgxError, device_count, find_best_call, parse_params)

__all__ = ["abi", "synth", "image_files", "Image", "Context", "KgxError", "device_count",
           "find_best_call", "parse_params", "HIT_DTYPE", "CALL_DTYPE", "OTU_DTYPE", "SIG_DTYPE",
           "WANT_HITS", "WANT_CALLS", "WANT_OTU"]
