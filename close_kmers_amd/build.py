"""Compile the gfx950 engine in-tree.

    libkgx.so   kernels (csrc/kgx_kernels.hip) + C ABI runtime + KmerGuts facade
    kgx_query   request-handler surface driver linked against libkgx.so

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU
container as well as on the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(PKG, "libkgx.so")
QUERY = os.path.join(PKG, "kgx_query")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

LIB_SOURCES = ["kgx_lookup.hip", "kgx_synth.hip", "kgx_tables.hip", "kgx_fq.hip", "kgx_runtime.cpp",
               "kguts_hip.cpp"]
HEADERS = ["kgx_internal.h", "kgx_device.h", "kguts_hip.h", "kgx_rt.h", "kgx_lstd.h"]
COMMON = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INCLUDE}", f"-I{CSRC}",
          "-Wall", "-Wno-unused-function"]


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build failed: {' '.join(cmd)}")


def build(force: bool = False, verbose: bool = False) -> None:
    deps = [os.path.join(CSRC, f) for f in LIB_SOURCES + HEADERS] + [os.path.join(INCLUDE, "kgx.h"),
                                                                     __file__]
    if force or _newer(LIB, deps):
        objs = []
        for src in LIB_SOURCES:
            obj = os.path.join(CSRC, "_obj", src + ".o")
            os.makedirs(os.path.dirname(obj), exist_ok=True)
            cmd = [HIPCC] + COMMON + ["-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj]
            if verbose:
                print(" ".join(cmd))
            _run(cmd)
            objs.append(obj)
        tmp = LIB + ".tmp"
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs)
        os.replace(tmp, LIB)
    qsrc = os.path.join(CSRC, "kgx_query.cpp")
    if force or _newer(QUERY, [qsrc, LIB] + deps):
        tmp = QUERY + ".tmp"
        _run([HIPCC] + COMMON + ["-x", "hip", qsrc, "-o", tmp, f"-L{PKG}", "-lkgx",
                                 "-Wl,-rpath,$ORIGIN"])
        os.replace(tmp, QUERY)


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
