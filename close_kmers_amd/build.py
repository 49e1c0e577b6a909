"""Compile the gfx950 engine in-tree.

    libkgx.so   kernels (csrc/kgx_kernels.hip) + C ABI runtime + KmerGuts facade
    kgx_query   request-handler surface driver linked against libkgx.so
    kgx_server  the kser HTTP request server (krequest2.cc routes) over libkgx.so

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU
container as well as on the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(PKG, "libkgx.so")
QUERY = os.path.join(PKG, "kgx_query")
SERVER = os.path.join(PKG, "kgx_server")
# the facade under T concurrent worker threads (tests/test_gpu_coalesce.py)
COALESCE_CHECK = os.path.join(ROOT, "tests", "native", "coalesce_check")
# per-sequence service callers beside a batch caller (tests/test_gpu_svc.py)
BESIDE_CHECK = os.path.join(ROOT, "tests", "native", "beside_check")
# the one-wave std::sort replay against the serial one (tests/test_gpu_svc.py)
WAVE_SORT_CHECK = os.path.join(ROOT, "tests", "native", "wave_sort_check")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

LIB_SOURCES = ["kgx_lookup.hip", "kgx_fused.hip", "kgx_synth.hip", "kgx_tables.hip", "kgx_fq.hip", "kgx_runtime.cpp",
               "kgx_pool.cpp", "kgx_svc.cpp", "kguts_hip.cpp", "kgx_handlers.cpp"]
HEADERS = ["kgx_internal.h", "kgx_device.h", "kguts_hip.h", "kgx_rt.h", "kgx_lstd.h", "kgx_handlers.h", "kgx_wave_sort.h"]
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
        objs, cmds = [], []
        for src in LIB_SOURCES:
            obj = os.path.join(CSRC, "_obj", src + ".o")
            os.makedirs(os.path.dirname(obj), exist_ok=True)
            objs.append(obj)
            # an object is rebuilt when its source, a header or this script changed
            obj_deps = [os.path.join(CSRC, src)] + [d for d in deps if not d.endswith((".hip", ".cpp"))]
            if not force and not _newer(obj, obj_deps):
                continue
            cmds.append([HIPCC] + COMMON + ["-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj])
        if verbose:
            for cmd in cmds:
                print(" ".join(cmd))
        # objects compile independently: one hipcc per source, a few at a time
        jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "0")) or min(8, os.cpu_count() or 1)))
        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(_run, cmds))
        tmp = LIB + ".tmp"
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs)
        os.replace(tmp, LIB)
    for exe, esrc in ((QUERY, os.path.join(CSRC, "kgx_query.cpp")), (SERVER, os.path.join(CSRC, "kgx_server.cpp")),
                      (COALESCE_CHECK, os.path.join(ROOT, "tests", "native", "coalesce_check.cpp")),
                      (BESIDE_CHECK, os.path.join(ROOT, "tests", "native", "beside_check.cpp")),
                      (WAVE_SORT_CHECK, os.path.join(ROOT, "tests", "native", "wave_sort_check.cpp"))):
        if not os.path.exists(esrc):
            continue
        if force or _newer(exe, [esrc, LIB] + deps):
            tmp = exe + ".tmp"
            rpath = os.path.join("$ORIGIN", os.path.relpath(PKG, os.path.dirname(exe)))  # libkgx.so, in-tree
            _run([HIPCC] + COMMON + ["-x", "hip", esrc, "-o", tmp, f"-L{PKG}", "-lkgx", f"-Wl,-rpath,{rpath}",
                                     "-pthread"])
            os.replace(tmp, exe)


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
