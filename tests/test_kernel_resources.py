"""Build-time guard: the resident call service's kernel (svc_kernel in
kgx_fused.hip) must use no scratch memory.  It stays resident, so scratch
set-up and spills are paid by every call (a local partition stack once cost
~1 us per call; a select of two structs once put 12 B/lane there).  Compiles
the file for gfx950 with the compiler's resource remarks.  No GPU."""
import os
import re
import subprocess

from close_kmers_amd import build as kbuild


def test_svc_kernel_has_no_scratch(tmp_path):
    src = os.path.join(kbuild.CSRC, "kgx_fused.hip")
    cmd = [kbuild.HIPCC, "-O3", "-std=c++17", f"--offload-arch={kbuild.ARCH}", f"-I{kbuild.INCLUDE}",
           f"-I{kbuild.CSRC}", "-x", "hip", "-c", src, "-o", str(tmp_path / "f.o"),
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    kernels = {}
    name = None
    for ln in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            name = m.group(1)
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", ln)
        if m and name:
            kernels[name] = int(m.group(1))
    svc = {k: v for k, v in kernels.items() if "svc_kernel" in k}
    assert len(svc) == 2, kernels  # the thread and the quad probe instances
    assert all(v == 0 for v in svc.values()), svc
    small = {k: v for k, v in kernels.items() if "fused_small" in k}
    assert small and all(v == 0 for v in small.values()), small
