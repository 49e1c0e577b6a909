"""Process exit with live handles (images, contexts, the host path's twin
contexts and copy streams, a running call service, a thread still calling
it).  The reference's server ends from a signal with its workers and their
KmerGuts alive (/root/reference/kserver.cc:206-214), so the library must
let a process end without closing anything.

Round 4 found two faults there, both under rocprofv3 (r5a/r5c records):
the service's exit hook called hipStreamSynchronize after the exiting
thread's thread_local objects were gone (the profiler aborted, the process
hung), and a full-CU-mask copy stream left alive faulted in the profiler's
finalisation.  The hook now uses no runtime call and the copy streams are
priority streams; these tests run the child (tests/exit_child.py) plainly and
under the profiler, with the program itself after `--`."""
import os
import shutil
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CHILD = os.path.join(HERE, "exit_child.py")


def _run(cmd, tmp_path):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd=str(tmp_path))
    assert r.returncode == 0, f"rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    assert "leaving every handle open" in r.stdout
    return r


@pytest.mark.parametrize("flags", [[], ["--threads"], ["--no-host"]])
def test_exit_with_live_handles(gpu, tmp_path, flags):
    _run([sys.executable, CHILD] + flags, tmp_path)


def test_exit_with_live_handles_under_rocprofv3(gpu, tmp_path):
    prof = shutil.which("rocprofv3")
    if not prof:
        pytest.skip("rocprofv3 not on PATH")
    r = _run([prof, "--kernel-trace", "--stats", "-d", str(tmp_path / "kt"), "-o", "kt", "--",
              sys.executable, CHILD, "--threads"], tmp_path)
    assert "Segmentation fault" not in r.stderr and "Check failed" not in r.stderr
