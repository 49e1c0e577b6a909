"""Sharding of query batches over ranks.

The path is embarrassingly parallel over sequences (lookup_request.cc:153
processes each independently; KmerGuts state is per sequence), so every rank
holds a replica of the read-only image and processes a contiguous shard of
the batch.  There is no collective on the data path: results are concatenated
in rank order, which is input order.  torch.distributed (gloo, CPU tensors) is
used only for the barrier and the max / sum reductions of timings and counts.
"""
from __future__ import annotations

import contextlib
import os
import socket
import sys

import numpy as np


def balanced_shards(offsets: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous sequence ranges [lo, hi) per rank with about equal residue
    counts (offsets: uint64 CSR over the batch, len n_seq + 1)."""
    offsets = np.asarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    if world < 1:
        raise ValueError("world must be >= 1")
    total = int(offsets[-1] - offsets[0])
    cuts = [0]
    for r in range(1, world):
        target = offsets[0] + np.uint64(total * r // world)
        cuts.append(max(cuts[-1], int(np.searchsorted(offsets[:n], target, side="left"))))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def weak_shard(rank: int, n_per_rank: int) -> tuple[int, int]:
    """Weak scaling: rank r owns queries [r*n, (r+1)*n) of the global stream."""
    return rank * n_per_rank, (rank + 1) * n_per_rank


@contextlib.contextmanager
def _stdout_to_stderr():
    """fd 1 -> fd 2 for the duration: gloo prints its connection report
    ("[Gloo] Rank 0 is connected to ...") on stdout, where bench.py's one
    JSON line must stand alone."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


class Dist:
    """Rank / world from the torchrun environment; gloo for control only."""

    def __init__(self, backend: str = "gloo"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            with _stdout_to_stderr():
                if not dist.is_initialized():
                    dist.init_process_group(backend)
                dist.barrier()  # the mesh is connected (and reported) here
            self.pg = dist

    def barrier(self) -> None:
        if self.pg:
            self.pg.barrier()

    def _reduce(self, x: float, op) -> float:
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.pg.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.pg.ReduceOp.MAX) if self.pg else float(x)

    def sum(self, x: float) -> float:
        return self._reduce(x, self.pg.ReduceOp.SUM) if self.pg else float(x)

    def gather_objects(self, obj):
        """All ranks' objects in rank order (control-plane use only)."""
        if not self.pg:
            return [obj]
        out = [None] * self.world
        self.pg.all_gather_object(out, obj)
        return out

    def close(self) -> None:
        if self.pg:
            self.pg.destroy_process_group()
            self.pg = None


def job_throughput(world: int, residues_per_rank: int, steps: int, max_seconds: float) -> float:
    """Whole-job residues/s: all ranks' residues over the slowest rank's time."""
    return world * residues_per_rank * steps / max_seconds


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank: int, world: int, port: int, base: dict | None = None) -> dict:
    """The environment torchrun gives rank `rank` of a one-node job of `world`
    ranks (one rank per GPU: LOCAL_RANK = RANK = the device index)."""
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0",
                "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    return env


def launch_ranks(cmd: list[str], world: int, out=None, grace_s: float = 10.0,
                 poll_s: float = 0.05) -> int:
    """Run `cmd` as `world` ranks of one node, the way torchrun would, from a
    parent that never touches the GPU (the reference's analogue is one worker
    per execution resource over a shared image, threadpool.cc:18-44).

    Each rank's stderr goes straight to ours; rank 0's stdout is relayed line
    by line to `out` (default sys.stdout), the other ranks' stdout goes to our
    stderr.  When a rank fails, the others are terminated (then killed after
    `grace_s`): a rank left waiting in a barrier for a dead peer would hang.
    Returns 0 when every rank exits 0, else the first failing rank's code
    (or 1 when a rank was killed by a signal)."""
    import subprocess
    import threading
    import time

    out = out or sys.stdout
    port = free_port()
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen(cmd, env=rank_env(r, world, port), stdout=subprocess.PIPE,
                                      stderr=None, text=True, bufsize=1))

    def relay(p, sink):
        for line in p.stdout:
            sink.write(line)
            sink.flush()

    relays = [threading.Thread(target=relay, args=(p, out if r == 0 else sys.stderr), daemon=True)
              for r, p in enumerate(procs)]
    for t in relays:
        t.start()
    rc = 0
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed, code = bad[0]
            rc = code if code > 0 else 1
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(poll_s)
    if failed is not None:
        sys.stderr.write(f"[launch] rank {failed} exited with {procs[failed].returncode}; "
                         f"stopping the other ranks\n")
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    for t in relays:
        t.join(timeout=5)
    return rc
