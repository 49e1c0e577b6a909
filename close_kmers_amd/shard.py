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
