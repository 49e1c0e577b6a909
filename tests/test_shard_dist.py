"""The N>1 path on CPU: world_size-2 gloo ranks each process their own shard
(no data-path collective) and the concatenation equals the one-rank result."""
import os
import socket

import numpy as np
import pytest

from close_kmers_amd import shard, synth


def test_balanced_shards_cover_and_balance():
    rng = np.random.default_rng(0)
    lens = rng.integers(0, 2000, 997)
    off = np.zeros(len(lens) + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    for world in (1, 2, 3, 4, 8, 16):
        sh = shard.balanced_shards(off, world)
        assert sh[0][0] == 0 and sh[-1][1] == len(lens)
        assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
        res = [int(off[hi] - off[lo]) for lo, hi in sh]
        assert max(res) - min(res) <= 2 * lens.max() + 1
    assert shard.balanced_shards(np.zeros(1, np.uint64), 4) == [(0, 0)] * 4


def test_weak_shard_and_throughput():
    assert shard.weak_shard(0, 100) == (0, 100)
    assert shard.weak_shard(3, 100) == (300, 400)
    assert shard.job_throughput(8, 30_000_000, 20, 2.0) == 8 * 30_000_000 * 20 / 2.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    import oracle
    from helpers import synthetic_table
    d = shard.Dist("gloo")
    spec, table = synthetic_table(20000)
    n = 120
    lo, hi = shard.weak_shard(d.rank, n)
    res, off = synth.make_queries(spec, n, q0=lo, x_permille=5)
    r = oracle.process_batch(table, res, off)
    d.barrier()
    t = d.max(float(rank + 1))
    total_hits = d.sum(float(len(r.hits)))
    parts = d.gather_objects((lo, hi, r.hits["pos"].tolist(), r.hits["which_kmer"].tolist(),
                              np.diff(r.call_offsets).tolist()))
    if d.rank == 0:
        q.put((t, total_hits, parts))
    d.close()


def test_two_rank_gloo_shards_equal_single_rank():
    import torch.multiprocessing as mp
    import oracle
    from helpers import synthetic_table
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    t, total_hits, parts = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 2.0
    spec, table = synthetic_table(20000)
    res, off = synth.make_queries(spec, 240, x_permille=5)
    whole = oracle.process_batch(table, res, off)
    assert total_hits == len(whole.hits)
    assert [p[0] for p in parts] == [0, 120]
    pos = sum((p[2] for p in parts), [])
    keys = sum((p[3] for p in parts), [])
    calls = sum((p[4] for p in parts), [])
    assert pos == whole.hits["pos"].tolist()
    assert keys == whole.hits["which_kmer"].tolist()
    assert calls == np.diff(whole.call_offsets).tolist()


def _strong_worker(rank, world, port, q):
    """bench.py --strong (C5) on CPU: every rank takes its residue-balanced
    shard of one global batch of mixed lengths."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    import oracle
    from helpers import synthetic_table
    d = shard.Dist("gloo")
    spec, table = synthetic_table(20000)
    res, off = _mixed_global(spec)
    lo, hi = shard.balanced_shards(off, d.world)[d.rank]
    r0, r1 = int(off[lo]), int(off[hi])
    r = oracle.process_batch(table, res[r0:r1], off[lo:hi + 1] - off[lo])
    parts = d.gather_objects((lo, hi, r1 - r0, r.hits["pos"].tolist(), r.hits["which_kmer"].tolist(),
                              np.diff(r.call_offsets).tolist(), r.calls["weighted_hits"].tolist()))
    if d.rank == 0:
        q.put(parts)
    d.close()


def _mixed_global(spec):
    rng = np.random.default_rng(3)
    res, off = synth.make_queries(spec, 301, x_permille=5, q0=17)
    lens = rng.integers(0, 300, 301)
    seqs = [bytes(res[int(off[i]):int(off[i]) + int(lens[i])]) for i in range(301)]
    o = np.zeros(302, np.uint64)
    o[1:] = np.cumsum([len(x) for x in seqs])
    return np.frombuffer(b"".join(seqs), np.uint8).copy(), o


@pytest.mark.parametrize("world", [2, 3])
def test_strong_split_ranks_concatenate_to_one_pass(world):
    import torch.multiprocessing as mp
    import oracle
    from helpers import synthetic_table
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strong_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spec, table = synthetic_table(20000)
    res, off = _mixed_global(spec)
    whole = oracle.process_batch(table, res, off)
    assert [p[0] for p in parts][0] == 0 and parts[-1][1] == 301
    assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
    sizes = [p[2] for p in parts]
    assert max(sizes) - min(sizes) <= 2 * 300  # residue-balanced
    assert sum((p[3] for p in parts), []) == whole.hits["pos"].tolist()
    assert sum((p[4] for p in parts), []) == whole.hits["which_kmer"].tolist()
    assert sum((p[5] for p in parts), []) == np.diff(whole.call_offsets).tolist()
    got_w = np.array(sum((p[6] for p in parts), []), np.float32)
    assert np.array_equal(got_w.view(np.uint32), whole.calls["weighted_hits"].view(np.uint32))


# ---- bench.py --gpus N: the rank launcher (shard.launch_ranks) ----------

_RANK_SCRIPT = r'''
import json, os, sys
sys.path.insert(0, {root!r})
from close_kmers_amd import shard
assert "close_kmers_amd.abi" not in sys.modules
d = shard.Dist("gloo")
env = {{k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}}
envs = d.gather_objects(env)
t = d.max(float(d.rank + 1))
if d.rank == 0:
    print(json.dumps({{"world": d.world, "max": t, "envs": envs}}), flush=True)
else:
    print("not relayed to stdout", flush=True)
d.close()
'''


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(body)
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_launch_ranks_plumbs_torchrun_env(tmp_path, world):
    import io
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = _script(tmp_path, _RANK_SCRIPT.format(root=root))
    out = io.StringIO()
    rc = shard.launch_ranks([sys.executable, str(p)], world, out=out)
    assert rc == 0
    lines = out.getvalue().splitlines()
    assert len(lines) == 1  # rank 0's line alone
    got = json.loads(lines[0])
    assert got["world"] == world and got["max"] == float(world)
    assert [e["RANK"] for e in got["envs"]] == [str(r) for r in range(world)]
    assert [e["LOCAL_RANK"] for e in got["envs"]] == [str(r) for r in range(world)]
    assert all(e["WORLD_SIZE"] == str(world) and e["MASTER_ADDR"] == "127.0.0.1" for e in got["envs"])


def test_launch_ranks_failing_rank_stops_the_others(tmp_path):
    import io
    import sys
    import time
    p = _script(tmp_path, "import os, sys, time\n"
                          "if os.environ['RANK'] == '1': sys.exit(3)\n"
                          "time.sleep(120)\n")
    t0 = time.time()
    rc = shard.launch_ranks([sys.executable, str(p)], 2, out=io.StringIO(), grace_s=5)
    assert rc == 3
    assert time.time() - t0 < 30


def test_rank_env():
    env = shard.rank_env(2, 4, 1234, base={"PATH": "/bin"})
    assert env == {"PATH": "/bin", "RANK": "2", "LOCAL_RANK": "2", "WORLD_SIZE": "4",
                   "LOCAL_WORLD_SIZE": "4", "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                   "MASTER_PORT": "1234"}


def _bench(args, env_extra=None):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=120)


def test_bench_gpus_n_launches_n_ranks_and_fails_without_devices():
    """No GPU in this container: `bench.py --gpus 2` must start two ranks
    (each reporting its missing device), print no JSON line and fail."""
    r = _bench(["--gpus", "2", "--no-cpu-baseline"])
    assert r.returncode != 0
    assert r.stdout == ""
    assert "no device" in r.stderr
    assert "rank 1" in r.stderr or "rank 0" in r.stderr


def test_bench_gpus_must_match_torchrun_world():
    r = _bench(["--gpus", "3"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 3 but the launcher started 2 ranks" in r.stderr


def _canary_worker(rank, world, port, q, corrupt_rank, same_device):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    from close_kmers_amd import canary
    d = shard.Dist("gloo")
    want = canary.expected()["digest"]
    mine = {"rank": d.rank, "device": 0 if same_device else d.rank,
            "digest": ("0" * 64) if d.rank == corrupt_rank else want, "hits": 1, "calls": 1}
    recs = d.gather_objects(mine)
    q.put((d.rank, canary.verdict(recs, want, True)))
    d.close()


@pytest.mark.parametrize("corrupt_rank,same_device,ok", [(-1, False, True), (1, False, False), (-1, True, False)])
def test_canary_verdict_over_gloo_ranks(corrupt_rank, same_device, ok):
    """bench.py's canary plumbing at world size 2: every rank's digest is
    gathered and every rank reaches the same verdict -- a rank whose digest
    is not the oracle's, or two ranks on one device, fail the whole job."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_canary_worker, args=(r, 2, port, q, corrupt_rank, same_device)) for r in range(2)]
    for p in ps:
        p.start()
    got = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(v[0] == ok for _, v in got), got
