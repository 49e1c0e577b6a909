"""End-to-end HTTP serving through kgx_server (the kser drop-in), C2 data.

    python tools/bench_server.py [--n-keys 1e9] [--clients 1,4,8,16] [--threads 8]

Starts close_kmers_amd/kgx_server on 127.0.0.1 with the C2 synthetic image
(--synthetic-image: 1B keys built in HBM, PACKED16) and --threads KmerGuts
workers, then runs tools/load_gen (native C++, its own process: C client
threads, one connection per request as in krequest2.cc) POSTing FASTA bodies
of the C2 query set to /query (query_request.cc: PROTEIN-ID / CALL /
OTU-COUNTS text back) and reading the responses to the end.  Bodies are cut
at record boundaries to at most --body-bytes (default 1 MiB, the reference's
request buffer, krequest2.cc:41).  Server and load generator share the
box's CPU share (16 CPUs on the GPU box's cgroup).  Reports per C the
aggregate residues/s (residues in the bodies completed / wall time), the
request latency (median, p99) and the server's own per-stage clocks (GET
/server_stats: recv, parse, gpu, handle, send per request).  Prints one JSON
line.

With --families N a synthetic family DB is loaded (families.tsv, genus.map
and nr.fasta over source proteins 0..N-1 of the synthetic image; each family
holds one protein) so that /lookup runs in family mode
(lookup_request.cc:153-400), e.g.
    python tools/bench_server.py --families 100000 --path "/lookup?family_mode=1&find_best_match=1"
"""
from __future__ import annotations

import argparse
import resource
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fasta_bodies(res: np.ndarray, off: np.ndarray, body_bytes: int):
    """FASTA records '>q<i>\\n<seq>\\n' grouped into bodies of <= body_bytes."""
    raw = res.tobytes()
    bodies, cur, cur_len, cur_res = [], [], 0, 0
    out = []
    for i in range(len(off) - 1):
        rec = b">q%d\n" % i + raw[off[i]:off[i + 1]] + b"\n"
        if cur and cur_len + len(rec) > body_bytes:
            bodies.append(b"".join(cur))
            out.append(cur_res)
            cur, cur_len, cur_res = [], 0, 0
        cur.append(rec)
        cur_len += len(rec)
        cur_res += int(off[i + 1] - off[i])
    if cur:
        bodies.append(b"".join(cur))
        out.append(cur_res)
    return bodies, out


GENERA = [("Escherichia", 561), ("Bacillus", 1386), ("Mycoplasma", 2093), ("Streptomyces", 1883)]


def write_family_db(d: str, n: int) -> list:
    """families.tsv / genus.map / nr.fasta (the golden fq data set's formats)
    with family i = source protein i of the synthetic image."""
    from close_kmers_amd import synth
    with open(os.path.join(d, "genus.map"), "w") as f:
        for g, t in GENERA:
            f.write(f"{g}\t{t}\n")
    with open(os.path.join(d, "families.tsv"), "w") as fam, open(os.path.join(d, "nr.fasta"), "wb") as nr:
        for a in range(0, n, 20000):
            ids = np.arange(a, min(n, a + 20000))
            seqs = synth.ALPHA[synth.source_residue_codes(ids)]
            for i, row in zip(ids, seqs):
                g = GENERA[int(i) % len(GENERA)][0]
                peg = f"fig|{1000 + int(i) % 97}.{int(i) % 7}.peg.{int(i)}"
                fam.write(f"GF{int(i):08d}\t1\t1\t{peg}\t{len(row)}\tfunction {int(i) % 100000}\t100\t{g}\t100\n")
                nr.write(b">" + peg.encode() + b"\n" + row.tobytes() + b"\n")
    # (--families-nr takes every following non-option word: it goes after the positionals)
    return (["--families-genus-mapping", os.path.join(d, "genus.map"),
             "--families-file", os.path.join(d, "families.tsv")],
            ["--families-nr", os.path.join(d, "nr.fasta")])


def post(port: int, path: str, body: bytes) -> bytes:
    with socket.create_connection(("127.0.0.1", port), timeout=300) as s:
        s.sendall(b"POST %s HTTP/1.1\r\nContent-Length: %d\r\n\r\n" % (path.encode(), len(body)) + body)
        chunks = []
        while True:
            c = s.recv(1 << 20)
            if not c:
                break
            chunks.append(c)
    return b"".join(chunks)


LOAD_GEN_SRC = os.path.join(ROOT, "tools", "load_gen.cpp")
LOAD_GEN = os.path.join(ROOT, "tools", "load_gen")


def build_load_gen() -> str:
    if not os.path.exists(LOAD_GEN) or os.path.getmtime(LOAD_GEN) < os.path.getmtime(LOAD_GEN_SRC):
        subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", LOAD_GEN_SRC, "-o", LOAD_GEN], check=True)
    return LOAD_GEN


def get(port: int, path: str) -> bytes:
    with socket.create_connection(("127.0.0.1", port), timeout=60) as s:
        s.sendall(b"GET %s HTTP/1.1\r\n\r\n" % path.encode())
        chunks = []
        while True:
            c = s.recv(1 << 16)
            if not c:
                break
            chunks.append(c)
    return b"".join(chunks)


def server_stats(port: int, reset: bool = False) -> dict:
    r = get(port, "/server_stats" + ("?reset=1" if reset else ""))
    return json.loads(r.split(b"\n\n", 1)[1])


def cpu_snapshot(pid):
    """CPU seconds of the server process, the children waited for so far (the
    load generator) and the cgroup's usage/throttling where it shows them:
    the box runs in a CPU share, and a server and its load generator that
    together need more than that share are bound by it, not by the GPU"""
    snap = {"t": time.time()}
    try:
        f = open(f"/proc/{pid}/stat").read().rsplit(")", 1)[1].split()
        tck = os.sysconf("SC_CLK_TCK")
        snap["server_cpu_s"] = (int(f[11]) + int(f[12])) / tck
    except OSError:
        pass
    ru = resource.getrusage(resource.RUSAGE_CHILDREN)
    snap["children_cpu_s"] = ru.ru_utime + ru.ru_stime
    for path in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat", "/sys/fs/cgroup/cpuacct/cpuacct.usage"):
        try:
            for ln in open(path).read().split("\n"):
                kv = ln.split()
                if len(kv) == 2:
                    snap[path.rsplit("/", 1)[1] + ":" + kv[0]] = int(kv[1])
                elif len(kv) == 1:
                    snap[path.rsplit("/", 1)[1]] = int(kv[0])
        except (OSError, ValueError):
            pass
    return snap


def cpu_delta(a, b):
    dt = b["t"] - a["t"]
    out = {k: round((b[k] - a[k]) / dt, 3) for k in b if k != "t" and k in a}
    out["wall_s"] = round(dt, 3)
    return out


def cpu_limits():
    lim = {"affinity_cpus": len(os.sched_getaffinity(0))}
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us"):
        try:
            lim[path] = open(path).read().strip()
        except OSError:
            pass
    return lim


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-keys", type=float, default=1e9)
    ap.add_argument("--n-seq", type=int, default=100000)
    ap.add_argument("--clients", default="1,4,8,16")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--body-bytes", type=int, default=1 << 20)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--path", default="/query")
    ap.add_argument("--allow-failures", action="store_true", help="report failed requests instead of raising")
    ap.add_argument("--server-prefix", default="", help="command words put before the server (a profiler)")
    ap.add_argument("--families", type=int, default=0, help="synthetic family DB over this many source proteins")
    args = ap.parse_args()
    from close_kmers_amd import build as kbuild
    from close_kmers_amd import image_files, synth

    kbuild.build()
    load_gen = build_load_gen()
    spec = synth.ImageSpec(int(args.n_keys))
    res, off = synth.make_queries(spec, args.n_seq)
    bodies, body_res = fasta_bodies(res, off, args.body_bytes)
    tmp = tempfile.TemporaryDirectory()
    bodies_file = os.path.join(tmp.name, "bodies.bin")
    with open(bodies_file, "wb") as f:
        f.write(np.uint64(len(bodies)).tobytes())
        for b, r in zip(bodies, body_res):
            f.write(np.array([r, len(b)], np.uint64).tobytes() + b)
    image_files.write_index(os.path.join(tmp.name, "function.index"), [f"function {i}" for i in range(100000)])
    image_files.write_index(os.path.join(tmp.name, "otu.index"), ["otu0"])
    port_file = os.path.join(tmp.name, "port")
    fam_pre, fam_post = [], []
    if args.families:
        fam_pre, fam_post = write_family_db(tmp.name, min(args.families, spec.n_src))
    t0 = time.time()
    srv = subprocess.Popen(args.server_prefix.split() + [kbuild.SERVER, "--bind", "127.0.0.1", "--listen-port-file", port_file,
                            "--n-kmer-threads", str(args.threads),
                            "--synthetic-image", f"{spec.n_keys}:{spec.num_sigs}"] + fam_pre + ["0", tmp.name] + fam_post,
                           stderr=subprocess.PIPE)
    port = None
    while time.time() - t0 < 300:
        if srv.poll() is not None:
            raise RuntimeError(srv.stderr.read().decode())
        if os.path.exists(port_file) and open(port_file).read().strip():
            port = int(open(port_file).read())
            break
        time.sleep(0.1)
    assert port, "server did not start"
    startup_s = time.time() - t0
    print(f"[bench_server] server up in {startup_s:.1f} s, {len(bodies)} bodies", file=sys.stderr)
    try:
        # warm-up and a sanity check on the first body
        r = post(port, args.path, bodies[0])
        assert r.startswith(b"HTTP/1.1 200 OK"), r[:200]
        assert r.count(b"PROTEIN-ID") == bodies[0].count(b">") or args.path != "/query"
        rows = {}
        for c in [int(x) for x in args.clients.split(",")]:
            server_stats(port, reset=True)
            c0 = cpu_snapshot(srv.pid)
            r = subprocess.run([load_gen, str(port), args.path, bodies_file, str(c), str(args.seconds)],
                               capture_output=True, text=True, timeout=args.seconds + 600)
            if r.returncode != 0 and not (args.allow_failures and r.stdout.strip()):
                raise RuntimeError(f"load_gen: {r.stdout} {r.stderr}")
            row = json.loads(r.stdout)
            row["cpu_per_s"] = cpu_delta(c0, cpu_snapshot(srv.pid))
            row["server_stages"] = server_stats(port)
            rows[str(c)] = row
            print(f"[bench_server] clients={c}: {rows[str(c)]}", file=sys.stderr)
        best = max(rows.values(), key=lambda r: r["residues_per_s"])
        print(json.dumps({
            "metric": "HTTP serving residues/s through kgx_server (kser drop-in), C2 image",
            "value": best["residues_per_s"], "unit": "residues/s", "load_generator": "tools/load_gen.cpp",
            "config": {"n_keys": spec.n_keys, "num_sigs": spec.num_sigs, "path": args.path,
                       "families": args.families,
                       "body_bytes": args.body_bytes, "proteins_per_body": round(args.n_seq / len(bodies), 1),
                       "server_threads": args.threads, "startup_s": startup_s, "cpu_limits": cpu_limits()},
            "by_clients": rows,
            "note": "loopback TCP, native load generator (tools/load_gen) as its own process in the same CPU "
                    "share; server parses FASTA, one GPU pass per body piece, writes query_request text; "
                    "server_stages: the server's clocks per request (ms), gpu summed over a body's pieces"}))
    finally:
        try:
            with socket.create_connection(("127.0.0.1", port), timeout=60) as s:
                s.sendall(b"GET /quit HTTP/1.1\r\n\r\n")
                s.recv(1024)
        except OSError:
            pass
        try:
            srv.wait(timeout=60)
        except subprocess.TimeoutExpired:
            srv.kill()
        tmp.cleanup()


if __name__ == "__main__":
    main()
