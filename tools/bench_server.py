"""End-to-end HTTP serving through kgx_server (the kser drop-in), C2 data.

    python tools/bench_server.py [--n-keys 1e9] [--clients 1,4,8,16] [--threads 8]

Starts close_kmers_amd/kgx_server on 127.0.0.1 with the C2 synthetic image
(--synthetic-image: 1B keys built in HBM, PACKED16) and --threads KmerGuts
workers, then C client threads POST FASTA bodies of the C2 query set to
/query (query_request.cc: PROTEIN-ID / CALL / OTU-COUNTS text back) and
read the responses to the end.  Bodies are cut at record boundaries to at
most --body-bytes (default 1 MiB, the reference's request buffer,
krequest2.cc:41).  Each request is one connection, as in krequest2.cc.
Reports per C the aggregate residues/s (residues in the bodies completed ÷
wall time) and the request latency (median, p99).  Prints one JSON line.

With --families N a synthetic family DB is loaded (families.tsv, genus.map
and nr.fasta over source proteins 0..N-1 of the synthetic image; each family
holds one protein) so that /lookup runs in family mode
(lookup_request.cc:153-400), e.g.
    python tools/bench_server.py --families 100000 --path "/lookup?family_mode=1&find_best_match=1"

Everything on the path is timed: loopback TCP, the server's FASTA parse,
the GPU pass (H2D, kernels, D2H of calls and OTU tallies), the text output.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-keys", type=float, default=1e9)
    ap.add_argument("--n-seq", type=int, default=100000)
    ap.add_argument("--clients", default="1,4,8,16")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--body-bytes", type=int, default=1 << 20)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--path", default="/query")
    ap.add_argument("--families", type=int, default=0, help="synthetic family DB over this many source proteins")
    args = ap.parse_args()
    from close_kmers_amd import build as kbuild
    from close_kmers_amd import image_files, synth

    kbuild.build()
    spec = synth.ImageSpec(int(args.n_keys))
    res, off = synth.make_queries(spec, args.n_seq)
    bodies, body_res = fasta_bodies(res, off, args.body_bytes)
    tmp = tempfile.TemporaryDirectory()
    image_files.write_index(os.path.join(tmp.name, "function.index"), [f"function {i}" for i in range(100000)])
    image_files.write_index(os.path.join(tmp.name, "otu.index"), ["otu0"])
    port_file = os.path.join(tmp.name, "port")
    fam_pre, fam_post = [], []
    if args.families:
        fam_pre, fam_post = write_family_db(tmp.name, min(args.families, spec.n_src))
    t0 = time.time()
    srv = subprocess.Popen([kbuild.SERVER, "--bind", "127.0.0.1", "--listen-port-file", port_file,
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
            lat, done_res, nxt = [], [0], [0]
            lock = threading.Lock()
            stop = time.perf_counter() + args.seconds

            def worker():
                while time.perf_counter() < stop:
                    with lock:
                        i = nxt[0] % len(bodies)
                        nxt[0] += 1
                    t = time.perf_counter()
                    out = post(port, args.path, bodies[i])
                    dt = time.perf_counter() - t
                    assert out.startswith(b"HTTP/1.1 200 OK")
                    with lock:
                        lat.append(dt)
                        done_res[0] += body_res[i]

            ths = [threading.Thread(target=worker) for _ in range(c)]
            t = time.perf_counter()
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            wall = time.perf_counter() - t
            lat_ms = np.array(lat) * 1e3
            rows[str(c)] = {"residues_per_s": done_res[0] / wall, "requests": len(lat),
                            "ms_median": float(np.median(lat_ms)), "ms_p99": float(np.percentile(lat_ms, 99))}
            print(f"[bench_server] clients={c}: {rows[str(c)]}", file=sys.stderr)
        best = max(rows.values(), key=lambda r: r["residues_per_s"])
        print(json.dumps({
            "metric": "HTTP serving residues/s through kgx_server (kser drop-in), C2 image",
            "value": best["residues_per_s"], "unit": "residues/s",
            "config": {"n_keys": spec.n_keys, "num_sigs": spec.num_sigs, "path": args.path,
                       "families": args.families,
                       "body_bytes": args.body_bytes, "proteins_per_body": round(args.n_seq / len(bodies), 1),
                       "server_threads": args.threads, "startup_s": startup_s},
            "by_clients": rows,
            "note": "loopback TCP; server parses FASTA, one GPU pass per body, writes query_request text"}))
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
