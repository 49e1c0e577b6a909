"""The kser request surface over HTTP (kgx_server, krequest2.cc:273-489 routes).

GPU tests drive every golden handler case through a running server and
compare the response body with the same golden text the kgx_query driver and
the oracle reproduce; CPU tests cover the command line and the start-up
errors, which need no device."""
import os
import socket
import subprocess
import tempfile
import time

import pytest

from close_kmers_amd import build as kbuild
from helpers import GOLDEN
from test_oracle_golden import FQ_FILES, PARAMS, parse_case

HEADER = b"HTTP/1.1 200 OK\nContent-type: text/plain\n\n"


def _server_exe():
    kbuild.build()
    return kbuild.SERVER


def test_server_usage_and_bad_data_dir():
    exe = _server_exe()
    r = subprocess.run([exe, "--help"], capture_output=True, timeout=60)
    assert r.returncode == 2 and b"listen-port kmer-data-dir" in r.stderr
    r = subprocess.run([exe, "--bind", "127.0.0.1", "0", "/nonexistent-kmer-dir"], capture_output=True,
                       timeout=60)
    assert r.returncode == 1 and b"kmer.table.mem_map" in r.stderr
    r = subprocess.run([exe, "--bogus", "0", "x"], capture_output=True, timeout=60)
    assert r.returncode == 2
    for bad in ("3-1", "", "a", "0,,1", "-2"):
        r = subprocess.run([exe, "--devices", bad, "0", "x"], capture_output=True, timeout=60)
        assert r.returncode == 2 and b"--devices" in r.stderr, bad


class Server:
    """A kgx_server on 127.0.0.1 with an ephemeral port."""

    def __init__(self, data_dir, family_db=False, threads=2, devices=None, extra=()):
        self.tmp = tempfile.TemporaryDirectory()
        port_file = os.path.join(self.tmp.name, "port")
        args = [_server_exe(), "--bind", "127.0.0.1", "--listen-port-file", port_file,
                "--n-kmer-threads", str(threads), "--kmer-version", "kv1"]
        if devices:
            args += ["--devices", devices]
        args += list(extra)
        if family_db:
            fq = os.path.join(GOLDEN, "fq")
            args += ["--families-genus-mapping", os.path.join(fq, FQ_FILES["genus"]),
                     "--families-file", os.path.join(fq, FQ_FILES["families"]),
                     "--families-version", "fv1"]
        args += ["0", data_dir]
        if family_db:
            args += ["--families-nr", os.path.join(GOLDEN, "fq", FQ_FILES["nr"])]
        self.err_path = os.path.join(self.tmp.name, "stderr")
        self.err = open(self.err_path, "wb")
        self.proc = subprocess.Popen(args, stderr=self.err)
        deadline = time.time() + 120
        self.port = None
        while time.time() < deadline:
            if self.proc.poll() is not None:
                raise RuntimeError(open(self.err_path, "rb").read().decode())
            try:
                txt = open(port_file).read().strip()
                if txt:
                    self.port = int(txt)
                    break
            except FileNotFoundError:
                pass
            time.sleep(0.05)
        assert self.port, "server did not start"

    def request(self, method, path, body=b"", headers=b"", length=None):
        with socket.create_connection(("127.0.0.1", self.port), timeout=120) as s:
            head = f"{method} {path} HTTP/1.1\r\nHost: x\r\n"
            if method == "POST":
                head += f"Content-Length: {len(body) if length is None else length}\r\n"
            s.sendall(head.encode() + headers + b"\r\n" + body)
            out = b""
            while True:
                chunk = s.recv(1 << 16)
                if not chunk:
                    return out
                out += chunk

    def log(self) -> bytes:
        self.err.flush()
        return open(self.err_path, "rb").read()

    def close(self):
        if self.proc.poll() is None:
            r = self.request("GET", "/quit")
            assert b"OK, quitting" in r
            self.proc.wait(timeout=60)
        self.err.close()
        assert self.proc.returncode == 0
        self.tmp.cleanup()


def _query_string(pname):
    p = {k: v for k, v in PARAMS[pname].items() if k != "family_mode"}
    return "&".join(f"{k}={v}" for k, v in p.items())


def _cases(ds):
    d = os.path.join(GOLDEN, ds)
    return sorted(f for f in os.listdir(d) if f.startswith("expected_") and f.endswith(".txt"))


QUERY_FLAGS = {"query": "", "query_details": "details=1", "query_best": "find_best_call=1"}


@pytest.mark.gpu
@pytest.mark.parametrize("ds", ["scoring", "edge", "cap"])
def test_query_and_add_routes_match_golden(gpu, ds):
    d = os.path.join(GOLDEN, ds)
    fasta = open(os.path.join(d, "input.fasta"), "rb").read()
    srv = Server(os.path.join(d, "data"))
    try:
        for fname in _cases(ds):
            mode, pname = parse_case(fname)
            qs = "&".join(x for x in (QUERY_FLAGS.get(mode, ""), _query_string(pname)) if x)
            route = "/query" if mode in QUERY_FLAGS else "/mapping/m_%s/add" % pname
            got = srv.request("POST", route + ("?" + qs if qs else ""), fasta)
            assert got.startswith(HEADER), (fname, got[:80])
            assert got[len(HEADER):] == open(os.path.join(d, fname), "rb").read(), fname
    finally:
        srv.close()


@pytest.mark.gpu
def test_server_stats_count_the_request_stages(gpu):
    """GET /server_stats: the server's per-stage clocks (recv, parse, gpu,
    handle, send) over the requests served since the last ?reset=1."""
    import json
    d = os.path.join(GOLDEN, "edge")
    fasta = open(os.path.join(d, "input.fasta"), "rb").read()
    srv = Server(os.path.join(d, "data"))
    try:
        srv.request("GET", "/server_stats?reset=1")
        for _ in range(3):
            assert srv.request("POST", "/query", fasta).startswith(HEADER)
        r = srv.request("GET", "/server_stats")
        st = json.loads(r.split(b"\n\n", 1)[1])
        assert st["requests"] == 3 and st["bytes_in"] == 3 * len(fasta) and st["gpu_passes"] >= 3
        ms = st["ms_per_request"]
        assert all(ms[k] > 0 for k in ("recv", "parse", "gpu", "handle", "send"))
        assert ms["handle"] >= ms["gpu"]
        srv.request("GET", "/server_stats?reset=1")
        st = json.loads(srv.request("GET", "/server_stats").split(b"\n\n", 1)[1])
        assert st["requests"] == 0
    finally:
        srv.close()


@pytest.mark.gpu
def test_concurrent_requests_match_golden(gpu):
    """Requests on 8 connections at once (4 KmerGuts workers) get the same
    bytes as one at a time; a client sending Expect: 100-continue gets the
    interim response first (krequest2.cc:262-270)."""
    import threading
    d = os.path.join(GOLDEN, "edge")
    fasta = open(os.path.join(d, "input.fasta"), "rb").read()
    cases = [f for f in _cases("edge") if parse_case(f)[0] in QUERY_FLAGS]
    srv = Server(os.path.join(d, "data"), threads=4)
    errors = []

    def run(fname):
        mode, pname = parse_case(fname)
        qs = "&".join(x for x in (QUERY_FLAGS[mode], _query_string(pname)) if x)
        for _ in range(3):
            got = srv.request("POST", "/query" + ("?" + qs if qs else ""), fasta)
            if got != HEADER + open(os.path.join(d, fname), "rb").read():
                errors.append(fname)

    try:
        ths = [threading.Thread(target=run, args=(f,)) for f in cases[:8]]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert not errors, errors
        with socket.create_connection(("127.0.0.1", srv.port), timeout=120) as s:
            s.sendall(b"POST /query HTTP/1.1\r\nExpect: 100-continue\r\nContent-Length: %d\r\n\r\n"
                      % len(fasta))
            assert s.recv(64).startswith(b"HTTP/1.1 100 Continue")
            s.sendall(fasta)
            out = b""
            while True:
                c = s.recv(1 << 16)
                if not c:
                    break
                out += c
        assert out.endswith(open(os.path.join(d, "expected_query_default.txt"), "rb").read())
    finally:
        srv.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mib", [5, 1])
def test_large_query_body_runs_in_pieces_and_matches_oracle(gpu, oracle_lib, tmp_path, mib):
    """A 5-MiB /query body is cut at record starts and its pieces run on 4
    workers at once; a 1-MiB body is one GPU pass whose parse and text run in
    sub-pieces on the router's helper threads.  Either way the response is
    the oracle's text for the whole body."""
    import numpy as np
    from helpers import random_protein
    d = os.path.join(GOLDEN, "scoring")
    base = open(os.path.join(d, "input.fasta"), "rb").read()
    rng = np.random.default_rng(99)
    recs = [base]
    size = len(base)
    i = 0
    while size < mib << 20:
        r = b">p%d\n%s\n" % (i, random_protein(rng, int(rng.integers(5, 600))).encode())
        recs.append(r)
        size += len(r)
        i += 1
        if i % 50 == 0:
            recs.append(base)
            size += len(base)
    body = b"".join(recs)
    fasta = tmp_path / "big.fasta"
    fasta.write_bytes(body)
    want = oracle_lib.query_text(os.path.join(d, "data"), str(fasta), "query", {})
    srv = Server(os.path.join(d, "data"), threads=4)
    try:
        got = srv.request("POST", "/query", body)
        assert got == HEADER + want
        got = srv.request("POST", "/query?details=1", body)
        want_d = oracle_lib.query_text(os.path.join(d, "data"), str(fasta), "query_details", {})
        assert got == HEADER + want_d
        if mib == 1:
            got = srv.request("POST", "/query?find_best_call=1", body)
            want_b = oracle_lib.query_text(os.path.join(d, "data"), str(fasta), "query_best", {})
            assert got == HEADER + want_b
    finally:
        srv.close()


@pytest.mark.gpu
def test_matrix_route_after_add_matches_golden(gpu):
    d = os.path.join(GOLDEN, "matrix")
    fasta = open(os.path.join(d, "input.fasta"), "rb").read()
    srv = Server(os.path.join(d, "data"))
    try:
        r = srv.request("POST", "/mapping/mx/add?silent=1", fasta)
        assert r == HEADER  # silent: header only
        got = srv.request("POST", "/mapping/mx/matrix", fasta)
        assert got == HEADER + open(os.path.join(d, "expected_matrix_default.txt"), "rb").read()
        # a mapping key nobody /add-ed: no partners, empty matrix
        assert srv.request("POST", "/mapping/other/matrix", fasta) == HEADER
        sizes = srv.request("GET", "/dump_sizes")
        assert b"Mapping 'mx':" in sizes and b"peg_to_id_: size=" in sizes
    finally:
        srv.close()


@pytest.mark.gpu
def test_lookup_peg_mode_routes_match_oracle(gpu, oracle_lib):
    """A server without --families-file is in peg mode (kser.cc:289) and its
    mappings carry no family data, so the expected text is the oracle's
    /add + /lookup without a family DB (the golden peg files were made with
    one, which only kgx_query's file arguments can combine with peg mode)."""
    d = os.path.join(GOLDEN, "lookup")
    fasta_path = os.path.join(d, "input.fasta")
    fasta = open(fasta_path, "rb").read()
    srv = Server(os.path.join(d, "data"))
    try:
        assert srv.request("POST", "/add?silent=1", fasta) == HEADER
        for pname in ("peg", "peg_all"):
            qs = _query_string(pname)
            got = srv.request("POST", "/lookup" + ("?" + qs if qs else ""), fasta)
            want = oracle_lib.query_text(os.path.join(d, "data"), fasta_path, "lookup", PARAMS[pname])
            assert want.count(b"//") > 5
            assert got == HEADER + want, pname
        v = srv.request("GET", "/version")
        assert v.endswith(b"kmer\tkv1\nfamily-mode\t0\n")
    finally:
        srv.close()


@pytest.mark.gpu
def test_family_mode_lookup_and_fq_routes_match_golden(gpu):
    d = os.path.join(GOLDEN, "lookup")
    fasta = open(os.path.join(d, "input.fasta"), "rb").read()
    srv = Server(os.path.join(d, "data"), family_db=True)
    try:
        for fname in _cases("lookup"):
            mode, pname = parse_case(fname)
            if not pname.startswith("fam_"):
                continue
            got = srv.request("POST", "/lookup?" + _query_string(pname), fasta)
            assert got == HEADER + open(os.path.join(d, fname), "rb").read(), fname
        v = srv.request("GET", "/version")
        assert v.endswith(b"kmer\tkv1\nfamilies\tfv1\nfamily-mode\t1\n")
        assert srv.request("GET", "/genus_lookup/Escherichia").endswith(b"\n\n561\n")
        assert srv.request("GET", "/genus_lookup/no_such_genus").startswith(b"HTTP/1.1 404 Not Found")
        # lookup_request.cc:74 resolves target_genus with genus_map_[...] (kmer.h:136), which
        # inserts an unknown genus with an empty id: /genus_lookup finds it afterwards
        srv.request("POST", "/lookup?target_genus=Nogenus", fasta)
        assert srv.request("GET", "/genus_lookup/Nogenus").endswith(b"\n\n\n")
        assert srv.request("GET", "/nowhere").startswith(b"HTTP/1.1 404 Not found")
        assert srv.request("POST", "/nowhere", b"x").startswith(b"HTTP/1.1 404 Not found")
        assert srv.request("POST", "/fq_lookup", b"").endswith(b"\n\ndata done\n")
    finally:
        srv.close()
    fq = os.path.join(GOLDEN, "fq")
    srv = Server(os.path.join(fq, "data"), family_db=True)
    try:
        got = srv.request("POST", "/fq_lookup", open(os.path.join(fq, "input.fasta"), "rb").read())
        assert got == HEADER + open(os.path.join(fq, "expected_fq_default.txt"), "rb").read()
    finally:
        srv.close()


@pytest.mark.gpu
def test_concurrent_family_lookups_share_passes_and_match_golden(gpu):
    """Family /lookup requests on 12 connections at once (6 workers): the
    pieces of requests in flight share device passes (LookupBatcher: one
    staging area fills while the other's pass runs) and every response is the
    golden text byte for byte, whatever it shared a pass with; /server_stats
    shows pieces carried by shared passes.  KGX_LOOKUP_BATCH=0 (the default)
    gives the same bytes with every piece alone."""
    import json
    import threading
    d = os.path.join(GOLDEN, "lookup")
    fasta = open(os.path.join(d, "input.fasta"), "rb").read()
    cases = [f for f in _cases("lookup") if parse_case(f)[1].startswith("fam_")]
    assert len(cases) >= 3
    for batch in ("1", "0"):
        before = os.environ.get("KGX_LOOKUP_BATCH")
        os.environ["KGX_LOOKUP_BATCH"] = batch
        try:
            srv = Server(os.path.join(d, "data"), family_db=True, threads=6)
        finally:
            if before is None:
                del os.environ["KGX_LOOKUP_BATCH"]
            else:
                os.environ["KGX_LOOKUP_BATCH"] = before
        errors = []

        def run(k):
            for i in range(6):
                fname = cases[(k + i) % len(cases)]
                got = srv.request("POST", "/lookup?" + _query_string(parse_case(fname)[1]), fasta)
                if got != HEADER + open(os.path.join(d, fname), "rb").read():
                    errors.append(fname)

        try:
            srv.request("GET", "/server_stats?reset=1")
            ths = [threading.Thread(target=run, args=(k,)) for k in range(12)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            assert not errors, (batch, errors[:4])
            st = json.loads(srv.request("GET", "/server_stats").split(b"\n\n", 1)[1])
            print(batch, st)
            if batch == "1":
                assert st["batched_pieces"] >= st["batched_passes"] > 0, st
            else:
                assert st["batched_pieces"] == 0, st
        finally:
            srv.close()


@pytest.mark.gpu
def test_family_lookup_text_parts_equal_serial_text(gpu):
    """A family /lookup with find_best_match over a 3-MiB body (the golden
    proteins again and again between random ones: pieces of thousands of
    sequences, some with many rollup rows): the text written in parts on the
    text helpers (each part's map grown as the request's map would be at the
    part's first sequence, kgx_score_map.h) is the text of one thread
    (KGX_TEXT_HELPERS=0) byte for byte, for every golden family parameter set."""
    d = os.path.join(GOLDEN, "lookup")
    cases = [f for f in _cases("lookup") if parse_case(f)[1].startswith("fam_")]
    body = _big_body(seed=5, mib=3, base_name=os.path.join("lookup", "input.fasta"), every=3)
    outs = {}
    for helpers in ("0", "8"):
        before = os.environ.get("KGX_TEXT_HELPERS")
        os.environ["KGX_TEXT_HELPERS"] = helpers
        try:
            srv = Server(os.path.join(d, "data"), family_db=True, threads=2)
        finally:
            if before is None:
                del os.environ["KGX_TEXT_HELPERS"]
            else:
                os.environ["KGX_TEXT_HELPERS"] = before
        try:
            outs[helpers] = [srv.request("POST", "/lookup?" + _query_string(parse_case(f)[1]), body) for f in cases]
        finally:
            srv.close()
    for f, a, b in zip(cases, outs["0"], outs["8"]):
        assert a.startswith(HEADER) and a.count(b"\n") > 3000, f
        assert a == b, f


def _big_body(seed=99, mib=5, base_name=os.path.join("scoring", "input.fasta"), every=50):
    import numpy as np
    from helpers import random_protein
    base = open(os.path.join(GOLDEN, base_name), "rb").read()
    rng = np.random.default_rng(seed)
    recs, size, i = [base], len(base), 0
    while size < mib << 20:
        r = b">p%d\n%s\n" % (i, random_protein(rng, int(rng.integers(5, 600))).encode())
        recs.append(r)
        size += len(r)
        i += 1
        if i % every == 0:
            recs.append(base)
            size += len(base)
    return b"".join(recs)


@pytest.mark.gpu
def test_devices_replicas_serve_every_route(gpu, oracle_lib, tmp_path):
    """kgx_server --devices: one image replica per listed device (here three
    replicas on device 0 of a one-GPU box, the same code an 8-GPU node runs),
    workers spread over them, a large /query cut into pieces that run on
    several replicas at once, /add + /matrix on the mappings' device, family
    /lookup and /fq_lookup on any replica: every response is the golden /
    oracle text."""
    import threading
    d = os.path.join(GOLDEN, "scoring")
    body = _big_body(7, 5)
    fasta = tmp_path / "big.fasta"
    fasta.write_bytes(body)
    want = oracle_lib.query_text(os.path.join(d, "data"), str(fasta), "query", {})
    srv = Server(os.path.join(d, "data"), threads=5, devices="0,0,0")
    try:
        assert b"workers on devices 0 0 0 0 0" in srv.log()
        outs = [None] * 3

        def run(i):
            outs[i] = srv.request("POST", "/query", body)

        ths = [threading.Thread(target=run, args=(i,)) for i in range(3)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert all(o == HEADER + want for o in outs)
        md = os.path.join(GOLDEN, "matrix")
        mfasta = open(os.path.join(md, "input.fasta"), "rb").read()
    finally:
        srv.close()
    srv = Server(os.path.join(md, "data"), threads=3, devices="0,0")
    try:
        assert srv.request("POST", "/mapping/mx/add?silent=1", mfasta) == HEADER
        got = srv.request("POST", "/mapping/mx/matrix", mfasta)
        assert got == HEADER + open(os.path.join(md, "expected_matrix_default.txt"), "rb").read()
    finally:
        srv.close()
    ld = os.path.join(GOLDEN, "lookup")
    lfasta = open(os.path.join(ld, "input.fasta"), "rb").read()
    srv = Server(os.path.join(ld, "data"), family_db=True, threads=4, devices="0,0")
    try:
        cases = [f for f in _cases("lookup") if parse_case(f)[1].startswith("fam_")]
        errors = []

        def look(fname):
            got = srv.request("POST", "/lookup?" + _query_string(parse_case(fname)[1]), lfasta)
            if got != HEADER + open(os.path.join(ld, fname), "rb").read():
                errors.append(fname)

        ths = [threading.Thread(target=look, args=(f,)) for f in cases]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert cases and not errors, errors
    finally:
        srv.close()
    fq = os.path.join(GOLDEN, "fq")
    srv = Server(os.path.join(fq, "data"), family_db=True, threads=2, devices="0,0")
    try:
        got = srv.request("POST", "/fq_lookup", open(os.path.join(fq, "input.fasta"), "rb").read())
        assert got == HEADER + open(os.path.join(fq, "expected_fq_default.txt"), "rb").read()
    finally:
        srv.close()


@pytest.mark.gpu
def test_request_size_and_mapping_caps(gpu):
    """Oversized headers answer 431, an oversized Content-length 413 (before
    any body is read), a new /mapping key past --max-mappings 503; the server
    keeps serving afterwards."""
    d = os.path.join(GOLDEN, "scoring")
    fasta = open(os.path.join(d, "input.fasta"), "rb").read()
    srv = Server(os.path.join(d, "data"), extra=["--max-header-kb", "4", "--max-body-mb", "1",
                                                 "--max-mappings", "2"])
    try:
        r = srv.request("GET", "/version", headers=b"X-Big: " + b"a" * 8000 + b"\r\n")
        assert r.startswith(b"HTTP/1.1 431 "), r[:80]
        r = srv.request("POST", "/query", body=b"", length=2 << 20)
        assert r.startswith(b"HTTP/1.1 413 "), r[:80]
        ok = srv.request("POST", "/query", fasta)
        assert ok.startswith(HEADER)
        for key, code in (("a", b"200"), ("b", b"200"), ("a", b"200"), ("c", b"503")):
            r = srv.request("POST", f"/mapping/{key}/add?silent=1", fasta)
            assert r.startswith(b"HTTP/1.1 " + code), (key, r[:80])
        assert srv.request("POST", "/query", fasta) == ok
    finally:
        srv.close()
