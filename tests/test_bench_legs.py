"""bench.py's pool_e2e and host_path_lookup legs on CPU, over stand-ins for
the ABI (no device here): which devices the C5 pool spans at N ranks, the
per-configuration sweep, the byte comparison against one context's pass
(and its failure), and the fields the bench line carries."""
import types

import numpy as np

import bench


class _Compact:
    def __init__(self, off, n_hits_per_seq, best, tamper=False):
        n = len(off) - 1
        ho = np.zeros(n + 1, np.uint64)
        ho[1:] = np.cumsum(n_hits_per_seq)
        self.result = types.SimpleNamespace(hit_offsets=ho, call_offsets=ho // 3, calls=np.arange(int(ho[-1] // 3)),
                                            best=best)
        self._tamper = tamper

    def expand(self, a, b):
        h = np.arange(int(self.result.hit_offsets[a]), int(self.result.hit_offsets[b]), dtype=np.uint64)
        if self._tamper and len(h):
            h[0] += 1
        return h


class _FakeABI:
    WANT_BEST = 8
    ROLLUP_FAMILY = 1

    def __init__(self, tamper_pool=False):
        self.tamper_pool = tamper_pool
        self.pools = []
        self.replicated = []

    @staticmethod
    def check(rc, what):
        assert rc == 0, what

    @staticmethod
    def pinned_empty(n, dtype=np.uint8):
        return np.zeros(n, dtype)

    def _hits(self, off):
        return (np.diff(off).astype(np.uint64) % 7)

    def Context(self, img):
        abi = self

        class C:
            handle = 1

            def synchronize(self):
                pass

            def process_batch_compact(self, res, off, params, want):
                return _Compact(off, abi._hits(off), np.arange(len(off) - 1))

            def close(self):
                pass
        return C()

    def Pool(self, images, n_ctx):
        abi = self
        abi.pools.append((len(images), n_ctx))

        class P:
            def __enter__(self):
                return self

            def __exit__(self, *a):
                pass

            def process_batch_compact(self, res, off, params, want):
                return _Compact(off, abi._hits(off), np.arange(len(off) - 1), tamper=abi.tamper_pool)
        return P()


class _Img:
    def __init__(self, dev, log):
        self.dev, self.log = dev, log

    def replicate(self, dv):
        self.log.append(dv)
        return _Img(dv, self.log)

    def close(self):
        pass


class _L:
    @staticmethod
    def kgx_device_alloc(dev, n, p):
        return 0

    @staticmethod
    def kgx_synth_queries(*a):
        return 0

    @staticmethod
    def kgx_memcpy_d2h(dst, src, n):
        return 0

    @staticmethod
    def kgx_device_free(p):
        return 0


def _offsets_writer(monkeypatch, n, Ls):
    """kgx_memcpy_d2h of the offsets: fill them as the device generator does"""
    real = np.empty

    def fake_empty(shape, dtype=float, *a, **k):
        out = real(shape, dtype, *a, **k)
        if dtype is np.uint64 and shape == n + 1:
            out[:] = np.arange(n + 1, dtype=np.uint64) * np.uint64(Ls)
        return out
    monkeypatch.setattr(bench.np, "empty", fake_empty)


def test_pool_devices_by_world():
    assert bench.pool_devices(0, 1, 1) == [0]
    assert bench.pool_devices(0, 8, 1) == [0]
    assert bench.pool_devices(0, 8, 8) == list(range(8))
    assert bench.pool_devices(3, 8, 2) == [3, 0]
    assert bench.pool_devices(0, 2, 8) == [0, 1]  # never more devices than are visible


def _run_pool_leg(monkeypatch, tamper):
    n, Ls = 4000, 300
    _offsets_writer(monkeypatch, n, Ls)
    abi = _FakeABI(tamper_pool=tamper)
    log = []
    spec = types.SimpleNamespace(n_keys=10 ** 6)
    out = bench.pool_e2e_leg(abi, _L, None, _Img(0, log), spec, [0, 1, 2], None, 11, n, Ls, 0)
    return abi, log, out


def test_pool_e2e_leg_fields_and_sweep(monkeypatch):
    abi, log, out = _run_pool_leg(monkeypatch, False)
    assert log == [1, 2]  # one replica per further device
    assert abi.pools == [(3, 3), (3, 6), (3, 12), (3, 24)]  # 1, 2, 4, 8 contexts per device
    assert out["match_single_context"] is True
    assert out["devices"] == [0, 1, 2]
    assert set(out["ms_by_config"]) == {f"{k}_ctx{c}" for k in ("pinned", "pageable") for c in (3, 6, 12, 24)}
    assert out["value"] == 4000 * 300 / (out["ms_per_batch"] / 1e3)
    assert out["contexts"] in (3, 6, 12, 24) and out["unit"] == "residues/s"


def test_pool_e2e_leg_reports_a_mismatch(monkeypatch):
    _, _, out = _run_pool_leg(monkeypatch, True)
    assert out["match_single_context"] is False
    assert not any(out["checks"].values())
