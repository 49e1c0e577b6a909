"""bench.py's C5 legs (pool_e2e, pool_lookup) on CPU, over stand-ins for the
ABI (no device here): which devices the C5 pool spans at N ranks, the
per-configuration sweep, the byte comparison against one context's pass
(and its failure), the per-device family maps, the HBM budget checks, and
the fields the bench line carries."""
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
        self.lookups = []
        self.kmaps = []
        self.free = {}

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

            def set_option(self, name, value):
                pass

            def process_batch_compact(self, res, off, params, want):
                return _Compact(off, abi._hits(off), np.arange(len(off) - 1))

            def process_batch(self, res, off, params, want):
                self.off = off
                return types.SimpleNamespace(best=np.arange(len(off) - 1, dtype=np.int64))

            def close(self):
                pass

            def __enter__(self):
                return self

            def __exit__(self, *a):
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

            def numa_nodes(self):
                return [im.device % 2 for im in images] * (n_ctx // len(images))

            def process_batch_compact(self, res, off, params, want):
                return _Compact(off, abi._hits(off), np.arange(len(off) - 1), tamper=abi.tamper_pool)

            def lookup(self, maps, res, off, params, want, copy=True):
                abi.lookups.append(sorted(m.dev for m in maps))
                ro, rows = _rollup(off)
                if abi.tamper_pool:
                    rows = rows.copy()
                    rows[-1] += 1
                return types.SimpleNamespace(best=np.arange(len(off) - 1, dtype=np.int64)), ro, rows
        return P()

    KMAP_SET = 1

    def Kmap(self, dev, mode):
        abi = self

        class K:
            def __init__(self):
                self.dev = dev
                abi.kmaps.append(dev)

            def add(self, keys, ids):
                assert len(keys) == len(ids) > 0

            def rollup(self, ctx, mode):
                return _rollup(ctx.off)

            def close(self):
                pass
        return K()

    def device_memory(self, dev):
        return self.free.get(dev, 200e9), 288e9


def _rollup(off):
    n = len(off) - 1
    ro = np.arange(n + 1, dtype=np.uint64) * np.uint64(2)
    return ro, np.arange(2 * n, dtype=np.uint32)


class _Img:
    def __init__(self, dev, log):
        self.dev, self.log = dev, log
        self.device = dev

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


def _c5(monkeypatch, n=4000, Ls=300):
    _offsets_writer(monkeypatch, n, Ls)
    abi = _FakeABI()
    spec = types.SimpleNamespace(n_keys=10 ** 6)
    return bench.c5_batch(abi, _L, _Img(0, []), spec, n, Ls, 0)


def _run_pool_leg(monkeypatch, tamper):
    pin, off = _c5(monkeypatch)
    abi = _FakeABI(tamper_pool=tamper)
    log = []
    img = _Img(0, log)
    images = [img] + [img.replicate(dv) for dv in (1, 2)]
    out = bench.pool_e2e_leg(abi, images, pin, off, None, 11)
    return abi, log, out


def test_pool_e2e_leg_fields_and_sweep(monkeypatch):
    abi, log, out = _run_pool_leg(monkeypatch, False)
    assert log == [1, 2]  # one replica per further device
    assert abi.pools == [(3, 3), (3, 6), (3, 12), (3, 24)]  # 1, 2, 4, 8 contexts per device
    assert out["match_single_context"] is True
    assert out["devices"] == [0, 1, 2] and out["numa_nodes"] == [0, 1, 0]
    assert set(out["ms_by_config"]) == {f"{k}_ctx{c}" for k in ("pinned", "pageable") for c in (3, 6, 12, 24)}
    assert out["value"] == 4000 * 300 / (out["ms_per_batch"] / 1e3)
    assert out["contexts"] in (3, 6, 12, 24) and out["unit"] == "residues/s"


def test_pool_e2e_leg_reports_a_mismatch(monkeypatch):
    _, _, out = _run_pool_leg(monkeypatch, True)
    assert out["match_single_context"] is False
    assert not any(out["checks"].values())


def _run_lookup_leg(monkeypatch, tamper):
    from close_kmers_amd import synth
    pin, off = _c5(monkeypatch, n=2000)
    abi = _FakeABI(tamper_pool=tamper)
    img = _Img(0, [])
    images = [img, _Img(3, []), _Img(5, [])]
    out = bench.pool_lookup_leg(abi, synth, images, synth.ImageSpec(10 ** 6), pin, off, None, n_fam=40)
    return abi, out


def test_pool_lookup_leg_one_map_per_device(monkeypatch):
    abi, out = _run_lookup_leg(monkeypatch, False)
    assert abi.kmaps == [0, 3, 5]  # a family map on every device of the pool
    assert abi.lookups and all(m == [0, 3, 5] for m in abi.lookups)  # every call gets all of them
    assert abi.pools == [(3, 12), (3, 24)]  # 4 and 8 contexts per device
    assert out["match_single_context"] is True and out["devices"] == [0, 3, 5]
    assert out["rollup_rows"] == 2 * 2000 and out["families"] == 40
    assert out["value"] == 2000 * 300 / (out["ms_per_batch"] / 1e3)


def test_pool_lookup_leg_reports_a_mismatch(monkeypatch):
    _, out = _run_lookup_leg(monkeypatch, True)
    assert out["match_single_context"] is False and not any(out["checks"].values())


def test_hbm_budget(monkeypatch):
    """The image's HBM at C2 (57 GB packed + 114 GB line index at load 36,
    85.4 GB while built) and the check's message."""
    import pytest
    b = bench.image_bytes(10 ** 9, 3_559_786_523, 36)
    assert round(b["packed16"] / 1e9, 1) == 57.0 and round(b["aos24"] / 1e9, 1) == 85.4
    assert round(b["line_index"] / 1e9, 1) == 113.8 and bench.image_bytes(10 ** 9, 10, 0)["line_index"] == 0
    abi = _FakeABI()
    abi.free = {2: 100e9}
    bench.hbm_check(abi, [0, 1], 180e9, "x")
    with pytest.raises(SystemExit) as e:
        bench.hbm_check(abi, [0, 2], 180e9, "an image replica")
    assert "device 2: 100.0 GB of 288.0 GB HBM free, but an image replica needs 180.0 GB" in str(e.value)
