"""Random-read rate of cooperative line reads (4 or 8 lanes per 64/128-B line)
vs per-lane 16-B record reads, whole table and cache-sized spans."""
import ctypes, json, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from close_kmers_amd import abi, synth
spec = synth.ImageSpec(10 ** 9)
img, _ = abi.Image.synthetic(spec.n_keys, spec.num_sigs)
img.set_layout(abi.Image.PACKED16)
ctx = abi.Context(img)
L = abi.lib()
out = {}
for span_mb in (64, 0):
    ctx.set_option("microbench_span", span_mb << 20)
    for mode, name in ((3, "rec16"), (4, "line64_quad"), (5, "line128_oct"), (2, "sector64_lane")):
        ms, reads = ctypes.c_float(), ctypes.c_uint64()
        for _ in range(2):
            abi.check(L.kgx_microbench_random_read(ctx.handle, 40_000_000, mode, ctypes.byref(ms),
                                                   ctypes.byref(reads)), "mb")
        out[f"{span_mb or 'all'}MB_{name}"] = round(reads.value / (ms.value / 1e3) / 1e9, 2)
        print(json.dumps(out), flush=True)
print(json.dumps(out))
