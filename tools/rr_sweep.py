"""Random-read ceiling of the resident 1B-entry image vs reads in flight per
lane (ILP) and workgroups per CU; modes key8 and rec16."""
import ctypes, json, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from close_kmers_amd import abi, synth
spec = synth.ImageSpec(10 ** 9)
img, _ = abi.Image.synthetic(spec.n_keys, spec.num_sigs)
ctx = abi.Context(img)
L = abi.lib()
out = {}
for wgs in (1, 2, 4, 8, 16):
    for ilp in (1, 2, 4, 8, 16):
        ctx.set_option("microbench_wgs", wgs)
        ctx.set_option("microbench_ilp", ilp)
        for mode, name in ((1, "key8"), (3, "rec16")):
            ms, reads = ctypes.c_float(), ctypes.c_uint64()
            for _ in range(2):
                abi.check(L.kgx_microbench_random_read(ctx.handle, 40_000_000, mode, ctypes.byref(ms),
                                                       ctypes.byref(reads)), "mb")
            out[f"wgs{wgs}_ilp{ilp}_{name}"] = round(reads.value / (ms.value / 1e3) / 1e9, 2)
    print(json.dumps({k: v for k, v in out.items() if k.startswith(f"wgs{wgs}_")}), file=sys.stderr, flush=True)
print(json.dumps(out))
