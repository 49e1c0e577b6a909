"""Device phases of the call service with OTU stats on images whose k-mers
carry varied OTUs (the C2 bench image's are all -1, so its calls always take
the one-OTU fast path).  Not a test: run by hand on a GPU box,

    KGX_SVC_DEBUG=1 python3 tests/perf_svc_otu_phases.py

prints, per OTU modulus, the mean store+score+tally phase per call (us) and
the distinct OTUs per call.  Lives in tests/ because it builds its tables with
the oracle's table builder."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import oracle
    from close_kmers_amd import abi, synth
    assert os.environ.get("KGX_SVC_DEBUG") == "1", "set KGX_SVC_DEBUG=1"
    oracle.build(ref=None)
    spec = synth.ImageSpec(30000)
    k, f, o, av, w = spec.unique_entries()
    res, off = synth.make_queries(spec, 400, x_permille=0, q0=9)
    seqs = [bytes(res[int(off[i]):int(off[i + 1])]) for i in range(400)]
    out = {}
    for mod in (0, 6, 97):
        oo = np.full_like(o, -1) if mod == 0 else (k % np.uint64(mod)).astype(np.int32)
        table = oracle.build_table(spec.num_sigs, k, f, oo, av, w)
        with abi.Image.from_table(table, device=0) as img:
            for otus in (False, True):
                for s in seqs[:50]:  # warm up
                    img.svc_call(s, None, want=3, otus=otus)
                c0 = img.svc_stat("calls")
                p0 = [img.svc_stat(f"phase_n{i}") for i in range(16)]
                n_otu = 0
                for s in seqs:
                    r = img.svc_call(s, None, want=3, otus=otus)
                    n_otu += len(r[2]) if otus else 0
                n = img.svc_stat("calls") - c0
                ph = [(img.svc_stat(f"phase_n{i}") - p0[i]) / n / 1e3 for i in range(16)]
                out[f"mod{mod}_otu{int(otus)}"] = {"calls": n, "wall_us": round(ph[0], 2),
                                                   "store_score_tally_us": round(ph[4], 2),
                                                   "tally_us": round(ph[6], 2),
                                                   "count_sort_us": round(ph[7], 2),
                                                   "fence_us": round(ph[14], 2),
                                                   "sort_clock_mhz": round(ph[15] * 1e3 / max(ph[7], 1e-9), 0),
                                                   "otus_per_call": round(n_otu / n, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
