"""The expected digest of the bench's per-device canary pass
(close_kmers_amd/canary.py), computed by the CPU oracle.

    python tests/golden/make_canary.py [--check]

The image is the synthetic generator's CANARY_KEYS entries (duplicates
dropped, lowest entry id kept) inserted sequentially into the builder-sized
table (oracle.build_table, kguts.cc:202-222) -- the device builder
(kgx_image_build_synthetic) stores the same entries, and a probe's results do
not depend on which bucket of a chain holds a key.  The batch is CANARY_SEQ
synthetic 300-aa proteins; the oracle runs hits + calls + find_best_call per
sequence (want 11, lookup_request.cc:166-210) and the result is digested in
canary.digest's canonical layout.  Writes tests/golden/canary/digest.json;
--check recomputes and compares instead.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from close_kmers_amd import canary, synth  # noqa: E402


def compute() -> dict:
    oracle.build(ref=None)
    t0 = time.time()
    spec = synth.ImageSpec(canary.CANARY_KEYS)
    keys, fI, oI, avg, wt = spec.unique_entries()
    table = oracle.build_table(spec.num_sigs, keys, fI, oI, avg, wt)
    res, off = synth.make_queries(spec, canary.CANARY_SEQ, length=canary.CANARY_LEN,
                                  x_permille=canary.CANARY_X_PERMILLE, q0=canary.CANARY_Q0)
    r = oracle.process_batch(table, res, off, want=canary.CANARY_WANT)
    dg = canary.digest(r.hit_offsets, r.hits, r.call_offsets, r.calls, r.best)
    return {"digest": dg, "hits": int(r.hit_offsets[-1]), "calls": int(r.call_offsets[-1]),
            "n_keys": canary.CANARY_KEYS, "keys_stored": int(len(keys)), "num_sigs": spec.num_sigs,
            "n_seq": canary.CANARY_SEQ, "length": canary.CANARY_LEN, "x_permille": canary.CANARY_X_PERMILLE,
            "q0": canary.CANARY_Q0, "want": canary.CANARY_WANT,
            "generator": "tests/golden/make_canary.py (CPU oracle)", "seconds": round(time.time() - t0, 1)}


if __name__ == "__main__":
    got = compute()
    if "--check" in sys.argv:
        want = canary.expected()
        ok = got["digest"] == want["digest"]
        print(json.dumps({"ok": ok, "got": got["digest"], "want": want["digest"]}))
        sys.exit(0 if ok else 1)
    os.makedirs(os.path.dirname(canary.DIGEST_JSON), exist_ok=True)
    got.pop("seconds")
    with open(canary.DIGEST_JSON, "w") as f:
        json.dump(got, f, indent=1)
    print(json.dumps(got))
