"""Per-launch HBM traffic of the probe kernel from two rocprofv3 --pmc passes.

    python profiles/traffic.py FETCH_DIR WRITE_DIR BENCH_JSON > probe_traffic.json

FETCH_DIR / WRITE_DIR hold the *_counter_collection.csv of a `--pmc FETCH_SIZE`
and a `--pmc WRITE_SIZE` pass over `bench.py` (separate passes: the two do not
fit one TCC pass on gfx950).  BENCH_JSON is the JSON line that pass printed; it
supplies the workload (so bench.py only picks the file up for the same config)
and the read counts of the random-read microbenchmark, which calibrate the
counter for this access pattern (MI355X_MICROARCH.md, HBM: FETCH_SIZE is
TCC_EA0_RDREQ x 64 B; exact for 64-B random requests, half the bytes of wide
streaming reads; other widths must be calibrated on a known byte count).
The probe's reads are 8/16-B random loads, one 64-B request each, so its
FETCH_SIZE is taken as measured once the sector64 calibration reads ~64 B/read.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            rows.setdefault(r["Kernel_Name"], []).append(
                (int(r["Grid_Size"]), float(r["Counter_Value"]) * 1024.0))  # KiB
    return rows


def mean_of(rows, pred, full_grid_only=False):
    """Mean counter value over the dispatches of the matching kernels.  With
    full_grid_only, only the largest grid counts: bench.py's timed batch, not
    the smaller chunks of its host-buffer leg."""
    vals = [gv for k, vs in rows.items() if pred(k) for gv in vs]
    if full_grid_only and vals:
        g = max(gv[0] for gv in vals)
        vals = [gv for gv in vals if gv[0] == g]
    vals = [v for _, v in vals]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    fdir, wdir, bjson = sys.argv[1:4]
    bench = json.loads(open(bjson).read().strip().splitlines()[-1])
    fetch, write = per_dispatch(fdir, "FETCH_SIZE"), per_dispatch(wdir, "WRITE_SIZE")
    is_probe = lambda k: "probe_kernel" in k or "probe_line_kernel" in k
    pf, nf = mean_of(fetch, is_probe, True)
    pw, nw = mean_of(write, is_probe, True)
    calib = {}
    ceil = (bench.get("roofline") or {}).get("random_read_ceiling") or {}
    for mode, name in ((0, "bucket24"), (1, "key8"), (2, "sector64"), (3, "rec16"), (4, "line64")):
        b, n = mean_of(fetch, lambda k, m=mode: f"random_read_kernel<{m}," in k)
        reads = (ceil.get(name) or {}).get("reads")
        if b is not None and reads:
            calib[name] = {"fetch_bytes_per_read": b / reads, "dispatches": n}
    cfg = bench["config"]
    out = {
        "n_keys": cfg["n_keys"], "keys_stored": cfg.get("keys_stored"), "n_seq": cfg["n_seq_per_gpu"],
        "length": cfg["seq_len"],
        "image_layout": (bench.get("roofline") or {}).get("image_layout", "AOS24"),
        "line_index": (bench.get("roofline") or {}).get("line_index", 0),
        "fetch_bytes_per_launch": pf, "write_bytes_per_launch": pw,
        "hbm_bytes_per_launch": (pf or 0) + (pw or 0) if pf is not None else None,
        "probe_dispatches": {"fetch": nf, "write": nw},
        "random_read_calibration": calib,
        "windows_per_launch": cfg["n_seq_per_gpu"] * max(0, cfg["seq_len"] - 8),
    }
    if pf is not None:
        out["hbm_bytes_per_window"] = out["hbm_bytes_per_launch"] / out["windows_per_launch"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
