"""Device occupancy of a server under load from a rocprofv3 --kernel-trace CSV
(bench_server.py --server-prefix "rocprofv3 --kernel-trace ... --"): per
kernel the count and mean duration, and over the busiest 2-s window the
fraction of time with any kernel running (the union of kernel intervals) and
with a probe running.  python tools/server_trace.py DIR [requests]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def union(iv):
    iv.sort()
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:48]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    # the load window: kernels between the first and last probe launch after startup
    probes = [r for r in rows if "probe" in r[2]]
    t0 = probes[len(probes) // 10][0] if probes else rows[0][0]
    t1 = probes[-1][1] if probes else rows[-1][1]
    win = [r for r in rows if t0 <= r[0] and r[1] <= t1]
    agg = defaultdict(list)
    for s, e, n in win:
        agg[n].append((e - s) / 1e3)
    span = (t1 - t0) / 1e3
    out = {"window_us": round(span), "kernels": len(win),
           "busy_frac": round(union([(s, e) for s, e, _ in win]) / 1e3 / span, 3),
           "probe_busy_frac": round(union([(s, e) for s, e, n in win if "probe" in n]) / 1e3 / span, 3),
           "by_kernel": {n: {"count": len(v), "mean_us": round(sum(v) / len(v), 2), "sum_frac": round(sum(v) / span, 3)}
                         for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))}}
    if len(sys.argv) > 2:
        out["probe_launches_per_s"] = round(len([1 for r in win if "probe" in r[2]]) / span * 1e6)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
