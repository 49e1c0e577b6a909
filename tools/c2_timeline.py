"""C2 step timeline from a rocprofv3 --kernel-trace run of bench.py: the last N
probe launches, each probe's duration, the gap to the next probe, and the
other kernels that start while it runs (name@start offset+duration, us).

    python tools/c2_timeline.py DIR [--last 12] [--marker probe_line_kernel]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re


def short(name):
    name = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))
    return name.split("::")[-1][:32]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=12)
    ap.add_argument("--marker", default="probe_line_kernel")
    args = ap.parse_args()
    f = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(open(f)))
    allp = [e for e in ev if args.marker in e[2]]
    # the timed steps: the longest run of probes each starting within 200 us
    # of the previous one's end (the later legs of bench.py probe too)
    best, cur = (0, 0), 0
    for i in range(1, len(allp)):
        if allp[i][0] - allp[i - 1][1] > 200_000:
            cur = i
        if i - cur > best[1] - best[0]:
            best = (cur, i)
    probes = allp[best[0]:best[1] + 1][-(args.last + 1):]
    busy = []
    for p, q in zip(probes, probes[1:]):
        others = [e for e in ev if p[0] <= e[0] < q[0] and args.marker not in e[2]]
        desc = ", ".join(f"{e[2]}@{(e[0] - p[0]) / 1e3:.0f}+{(e[1] - e[0]) / 1e3:.0f}" for e in others)
        dur, gap = (p[1] - p[0]) / 1e3, (q[0] - p[1]) / 1e3
        busy.append((dur, gap))
        print(f"probe {dur:7.1f} us, gap {gap:6.1f} us; {desc}")
    if busy:
        print(f"mean probe {sum(b[0] for b in busy) / len(busy):.1f} us, mean gap {sum(b[1] for b in busy) / len(busy):.1f} us")


if __name__ == "__main__":
    main()
