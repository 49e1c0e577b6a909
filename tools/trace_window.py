"""Print the last lookup call's kernels and copies from a rocprofv3 CSV trace:

    python tools/trace_window.py DIR/kt [--marker probe_line] [--calls 1]

The window starts at the last H2D copy burst before the final `calls` groups
of the marker kernel; times in us from the window's first event, one line per
kernel or copy with its queue (or stream) and duration."""
from __future__ import annotations

import argparse
import csv
import re


def short(name):
    name = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", ""))
    name = re.sub(r"<.*>", "<>", name)
    return name.split("::")[-1][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--span-us", type=float, default=3000.0)
    args = ap.parse_args()
    ev = []
    with open(args.prefix + "_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "q%s" % r["Queue_Id"],
                       short(r["Kernel_Name"])))
    try:
        with open(args.prefix + "_memory_copy_trace.csv") as f:
            for r in csv.DictReader(f):
                d = "H2D" if "HOST_TO_DEVICE" in r["Direction"] else "D2H" if "DEVICE_TO_HOST" in r["Direction"] else "copy"
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "s%s" % r["Stream_Id"], d))
    except FileNotFoundError:
        pass
    ev.sort()
    # the last window: back from the final event by span-us, snapped to the first H2D in it
    end = max(e[1] for e in ev)
    lo = end - args.span_us * 1000
    h2d = [e for e in ev if e[3] == "H2D" and e[0] >= lo]
    t0 = min(e[0] for e in h2d) if h2d else lo
    busy = []
    for s, e, q, n in ev:
        if s >= t0 - 50_000:
            print("%9.1f %9.1f %7.1f  %-4s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, q, n))
            if e >= t0:
                busy.append((max(s, t0), e))
    busy.sort()
    tot, cur_s, cur_e = 0, None, None
    for s, e in busy:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    print("busy (union of kernels and copies) %.1f us" % (tot / 1e3))


if __name__ == "__main__":
    main()
