"""Per-kernel average durations (us) from rocprofv3 --kernel-trace CSVs, one
column per run directory: python tools/trace_summary.py DIR [DIR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    agg = defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[:48]
        agg[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return agg


runs = [(os.path.basename(os.path.normpath(d)), load(d)) for d in sys.argv[1:]]
names = sorted({n for _, a in runs for n in a}, key=lambda n: -max(sum(a.get(n, [0])) for _, a in runs))
print(f"{'kernel':48s} " + " ".join(f"{r:>14s}" for r, _ in runs))
for n in names[:25]:
    print(f"{n:48s} " + " ".join(f"{(sum(a[n]) / len(a[n]) if n in a else 0):9.1f}x{len(a.get(n, [])):<4d}" for _, a in runs))
