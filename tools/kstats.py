"""Summarise a rocprofv3 kernel trace: median duration per (kernel, grid).

Accepts the CSV (`--output-format csv`, *_kernel_trace.csv) or the rocpd
SQLite database rocprofv3 writes by default (*_results.db).
"""
import collections
import csv
import sqlite3
import statistics
import sys


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, dur, gx, wx in c.execute("select name, duration, grid_x, workgroup_x from kernels"):
            yield name, dur / 1e3, gx // wx
    else:
        for r in csv.DictReader(open(path)):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            yield r["Kernel_Name"], dur, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])


d = collections.defaultdict(list)
for name, dur, blocks in rows(sys.argv[1]):
    name = name.replace("void dlq::(anonymous namespace)::", "").replace("dlq::(anonymous namespace)::", "")
    d[(name[:60], blocks)].append(dur)
tot = 0.0
out = []
for k, v in d.items():
    if len(v) < 5:
        continue
    out.append((statistics.median(v), len(v), k))
n_fwd = max(len(v) for v in d.values())
for med, n, k in sorted(out, key=lambda t: -t[0] * t[1]):
    per_fwd = n / n_fwd
    tot += med * per_fwd
    print(f"{med:9.1f} us  x{per_fwd:4.1f}/fwd  blocks={k[1]:6d}  {k[0]}")
print(f"sum of medians per forward: {tot:.1f} us")
