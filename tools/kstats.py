"""Summarise a rocprofv3 kernel trace: median duration per (kernel, grid)."""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"]
    name = name.replace("void dlq::(anonymous namespace)::", "").replace("dlq::(anonymous namespace)::", "")
    d[(name[:60], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))].append(dur)
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
