"""Per-position kernel times of the ResNet-18 forward from a rocprofv3 kernel
trace (CSV or rocpd .db): forwards are split at each stem launch."""
import collections
import statistics
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from kstats import rows  # noqa: E402

seq = [(n, d) for n, d, _ in rows(sys.argv[1]) if "dlq" in n or "stem" in n or "conv" in n or "gap" in n]
fwds, cur = [], []
for n, d in seq:
    if "stem" in n and cur:
        fwds.append(cur)
        cur = []
    cur.append((n, d))
if cur:
    fwds.append(cur)
L = collections.Counter(len(f) for f in fwds).most_common(1)[0][0]
fwds = [f for f in fwds if len(f) == L][1:]
tot = 0.0
for i in range(L):
    ds = [f[i][1] for f in fwds]
    med = statistics.median(ds)
    tot += med
    name = fwds[0][i][0].replace("void dlq::(anonymous namespace)::", "").replace("dlq::(anonymous namespace)::", "")
    print(f"{i:2d} {med:8.1f} us  {name[:70]}")
print(f"forwards {len(fwds)}, kernels/forward {L}, sum of medians {tot:.1f} us")
