"""Per-kernel-family HBM traffic and launch durations from rocprofv3 output.

Parses (no GPU work here -- the rocprofv3 passes run from the shell, see
tools/gpu_pmc.sh):
  --fetch DIR   a `rocprofv3 --pmc FETCH_SIZE --output-format csv` run
  --write DIR   a `rocprofv3 --pmc WRITE_SIZE --output-format csv` run
  --trace DIR   a `rocprofv3 --kernel-trace --stats --output-format csv` run
and writes a JSON summary keyed by the families of dlq_amd.lib.FAMILIES:

  hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024

FETCH_SIZE / WRITE_SIZE are KiB per dispatch measured at the L2's fabric side
(Infinity-Cache hits included).  On gfx950 FETCH_SIZE reports half the bytes
of a 16 B/lane streaming read (MI355X_MICROARCH.md, HBM section), hence the 2x;
WRITE_SIZE is exact for 16 B/lane stores.  Two separate passes because the two
counters do not fit one TCC pass.

bench.py reads `families[<name>]["hbm_bytes_per_launch"]` for the dominant
kernel's roofline.traffic; `avg_launch_us` from the kernel trace is the
rocprof-side duration to compare with bench.py's hipEvent figure.
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dlq_amd.lib import FAMILIES  # noqa: E402  (pure-Python constant; loads no library)

PREFIX = [("stem_fused_kernel", 0), ("stem2_kernel", 0), ("block_l1_kernel", 1), ("block_l1_sp_kernel", 1), ("conv3x3s1_kernel", 1), ("conv3x3s2i_kernel", 2),
          ("conv3x3s2_kernel", 2), ("conv3x3i_kernel", 3), ("conv3x3w_kernel", 3), ("gap16_kernel", 4), ("gap_fc_kernel", 4),
          ("linear_kernel", 5)]


def family_of(kernel_name):
    n = kernel_name.replace("void ", "").replace("dlq::(anonymous namespace)::", "")
    if n.startswith("conv_s8_kernel") and ", true>" in n:  # the F8 instantiations
        return 7
    for p, f in PREFIX:
        if n.startswith(p):
            return f
    return 6


def find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    if not hits:
        raise SystemExit(f"no {pattern} under {d}")
    return hits[0]


def counter_per_dispatch(d, counter):
    """{dispatch_id: (kernel_name, value)} summed over the counter's instances."""
    out = {}
    for r in csv.DictReader(open(find(d, "*counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        k = r.get("Dispatch_Id") or r.get("Correlation_Id")
        name, v = out.get(k, (r["Kernel_Name"], 0.0))
        out[k] = (name, v + float(r["Counter_Value"]))
    return out


def per_family(disp, skip_first):
    """Mean per launch per family, dropping each family's first `skip_first`
    launches (warm-up: first touches of the weights and buffers)."""
    seen = collections.Counter()
    vals = collections.defaultdict(list)
    for k in sorted(disp, key=lambda s: int(s)):
        name, v = disp[k]
        f = family_of(name)
        seen[f] += 1
        if seen[f] > skip_first[f]:
            vals[f].append(v)
    return {f: (statistics.fmean(v), len(v)) for f, v in vals.items() if v}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--trace")
    ap.add_argument("--warm-forwards", type=int, default=1,
                    help="forwards at the start of each run to leave out")
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--cmd", default="", help="the profiled command, recorded in the JSON")
    a = ap.parse_args()

    fetch = counter_per_dispatch(a.fetch, "FETCH_SIZE")
    write = counter_per_dispatch(a.write, "WRITE_SIZE")
    # launches per forward per family, from the fetch pass (the stem runs once per forward)
    cnt = collections.Counter(family_of(n) for n, _ in fetch.values())
    n_fwd = max(cnt[0], 1)
    skip = {f: a.warm_forwards * cnt[f] // n_fwd for f in range(len(FAMILIES))}
    fe, wr = per_family(fetch, skip), per_family(write, skip)
    dur = {}
    if a.trace:
        d = collections.defaultdict(list)
        for r in csv.DictReader(open(find(a.trace, "*kernel_trace.csv"))):
            d[family_of(r["Kernel_Name"])].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for f, v in d.items():
            v = v[skip[f]:] if len(v) > skip[f] else v
            dur[f] = (statistics.fmean(v), len(v))
    fams = {}
    for f, name in enumerate(FAMILIES):
        if f not in fe or f not in wr:
            continue
        ent = {"fetch_kib_per_launch": round(fe[f][0], 1), "write_kib_per_launch": round(wr[f][0], 1),
               "hbm_bytes_per_launch": round((2.0 * fe[f][0] + wr[f][0]) * 1024.0),
               "launches_per_forward": round(cnt[f] / n_fwd, 2), "launches_counted": fe[f][1]}
        if f in dur:
            ent["avg_launch_us"] = round(dur[f][0], 2)
            ent["trace_launches"] = dur[f][1]
        fams[name] = ent
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                     "--kernel-trace for durations",
           "formula": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024 "
                      "(gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md HBM section)",
           "note": "fabric-side L2 misses; Infinity-Cache (256 MiB) hits are counted as traffic",
           "command": a.cmd, "families": fams}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    for name, e in fams.items():
        print(f"{name:34s} {e['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch  "
              f"x{e['launches_per_forward']}/fwd  {e.get('avg_launch_us', float('nan')):8.2f} us")


if __name__ == "__main__":
    main()
