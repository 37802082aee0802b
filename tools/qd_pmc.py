"""HBM bytes and GB/s of the standalone quantise / dequant passes from
rocprofv3 counters (north_star: "achieved HBM GB/s on the quant/dequant
passes", evidenced by rocprof counters, not events).  Test/measurement
tooling, not product code.

  python tools/qd_pmc.py --fetch DIR --write DIR --trace DIR [-o out.json]

DIRs are three separate rocprofv3 runs of `python3 tools/qd_time.py` (the
program directly after `--`): `--pmc FETCH_SIZE`, `--pmc WRITE_SIZE` and
`--kernel-trace --stats` (tools/qd_pmc.sh).  Per dispatch of the v4
(16-byte streaming) kernels (and the 4-byte dequant for HW % 4 != 0):

  counter bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024

(MI355X_MICROARCH.md, HBM: on gfx950 FETCH_SIZE counts half the bytes of a
16-B-per-lane streaming read; WRITE_SIZE is exact for 16-B stores), against
the algorithmic bytes of the call (quantise: 4 B in + 1 B out per element;
dequant: 4 B int32 in + 4 B fp32 out per element), and GB/s = counter bytes
/ the kernel's mean duration from the trace.
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    if not hits:
        raise SystemExit(f"no {pattern} under {d}")
    return hits[0]


def per_dispatch(d, counter):
    out = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(find(d, "*counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        out[k] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
    return out, names


def short(name):
    for key in ("quantize_f32_s8_v4_kernel", "dequant_s32_f32_v4_kernel", "dequant_s32_f32_kernel"):
        if key in name:
            return key
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("-o", default=None)
    a = ap.parse_args()
    fetch, fnames = per_dispatch(a.fetch, "FETCH_SIZE")
    write, wnames = per_dispatch(a.write, "WRITE_SIZE")
    # kernel durations (ns) from the trace, in dispatch order per kernel: the
    # qd_time.py calls in order are quantise (n), dequant (256x64x3136),
    # dequant (256x512x49), each 5 warm + 20 timed
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(find(a.trace, "*kernel_trace.csv"))):
        k = short(r["Kernel_Name"])
        if k:
            durs[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    n_q = 256 * 3 * 224 * 224
    shapes = [("quantize_f32_s8_v4_kernel", n_q, 5 * n_q),
              ("dequant_s32_f32_v4_kernel", 256 * 64 * 3136, 8 * 256 * 64 * 3136),
              # HW = 49 is not a multiple of 4: the 4-byte-per-lane kernel, whose
              # FETCH_SIZE scale is uncalibrated (the 2x is the 16-B rule)
              ("dequant_s32_f32_kernel", 256 * 512 * 49, 8 * 256 * 512 * 49)]
    fd = {k: [(i, fetch[i]) for i in sorted(fetch) if short(fnames[i]) == k] for k in set(s[0] for s in shapes)}
    wd = {k: [(i, write[i]) for i in sorted(write) if short(wnames[i]) == k] for k in set(s[0] for s in shapes)}
    rows = []
    used = collections.Counter()
    for kname, elems, alg in shapes:
        lo = used[kname] * 25
        used[kname] += 1
        fv = [v for _, v in fd[kname][lo + 5:lo + 25]]
        wv = [v for _, v in wd[kname][lo + 5:lo + 25]]
        dv = [d for _, d in sorted(durs[kname])[lo + 5:lo + 25]]
        if not fv or not wv or not dv:
            raise SystemExit(f"{kname}: missing dispatches (fetch {len(fv)}, write {len(wv)}, trace {len(dv)})")
        fetch_b = 2 * statistics.median(fv) * 1024
        write_b = statistics.median(wv) * 1024
        us = statistics.median(dv) / 1e3
        rows.append({"kernel": kname, "elements": elems, "algorithmic_bytes": alg,
                     "fetch_bytes_x2": round(fetch_b), "write_bytes": round(write_b),
                     "counter_bytes": round(fetch_b + write_b),
                     "counter_over_algorithmic": round((fetch_b + write_b) / alg, 4),
                     "median_us": round(us, 2), "counter_GBps": round((fetch_b + write_b) / (us * 1e3), 1),
                     "algorithmic_GBps": round(alg / (us * 1e3), 1)})
    out = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / --kernel-trace, three runs of "
                     "tools/qd_time.py; bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB) per dispatch, median of the 20 "
                     "timed dispatches per shape", "passes": rows}
    txt = json.dumps(out, indent=1)
    if a.o:
        open(a.o, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
