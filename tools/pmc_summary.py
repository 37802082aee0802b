"""Per-launch-position summary of a rocprofv3 `--pmc` run of bench.py
(`--output-format csv`), MFMA utilisation per kernel family.

Takes the LAST forward's dispatches (one launch per position of the
16-launch int8 forward) and, for the counters present, reports per launch:
  mfma_busy_per_simd = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs  (cycles; the
                       counter adds 32 per v_mfma_i32_32x32x32_i8, checked
                       against the kernels' MFMA counts)
  wave_cycles        = SQ_WAVE_CYCLES * 4 / SQ_WAVES (SQ_WAVE_CYCLES counts
                       quad-cycles, MI355X_MICROARCH.md): a wave's lifetime
  mfma_util          = mfma_busy_per_simd / wave_cycles  (the kernels run
                       one workgroup per CU for their whole duration, so a
                       wave's lifetime is the launch's length in shader cycles)
  i8_mfma_insts      = SQ_INSTS_VALU_MFMA_I8 (when collected)
and the same per family (launch-weighted).  GRBM_GUI_ACTIVE is reported raw
but not used: on gfx950 it does not tick at the shader clock.

  python tools/pmc_summary.py DIR [-o out.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tools.pmc_traffic import family_of  # noqa: E402
from dlq_amd.lib import FAMILIES  # noqa: E402


def load(d):
    path = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(path)):
        k = int(r["Dispatch_Id"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        name = r["Kernel_Name"].replace("void ", "").replace("dlq::(anonymous namespace)::", "")
        meta[k] = (name, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, int(r["Grid_Size"]))
    return agg, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("-o", default=None)
    ap.add_argument("--launches", type=int, default=16, help="launches of one forward")
    a = ap.parse_args()
    agg, meta = load(a.dir)
    ids = [k for k in sorted(agg) if not meta[k][0].startswith("__amd")]
    last = ids[-a.launches:]
    rows, fam = [], collections.defaultdict(list)
    for k in last:
        c = agg[k]
        name, dur_us, grid = meta[k]
        r = {"kernel": name[:70], "dur_us_profiled": round(dur_us, 2)}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            r["mfma_busy_per_simd"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024)
        if "SQ_WAVE_CYCLES" in c and c.get("SQ_WAVES"):
            r["wave_cycles"] = round(c["SQ_WAVE_CYCLES"] * 4 / c["SQ_WAVES"])
        if "mfma_busy_per_simd" in r and r.get("wave_cycles"):
            r["mfma_util"] = round(r["mfma_busy_per_simd"] / r["wave_cycles"], 4)
            r["clock_ghz_est"] = round(r["wave_cycles"] / (dur_us * 1e3), 3)
        for cn in ("SQ_INSTS_VALU_MFMA_I8", "SQ_INSTS_VALU_MFMA_MOPS_I8", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                   "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_INSTS_LDS",
                   "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"):
            if cn in c:
                r[cn] = int(c[cn])
        if "SQ_WAVE_CYCLES" in c:
            tot = c["SQ_WAVE_CYCLES"]
            for cn, short in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "issue_stall_frac"),
                              ("SQ_ACTIVE_INST_ANY", "active_frac")):
                if cn in c:
                    r[short] = round(c[cn] / tot, 3)
        rows.append(r)
        fam[FAMILIES[family_of(name)]].append(r)
    fams = {}
    for f, rs in fam.items():
        ent = {"launches": len(rs)}
        if all("mfma_util" in r for r in rs):
            busy = sum(r["mfma_busy_per_simd"] for r in rs)
            cyc = sum(r["wave_cycles"] for r in rs)
            ent["mfma_util"] = round(busy / cyc, 4)
            ent["mfma_busy_per_simd"] = busy
            ent["wave_cycles"] = cyc
        fams[f] = ent
    out = {"source": os.path.abspath(a.dir), "per_launch": rows, "families": fams}
    txt = json.dumps(out, indent=1)
    if a.o:
        open(a.o, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
