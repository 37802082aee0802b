"""Issue / LDS counters per launch position of the int8 forward (measurement
tooling): two rocprofv3 --pmc passes of bench.py (each with SQ_WAVES and
SQ_WAVE_CYCLES so both normalise alike), the LAST forward's 16 dispatches.

  wave_cycles   SQ_WAVE_CYCLES * 4 / SQ_WAVES (quad-cycles -> cycles)
  mfma_util     SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / wave_cycles
  coexec/mfma   SQ_VALU_MFMA_COEXEC_CYCLES / SQ_VALU_MFMA_BUSY_CYCLES: the
                share of MFMA-busy cycles in which a VALU op also executed
  valu_frac, lds_frac, sca_frac, wait_lds_frac
                SQ_ACTIVE_INST_VALU / _LDS / _SCA, SQ_WAIT_INST_LDS over
                SQ_WAVE_CYCLES (both summed over waves, same unit)
  bank_conf/lds_active  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
Raw sums are kept in the JSON.
  python tools/pmc_issue.py PASS1_DIR PASS2_DIR [-o out.json]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tools.pmc_summary import load  # noqa: E402


def last_forward(d, n=16):
    agg, meta = load(d)
    ids = [k for k in sorted(agg) if not meta[k][0].startswith("__amd")]
    return [(meta[k], agg[k]) for k in ids[-n:]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("p1")
    ap.add_argument("p2")
    ap.add_argument("-o", default=None)
    a = ap.parse_args()
    rows = []
    for (m1, c1), (m2, c2) in zip(last_forward(a.p1), last_forward(a.p2)):
        c = dict(c1)
        c.update({k: v for k, v in c2.items() if k not in ("SQ_WAVES", "SQ_WAVE_CYCLES")})
        wc = c["SQ_WAVE_CYCLES"]
        r = {"kernel": m1[0][:60], "wave_cycles": round(wc * 4 / c["SQ_WAVES"])}
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        r["mfma_util"] = round(busy / 1024 / r["wave_cycles"], 3)
        if busy:
            r["coexec/mfma"] = round(c.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / busy, 3)
        for cn, short in (("SQ_ACTIVE_INST_VALU", "valu_frac"), ("SQ_ACTIVE_INST_LDS", "lds_frac"),
                          ("SQ_ACTIVE_INST_SCA", "sca_frac"), ("SQ_WAIT_INST_LDS", "wait_lds_frac")):
            if cn in c:
                r[short] = round(c[cn] / wc, 3)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            r["bank_conf/lds_active"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 3)
        r["raw"] = {k: int(v) for k, v in c.items()}
        rows.append(r)
    out = {"passes": [os.path.abspath(a.p1), os.path.abspath(a.p2)], "per_launch": rows}
    if a.o:
        open(a.o, "w").write(json.dumps(out, indent=1) + "\n")
    for r in rows:
        print(" ".join(f"{k}={v}" for k, v in r.items() if k != "raw"))


if __name__ == "__main__":
    main()
