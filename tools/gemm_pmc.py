"""MFMA utilisation of the exported int8 GEMM (dlq_gemm_s8s8s32, tile chosen
by shape) from rocprofv3 counters -- the north star's "MFMA utilisation on
the GEMM against gfx950 peak" (kernel work, not product).

  run:  rocprofv3 --pmc SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES \\
            --output-format csv -d DIR -o run -- python3 tools/gemm_pmc.py run
  sum:  python3 tools/gemm_pmc.py sum DIR -o out.json

`run` makes CALLS calls per shape (NN, then NT), in SHAPES order; `sum`
takes each (shape, layout)'s last dispatch and reports, per launch:
  mfma_insts     SQ_INSTS_VALU_MFMA_I8, checked against M N K / 32^3 padded
                 to whole tiles (one v_mfma_i32_32x32x32_i8 per 32x32x32 block)
  busy_per_simd  SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs (32 per MFMA)
  dur_us         the dispatch's duration in the counter run
  of_nominal     busy_per_simd / (dur_us x 2.4 GHz): the MFMA pipe's share of
                 the launch at the nominal clock (= TOPS / 5,033 with padding)
  clock_ghz_est  SQ_WAVE_CYCLES x 4 / (waves resident at once) / dur: waves
                 live for the whole launch when the tiles fit one round
  of_clock       busy_per_simd / (dur_us x clock_ghz_est): MFMA utilisation
                 at the clock the chip actually ran
"""
import collections
import csv
import glob
import json
import os
import sys

SHAPES = ((8192, 8192, 8192), (256, 50176, 2304), (12544, 512, 4608), (50176, 256, 2304))
CALLS = 3
NOMINAL_GHZ = 2.4
TILES = {1: (256, 256, 8), 2: (256, 128, 8), 3: (128, 128, 4), 4: (256, 224, 8), 5: (224, 128, 4), 6: (224, 256, 8)}


def run():
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from dlq_amd.lib import check, lib
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    for (M, N, K) in SHAPES:
        A = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        B = torch.randint(-127, 128, (K, N), dtype=torch.int8, device=dev)
        C = torch.empty((M, N), dtype=torch.int32, device=dev)
        for fn in (lib.dlq_gemm_s8s8s32, lib.dlq_gemm_s8s8s32_nt):
            for _ in range(CALLS):
                check(fn(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, st), "gemm")
        torch.cuda.synchronize()
        del A, B, C


def tile_of(name):
    # gemm_s8s8s32_k128_kernel<WM, WN, MI, NJ, WPS, BT>
    t = name.split("<")[1].split(">")[0].split(",")
    wm, wn, mi, nj = (int(x) for x in t[:4])
    return 32 * wm * mi, 32 * wn * nj, wm * wn


def summarize(d, out):
    path = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))[0]
    agg = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        k = int(r["Dispatch_Id"])
        agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ids = [k for k in sorted(agg) if "gemm_s8s8s32" in meta[k][0]]
    assert len(ids) == len(SHAPES) * 2 * CALLS, (len(ids), "dispatches")
    res = {}
    for si, (M, N, K) in enumerate(SHAPES):
        for li, lay in enumerate(("nn", "nt")):
            k = ids[(si * 2 + li) * CALLS + CALLS - 1]
            c, (name, dur) = agg[k], meta[k]
            TM, TN, nw = tile_of(name)
            tiles = -(-M // TM) * -(-N // TN)
            expect = tiles * (TM // 32) * (TN // 32) * -(-K // 128) * 4
            r = {"kernel": name.replace("void ", "").replace("dlq::(anonymous namespace)::", "")[:80],
                 "tile": f"{TM}x{TN}", "tiles": tiles, "dur_us": round(dur, 2),
                 "tops": round(2 * M * N * K / (dur * 1e-6) / 1e12, 1)}
            if "SQ_INSTS_VALU_MFMA_I8" in c:
                r["mfma_insts"] = int(c["SQ_INSTS_VALU_MFMA_I8"])
                r["mfma_insts_expected"] = expect
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024
                r["busy_per_simd"] = round(busy)
                r["of_nominal"] = round(busy / (dur * 1e3 * NOMINAL_GHZ), 4)
                if c.get("SQ_WAVE_CYCLES"):
                    resident = min(tiles, 256) * nw
                    clk = c["SQ_WAVE_CYCLES"] * 4 / resident / (dur * 1e3)
                    r["clock_ghz_est"] = round(clk, 3)
                    r["of_clock"] = round(busy / (dur * 1e3 * clk), 4)
            res[f"{M}x{N}x{K}_{lay}"] = r
            print(f"{M}x{N}x{K} {lay}: " + json.dumps(r), flush=True)
    json.dump({"source": d, "method": __doc__.split("\n\n")[0], "launches": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2], sys.argv[4] if len(sys.argv) > 4 else "gemm_pmc.json")
