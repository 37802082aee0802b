"""dlq_gemm_s8s8s32 (NN: B[K][N]) and dlq_gemm_s8s8s32_nt (NT: Bt[N][K]) TOPS
per tile configuration (knob gemm_tile 0 = the by-shape choice, 1 = 256 x 256,
2 = 256 x 128, 3 = 128 x 128, 4 = 256 x 224, 5 = 224 x 128, 6 = 224 x 256) on the bench's GEMM shapes and the conv-shaped
calibration cases: hipEvents over back-to-back calls, one process.  Every
configuration is timed in ROUNDS rounds whose order rotates (the first
configuration timed in a process used to read low: the clock ramp), after a
global warmup of the first shape; the median over rounds is reported.
python tools/gemm_tiles.py [reps] [rounds]"""
import statistics
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dlq_amd.lib import check, lib, set_knob  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda")
out = {}
for (M, N, K) in ((8192, 8192, 8192), (4096, 4096, 4096), (256, 50176, 2304), (12544, 512, 4608),
                  (50176, 256, 2304), (128, 200704, 1152)):
    A = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
    B = torch.randint(-127, 128, (K, N), dtype=torch.int8, device=dev)
    C = torch.empty((M, N), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    configs = [(lay, t) for lay in ("nn", "nt") for t in (0, 1, 2, 3, 4, 5, 6)]
    times = {f"{lay}{t}": [] for lay, t in configs}
    st = torch.cuda.current_stream().cuda_stream

    def run(lay, tile, n):
        set_knob("gemm_tile", tile)
        fn = lib.dlq_gemm_s8s8s32 if lay == "nn" else lib.dlq_gemm_s8s8s32_nt  # B's bytes reused as Bt[N][K]
        for _ in range(n):
            check(fn(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, st), "gemm")

    run("nn", 0, 3 * reps)  # warm the clock before the first timed configuration
    torch.cuda.synchronize()
    for r in range(rounds):
        order = configs[r % len(configs):] + configs[:r % len(configs)]
        for lay, tile in order:
            run(lay, tile, 3)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(lay, tile, reps)
            e1.record()
            e1.synchronize()
            times[f"{lay}{tile}"].append(e0.elapsed_time(e1) / reps)
    for k, v in times.items():
        ms = statistics.median(v)
        res[k] = {"ms": round(ms, 4), "tops": round(2 * M * N * K / (ms * 1e-3) / 1e12, 1)}
    set_knob("gemm_tile", 0)
    out[f"{M}x{N}x{K}"] = res
    print(f"{M}x{N}x{K}: " + "  ".join(f"{k} {v['tops']:7.1f}" for k, v in res.items()), flush=True)
    del A, B, C
print(json.dumps(out))
