"""Stream-K against data-parallel for dlq_gemm_s8s8s32 / _nt on the bench's
GEMM shapes: TOPS per (layout, gemm_tile, gemm_sk) -- sk 1 = data-parallel,
2 = stream-K, and the default (tile 0, sk 0) -- hipEvents over back-to-back
calls, ROUNDS rounds in rotating order, median reported (as
tools/gemm_tiles.py).  Also checks that every configuration's C is
identical (int32 sums: exact in any order).
python tools/gemm_sk.py [reps] [rounds]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dlq_amd.lib import check, lib, set_knob  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda")
out = {}
for (M, N, K) in ((256, 50176, 2304), (12544, 512, 4608), (50176, 256, 2304), (8192, 8192, 8192)):
    A = torch.randint(-128, 128, (M, K), dtype=torch.int8, device=dev)
    B = torch.randint(-128, 128, (K, N), dtype=torch.int8, device=dev)
    C = torch.empty((M, N), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    configs = [(lay, t, sk) for lay in ("nn", "nt") for (t, sk) in ((0, 0), (1, 1), (1, 2), (2, 1), (2, 2))]
    times = {c: [] for c in configs}
    digest = {}

    def run(lay, tile, sk, n):
        set_knob("gemm_tile", tile)
        set_knob("gemm_sk", sk)
        fn = lib.dlq_gemm_s8s8s32 if lay == "nn" else lib.dlq_gemm_s8s8s32_nt  # B's bytes reused as Bt[N][K]
        for _ in range(n):
            check(fn(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, st), "gemm")

    run("nn", 0, 0, 3 * reps)  # warm the clock before the first timed configuration
    torch.cuda.synchronize()
    for r in range(rounds):
        order = configs[r % len(configs):] + configs[:r % len(configs)]
        for c in order:
            C.fill_(-1)
            run(*c, 3)
            torch.cuda.synchronize()
            if r == 0:
                digest[c] = (C.view(-1)[::97].double().sum().item(), C.double().abs().sum().item())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(*c, reps)
            e1.record()
            e1.synchronize()
            times[c].append(e0.elapsed_time(e1) / reps)
    res = {}
    for lay in ("nn", "nt"):
        ds = {digest[c] for c in configs if c[0] == lay}
        assert len(ds) == 1, f"{M}x{N}x{K} {lay}: configurations disagree: {ds}"
    for c, v in times.items():
        ms = statistics.median(v)
        res[f"{c[0]} tile{c[1]} sk{c[2]}"] = {"ms": round(ms, 4), "tops": round(2 * M * N * K / (ms * 1e-3) / 1e12, 1)}
    set_knob("gemm_tile", 0)
    set_knob("gemm_sk", 0)
    out[f"{M}x{N}x{K}"] = res
    print(f"{M}x{N}x{K}: " + "  ".join(f"{k} {v['tops']:7.1f}" for k, v in res.items()), flush=True)
    del A, B, C
print(json.dumps(out))
