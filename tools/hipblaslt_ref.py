"""Calibration (not product code): the vendor int8 GEMM (torch._int_mm ->
hipBLASLt on ROCm) at the shapes the round's GEMM numbers are quoted on, next
to dlq_gemm_s8s8s32 (NN) and dlq_gemm_s8s8s32_nt (NT), so the kernels' MFMA
fraction can be read against what the library reaches on the same box at the
same loaded clock."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dev = torch.device("cuda", 0)
    out = {}
    from dlq_amd.lib import lib, check
    for (M, N, K) in ((8192, 8192, 8192), (4096, 4096, 4096), (50176, 256, 2304), (200704, 128, 1152),
                      (12544, 512, 4608)):
        A = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        Bt = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        ent = {}
        try:
            ms = timed(lambda: torch._int_mm(A, Bt.t()))
            ent["int_mm_NT_ms"] = round(ms, 4)
            ent["int_mm_NT_tops"] = round(2.0 * M * N * K / (ms * 1e-3) / 1e12, 1)
        except Exception as e:
            ent["int_mm_error"] = repr(e)[:200]
        try:
            Bn = Bt.t().contiguous()
            ms = timed(lambda: torch._int_mm(A, Bn))
            ent["int_mm_NN_tops"] = round(2.0 * M * N * K / (ms * 1e-3) / 1e12, 1)
            C = torch.empty((M, N), dtype=torch.int32, device=dev)
            st = torch.cuda.current_stream().cuda_stream
            ms = timed(lambda: check(lib.dlq_gemm_s8s8s32(A.data_ptr(), Bn.data_ptr(), C.data_ptr(), M, N, K, st),
                                     "gemm"))
            ent["dlq_gemm_tops"] = round(2.0 * M * N * K / (ms * 1e-3) / 1e12, 1)
            ms = timed(lambda: check(lib.dlq_gemm_s8s8s32_nt(A.data_ptr(), Bt.data_ptr(), C.data_ptr(), M, N, K, st),
                                     "gemm_nt"))
            ent["dlq_gemm_nt_tops"] = round(2.0 * M * N * K / (ms * 1e-3) / 1e12, 1)
            ref = torch._int_mm(A[:256], Bt.t())
            check(lib.dlq_gemm_s8s8s32_nt(A.data_ptr(), Bt.data_ptr(), C.data_ptr(), M, N, K, st), "gemm_nt")
            torch.cuda.synchronize()
            ent["dlq_nt_equals_int_mm_rows0_255"] = bool(torch.equal(C[:256], ref))
        except Exception as e:
            ent["nn_error"] = repr(e)[:200]
        out[f"{M}x{N}x{K}"] = ent
        print(f"{M}x{N}x{K}", ent, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
