"""Run dlq_gemm_s8s8s32 (the exported sgemm_tiled replacement) on the GPU a few
times for profiling (rocprofv3) and print TOPS: python tools/gemm_run.py [M N K reps]."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dlq_amd.lib import check, lib  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (8192, 8192, 8192)
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
dev = torch.device("cuda")
A = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
B = torch.randint(-127, 128, (K, N), dtype=torch.int8, device=dev)
C = torch.empty((M, N), dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
for _ in range(2):
    check(lib.dlq_gemm_s8s8s32(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, st), "gemm")
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    check(lib.dlq_gemm_s8s8s32(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, st), "gemm")
e1.record()
e1.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"gemm {M}x{N}x{K}: {ms:.3f} ms  {2 * M * N * K / (ms * 1e-3) / 1e12:.1f} TOPS")
