"""HBM GB/s of the standalone quantise / dequant passes (dlq_quantize_f32_s8,
dlq_dequant_s32_f32) on the bench's shapes: hipEvents over back-to-back calls."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dlq_amd.lib import check, lib  # noqa: E402

dev = torch.device("cuda")
st = torch.cuda.current_stream().cuda_stream


def timed(fn, iters=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters


n = 256 * 3 * 224 * 224
x = torch.randn(n, device=dev)
q = torch.empty(n, dtype=torch.int8, device=dev)
ms = timed(lambda: check(lib.dlq_quantize_f32_s8(x.data_ptr(), n, 50.0, q.data_ptr(), st), "q"))
print(f"quantize_f32_s8 n={n}: {ms * 1e3:.1f} us, {5 * n / (ms * 1e-3) / 1e9:.0f} GB/s")
for (NB, CC, HW) in ((256, 64, 3136), (256, 512, 49)):
    acc = torch.randint(-(1 << 20), 1 << 20, (NB, CC, HW), dtype=torch.int32, device=dev)
    sc = torch.rand(CC, device=dev)
    y = torch.empty((NB, CC, HW), dtype=torch.float32, device=dev)
    ms = timed(lambda: check(lib.dlq_dequant_s32_f32(acc.data_ptr(), NB, CC, HW, sc.data_ptr(), y.data_ptr(), st), "d"))
    e = NB * CC * HW
    print(f"dequant_s32_f32 {NB}x{CC}x{HW}: {ms * 1e3:.1f} us, {8 * e / (ms * 1e-3) / 1e9:.0f} GB/s")
