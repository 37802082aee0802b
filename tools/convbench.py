"""Per-layer conv microbenchmark (HIP-event timed) for kernel A/B work.

usage: python tools/convbench.py [--batch 256] [--iters 50] [--only l2,l3,...]
(A/B of library builds: DLQ_LIB_PATH selects the libdlq.so, tools/ab.py.)
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlq_amd import ops  # noqa: E402

# (name, IC, OC, k, s, p, H, residual)
LAYERS = [
    ("stem", 3, 64, 7, 2, 3, 224, False),
    ("l1", 64, 64, 3, 1, 1, 56, True),
    ("l2_0c1", 64, 128, 3, 2, 1, 56, False),
    ("l2_ds", 64, 128, 1, 2, 0, 56, False),
    ("l2", 128, 128, 3, 1, 1, 28, True),
    ("l3_0c1", 128, 256, 3, 2, 1, 28, False),
    ("l3", 256, 256, 3, 1, 1, 14, True),
    ("l4_0c1", 256, 512, 3, 2, 1, 14, False),
    ("l4", 512, 512, 3, 1, 1, 7, True),
]


def bench(name, f, iters, tag, macs):
    """Kernel time without host launch overhead: `iters` launches captured in
    one graph, replayed (a Python-driven loop is launch-bound below ~30 us)."""
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    print(f"{tag:16s} {name:8s} {us:8.1f} us  {2 * macs / us / 1e6:7.1f} TOPS", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    tag = os.path.basename(os.path.dirname(os.environ.get("DLQ_LIB_PATH", "dlq_amd/libdlq.so")))
    if "stemf" in args.only.split(","):
        x = torch.randn(args.batch, 3, 224, 224, device="cuda")
        q = rng.integers(-127, 128, size=(64, 3, 7, 7), dtype=np.int8)
        wp, alp = ops.pack_stem_weights(q, np.full(64, 1e-3, np.float32))
        w = torch.from_numpy(wp).cuda()
        alpha = torch.from_numpy(alp).cuda()
        beta = torch.zeros(64, device="cuda")
        bench("stemf", lambda: ops.stem_fused_s8(x, w, alpha, beta, 0.02), args.iters, tag,
              args.batch * 112 * 112 * 64 * 3 * 49)
    for name, IC, OC, k, s, p, H, res in LAYERS:
        if args.only and name not in args.only.split(","):
            continue
        c_store = 4 if IC == 3 else IC
        x = torch.randint(-127, 128, (args.batch, H, H, c_store), dtype=torch.int8, device="cuda")
        q = rng.integers(-127, 128, size=(OC, IC, k, k), dtype=np.int8)
        w = torch.from_numpy(ops.pack_conv_weights(q, c_store, H, s, p)).cuda()
        ocp = ops.packed_oc(OC)
        alpha = torch.full((ocp,), 1e-4, device="cuda")
        beta = torch.zeros(ocp, device="cuda")
        OH = ops.out_dim(H, k, s, p)
        r = torch.randint(-127, 128, (args.batch, OH, OH, OC), dtype=torch.int8, device="cuda") if res else None
        f = lambda: ops.conv2d_nhwc_s8(x, w, OC, k, s, p, alpha, beta, residual=r, res_scale=0.01,  # noqa: E731
                                       relu=True)
        bench(name, f, args.iters, tag, args.batch * OH * OH * OC * IC * k * k)


if __name__ == "__main__":
    main()
