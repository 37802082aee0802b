"""Probe: how does v_mfma_f32_32x32x64_f8f6f4 round?  Runs the fp8 conv's raw
fp32 accumulators (dlq_conv2d_nhwc_f8_acc) on random e4m3 data and compares
them with candidate emulations computed on the host:
  H_exact : the exact sum rounded once to fp32
  H_step  : per K step (64 products, one MFMA) the exact dot, added to the
            fp32 accumulator with one rounding (a fused dot-accumulate)
  H_step2 : per K step the dot rounded to fp32, then an fp32 add
Writes gpurun_out/f8_acc_probe.json.  Test infrastructure only."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle as O  # noqa: E402
from dlq_amd import ops  # noqa: E402


def emulate(x, w, s, p):
    """x [N,C,H,W] codes, w [OC,C,k,k] codes -> per-K-step exact dots in kernel order."""
    xd = O.decode_f8(x).astype(np.float64)
    wd = O.decode_f8(w).astype(np.float64)
    N, Cc, H, W = x.shape
    OC, _, k, _ = w.shape
    xp = np.pad(xd, ((0, 0), (0, 0), (p, p), (p, p)))
    OH = (H + 2 * p - k) // s + 1
    dots = []
    for kh in range(k):
        for kw in range(k):
            patch = xp[:, :, kh:kh + s * OH:s, kw:kw + s * OH:s]  # [N,C,OH,OW]
            for c0 in range(0, Cc, 64):
                dots.append(np.einsum("nchw,oc->nohw", patch[:, c0:c0 + 64], wd[:, c0:c0 + 64, kh, kw]))
    return dots


def main():
    rng = np.random.default_rng(5)
    res = {}
    tag = ""
    for (Cc, OC, k, s, p, H) in [(256, 128, 3, 1, 1, 14), (128, 128, 3, 1, 1, 28), (512, 128, 3, 1, 1, 7),
                                 (256, 256, 3, 1, 1, 14)]:
        x = O.quantize_f32_f8(np.abs(rng.standard_normal((1, Cc, H, H))).astype(np.float32) * 40, 1.0)
        w = O.quantize_f32_f8(rng.standard_normal((OC, Cc, k, k)).astype(np.float32) * 60, 1.0)
        packed = ops.pack_conv_weights_f8(w, Cc, H, s, p)
        xh = np.ascontiguousarray(np.transpose(x, (0, 2, 3, 1)))
        acc = ops.conv2d_nhwc_f8_acc(torch.from_numpy(xh).cuda(), torch.from_numpy(packed).cuda(), OC, k, s, p)
        got = np.transpose(acc.cpu().numpy(), (0, 3, 1, 2)).astype(np.float32)
        dots = emulate(x, w, s, p)
        exact = np.sum(dots, axis=0)
        h_exact = exact.astype(np.float32)
        a1 = np.zeros_like(h_exact)
        a2 = np.zeros_like(h_exact)
        for d in dots:
            a1 = (a1.astype(np.float64) + d).astype(np.float32)
            a2 = (a2 + d.astype(np.float32)).astype(np.float32)
        key = f"C{Cc}_OC{OC}_H{H}{tag}"
        res[key] = {"n": int(got.size),
                    "eq_exact": int(np.count_nonzero(got == h_exact)),
                    "eq_step_fused": int(np.count_nonzero(got == a1)),
                    "eq_step_twice": int(np.count_nonzero(got == a2)),
                    "max_rel_vs_exact": float(np.max(np.abs(got - exact) / np.maximum(np.abs(exact), 1)))}
        np.savez_compressed(f"gpurun_out/f8_probe_{key}.npz", x=x, w=w, got=got)
        print(key, res[key], flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open(f"gpurun_out/f8_acc_probe{tag}.json", "w"), indent=1)


if __name__ == "__main__":
    main()
