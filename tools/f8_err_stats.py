"""Probe (test infrastructure, not product code): the TYPICAL error of the
e4m3 conv's fp32 MFMA accumulators, for the fp8 flip-count bar of
tests/test_gpu_f8.py.

The tests bound every output by the worst-case accumulator error
|acc - exact| <= 2^-18 sum|w x| (ACC_EPS, tools/f8_acc_probe.py), and a
count of flipped e4m3 codes from it; that count is 3-140x what the cases
measure, because a sum's rounding error grows like a random walk, with the
root of the number of products, not with their count.  This probe runs the
raw fp32 accumulators of each test shape (dlq_conv2d_nhwc_f8_acc, the
tests' own seeds and data) against the oracle's exact sums and reports

  r = |acc_gpu - exact| / sqrt(sum (w x)^2)       per output

(mean, p99, max), so the tests can use E|err| = ACC_TYP sqrt(sum (w x)^2)
with ACC_TYP from here.  Writes gpurun_out/f8_err_stats.json.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as O  # noqa: E402
from dlq_amd import ops  # noqa: E402
from helpers import nchw_to_nhwc, rand_conv  # noqa: E402

SHAPES = [  # tests/test_gpu_f8.py CONV_SHAPES
    ("stem", 3, 64, 7, 2, 3, 224),
    ("l1_3x3", 64, 64, 3, 1, 1, 56),
    ("l2_0_conv1", 64, 128, 3, 2, 1, 56),
    ("l2_3x3", 128, 128, 3, 1, 1, 28),
    ("l2_ds", 64, 128, 1, 2, 0, 56),
    ("l3_3x3", 256, 256, 3, 1, 1, 14),
    ("l4_0_conv1", 256, 512, 3, 2, 1, 14),
    ("l4_3x3", 512, 512, 3, 1, 1, 7),
    ("l4_ds", 256, 512, 1, 2, 0, 14),
]


def conv_sq(x, wq, s, p):
    """sum over taps of (w x)^2 per output, float64 (im2col of the squares)."""
    xd = O.decode_f8(x).astype(np.float64) ** 2
    wd = O.decode_f8(wq).astype(np.float64) ** 2
    N, C, H, W = xd.shape
    OC, _, k, _ = wd.shape
    OH = (H + 2 * p - k) // s + 1
    xp = np.pad(xd, ((0, 0), (0, 0), (p, p), (p, p)))
    out = np.zeros((N, OC, OH, OH))
    for kh in range(k):
        for kw in range(k):
            patch = xp[:, :, kh:kh + s * OH:s, kw:kw + s * OH:s]
            out += np.einsum("nchw,oc->nohw", patch, wd[:, :, kh, kw], optimize=True)
    return out


def main():
    res = {}
    N = 2
    for name, IC, OC, k, s, p, H in SHAPES:
        rng = np.random.default_rng(17 + sum(map(ord, name)) + N)  # _run_conv's data
        x = O.quantize_f32_f8(np.abs(rng.standard_normal((N, IC, H, H))).astype(np.float32) * 40, 1.0)
        w, _ = rand_conv(rng, OC, IC, k)
        wq, _ = O.quantize_weights_f8(w)
        exact = O.conv_f8_acc(x, wq, s, p)
        c_store = 4 if IC == 3 else IC
        xh = nchw_to_nhwc(x)
        if c_store != IC:
            xh = np.concatenate([xh, np.zeros(xh.shape[:3] + (c_store - IC,), np.uint8)], axis=3)
        packed = ops.pack_conv_weights_f8(wq, c_store, H, s, p)
        acc = ops.conv2d_nhwc_f8_acc(torch.from_numpy(np.ascontiguousarray(xh)).cuda(),
                                     torch.from_numpy(packed).cuda(), OC, k, s, p)
        got = np.transpose(acc.cpu().numpy(), (0, 3, 1, 2)).astype(np.float64)
        rms = np.sqrt(conv_sq(x, wq, s, p))
        sabs = O.conv_f8_acc(x & 0x7F, wq & 0x7F, s, p)
        err = np.abs(got - exact)
        ok = rms > 0
        r = err[ok] / rms[ok]
        res[name] = {"K": IC * k * k, "n": int(err.size), "exact_outputs": int(np.count_nonzero(err == 0)),
                     "mean_r": float(r.mean()), "p99_r": float(np.quantile(r, 0.99)), "max_r": float(r.max()),
                     "max_err_over_sum_abs_x2^18": float(np.max(err[sabs > 0] / sabs[sabs > 0]) * 2.0 ** 18)}
        print(name, res[name], flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/f8_err_stats.json", "w"), indent=1)


if __name__ == "__main__":
    main()
