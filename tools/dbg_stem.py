"""Debug helper: where does the fused stem differ from the oracle?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlq_amd import ops  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.helpers import nhwc_to_nchw, rand_conv  # noqa: E402

rng = np.random.default_rng(42)
N = 1
x = (rng.standard_normal((N, 3, 224, 224), dtype=np.float32) * 1.7).astype(np.float32)
w, bn = rand_conv(rng, 64, 3, 7)
neg = len(sys.argv) > 1 and sys.argv[1] == "neg"
if neg:
    bn[0][::3] *= -1
wq, sw = O.quantize_weights_s8(w)
s_in, s_y = 2.64 / 127, 0.043
alpha, beta = O.fold_bn(s_in, sw, bn, s_y)
xq = O.quantize_f32_s8(x, s_in)
acc = O.conv_s8_acc(xq, wq, 2, 3)
conv = O.epilogue_s8(acc, alpha, beta, None, 0.0, True)
ref = O.maxpool_s8(conv)
wst, al_p = ops.pack_stem_weights(wq, alpha)
y = ops.stem_fused_s8(torch.from_numpy(x).cuda(), torch.from_numpy(wst).cuda(), torch.from_numpy(al_p).cuda(),
                      torch.from_numpy(beta).cuda(), s_in)
got = nhwc_to_nchw(y.cpu().numpy())
bad = got != ref
print("neg" if neg else "pos", "mismatches", bad.sum(), "of", bad.size)
b = bad[0]  # [64][56][56]
print("by channel tile:", b[:32].sum(), b[32:].sum())
print("by pooled row (first 8):", b.sum(axis=(0, 2))[:8], "last:", b.sum(axis=(0, 2))[-4:])
cols = b.sum(axis=(0, 1))
print("by pooled col:", cols.tolist())
print("by channel:", b.sum(axis=(1, 2)).tolist())
# sample diffs
idx = np.argwhere(b)[:10]
for c, r, cc in idx:
    win = conv[0, c, max(0, 2 * r - 1):2 * r + 2, max(0, 2 * cc - 1):2 * cc + 2]
    print(c, r, cc, "got", got[0, c, r, cc], "ref", ref[0, c, r, cc], "win", win.ravel().tolist())
