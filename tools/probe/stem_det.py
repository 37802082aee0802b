"""Stem determinism / build-equality probe (kernel work, not product).

usage: DLQ_LIB_PATH=<lib> python tools/probe/stem_det.py OUT.npy [REPS]
Runs the int8 stem (dlq_stem_fused_s8) REPS times on one seeded B=256 input,
reports whether the runs agree byte for byte, and saves the first run's
output so two builds can be compared (np.array_equal on the two files).
"""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dlq_amd import ops  # noqa: E402

out, reps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3
rng = np.random.default_rng(7)
B = 256
x = torch.from_numpy((rng.standard_normal((B, 3, 224, 224), dtype=np.float32) * 1.7)).cuda()
wq = rng.integers(-127, 128, size=(64, 3, 7, 7), dtype=np.int8)
alpha = (rng.uniform(0.002, 0.02, 64) * np.where(np.arange(64) % 3 == 0, -1, 1)).astype(np.float32)
beta = rng.uniform(-3, 3, 64).astype(np.float32)
wst, al_p = ops.pack_stem_weights(wq, alpha)
wst, al_p, be = (torch.from_numpy(v).cuda() for v in (wst, al_p, beta))
ys = []
for _ in range(reps):
    y = ops.stem_fused_s8(x, wst, al_p, be, 2.64 / 127)
    torch.cuda.synchronize()
    ys.append(y.cpu().numpy())
hs = [hashlib.sha1(y.tobytes()).hexdigest()[:16] for y in ys]
bad = [int(np.count_nonzero(y != ys[0])) for y in ys[1:]]
print("hashes", hs, "mismatching bytes vs run 0:", bad)
np.save(out, ys[0])
