"""Per-stage comparison of two dump directories (bin/dlq_e2e --dump_dir,
the reference's step8_e2e --dump_dir, or a torch run): for each of the seven
checkpoints max_abs, mean_abs and cosine, the metrics of the reference's
tools/diag_e2e_compare.py:5-40 (checkpoints stem_pool .. logits, fp32 raw).

  python tools/diag_compare.py --torch_dir A --cuda_dir B
"""
import argparse
import os

import numpy as np

CKPTS = [("stem_pool.bin", (64, 56, 56)), ("layer1.bin", (64, 56, 56)), ("layer2.bin", (128, 28, 28)),
         ("layer3.bin", (256, 14, 14)), ("layer4.bin", (512, 7, 7)), ("gap.bin", (512,)), ("logits.bin", (1000,))]


def load(path, shape):
    x = np.fromfile(path, dtype=np.float32)
    if x.size != int(np.prod(shape)):
        raise RuntimeError(f"size mismatch for {path}: got {x.size}, want {int(np.prod(shape))}")
    return x.reshape(shape)


def metrics(a, b):
    """(max_abs, mean_abs, cosine) in float64; cosine 0 when either norm is 0."""
    d = np.abs(a.astype(np.float64) - b.astype(np.float64)).reshape(-1)
    a64, b64 = a.reshape(-1).astype(np.float64), b.reshape(-1).astype(np.float64)
    na, nb = np.linalg.norm(a64), np.linalg.norm(b64)
    cos = 0.0 if na == 0 or nb == 0 else float(np.dot(a64, b64) / (na * nb))
    return float(d.max()), float(d.mean()), cos


def compare(dir_a, dir_b):
    out = {}
    for name, shape in CKPTS:
        out[name] = metrics(load(os.path.join(dir_a, name), shape), load(os.path.join(dir_b, name), shape))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--torch_dir", required=True)
    ap.add_argument("--cuda_dir", required=True)
    a = ap.parse_args()
    print(f"[COMPARE] torch_dir={a.torch_dir}")
    print(f"[COMPARE]  cuda_dir={a.cuda_dir}")
    for name, (mx, mn, cs) in compare(a.torch_dir, a.cuda_dir).items():
        print(f"{name:<14}  max_abs={mx:.6g}  mean_abs={mn:.6g}  cosine={cs:.6f}")


if __name__ == "__main__":
    main()
