"""Write a ResNet-18 manifest directory for bin/dlq_e2e (and the reference's
own launcher format): seeded synthetic weights with torchvision's state_dict
names (no pretrained download is possible offline), CPU-calibrated activation
scales, and one preprocessed input image.

  python tools/export_manifest.py --out DIR [--int8] [--seed S]

DIR/<name>.bin + DIR/manifest.json   (export_resnet18.py:57-113 layout;
                                      --int8: int8 weights + .scale.bin)
DIR/scales.txt                        (dlq_resnet18_load_scales format)
DIR/input.bin                         (fp32 [1,3,224,224], preprocess_to_bin.py)
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlq_amd.manifest import Manifest  # noqa: E402
from dlq_amd.models import resnet18_state_dict, synthetic_images  # noqa: E402
from dlq_amd.quant import calibrate_resnet18  # noqa: E402

SEED = 0x20260306


def export(out, int8=False, seed=SEED, image_seed=SEED + 7):
    sd = resnet18_state_dict(seed)
    scales = calibrate_resnet18(sd, synthetic_images(2, seed=seed + 1), device="cpu")
    m = Manifest.from_state_dict(sd, scales)
    m.save(out, int8=int8)
    m.save_scales(os.path.join(out, "scales.txt"))
    x = synthetic_images(1, seed=image_seed).numpy().astype(np.float32)
    x.tofile(os.path.join(out, "input.bin"))
    return sd, scales, x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--int8", action="store_true")
    ap.add_argument("--seed", type=int, default=SEED)
    a = ap.parse_args()
    export(a.out, a.int8, a.seed)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
