"""Activation-scale calibration: the int8 "quant block" the reference
anticipates (CUDA/resnet18-kernel-lab/reports/Step1.md:92) but never built.

Symmetric per-tensor scales s = max|a| / 127 at every site the int8 net
requantises (dlq_amd.models.conv_sites()), measured by a forward of the fp32
torch model on calibration images.  This is offline model preparation, not
part of the timed path; the scales are then plain inputs of both the HIP
engine and the CPU oracle, so parity does not depend on how they were made.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .models import BLOCKS, torch_resnet18


@torch.inference_mode()
def calibrate_resnet18(sd, x: torch.Tensor, device=None, qmax: float = 127.0) -> dict[str, float]:
    """Per-site scales amax / qmax: qmax 127 for int8, 448 (the e4m3 maximum)
    for the fp8 path."""
    device = device or x.device
    m = torch_resnet18(sd, device)
    x = x.to(device)
    amax: dict[str, float] = {}

    def upd(site, t):
        v = float(t.detach().abs().max())
        amax[site] = max(amax.get(site, 0.0), v)

    upd("input", x)
    y = F.relu(m.bn1(m.conv1(x)))
    upd("conv1", y)
    y = F.max_pool2d(y, 3, 2, 1)
    for name, _, _, _, ds in BLOCKS:
        layer, idx = name.split(".")
        blk = getattr(m, layer)[int(idx)]
        h = F.relu(blk.bn1(blk.conv1(y)))
        upd(f"{name}.conv1", h)
        o = blk.bn2(blk.conv2(h))
        if ds:
            skip = blk.downsample(y)
            upd(f"{name}.downsample", skip)
        else:
            skip = y
        y = F.relu(o + skip)
        upd(f"{name}.conv2", y)
    g = F.adaptive_avg_pool2d(y, 1).flatten(1)
    upd("gap", g)
    return {k: float(np.float32(max(v, 1e-8) / qmax)) for k, v in amax.items()}


def save_scales(scales: dict[str, float], path: str) -> None:
    """Write the '<site> <scale>' text read by dlq_resnet18_load_scales."""
    with open(path, "w") as f:
        f.write("# dlq int8 activation scales (site scale)\n")
        for k, v in scales.items():
            f.write(f"{k} {float(np.float32(v))!r}\n")


def load_scales(path: str) -> dict[str, float]:
    out = {}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            k, v = line.split()
            out[k] = float(v)
    return out


@torch.inference_mode()
def calibrate_mlp(W1, b1, x: np.ndarray):
    """(s_in, s_hidden) for the MNIST MLP from fp32 activations."""
    xt = torch.from_numpy(np.ascontiguousarray(x, np.float32))
    h = torch.relu(xt @ torch.from_numpy(W1) + torch.from_numpy(b1))
    return (float(np.float32(float(xt.abs().max()) / 127.0)),
            float(np.float32(float(h.abs().max()) / 127.0)))
