"""Shared test utilities (layout conversions, seeded inputs, cached scales)."""
from __future__ import annotations

import functools
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name, shape=None):
    a = np.fromfile(os.path.join(GOLDEN, name), dtype=np.float32)
    return a.reshape(shape) if shape is not None else a


def nchw_to_nhwc(a):
    return np.ascontiguousarray(np.transpose(a, (0, 2, 3, 1)))


def nhwc_to_nchw(a):
    return np.ascontiguousarray(np.transpose(a, (0, 3, 1, 2)))


def rand_s8(rng, shape, lo=-127, hi=127):
    return rng.integers(lo, hi + 1, size=shape, dtype=np.int8)


def rand_conv(rng, oc, ic, k):
    w = rng.standard_normal((oc, ic, k, k), dtype=np.float32) * np.float32((2.0 / (oc * k * k)) ** 0.5)
    g = (rng.random(oc, dtype=np.float32) + 0.5).astype(np.float32)
    b = ((rng.random(oc, dtype=np.float32) - 0.5) * 0.2).astype(np.float32)
    m = (rng.standard_normal(oc, dtype=np.float32) * 0.1).astype(np.float32)
    v = (rng.random(oc, dtype=np.float32) + 0.5).astype(np.float32)
    return w, (g, b, m, v)


@functools.lru_cache(maxsize=None)
def model_and_scales(seed=0x20260306, n_calib=2):
    """Synthetic ResNet-18 weights + activation scales calibrated on the CPU
    with the fp32 torch model (deterministic)."""
    import torch
    from dlq_amd.models import resnet18_state_dict, synthetic_images
    from dlq_amd.quant import calibrate_resnet18
    sd = resnet18_state_dict(seed)
    torch.manual_seed(0)
    scales = calibrate_resnet18(sd, synthetic_images(n_calib, seed=seed + 1), device="cpu")
    return sd, scales
