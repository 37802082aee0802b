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


@functools.lru_cache(maxsize=None)
def model_and_scales_f8(seed=0x20260306, n_calib=2):
    """Same weights, activation scales for the e4m3 range (amax / 448)."""
    import torch
    from dlq_amd.models import resnet18_state_dict, synthetic_images
    from dlq_amd.quant import calibrate_resnet18
    sd = resnet18_state_dict(seed)
    torch.manual_seed(0)
    scales = calibrate_resnet18(sd, synthetic_images(n_calib, seed=seed + 1), device="cpu", qmax=448.0)
    return sd, scales


def f8_ordinal(q):
    """e4m3 codes -> signed ordinal (adjacent values differ by 1; +-0 -> 0)."""
    q = np.asarray(q, np.uint8).astype(np.int32)
    return np.where(q & 0x80, -(q & 0x7F), q)


def f8_sweep(rng, n=60000):
    """fp32 values covering the e4m3 range: random magnitudes over 2^-12..2^9
    (beyond +-448 too), every exact e4m3 value, every rounding midpoint and
    its two fp32 neighbours, both signs."""
    from oracle import oracle as O
    vals = O.decode_f8(np.arange(256, dtype=np.uint8))
    vals = vals[np.isfinite(vals)]
    pos = np.unique(np.abs(vals)).astype(np.float64)
    mids = ((pos[1:] + pos[:-1]) / 2).astype(np.float32)
    near = np.concatenate([mids, np.nextafter(mids, np.float32(0)), np.nextafter(mids, np.float32(1e9))])
    mag = (2.0 ** rng.uniform(-12, 9.5, n)).astype(np.float32)
    sgn = np.where(rng.random(n) < 0.5, -1, 1).astype(np.float32)
    x = np.concatenate([mag * sgn, vals, near, -near, np.float32([0.0, -0.0, 448.0, -448.0, 1e6, -1e6])])
    return x.astype(np.float32)


def synth_image(h, w, seed):
    """Seeded smooth + noisy u8 HWC RGB image (tools/make_preprocess_golden.py
    generated the preprocessing goldens from exactly these)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.empty((h, w, 3), np.float64)
    for c in range(3):
        a, b, f = rng.random(3)
        img[..., c] = 128 + 90 * np.sin(xx * (0.02 + 0.2 * a) + yy * (0.03 + 0.1 * b) + 6 * f)
    img += rng.normal(0, 12, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def preprocess_cases():
    """(h, w, seed, crop_sha256, fp32_sha256) of tests/golden/preprocess_golden.npz."""
    g = np.load(os.path.join(GOLDEN, "preprocess_golden.npz"))
    out, i = [], 0
    while f"case{i}_hws" in g:
        h, w, seed = (int(v) for v in g[f"case{i}_hws"])
        out.append((h, w, seed, g[f"case{i}_crop_sha256"].tobytes(), g[f"case{i}_sha256"].tobytes()))
        i += 1
    return out
