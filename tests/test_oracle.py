"""CPU: pin the oracle (the checker) to the reference's own golden vectors and
to the reference's own CPU code, and check the int8 restatement against
independent numpy arithmetic.  No GPU."""
import ctypes as C
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import oracle as O
from tests.helpers import golden, rand_conv, rand_s8

REF_V3 = os.path.join(os.path.dirname(O.__file__), "_ref", "libmnist_v3.so")


# ---------------------------------------------------------------- fp32 golden pins

def test_fc_golden_bitexact():
    """out/step8_logits.bin == sgemm_tiled (fmaf-sequential k) + host bias add
    (infer_e2e.cu:206-219) on the committed tmp_e2e/ inputs, 1000/1000 bit-exact."""
    W = golden("fc.weight.bin", (1000, 512))
    b = golden("fc.bias.bin")
    gap = golden("gap.bin")
    ref = golden("step8_logits.bin")
    out = O.fc_forward_f32(gap, W, b)
    assert np.array_equal(out.view(np.int32), ref.view(np.int32))
    assert int(out.argmax()) == 293 and abs(float(out.max()) - 15.774744) < 1e-5


def test_fc_golden_needs_fma_order():
    """The golden vector is NOT reproduced by mul-then-add -- i.e. it really
    pins the contracted (FMA) order of the reference build."""
    W = golden("fc.weight.bin", (1000, 512)).astype(np.float32)
    gap = golden("gap.bin")
    acc = np.zeros(1000, np.float32)
    for k in range(512):
        acc = (acc + (W[:, k] * gap[k]).astype(np.float32)).astype(np.float32)
    out = (acc + golden("fc.bias.bin")).astype(np.float32)
    assert np.count_nonzero(out.view(np.int32) != golden("step8_logits.bin").view(np.int32)) > 100


def test_gap_golden():
    """tmp_e2e/gap.bin vs the gap_global_ref tree order (infer_e2e.cu:37-61)
    on tmp_e2e/l4.bin: the fixture came from torch's mean, so equal to ~1 ulp."""
    l4 = golden("l4.bin", (512, 49))
    g = O.gap_f32(l4)
    assert np.abs(g - golden("gap.bin")).max() < 1e-6


def test_sgemm_is_fmaf_chain():
    rng = np.random.default_rng(0)
    A = rng.standard_normal((5, 37), dtype=np.float32)
    B = rng.standard_normal((37, 3), dtype=np.float32)
    Cm = O.sgemm_f32(A, B)
    ref = np.zeros((5, 3), np.float32)
    for k in range(37):  # sequential fused multiply-add in float64 then rounded == fmaf
        ref = (ref.astype(np.float64) + A[:, k:k + 1].astype(np.float64) * B[k:k + 1, :]).astype(np.float32)
    assert np.array_equal(Cm, ref)


@pytest.mark.parametrize("ic,oc,k,s,p,h", [(3, 8, 7, 2, 3, 33), (16, 8, 3, 1, 1, 13), (16, 8, 3, 2, 1, 14),
                                           (16, 8, 1, 2, 0, 14)])
def test_conv_bn_f32_vs_torch(ic, oc, k, s, p, h):
    """im2col + sgemm + bn (infer_e2e.cu:102-136, :83-97) vs torch within the
    reference's own gate, max_abs <= 1e-4 (infer_conv1_bn1_relu.cu:150)."""
    rng = np.random.default_rng(ic * 100 + k)
    x = rng.standard_normal((ic, h, h), dtype=np.float32)
    w, bn = rand_conv(rng, oc, ic, k)
    y = O.conv_bn_f32(x, w, bn, s, p)
    t = F.conv2d(torch.from_numpy(x)[None], torch.from_numpy(w), stride=s, padding=p)
    g, b, m, v = (torch.from_numpy(a) for a in bn)
    t = F.batch_norm(t, m, v, g, b, False, 0.0, 1e-5)[0].numpy()
    assert np.abs(y - t).max() <= 1e-4


def test_maxpool_f32_vs_torch():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((4, 17, 17), dtype=np.float32)
    assert np.array_equal(O.maxpool_f32(x), F.max_pool2d(torch.from_numpy(x), 3, 2, 1).numpy())


@pytest.mark.skipif(not os.path.exists(REF_V3), reason="oracle/_ref not built (reference absent)")
def test_mnist_layer_matches_reference_v3c():
    """ora_mlp_layer_f32 == the reference's own C code (CUDA/MNIST_on_GPU/v3.c
    matmul_a_b :125-134, bias_forward :168-174, relu_forward :161-165),
    compiled from its source into oracle/_ref -- bit-exact."""
    ref = C.CDLL(REF_V3)
    fp = C.POINTER(C.c_float)
    rng = np.random.default_rng(2)
    B, I, Oo = 8, 784, 256
    X = rng.standard_normal((B, I), dtype=np.float32)
    W = (rng.standard_normal((I, Oo), dtype=np.float32) * 0.05).astype(np.float32)
    bias = rng.standard_normal(Oo, dtype=np.float32)
    H = np.empty((B, Oo), np.float32)
    ref.matmul_a_b(X.ctypes.data_as(fp), W.ctypes.data_as(fp), H.ctypes.data_as(fp), B, I, Oo)
    ref.bias_forward(H.ctypes.data_as(fp), bias.ctypes.data_as(fp), B, Oo)
    ref.relu_forward(H.ctypes.data_as(fp), B * Oo)
    mine = np.empty((B, Oo), np.float32)
    O.lib().ora_mlp_layer_f32(X, W, bias, B, I, Oo, 1, mine)
    assert np.array_equal(mine.view(np.int32), H.view(np.int32))


# ---------------------------------------------------------------- int8 restatement

def test_quantize_weights_properties():
    rng = np.random.default_rng(3)
    w = rng.standard_normal((16, 3, 3, 3), dtype=np.float32)
    w[5] = 0.0
    q, s = O.quantize_weights_s8(w)
    assert q.dtype == np.int8 and np.abs(q).max() <= 127
    assert s[5] == 1.0 and not q[5].any()
    flat = w.reshape(16, -1)
    for o in range(16):
        if o == 5:
            continue
        assert np.float32(np.abs(flat[o]).max() / np.float32(127.0)) == s[o]
        assert np.abs(q[o]).max() == 127  # the max-abs element maps to +-127
        assert np.array_equal(q[o].reshape(-1), np.clip(np.rint(flat[o] / s[o]), -127, 127).astype(np.int8))


def test_conv_s8_acc_vs_numpy():
    rng = np.random.default_rng(4)
    for (ic, oc, k, s, p, h) in [(3, 8, 7, 2, 3, 21), (8, 4, 3, 1, 1, 9), (8, 4, 3, 2, 1, 10), (8, 4, 1, 2, 0, 10)]:
        x = rand_s8(rng, (2, ic, h, h), lo=-128)
        w = rand_s8(rng, (oc, ic, k, k))
        acc = O.conv_s8_acc(x, w, s, p)
        ref = F.conv2d(torch.from_numpy(x.astype(np.float64)), torch.from_numpy(w.astype(np.float64)),
                       stride=s, padding=p).numpy()
        assert np.array_equal(acc, ref.astype(np.int64))


def test_epilogue_s8_sequence():
    """The fp32 epilogue is exactly: fma, fma(residual), clamp to [0 or -127, 127], rne."""
    rng = np.random.default_rng(5)
    acc = rng.integers(-200000, 200000, size=(2, 8, 30), dtype=np.int32)
    alpha = (rng.random(8, dtype=np.float32) * 1e-2).astype(np.float32)
    beta = (rng.standard_normal(8, dtype=np.float32) * 3).astype(np.float32)
    res = rand_s8(rng, acc.shape)
    r_s = np.float32(1.4)
    for relu in (True, False):
        out = O.epilogue_s8(acc, alpha, beta, res, r_s, relu=relu)
        a64 = acc.astype(np.float32).astype(np.float64)
        y = (a64 * alpha[None, :, None].astype(np.float64) + beta[None, :, None]).astype(np.float32)  # == fmaf
        y = (res.astype(np.float64) * np.float64(r_s) + y).astype(np.float32)
        ref = np.rint(np.clip(y, 0 if relu else -127, 127)).astype(np.int8)
        assert np.array_equal(out, ref)
        assert (out.min() >= 0) == relu


def test_fold_bn_output_grid():
    """alpha/beta fold dequant, BN and the 1/s_y requant in a fixed fp32 order."""
    rng = np.random.default_rng(8)
    _, (g, b, m, v) = rand_conv(rng, 16, 4, 3)
    s_w = (rng.random(16, dtype=np.float32) * 0.01).astype(np.float32)
    a, bb = O.fold_bn(0.02, s_w, (g, b, m, v), 0.05)
    f = np.float32
    t = (g / np.sqrt((v + f(1e-5)).astype(f)).astype(f)).astype(f)
    inv = f(f(1) / f(0.05))
    assert np.array_equal(a, (((f(0.02) * s_w).astype(f) * t).astype(f) * inv).astype(f))
    assert np.array_equal(bb, ((b - (m * t).astype(f)).astype(f) * inv).astype(f))


def test_gap_and_maxpool_s8():
    rng = np.random.default_rng(6)
    x = rand_s8(rng, (2, 16, 7, 7), lo=-128)
    k = O.gap_k(0.1, 49, 0.02)
    g, sums = O.gap_s8(x, k)
    assert np.array_equal(sums, x.astype(np.int32).sum(axis=(2, 3)))
    ref = np.clip(np.rint((sums.astype(np.float32) * k).astype(np.float32)), -127, 127).astype(np.int8)
    assert np.array_equal(g, ref)
    xm = rand_s8(rng, (2, 16, 15, 15), lo=-128)
    ref = F.max_pool2d(torch.from_numpy(xm.astype(np.float32)), 3, 2, 1).numpy().astype(np.int8)
    assert np.array_equal(O.maxpool_s8(xm), ref)


def test_int8_resnet18_tracks_fp32_reference():
    """Accuracy of the int8 scheme vs the reference fp32 semantics on the same
    synthetic weights (the reference's own metrics: max_abs / cosine / top-1,
    tools/diag_e2e_compare.py:15-24)."""
    from dlq_amd.models import synthetic_images
    from tests.helpers import model_and_scales
    sd, scales = model_and_scales()
    x = synthetic_images(2, seed=123).numpy()
    q, dumps = O.resnet18_forward_s8(sd, scales, x)
    for i in range(2):
        f, fd = O.resnet18_forward_f32(sd, x[i])
        cos = float(np.dot(q[i], f) / np.linalg.norm(q[i]) / np.linalg.norm(f))
        assert cos > 0.999, cos
        assert int(q[i].argmax()) == int(f.argmax())
        # stage checkpoints dequantised vs fp32
        l4 = dumps["layer4"][i].astype(np.float32) * np.float32(scales["layer4.1.conv2"])
        c = float(np.dot(l4.ravel(), fd["layer4"].ravel()) / np.linalg.norm(l4) / np.linalg.norm(fd["layer4"]))
        assert c > 0.99, c
