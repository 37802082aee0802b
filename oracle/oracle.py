"""ctypes/numpy front end of the CPU oracle (oracle.c).

TEST INFRASTRUCTURE ONLY -- the checker, never the product.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  The shipped path (dlq_amd / libdlq.so) never imports it.

Layouts follow the reference: NCHW activations, OIHW weights
(CUDA/resnet18-kernel-lab/cpp/fp32/runtime/infer_e2e.cu:100-136).
The ResNet-18 wiring restates infer_e2e.cu:259-433 (stem, 8 BasicBlocks via
basic_block_forward :156-203, GAP :418-424, FC :206-219).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_s8p = np.ctypeslib.ndpointer(np.int8, flags="C_CONTIGUOUS")
_s32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i = C.c_int
_f = C.c_float

_SIGS = {
    "ora_im2col_nchw_f32": [_f32p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _f32p],
    "ora_sgemm_f32": [_f32p, _f32p, _f32p, _i, _i, _i],
    "ora_bn_inference_f32": [_f32p, _f32p, _f32p, _f32p, _f32p, _f, _i, _i],
    "ora_relu_f32": [_f32p, _i],
    "ora_add_f32": [_f32p, _f32p, _i],
    "ora_maxpool_f32": [_f32p, _i, _i, _i, _i, _f32p],
    "ora_gap_f32": [_f32p, _i, _i, _f32p],
    "ora_fc_forward_f32": [_f32p, _f32p, _f32p, _i, _i, _f32p],
    "ora_conv2d_f32": [_f32p, _i, _i, _i, _f32p, _i, _i, _i, _i, _i, _i, _i, _f32p, _f32p],
    "ora_mlp_layer_f32": [_f32p, _f32p, _f32p, _i, _i, _i, _i, _f32p],
    "ora_quantize_weights_s8": [_f32p, _i, _i, _s8p, _f32p],
    "ora_fold_bn": [_f, _f32p, _f32p, _f32p, _f32p, _f32p, _f, _f, _i, _f32p, _f32p],
    "ora_res_scale": [_f, _f],
    "ora_quantize_f32_s8": [_f32p, C.c_size_t, _f, _s8p],
    "ora_im2col_nchw_s8": [_s8p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _s8p],
    "ora_gemm_s8s8s32": [_s8p, _s8p, _s32p, _i, _i, _i],
    "ora_conv2d_nchw_s8_acc": [_s8p, _i, _i, _i, _i, _s8p, _i, _i, _i, _i, _i, _i, _i, _s32p],
    "ora_epilogue_s8": [_s32p, _i, _i, _i, _f32p, _f32p, C.c_void_p, _f, _i, _s8p],
    "ora_epilogue_f32": [_s32p, _i, _i, _i, _f32p, _f32p, _i, _f32p],
    "ora_add_requant_s8": [_s8p, _s8p, C.c_size_t, _f, _f, _i, _s8p],
    "ora_maxpool_s8": [_s8p, _i, _i, _i, _i, _s8p],
    "ora_gap_s8": [_s8p, _i, _i, _i, _f, C.c_void_p, _s8p],
    "ora_fc_s8": [_s8p, _i, _i, _s8p, _i, _f32p, _f32p, C.c_void_p, _f32p],
    "ora_mlp_layer_s8_acc": [_s8p, _s8p, _i, _i, _i, _s32p],
    "ora_encode_f8": [_f32p, C.c_size_t, _u8p],
    "ora_decode_f8": [_u8p, C.c_size_t, _f32p],
    "ora_quantize_f32_f8": [_f32p, C.c_size_t, _f, _u8p],
    "ora_quantize_weights_f8": [_f32p, _i, _i, _u8p, _f32p],
    "ora_conv2d_nchw_f8_acc": [_u8p, _i, _i, _i, _i, _u8p, _i, _i, _i, _i, _i, _i, _i, _f64p],
    "ora_epilogue_f8": [_f64p, _i, _i, _i, _f32p, _f32p, C.c_void_p, _f, _i, _u8p],
    "ora_gap_f8": [_u8p, _i, _i, _i, _f, C.c_void_p, _u8p],
    "ora_fc_f8": [_u8p, _i, _i, _u8p, _i, _f32p, _f32p, C.c_void_p, _f32p],
}


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-C", _HERE, "_build/liboracle.so"])
        L = C.CDLL(path)
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = {"ora_conv2d_nchw_s8_acc": C.c_int, "ora_conv2d_nchw_f8_acc": C.c_int,
                         "ora_res_scale": C.c_float}.get(name)
        _LIB = L
    return _LIB


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def out_dim(n, k, s, p):
    return (n + 2 * p - k) // s + 1


# --------------------------------------------------------------------------
# fp32 reference semantics
# --------------------------------------------------------------------------

def sgemm_f32(A, B):
    A = _c(A, np.float32); B = _c(B, np.float32)
    M, K = A.shape; N = B.shape[1]
    Cm = np.empty((M, N), np.float32)
    lib().ora_sgemm_f32(A, B, Cm, M, N, K)
    return Cm


def fc_forward_f32(gap, W, B):
    gap = _c(gap, np.float32); W = _c(W, np.float32); B = _c(B, np.float32)
    O, I = W.shape
    out = np.empty(O, np.float32)
    lib().ora_fc_forward_f32(gap, W, B, O, I, out)
    return out


def gap_f32(x):
    x = _c(x, np.float32)
    Cc = x.shape[0]; HW = int(np.prod(x.shape[1:]))
    y = np.empty(Cc, np.float32)
    lib().ora_gap_f32(x, Cc, HW, y)
    return y


def conv_bn_f32(x, w, bn, stride, pad, eps=1e-5):
    """conv2d_nchw_im2col_gemm + bn_launch for one image [C,H,W] (infer_e2e.cu:102-136, :83-97)."""
    x = _c(x, np.float32); w = _c(w, np.float32)
    IC, H, W = x.shape; OC, _, kH, kW = w.shape
    OH, OW = out_dim(H, kH, stride, pad), out_dim(W, kW, stride, pad)
    col = np.empty(IC * kH * kW * OH * OW, np.float32)
    y = np.empty((OC, OH, OW), np.float32)
    lib().ora_conv2d_f32(x, IC, H, W, w, OC, kH, kW, stride, stride, pad, pad, col, y)
    g, b, m, v = (_c(t, np.float32) for t in bn)
    lib().ora_bn_inference_f32(y, g, b, m, v, eps, OC, OH * OW)
    return y


def maxpool_f32(x):
    x = _c(x, np.float32)
    Cc, H, W = x.shape
    y = np.empty((Cc, out_dim(H, 3, 2, 1), out_dim(W, 3, 2, 1)), np.float32)
    lib().ora_maxpool_f32(x, 1, Cc, H, W, y)
    return y


# ResNet-18 topology (infer_e2e.cu:336-407): (name, in_c, out_c, stride, downsample)
BLOCKS = [
    ("layer1.0", 64, 64, 1, False), ("layer1.1", 64, 64, 1, False),
    ("layer2.0", 64, 128, 2, True), ("layer2.1", 128, 128, 1, False),
    ("layer3.0", 128, 256, 2, True), ("layer3.1", 256, 256, 1, False),
    ("layer4.0", 256, 512, 2, True), ("layer4.1", 512, 512, 1, False),
]
STAGE_END = {"layer1.1": "layer1", "layer2.1": "layer2", "layer3.1": "layer3", "layer4.1": "layer4"}


def _bn(sd, prefix):
    return tuple(sd[f"{prefix}.{k}"] for k in ("weight", "bias", "running_mean", "running_var"))


def resnet18_forward_f32(sd, x, record=None):
    """Reference fp32 forward of ONE image x[3,224,224] (infer_e2e.cu:259-438).

    record(name, tensor) is called with every conv/stage output; used for
    activation-scale calibration.  Returns (logits[1000], dumps dict)."""
    rec = record or (lambda n, t: None)
    dumps = {}
    y = conv_bn_f32(x, sd["conv1.weight"], _bn(sd, "bn1"), 2, 3)
    lib().ora_relu_f32(y, y.size)
    rec("conv1", y)
    y = maxpool_f32(y)
    dumps["stem_pool"] = y
    for name, ic, oc, s, ds in BLOCKS:
        h = conv_bn_f32(y, sd[f"{name}.conv1.weight"], _bn(sd, f"{name}.bn1"), s, 1)
        lib().ora_relu_f32(h, h.size)
        rec(f"{name}.conv1", h)
        o = conv_bn_f32(h, sd[f"{name}.conv2.weight"], _bn(sd, f"{name}.bn2"), 1, 1)
        if ds:
            skip = conv_bn_f32(y, sd[f"{name}.downsample.0.weight"], _bn(sd, f"{name}.downsample.1"), s, 0)
            rec(f"{name}.downsample", skip)
        else:
            skip = y.copy()
        lib().ora_add_f32(o, skip, o.size)
        lib().ora_relu_f32(o, o.size)
        rec(f"{name}.conv2", o)
        y = o
        if name in STAGE_END:
            dumps[STAGE_END[name]] = y
    gap = gap_f32(y)
    rec("gap", gap)
    dumps["gap"] = gap
    logits = fc_forward_f32(gap, sd["fc.weight"], sd["fc.bias"])
    dumps["logits"] = logits
    return logits, dumps


# --------------------------------------------------------------------------
# int8 path
# --------------------------------------------------------------------------

def quantize_weights_s8(w):
    w = _c(w, np.float32)
    OC = w.shape[0]; K = w.size // OC
    q = np.empty(w.shape, np.int8); s = np.empty(OC, np.float32)
    lib().ora_quantize_weights_s8(w, OC, K, q, s)
    return q, s


def fold_bn(s_x, s_w, bn, s_y, eps=1e-5):
    """alpha, beta of the fused epilogue in output-grid units (ora_fold_bn)."""
    g, b, m, v = (_c(t, np.float32) for t in bn)
    OC = g.size
    alpha = np.empty(OC, np.float32); beta = np.empty(OC, np.float32)
    lib().ora_fold_bn(np.float32(s_x), _c(s_w, np.float32), g, b, m, v, eps, np.float32(s_y), OC, alpha, beta)
    return alpha, beta


def res_scale(s_r, s_y):
    return np.float32(lib().ora_res_scale(np.float32(s_r), np.float32(s_y)))


def inv_scale(s):
    return np.float32(np.float32(1.0) / np.float32(s))


def quantize_f32_s8(x, s):
    x = _c(x, np.float32)
    q = np.empty(x.shape, np.int8)
    lib().ora_quantize_f32_s8(x, x.size, inv_scale(s), q)
    return q


def conv_s8_acc(x, wq, stride, pad):
    """int32 accumulators of an int8 conv, NCHW x[N,IC,H,W], wq[OC,IC,kH,kW]."""
    x = _c(x, np.int8); wq = _c(wq, np.int8)
    N, IC, H, W = x.shape; OC, _, kH, kW = wq.shape
    OH, OW = out_dim(H, kH, stride, pad), out_dim(W, kW, stride, pad)
    acc = np.empty((N, OC, OH, OW), np.int32)
    rc = lib().ora_conv2d_nchw_s8_acc(x, N, IC, H, W, wq, OC, kH, kW, stride, stride, pad, pad, acc)
    assert rc == 0
    return acc


def epilogue_s8(acc, alpha, beta, res=None, r_s=0.0, relu=True):
    """int8 epilogue with alpha/beta/r_s in output-grid units (fold_bn, res_scale)."""
    N, OC = acc.shape[:2]; HW = int(np.prod(acc.shape[2:]))
    out = np.empty(acc.shape, np.int8)
    r = None if res is None else _c(res, np.int8)
    lib().ora_epilogue_s8(_c(acc, np.int32), N, OC, HW, _c(alpha, np.float32), _c(beta, np.float32),
                          _ptr(r), np.float32(r_s), int(relu), out)
    return out


def add_requant_s8(a, r, a_s, r_s, relu=True):
    a = _c(a, np.int8); r = _c(r, np.int8)
    out = np.empty(a.shape, np.int8)
    lib().ora_add_requant_s8(a, r, a.size, np.float32(a_s), np.float32(r_s), int(relu), out)
    return out


def maxpool_s8(x):
    x = _c(x, np.int8)
    N, Cc, H, W = x.shape
    y = np.empty((N, Cc, out_dim(H, 3, 2, 1), out_dim(W, 3, 2, 1)), np.int8)
    lib().ora_maxpool_s8(x, N, Cc, H, W, y)
    return y


def gap_k(s_in, hw, s_out):
    """Host constant of the int8 GAP requant: k = s_in / hw / s_out (fp32, this order)."""
    return np.float32(np.float32(np.float32(s_in) / np.float32(hw)) / np.float32(s_out))


def gap_s8(x, k):
    x = _c(x, np.int8)
    N, Cc = x.shape[:2]; HW = int(np.prod(x.shape[2:]))
    sums = np.empty((N, Cc), np.int32); y = np.empty((N, Cc), np.int8)
    lib().ora_gap_s8(x, N, Cc, HW, np.float32(k), _ptr(sums), y)
    return y, sums


def fc_s8(x, wq, alpha, beta):
    x = _c(x, np.int8); wq = _c(wq, np.int8)
    N, I = x.shape; O = wq.shape[0]
    accs = np.empty((N, O), np.int32); out = np.empty((N, O), np.float32)
    lib().ora_fc_s8(x, N, I, wq, O, _c(alpha, np.float32), _c(beta, np.float32), _ptr(accs), out)
    return out, accs


def mlp_alpha_beta(s_x, s_w, bias, s_y):
    """Hidden-layer epilogue constants in output-grid units (mlp.cpp prep_layer):
    alpha = (s_x*s_w)*(1/s_y), beta = bias*(1/s_y), fp32 in this order."""
    inv = np.float32(np.float32(1.0) / np.float32(s_y))
    sa = (np.float32(s_x) * _c(s_w, np.float32)).astype(np.float32)
    return (sa * inv).astype(np.float32), (_c(bias, np.float32) * inv).astype(np.float32)


def fc_alpha(s_x, s_w):
    return (np.float32(s_x) * _c(s_w, np.float32)).astype(np.float32)


def resnet18_forward_s8(sd, scales, x, eps=1e-5):
    """int8 forward of a batch x[N,3,224,224] fp32 under activation scales
    `scales` (dict: 'input', 'conv1', '<block>.conv1', '<block>.conv2',
    '<block>.downsample', 'gap').  Returns (logits[N,1000], dumps) where dumps
    holds the int8 NCHW stage outputs and the int32 accumulators of every conv."""
    dumps = {}
    xq = quantize_f32_s8(x, scales["input"])
    dumps["input_q"] = xq

    def conv(name, xin, s_in, w, bn, stride, pad, res=None, s_res=0.0, relu=True):
        wq, sw = quantize_weights_s8(w)
        alpha, beta = fold_bn(s_in, sw, bn, scales[name], eps)
        acc = conv_s8_acc(xin, wq, stride, pad)
        dumps[name + ".acc"] = acc
        r_s = res_scale(s_res, scales[name]) if res is not None else 0.0
        out = epilogue_s8(acc, alpha, beta, res, r_s, relu=relu)
        dumps[name] = out
        return out

    y = conv("conv1", xq, scales["input"], sd["conv1.weight"], _bn(sd, "bn1"), 2, 3)
    y = maxpool_s8(y)
    dumps["stem_pool"] = y
    s_y = scales["conv1"]
    for name, ic, oc, s, ds in BLOCKS:
        h = conv(f"{name}.conv1", y, s_y, sd[f"{name}.conv1.weight"], _bn(sd, f"{name}.bn1"), s, 1)
        if ds:
            skip = conv(f"{name}.downsample", y, s_y, sd[f"{name}.downsample.0.weight"],
                        _bn(sd, f"{name}.downsample.1"), s, 0, relu=False)
            s_skip = scales[f"{name}.downsample"]
        else:
            skip, s_skip = y, s_y
        y = conv(f"{name}.conv2", h, scales[f"{name}.conv1"], sd[f"{name}.conv2.weight"],
                 _bn(sd, f"{name}.bn2"), 1, 1, res=skip, s_res=s_skip)
        s_y = scales[f"{name}.conv2"]
        if name in STAGE_END:
            dumps[STAGE_END[name]] = y
    k = gap_k(s_y, y.shape[2] * y.shape[3], scales["gap"])
    g, sums = gap_s8(y, k)
    dumps["gap_sum"] = sums
    dumps["gap"] = g
    wq, sw = quantize_weights_s8(sd["fc.weight"])
    logits, accs = fc_s8(g, wq, fc_alpha(scales["gap"], sw), sd["fc.bias"])
    dumps["fc.acc"] = accs
    dumps["logits"] = logits
    return logits, dumps


# ------------------------------------------------------------------ fp8 path
# Config 5 (BASELINE configs[4]): e4m3 activations and
# per-output-channel e4m3 weights.  No reference code exists; the scheme is
# the build's own and oracle.c's ora_*_f8 functions define
# it.  The e4m3 codec is pinned against torch.float8_e4m3fn
# (tests/test_oracle_f8.py); accumulators here are EXACT (see oracle.c), so
# the GPU's fp32 MFMA accumulation is checked with a stated tolerance.

F8_MAX = 448.0


def encode_f8(y):
    """RNE e4m3fn codes (uint8) of fp32 values with |y| <= 448."""
    y = _c(y, np.float32)
    q = np.empty(y.shape, np.uint8)
    lib().ora_encode_f8(y, y.size, q)
    return q


def decode_f8(q):
    q = _c(q, np.uint8)
    y = np.empty(q.shape, np.float32)
    lib().ora_decode_f8(q, q.size, y)
    return y


def quantize_f32_f8(x, s):
    x = _c(x, np.float32)
    q = np.empty(x.shape, np.uint8)
    lib().ora_quantize_f32_f8(x, x.size, inv_scale(s), q)
    return q


def quantize_weights_f8(w):
    w = _c(w, np.float32)
    OC = w.shape[0]; K = w.size // OC
    q = np.empty(w.shape, np.uint8); s = np.empty(OC, np.float32)
    lib().ora_quantize_weights_f8(w, OC, K, q, s)
    return q, s


def conv_f8_acc(x, wq, stride, pad):
    """Exact accumulators (float64) of an e4m3 conv, NCHW codes x, OIHW codes wq."""
    x = _c(x, np.uint8); wq = _c(wq, np.uint8)
    N, IC, H, W = x.shape; OC, _, kH, kW = wq.shape
    OH, OW = out_dim(H, kH, stride, pad), out_dim(W, kW, stride, pad)
    acc = np.empty((N, OC, OH, OW), np.float64)
    rc = lib().ora_conv2d_nchw_f8_acc(x, N, IC, H, W, wq, OC, kH, kW, stride, stride, pad, pad, acc)
    assert rc == 0
    return acc


def epilogue_f8(acc, alpha, beta, res=None, r_s=0.0, relu=True):
    N, OC = acc.shape[:2]; HW = int(np.prod(acc.shape[2:]))
    out = np.empty(acc.shape, np.uint8)
    r = None if res is None else _c(res, np.uint8)
    lib().ora_epilogue_f8(_c(acc, np.float64), N, OC, HW, _c(alpha, np.float32), _c(beta, np.float32),
                          _ptr(r), np.float32(r_s), int(relu), out)
    return out


def gap_k_f8(s_in, hw, s_out):
    """GAP constant on e4m3 units: gap_k(...) * 2^-9 (exact)."""
    return np.float32(gap_k(s_in, hw, s_out) * np.float32(2.0 ** -9))


def gap_f8(x, k):
    x = _c(x, np.uint8)
    N, Cc = x.shape[:2]; HW = int(np.prod(x.shape[2:]))
    sums = np.empty((N, Cc), np.int32); y = np.empty((N, Cc), np.uint8)
    lib().ora_gap_f8(x, N, Cc, HW, np.float32(k), _ptr(sums), y)
    return y, sums


def fc_f8(x, wq, alpha, beta):
    x = _c(x, np.uint8); wq = _c(wq, np.uint8)
    N, I = x.shape; O = wq.shape[0]
    accs = np.empty((N, O), np.float64); out = np.empty((N, O), np.float32)
    lib().ora_fc_f8(x, N, I, wq, O, _c(alpha, np.float32), _c(beta, np.float32), _ptr(accs), out)
    return out, accs


def resnet18_forward_f8(sd, scales, x, eps=1e-5):
    """fp8 (e4m3) forward of x[N,3,224,224] fp32 under activation scales
    calibrated for the e4m3 range (amax / 448).  Same wiring and dump names
    as resnet18_forward_s8; stage dumps are e4m3 codes (uint8), '.acc'
    dumps exact float64 accumulators."""
    dumps = {}
    xq = quantize_f32_f8(x, scales["input"])
    dumps["input_q"] = xq

    def conv(name, xin, s_in, w, bn, stride, pad, res=None, s_res=0.0, relu=True):
        wq, sw = quantize_weights_f8(w)
        alpha, beta = fold_bn(s_in, sw, bn, scales[name], eps)
        acc = conv_f8_acc(xin, wq, stride, pad)
        dumps[name + ".acc"] = acc
        r_s = res_scale(s_res, scales[name]) if res is not None else 0.0
        out = epilogue_f8(acc, alpha, beta, res, r_s, relu=relu)
        dumps[name] = out
        return out

    y = conv("conv1", xq, scales["input"], sd["conv1.weight"], _bn(sd, "bn1"), 2, 3)
    # max over non-negative e4m3 codes (post-ReLU, -0 canonicalised) = max of
    # the int8 bytes: the int8 maxpool applies unchanged
    y = maxpool_s8(y.view(np.int8)).view(np.uint8)
    dumps["stem_pool"] = y
    s_y = scales["conv1"]
    for name, ic, oc, s, ds in BLOCKS:
        h = conv(f"{name}.conv1", y, s_y, sd[f"{name}.conv1.weight"], _bn(sd, f"{name}.bn1"), s, 1)
        if ds:
            skip = conv(f"{name}.downsample", y, s_y, sd[f"{name}.downsample.0.weight"],
                        _bn(sd, f"{name}.downsample.1"), s, 0, relu=False)
            s_skip = scales[f"{name}.downsample"]
        else:
            skip, s_skip = y, s_y
        y = conv(f"{name}.conv2", h, scales[f"{name}.conv1"], sd[f"{name}.conv2.weight"],
                 _bn(sd, f"{name}.bn2"), 1, 1, res=skip, s_res=s_skip)
        s_y = scales[f"{name}.conv2"]
        if name in STAGE_END:
            dumps[STAGE_END[name]] = y
    k = gap_k_f8(s_y, y.shape[2] * y.shape[3], scales["gap"])
    g, sums = gap_f8(y, k)
    dumps["gap_sum"] = sums
    dumps["gap"] = g
    wq, sw = quantize_weights_f8(sd["fc.weight"])
    logits, accs = fc_f8(g, wq, fc_alpha(scales["gap"], sw), sd["fc.bias"])
    dumps["fc.acc"] = accs
    dumps["logits"] = logits
    return logits, dumps


# ------------------------------------------------------------------ the ends
# Preprocessing (RK/tools/preprocess_to_bin.py:5-33) and the head
# (RK/kernels/softmax.cu:5-47, launcher top-1 RK/runtime/infer_e2e.cu:436-438).
# The resize restates Pillow's 8-bit BILINEAR resampler (Pillow Resample.c:
# precompute_coeffs, normalize_coeffs_8bpc, ImagingResample{Horizontal,
# Vertical}_8bpc) -- the third-party algorithm under the reference's
# Image.resize call; pinned by tests/golden/preprocess_golden.npz, written by
# tools/make_preprocess_golden.py from the reference's own functions + PIL.

PREPROC_MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
PREPROC_STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)
_PREC = 22  # Resample.c PRECISION_BITS = 32 - 8 - 2


def preprocess_size(h, w, size=256):
    """resize_shorter_side's target (preprocess_to_bin.py:8-16): Python round."""
    if w < h:
        return int(round(h * size / w)), size
    return size, int(round(w * size / h))


def _bilinear_coeffs(in_size, out_size):
    """precompute_coeffs (box (0, in_size), support 1) + normalize_coeffs_8bpc:
    per output index (first source index, int32 fixed-point weights)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    out = []
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w.append(1.0 - t if t < 1.0 else 0.0)
        ww = 0.0
        for f in w:  # left-to-right double sum, as the C loop
            ww += f
        k = [(f / ww if ww != 0.0 else f) for f in w]
        kk = np.array([int(-0.5 + v * (1 << _PREC)) if v < 0 else int(0.5 + v * (1 << _PREC)) for v in k],
                      dtype=np.int64)
        out.append((xmin, kk))
    return out


def _clip8(v):
    return np.where(v >= (1 << _PREC) << 8, 255, np.where(v <= 0, 0, v >> _PREC)).astype(np.uint8)


def _resample_axis(img, out_size, axis):
    """One 8bpc pass along `axis` (1 = horizontal, 0 = vertical) of an HxWx3 u8 image."""
    coeffs = _bilinear_coeffs(img.shape[axis], out_size)
    src = np.moveaxis(img.astype(np.int64), axis, 0)
    res = np.empty((out_size,) + src.shape[1:], dtype=np.uint8)
    for xx, (xmin, kk) in enumerate(coeffs):
        acc = np.full(src.shape[1:], 1 << (_PREC - 1), dtype=np.int64)
        for i, k in enumerate(kk):
            acc += src[xmin + i] * k
        res[xx] = _clip8(acc)
    return np.ascontiguousarray(np.moveaxis(res, 0, axis))


def preprocess_resize_crop_u8(img, size=256, crop=224):
    """Image.resize((new_w, new_h), BILINEAR) then center_crop -> u8 HxWx3."""
    h, w = img.shape[:2]
    nh, nw = preprocess_size(h, w, size)
    x = img
    if nw != w:  # Resample.c: horizontal pass first
        x = _resample_axis(x, nw, 1)
    if nh != h:
        x = _resample_axis(x, nh, 0)
    top, left = (nh - crop) // 2, (nw - crop) // 2
    return np.ascontiguousarray(x[top:top + crop, left:left + crop])


def preprocess_u8(img):
    """u8 HWC RGB -> fp32 [3,224,224] (to_nchw_float32, preprocess_to_bin.py:24-33)."""
    x = preprocess_resize_crop_u8(img).astype(np.float32) / np.float32(255.0)
    x = (x - PREPROC_MEAN) / PREPROC_STD
    return np.ascontiguousarray(np.transpose(x, (2, 0, 1)))


def softmax_f64(x):
    """Exact-as-float64 softmax of each row (the tolerance anchor for softmax_1d)."""
    z = x.astype(np.float64) - x.astype(np.float64).max(axis=-1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=-1, keepdims=True)


def top1(x):
    """infer_e2e.cu:436-438: first index with logit > running best (from -1e30)."""
    idx = np.full(x.shape[0], -1, dtype=np.int32)
    val = np.full(x.shape[0], np.float32(-1e30), dtype=np.float32)
    for r in range(x.shape[0]):
        best, top = np.float32(-1e30), -1
        for i, v in enumerate(x[r]):
            if v > best:
                best, top = v, i
        idx[r], val[r] = top, best
    return idx, val
