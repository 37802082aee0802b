"""Per-layer int8 operators over the C ABI (torch tensors as device memory).

Names follow the reference's per-layer call sites
(CUDA/resnet18-kernel-lab/cpp/fp32/runtime/infer_e2e.cu and kernels/*.cu):
``conv2d_nchw_im2col_gemm`` -> :func:`conv2d_nhwc_s8`,
``maxpool2d_3x3_s2p1_nchw`` -> :func:`maxpool2d_3x3_s2p1_nhwc_s8`,
``gap_global``              -> :func:`gap_nhwc_s8`,
``fc_forward``              -> :func:`linear_s8`,
``im2col_nchw``             -> :func:`im2col_nchw_s8` (parity only).
Like the reference helpers they raise on failure instead of returning codes
(the reference exits the process, utils.hpp:23-32).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from .lib import (DLQ_OUT_F32, DLQ_OUT_S8, DLQ_OUT_S32, ConvDesc, check, lib, ptr,
                  stream_handle)


def out_dim(n, k, s, p):
    return (n + 2 * p - k) // s + 1


# ------------------------------------------------------------------ host prep

def quantize_weights(w: np.ndarray):
    """Per-output-channel int8 weights (dlq_quantize_weights_s8): (q, scale)."""
    w = np.ascontiguousarray(w, np.float32)
    OC = w.shape[0]; K = w.size // OC
    q = np.empty(w.shape, np.int8); s = np.empty(OC, np.float32)
    check(lib.dlq_quantize_weights_s8(ptr(w), OC, K, ptr(q), ptr(s)), "quantize_weights")
    return q, s


def fold_bn(s_x: float, s_w, g, b, m, v, s_y: float, eps=1e-5):
    """alpha/beta of the fused epilogue in output-grid units (dlq_fold_bn)."""
    arrs = [np.ascontiguousarray(a, np.float32) for a in (s_w, g, b, m, v)]
    OC = arrs[1].size
    alpha = np.empty(OC, np.float32); beta = np.empty(OC, np.float32)
    check(lib.dlq_fold_bn(float(s_x), *[ptr(a) for a in arrs], float(eps), float(s_y), OC, ptr(alpha),
                          ptr(beta)), "fold_bn")
    return alpha, beta


def res_scale(s_r: float, s_y: float) -> float:
    return lib.dlq_res_scale(float(s_r), float(s_y))


def packed_oc(OC: int) -> int:
    return lib.dlq_conv_packed_oc(OC)


def pack_conv_weights(q_oihw: np.ndarray, C_store: int, H: int, stride: int, pad: int) -> np.ndarray:
    """Weight image of the conv over NHWC [*, H, H, C_store] with this kernel /
    stride / pad -- the layout dlq_conv2d_nhwc_s8 expects for that descriptor."""
    q = np.ascontiguousarray(q_oihw, np.int8)
    OC, IC, kH, kW = q.shape
    d = ConvDesc(1, H, H, C_store, OC, kH, kW, stride, stride, pad, pad)
    nb = lib.dlq_conv_packed_bytes(C.byref(d))
    if nb == 0:
        raise ValueError(f"unsupported conv packing: C={C_store} k={kH}x{kW}")
    out = np.empty(nb, np.int8)
    check(lib.dlq_pack_conv_weights_s8(C.byref(d), ptr(q), IC, ptr(out)), "pack_conv_weights")
    return out


def pack_linear_weights(q: np.ndarray, K: int | None = None) -> np.ndarray:
    """Dense weights q[OC][IC] (IC <= K, K % 64 == 0) for dlq_linear_s8."""
    OC, IC = q.shape
    return pack_conv_weights(np.ascontiguousarray(q, np.int8).reshape(OC, IC, 1, 1), K or IC, 1, 1, 0)


def pack_stem_weights(q_oihw: np.ndarray, alpha: np.ndarray):
    """conv1 weights [64][3][7][7] int8 + conv1 alpha[64] -> (the fused stem's
    space-to-depth image, |alpha|) for stem_fused_s8 (see include/dlq.h)."""
    q = np.ascontiguousarray(q_oihw, np.int8)
    al = np.ascontiguousarray(alpha, np.float32)
    if q.shape != (64, 3, 7, 7) or al.shape != (64,):
        raise ValueError(f"stem weights must be [64,3,7,7] with alpha[64], got {q.shape}, {al.shape}")
    out = np.empty(lib.dlq_stem_packed_bytes(), np.int8)
    al_out = np.empty(64, np.float32)
    check(lib.dlq_pack_stem_weights_s8(ptr(q), ptr(al), ptr(out), ptr(al_out)), "pack_stem_weights")
    return out, al_out


def pack_downsample_weights(q_oc_ic: np.ndarray, C_store: int) -> np.ndarray:
    """1x1 downsample weights q[OC][IC] for conv2d_s2_ds_nhwc_s8."""
    q = np.ascontiguousarray(q_oc_ic, np.int8).reshape(q_oc_ic.shape[0], -1)
    OC, IC = q.shape
    nb = lib.dlq_downsample_packed_bytes(OC, C_store)
    if nb == 0:
        raise ValueError(f"unsupported downsample packing: C={C_store}")
    out = np.empty(nb, np.int8)
    check(lib.dlq_pack_downsample_weights_s8(ptr(q), OC, IC, C_store, ptr(out)), "pack_downsample_weights")
    return out


def pad_vec(v, n):
    out = np.zeros(n, np.float32)
    out[: len(v)] = v
    return out


# ------------------------------------------------------------------ device ops

def _dev(t: torch.Tensor, dtype) -> None:
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == dtype and t.is_contiguous()):
        raise TypeError(f"expected a contiguous CUDA tensor of {dtype}")


def quantize_nchw_to_nhwc(x: torch.Tensor, scale: float, c_out: int = 4) -> torch.Tensor:
    _dev(x, torch.float32)
    N, Cc, H, W = x.shape
    y = torch.empty((N, H, W, c_out), dtype=torch.int8, device=x.device)
    inv = float(np.float32(1.0) / np.float32(scale))
    check(lib.dlq_quantize_nchw_to_nhwc_s8(ptr(x), N, Cc, H, W, c_out, inv, ptr(y), stream_handle()),
          "quantize_nchw_to_nhwc")
    return y


def quantize_rows(x: torch.Tensor, scale: float, ld: int) -> torch.Tensor:
    _dev(x, torch.float32)
    rows, cols = x.shape
    y = torch.empty((rows, ld), dtype=torch.int8, device=x.device)
    inv = float(np.float32(1.0) / np.float32(scale))
    check(lib.dlq_quantize_rows_s8(ptr(x), rows, cols, ld, inv, ptr(y), stream_handle()), "quantize_rows")
    return y


def conv2d_nhwc_s8(x: torch.Tensor, w_packed: torch.Tensor, OC: int, k: int, stride: int, pad: int,
                   alpha: torch.Tensor | None = None, beta: torch.Tensor | None = None,
                   residual: torch.Tensor | None = None, res_scale: float = 0.0,
                   relu: bool = True, out_kind: int = DLQ_OUT_S8):
    """Implicit-GEMM int8 conv (+ fused epilogue) on NHWC x[N,H,W,C]; for int8
    output alpha/beta/res_scale are in output-grid units (fold_bn, res_scale)."""
    _dev(x, torch.int8)
    N, H, W, Cc = x.shape
    OH, OW = out_dim(H, k, stride, pad), out_dim(W, k, stride, pad)
    dt = {DLQ_OUT_S8: torch.int8, DLQ_OUT_F32: torch.float32, DLQ_OUT_S32: torch.int32}[out_kind]
    y = torch.empty((N, OH, OW, OC), dtype=dt, device=x.device)
    d = ConvDesc(N, H, W, Cc, OC, k, k, stride, stride, pad, pad)
    check(lib.dlq_conv2d_nhwc_s8(C.byref(d), ptr(x), ptr(w_packed), ptr(alpha), ptr(beta), ptr(residual),
                                 float(res_scale), int(relu), out_kind, ptr(y), stream_handle()),
          "conv2d_nhwc_s8")
    return y


def stem_fused_s8(x: torch.Tensor, w_stem: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor,
                  in_scale: float) -> torch.Tensor:
    """quantise + conv1 7x7/s2 + BN/ReLU/requant + maxpool 3x3/s2 in one launch:
    fp32 NCHW [N,3,224,224] -> int8 NHWC [N,56,56,64]; w_stem, alpha from
    pack_stem_weights, beta = conv1's beta (output-grid units)."""
    _dev(x, torch.float32)
    N = x.shape[0]
    if tuple(x.shape[1:]) != (3, 224, 224):
        raise ValueError(f"stem input must be [N,3,224,224], got {tuple(x.shape)}")
    y = torch.empty((N, 56, 56, 64), dtype=torch.int8, device=x.device)
    inv = float(np.float32(1.0) / np.float32(in_scale))
    check(lib.dlq_stem_fused_s8(ptr(x), N, ptr(w_stem), ptr(alpha), ptr(beta), inv, ptr(y), stream_handle()),
          "stem_fused_s8")
    return y


def conv2d_s2_ds_nhwc_s8(x: torch.Tensor, w_packed: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor,
                         w_ds: torch.Tensor, alpha_ds: torch.Tensor, beta_ds: torch.Tensor):
    """3x3/s2 conv (+BN+ReLU) and the fused 1x1/s2 downsample (+BN) of the same
    NHWC input: returns (y, y_ds), both int8 [N, H/2, W/2, 2C]."""
    _dev(x, torch.int8)
    N, H, W, Cc = x.shape
    OC = 2 * Cc
    y = torch.empty((N, H // 2, W // 2, OC), dtype=torch.int8, device=x.device)
    y_ds = torch.empty_like(y)
    d = ConvDesc(N, H, W, Cc, OC, 3, 3, 2, 2, 1, 1)
    check(lib.dlq_conv2d_s2_ds_nhwc_s8(C.byref(d), ptr(x), ptr(w_packed), ptr(alpha), ptr(beta), ptr(w_ds),
                                       ptr(alpha_ds), ptr(beta_ds), ptr(y), ptr(y_ds), stream_handle()),
          "conv2d_s2_ds_nhwc_s8")
    return y, y_ds


def conv2d_dsres_nhwc_s8(h: torch.Tensor, w_packed: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor,
                         x_blk: torch.Tensor, w_ds: torch.Tensor, alpha_ds: torch.Tensor, beta_ds: torch.Tensor,
                         res_scale: float) -> torch.Tensor:
    """A downsampling block's conv2 (3x3/s1 + BN) with the residual = the
    block input's 1x1/s2 downsample (+BN, requantised to int8) computed in the
    same launch, + ReLU (include/dlq.h dlq_conv2d_dsres_nhwc_s8): NHWC h[N,H,W,C],
    x_blk[N,2H,2W,C/2] -> int8 [N,H,W,C]."""
    _dev(h, torch.int8)
    _dev(x_blk, torch.int8)
    N, H, W, Cc = h.shape
    if tuple(x_blk.shape) != (N, 2 * H, 2 * W, Cc // 2):
        raise ValueError(f"conv2d_dsres_nhwc_s8: block input {tuple(x_blk.shape)} does not match h {tuple(h.shape)}")
    y = torch.empty_like(h)
    d = ConvDesc(N, H, W, Cc, Cc, 3, 3, 1, 1, 1, 1)
    check(lib.dlq_conv2d_dsres_nhwc_s8(C.byref(d), ptr(h), ptr(w_packed), ptr(alpha), ptr(beta), ptr(x_blk),
                                       ptr(w_ds), ptr(alpha_ds), ptr(beta_ds), float(res_scale), ptr(y),
                                       stream_handle()), "conv2d_dsres_nhwc_s8")
    return y


def block_l1_s8(x: torch.Tensor, w1: torch.Tensor, alpha1: torch.Tensor, beta1: torch.Tensor,
                w2: torch.Tensor, alpha2: torch.Tensor, beta2: torch.Tensor, res_scale: float) -> torch.Tensor:
    """Fused layer1 basic block on NHWC int8 x[N,56,56,64] (see include/dlq.h
    dlq_block_l1_nhwc_s8); w1/w2 from pack_conv_weights(q, 64, 56, 1, 1)."""
    _dev(x, torch.int8)
    if tuple(x.shape[1:]) != (56, 56, 64):
        raise ValueError(f"block_l1_s8: needs [N,56,56,64], got {tuple(x.shape)}")
    y = torch.empty_like(x)
    check(lib.dlq_block_l1_nhwc_s8(ptr(x), x.shape[0], ptr(w1), ptr(alpha1), ptr(beta1), ptr(w2), ptr(alpha2),
                                   ptr(beta2), float(res_scale), ptr(y), stream_handle()), "block_l1_s8")
    return y


def linear_s8(x: torch.Tensor, w_packed: torch.Tensor, OC: int, alpha=None, beta=None,
              relu: bool = False, out_kind: int = DLQ_OUT_F32):
    _dev(x, torch.int8)
    N, K = x.shape
    dt = {DLQ_OUT_S8: torch.int8, DLQ_OUT_F32: torch.float32, DLQ_OUT_S32: torch.int32}[out_kind]
    y = torch.empty((N, OC), dtype=dt, device=x.device)
    check(lib.dlq_linear_s8(ptr(x), N, K, ptr(w_packed), OC, ptr(alpha), ptr(beta), int(relu),
                            out_kind, ptr(y), stream_handle()), "linear_s8")
    return y


def maxpool2d_3x3_s2p1_nhwc_s8(x: torch.Tensor) -> torch.Tensor:
    _dev(x, torch.int8)
    N, H, W, Cc = x.shape
    y = torch.empty((N, out_dim(H, 3, 2, 1), out_dim(W, 3, 2, 1), Cc), dtype=torch.int8, device=x.device)
    check(lib.dlq_maxpool2d_3x3_s2p1_nhwc_s8(ptr(x), N, Cc, H, W, ptr(y), stream_handle()), "maxpool")
    return y


def gap_nhwc_s8(x: torch.Tensor, k: float) -> torch.Tensor:
    _dev(x, torch.int8)
    N, H, W, Cc = x.shape
    y = torch.empty((N, Cc), dtype=torch.int8, device=x.device)
    check(lib.dlq_gap_nhwc_s8(ptr(x), N, Cc, H * W, float(k), ptr(y), stream_handle()), "gap")
    return y


def gap_fc_s8(x: torch.Tensor, k: float, w_packed: torch.Tensor, OC: int, alpha: torch.Tensor,
              beta: torch.Tensor) -> torch.Tensor:
    """The network head in one launch (include/dlq.h dlq_gap_fc_s8): fp32
    logits [N, OC] from NHWC int8 x[N, H, W, 512], equal bit for bit to
    ``linear_s8(gap_nhwc_s8(x, k), w_packed, OC, alpha, beta)``."""
    _dev(x, torch.int8)
    N, H, W, Cc = x.shape
    y = torch.empty((N, OC), dtype=torch.float32, device=x.device)
    check(lib.dlq_gap_fc_s8(ptr(x), N, Cc, H * W, float(k), ptr(w_packed), OC, ptr(alpha), ptr(beta), ptr(y),
                            stream_handle()), "gap_fc")
    return y


def im2col_nchw_s8(x: torch.Tensor, k: int, stride: int, pad: int) -> torch.Tensor:
    _dev(x, torch.int8)
    N, Cc, H, W = x.shape
    OH, OW = out_dim(H, k, stride, pad), out_dim(W, k, stride, pad)
    col = torch.empty((N, Cc * k * k, OH * OW), dtype=torch.int8, device=x.device)
    check(lib.dlq_im2col_nchw_s8(ptr(x), N, Cc, H, W, k, k, stride, stride, pad, pad, ptr(col),
                                 stream_handle()), "im2col")
    return col


# ------------------------------------------------------------ the path's ends

def preprocess_u8(img: torch.Tensor) -> torch.Tensor:
    """u8 RGB images [N,H,W,3] (HWC, as np.array(PIL image)) on the device ->
    fp32 [N,3,224,224]: resize shorter side 256 (Pillow BILINEAR, bit-exact),
    centre crop 224, normalise (RK/tools/preprocess_to_bin.py:8-33)."""
    if not (img.is_cuda and img.dtype == torch.uint8 and img.dim() == 4 and img.shape[3] == 3):
        raise TypeError("img must be a CUDA uint8 [N,H,W,3] tensor")
    img = img.contiguous()
    N, H, W, _ = img.shape
    out = torch.empty((N, 3, 224, 224), dtype=torch.float32, device=img.device)
    check(lib.dlq_preprocess_u8(ptr(img), N, H, W, ptr(out), stream_handle()), "preprocess_u8")
    return out


def preprocess_size(H: int, W: int):
    nh, nw = C.c_int(), C.c_int()
    check(lib.dlq_preprocess_size(H, W, C.byref(nh), C.byref(nw)), "preprocess_size")
    return nh.value, nw.value


def softmax(x: torch.Tensor) -> torch.Tensor:
    """softmax_1d (RK/kernels/softmax.cu:5-47) on each row of fp32 [N,K]."""
    x = x.contiguous()
    y = torch.empty_like(x)
    check(lib.dlq_softmax_f32(ptr(x), x.shape[0], x.shape[1], ptr(y), stream_handle()), "softmax")
    return y


def top1(x: torch.Tensor):
    """The launcher's top-1 (RK/runtime/infer_e2e.cu:436-438) per row: (idx int32, logit)."""
    x = x.contiguous()
    idx = torch.empty(x.shape[0], dtype=torch.int32, device=x.device)
    val = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    check(lib.dlq_top1_f32(ptr(x), x.shape[0], x.shape[1], ptr(idx), ptr(val), stream_handle()), "top1")
    return idx, val


# ------------------------------------------------------------ fp8 (e4m3) path
# BASELINE configs[4]; include/dlq.h fp8 section.  e4m3 tensors are uint8
# code tensors (torch.float8_e4m3fn bytes).

def quantize_weights_f8(w: np.ndarray):
    w = np.ascontiguousarray(w, np.float32)
    OC = w.shape[0]
    K = w.size // OC
    q = np.empty(w.shape, np.uint8)
    s = np.empty(OC, np.float32)
    check(lib.dlq_quantize_weights_f8(w.ctypes.data, OC, K, q.ctypes.data, s.ctypes.data), "quantize_weights_f8")
    return q, s


def quantize_f32_f8(x: torch.Tensor, scale: float) -> torch.Tensor:
    _dev(x, torch.float32)
    y = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    inv = float(np.float32(1.0) / np.float32(scale))
    check(lib.dlq_quantize_f32_f8(ptr(x), x.numel(), inv, ptr(y), stream_handle()), "quantize_f32_f8")
    return y


def quantize_nchw_to_nhwc_f8(x: torch.Tensor, scale: float, c_out: int = 4) -> torch.Tensor:
    _dev(x, torch.float32)
    N, Cc, H, W = x.shape
    y = torch.empty((N, H, W, c_out), dtype=torch.uint8, device=x.device)
    inv = float(np.float32(1.0) / np.float32(scale))
    check(lib.dlq_quantize_nchw_to_nhwc_f8(ptr(x), N, Cc, H, W, c_out, inv, ptr(y), stream_handle()),
          "quantize_nchw_to_nhwc_f8")
    return y


def pack_conv_weights_f8(q_oihw: np.ndarray, C_store: int, H: int, stride: int, pad: int) -> np.ndarray:
    """Packed image of e4m3 OIHW codes for the conv {H x H, stride, pad}
    (dlq_pack_conv_weights_f8: the wide layout for the layer2-4 stride-1 3x3
    shapes, the generic one otherwise)."""
    q = np.ascontiguousarray(q_oihw, np.uint8)
    OC, IC, k, _ = q.shape
    d = ConvDesc(1, H, H, C_store, OC, k, k, stride, stride, pad, pad)
    nb = lib.dlq_conv_packed_bytes_f8(C.byref(d))
    if nb == 0:
        raise ValueError("unsupported conv shape for the fp8 path")
    out = np.empty(nb, np.uint8)
    check(lib.dlq_pack_conv_weights_f8(C.byref(d), q.ctypes.data, IC, out.ctypes.data), "pack_conv_weights_f8")
    return out


def conv2d_nhwc_f8(x: torch.Tensor, w_packed: torch.Tensor, OC: int, k: int, stride: int, pad: int,
                   alpha: torch.Tensor, beta: torch.Tensor, residual: torch.Tensor | None = None,
                   res_scale: float = 0.0, relu: bool = True) -> torch.Tensor:
    _dev(x, torch.uint8)
    N, H, W, Cc = x.shape
    OH, OW = out_dim(H, k, stride, pad), out_dim(W, k, stride, pad)
    y = torch.empty((N, OH, OW, OC), dtype=torch.uint8, device=x.device)
    d = ConvDesc(N, H, W, Cc, OC, k, k, stride, stride, pad, pad)
    check(lib.dlq_conv2d_nhwc_f8(C.byref(d), ptr(x), ptr(w_packed), ptr(alpha), ptr(beta), ptr(residual),
                                 float(res_scale), int(relu), ptr(y), stream_handle()), "conv2d_nhwc_f8")
    return y


def conv2d_nhwc_f8_acc(x: torch.Tensor, w_packed: torch.Tensor, OC: int, k: int, stride: int, pad: int):
    """Raw fp32 accumulators [N,OH,OW,OC] of the e4m3 conv (parity/debugging)."""
    _dev(x, torch.uint8)
    N, H, W, Cc = x.shape
    OH, OW = out_dim(H, k, stride, pad), out_dim(W, k, stride, pad)
    y = torch.empty((N, OH, OW, OC), dtype=torch.float32, device=x.device)
    d = ConvDesc(N, H, W, Cc, OC, k, k, stride, stride, pad, pad)
    check(lib.dlq_conv2d_nhwc_f8_acc(C.byref(d), ptr(x), ptr(w_packed), ptr(y), stream_handle()),
          "conv2d_nhwc_f8_acc")
    return y


def gap_nhwc_f8(x: torch.Tensor, k: float) -> torch.Tensor:
    _dev(x, torch.uint8)
    N, H, W, Cc = x.shape
    y = torch.empty((N, Cc), dtype=torch.uint8, device=x.device)
    check(lib.dlq_gap_nhwc_f8(ptr(x), N, Cc, H * W, float(k), ptr(y), stream_handle()), "gap_nhwc_f8")
    return y


def linear_f8(x: torch.Tensor, w: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor) -> torch.Tensor:
    _dev(x, torch.uint8)
    _dev(w, torch.uint8)
    N, K = x.shape
    O = w.shape[0]
    y = torch.empty((N, O), dtype=torch.float32, device=x.device)
    check(lib.dlq_linear_f8(ptr(x), N, K, ptr(w), O, ptr(alpha), ptr(beta), ptr(y), stream_handle()), "linear_f8")
    return y


def pack_stem_weights_f8(q_oihw: np.ndarray, alpha: np.ndarray):
    q = np.ascontiguousarray(q_oihw, np.uint8)
    a = np.ascontiguousarray(alpha, np.float32)
    out = np.empty(64 * 256, np.uint8)
    ap = np.empty(64, np.float32)
    check(lib.dlq_pack_stem_weights_f8(q.ctypes.data, a.ctypes.data, out.ctypes.data, ap.ctypes.data),
          "pack_stem_weights_f8")
    return out, ap


def stem_fused_f8(x: torch.Tensor, w_stem: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor,
                  in_scale: float) -> torch.Tensor:
    """e4m3 fused stem: fp32 NCHW [N,3,224,224] -> e4m3 NHWC [N,56,56,64]."""
    _dev(x, torch.float32)
    N = x.shape[0]
    if tuple(x.shape[1:]) != (3, 224, 224):
        raise ValueError(f"stem input must be [N,3,224,224], got {tuple(x.shape)}")
    y = torch.empty((N, 56, 56, 64), dtype=torch.uint8, device=x.device)
    inv = float(np.float32(1.0) / np.float32(in_scale))
    check(lib.dlq_stem_fused_f8(ptr(x), N, ptr(w_stem), ptr(alpha), ptr(beta), inv, ptr(y), stream_handle()),
          "stem_fused_f8")
    return y


def conv2d_s2_ds_nhwc_f8(x: torch.Tensor, w_packed: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor,
                         w_ds: torch.Tensor, alpha_ds: torch.Tensor, beta_ds: torch.Tensor):
    """e4m3 twin of conv2d_s2_ds_nhwc_s8 (w_ds = pack_downsample_weights of the
    e4m3 codes viewed as int8): returns (y, y_ds), uint8 [N, H/2, W/2, 2C]."""
    _dev(x, torch.uint8)
    N, H, W, Cc = x.shape
    OC = 2 * Cc
    y = torch.empty((N, H // 2, W // 2, OC), dtype=torch.uint8, device=x.device)
    y_ds = torch.empty_like(y)
    d = ConvDesc(N, H, W, Cc, OC, 3, 3, 2, 2, 1, 1)
    check(lib.dlq_conv2d_s2_ds_nhwc_f8(C.byref(d), ptr(x), ptr(w_packed), ptr(alpha), ptr(beta), ptr(w_ds),
                                       ptr(alpha_ds), ptr(beta_ds), ptr(y), ptr(y_ds), stream_handle()),
          "conv2d_s2_ds_nhwc_f8")
    return y, y_ds


def block_l1_f8(x: torch.Tensor, w1: torch.Tensor, alpha1: torch.Tensor, beta1: torch.Tensor,
                w2: torch.Tensor, alpha2: torch.Tensor, beta2: torch.Tensor, res_scale: float) -> torch.Tensor:
    """e4m3 layer1 basic block in one launch: NHWC [N,56,56,64] -> same."""
    _dev(x, torch.uint8)
    if tuple(x.shape[1:]) != (56, 56, 64):
        raise ValueError(f"block_l1 input must be [N,56,56,64], got {tuple(x.shape)}")
    y = torch.empty_like(x)
    check(lib.dlq_block_l1_nhwc_f8(ptr(x), x.shape[0], ptr(w1), ptr(alpha1), ptr(beta1), ptr(w2), ptr(alpha2),
                                   ptr(beta2), float(res_scale), ptr(y), stream_handle()), "block_l1_f8")
    return y
