"""ctypes binding of libdlq.so (include/dlq.h).

The product path: every call goes to the hand-written gfx950 kernels through
the C ABI.  There is NO fallback -- if the library is missing or was not
built, importing this module raises.  PyTorch is used only as plumbing
(device memory, streams, torch.distributed); it is imported first so that
libdlq.so binds to the same HIP runtime instance as torch (both load
libamdhip64.so.7 by soname).
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the CDLL: shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
# DLQ_LIB_PATH: load another build of the same library (A/B timing of two
# builds on one box); the default is the in-tree dlq_amd/libdlq.so.
LIB_PATH = os.environ.get("DLQ_LIB_PATH") or os.path.join(_HERE, "libdlq.so")

DLQ_OK = 0
DLQ_OUT_S8, DLQ_OUT_F32, DLQ_OUT_S32 = 0, 1, 2
DLQ_PREC_INT8, DLQ_PREC_FP8 = 0, 1
# kernel families of dlq_resnet18_timing (include/dlq.h DLQ_FAM_*)
# (the first word names the int8 forward's kernel; the fp8 forward runs
# stem_fused_kernel and block_l1_kernel in families 0 and 1)
FAMILIES = ["stem2_kernel (int8 stem; fp8: stem_fused_kernel)",
            "block_l1_sp_kernel (int8 layer1 block; fp8: block_l1_kernel)", "conv3x3s2i_kernel (layer2-4 .0 conv1; + downsample at layer4.0)",
            "conv3x3i_kernel (layer2-4 s1)", "head: gap_fc_kernel (int8 GAP+FC) / gap16 (fp8, split)", "linear_kernel (FC on the pooled codes; fp8 / split head)", "other",
            "conv_s8_kernel fp8 (all convs, fp8 path)"]


class DLQError(RuntimeError):
    pass


class ConvDesc(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("N", "H", "W", "C", "OC", "kH", "kW", "sH", "sW", "pH", "pW")]


_vp, _i, _f, _sz = C.c_void_p, C.c_int, C.c_float, C.c_size_t
_SIGS = {
    "dlq_version": ([], C.c_char_p),
    "dlq_last_error": ([], C.c_char_p),
    "dlq_device_arch": ([_i, C.c_char_p, _i], _i),
    "dlq_set_knob": ([C.c_char_p, _i], _i),
    "dlq_get_knob": ([C.c_char_p, C.POINTER(_i)], _i),
    "dlq_quantize_weights_s8": ([_vp, _i, _i, _vp, _vp], _i),
    "dlq_fold_bn": ([_f, _vp, _vp, _vp, _vp, _vp, _f, _f, _i, _vp, _vp], _i),
    "dlq_res_scale": ([_f, _f], _f),
    "dlq_conv_packed_oc": ([_i], _i),
    "dlq_conv_packed_bytes": ([C.POINTER(ConvDesc)], _sz),
    "dlq_pack_conv_weights_s8": ([C.POINTER(ConvDesc), _vp, _i, _vp], _i),
    "dlq_quantize_nchw_to_nhwc_s8": ([_vp, _i, _i, _i, _i, _i, _f, _vp, _vp], _i),
    "dlq_quantize_rows_s8": ([_vp, _i, _i, _i, _f, _vp, _vp], _i),
    "dlq_conv2d_nhwc_s8": ([C.POINTER(ConvDesc), _vp, _vp, _vp, _vp, _vp, _f, _i, _i, _vp, _vp], _i),
    "dlq_init": ([_i], _i),
    "dlq_finalize": ([], _i),
    "dlq_quantize_f32_s8": ([_vp, _sz, _f, _vp, _vp], _i),
    "dlq_gemm_s8s8s32": ([_vp, _vp, _vp, _i, _i, _i, _vp], _i),
    "dlq_gemm_s8s8s32_nt": ([_vp, _vp, _vp, _i, _i, _i, _vp], _i),
    "dlq_conv2d_nchw_workspace_bytes": ([_i] * 11, _sz),
    "dlq_conv2d_nchw_s8": ([_vp, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp,
                            _sz, _vp, C.POINTER(_i), C.POINTER(_i)], _i),
    "dlq_bn_relu_requant_s8": ([_vp, _i, _i, _i, _vp, _vp, _i, _vp, _vp], _i),
    "dlq_add_relu_requant_s8": ([_vp, _vp, _sz, _f, _f, _i, _vp, _vp], _i),
    "dlq_maxpool2d_3x3_s2p1_nchw_s8": ([_vp, _i, _i, _i, _i, _vp, _vp], _i),
    "dlq_gap_s8": ([_vp, _i, _i, _i, _f, _vp, _vp], _i),
    "dlq_fc_s8": ([_vp, _i, _i, _vp, _i, _vp, _vp, _vp, _vp], _i),
    "dlq_dequant_s32_f32": ([_vp, _i, _i, _i, _vp, _vp, _vp], _i),
    "dlq_basic_block_s8": ([_vp, _i, _vp, _i, _vp, _vp], _i),
    "dlq_downsample_packed_bytes": ([_i, _i], _sz),
    "dlq_pack_downsample_weights_s8": ([_vp, _i, _i, _i, _vp], _i),
    "dlq_block_l1_nhwc_s8": ([_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, C.c_float, _vp, _vp], _i),
    "dlq_conv2d_s2_ds_nhwc_s8": ([C.POINTER(ConvDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "dlq_conv2d_dsres_nhwc_s8": ([C.POINTER(ConvDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_float, _vp, _vp],
                                 _i),
    "dlq_stem_packed_bytes": ([], _sz),
    "dlq_pack_stem_weights_s8": ([_vp, _vp, _vp, _vp], _i),
    "dlq_stem_fused_s8": ([_vp, _i, _vp, _vp, _vp, _f, _vp, _vp], _i),
    "dlq_linear_s8": ([_vp, _i, _i, _vp, _i, _vp, _vp, _i, _i, _vp, _vp], _i),
    "dlq_maxpool2d_3x3_s2p1_nhwc_s8": ([_vp, _i, _i, _i, _i, _vp, _vp], _i),
    "dlq_gap_nhwc_s8": ([_vp, _i, _i, _i, _f, _vp, _vp], _i),
    "dlq_gap_fc_s8": ([_vp, _i, _i, _i, _f, _vp, _i, _vp, _vp, _vp, _vp], _i),
    "dlq_im2col_nchw_s8": ([_vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp], _i),
    "dlq_resnet18_create": ([C.POINTER(_vp)], _i),
    "dlq_resnet18_destroy": ([_vp], None),
    "dlq_resnet18_set_tensor": ([_vp, C.c_char_p, _vp, _sz], _i),
    "dlq_resnet18_set_scale": ([_vp, C.c_char_p, _f], _i),
    "dlq_resnet18_load_manifest": ([_vp, C.c_char_p], _i),
    "dlq_resnet18_load_scales": ([_vp, C.c_char_p], _i),
    "dlq_resnet18_set_keep_stages": ([_vp, _i], _i),
    "dlq_resnet18_prepare": ([_vp, _i, _vp], _i),
    "dlq_resnet18_forward": ([_vp, _vp, _i, _vp, _vp], _i),
    "dlq_resnet18_stage": ([_vp, C.c_char_p, _vp, _sz, C.POINTER(_sz), _vp], _i),
    "dlq_resnet18_set_timing": ([_vp, _i], _i),
    "dlq_resnet18_timing": ([_vp, _vp, _vp, C.POINTER(_i)], _i),
    "dlq_resnet18_family_work": ([_vp, _vp, _vp], _i),
    "dlq_resnet18_macs_per_image": ([_vp, C.POINTER(C.c_double), C.POINTER(C.c_double)], _i),
    "dlq_resnet18_forward_f32": ([_vp, _vp, _i, _vp, _vp], _i),
    "dlq_resnet18_stage_f32": ([_vp, C.c_char_p, _vp, _sz, C.POINTER(_sz), _vp], _i),
    "dlq_resnet18_calibrate": ([_vp, _vp, _i, _f, _vp], _i),
    "dlq_mlp_create": ([_i, _i, _i, _vp, _vp, _vp, _vp, _f, _f, _i, _vp, C.POINTER(_vp)], _i),
    "dlq_mlp_destroy": ([_vp], None),
    "dlq_mlp_forward": ([_vp, _vp, _i, _vp, _vp], _i),
    "dlq_mlp_copy_hidden": ([_vp, _i, _vp, _sz, _vp], _i),
    "dlq_resnet18_set_tensor_s8": ([_vp, C.c_char_p, _vp, _sz, _vp, _sz], _i),
    "dlq_resnet18_save_manifest": ([_vp, C.c_char_p, _i], _i),
    "dlq_resnet18_save_scales": ([_vp, C.c_char_p], _i),
    "dlq_preprocess_size": ([_i, _i, C.POINTER(_i), C.POINTER(_i)], _i),
    "dlq_preprocess_u8": ([_vp, _i, _i, _i, _vp, _vp], _i),
    "dlq_softmax_f32": ([_vp, _i, _i, _vp, _vp], _i),
    "dlq_top1_f32": ([_vp, _i, _i, _vp, _vp, _vp], _i),
    "dlq_quantize_weights_f8": ([_vp, _i, _i, _vp, _vp], _i),
    "dlq_quantize_f32_f8": ([_vp, _sz, _f, _vp, _vp], _i),
    "dlq_quantize_nchw_to_nhwc_f8": ([_vp, _i, _i, _i, _i, _i, _f, _vp, _vp], _i),
    "dlq_conv_packed_bytes_f8": ([C.POINTER(ConvDesc)], _sz),
    "dlq_pack_conv_weights_f8": ([C.POINTER(ConvDesc), _vp, _i, _vp], _i),
    "dlq_conv2d_nhwc_f8": ([C.POINTER(ConvDesc), _vp, _vp, _vp, _vp, _vp, _f, _i, _vp, _vp], _i),
    "dlq_conv2d_nhwc_f8_acc": ([C.POINTER(ConvDesc), _vp, _vp, _vp, _vp], _i),
    "dlq_gap_nhwc_f8": ([_vp, _i, _i, _i, _f, _vp, _vp], _i),
    "dlq_linear_f8": ([_vp, _i, _i, _vp, _i, _vp, _vp, _vp, _vp], _i),
    "dlq_resnet18_set_precision": ([_vp, _i], _i),
    "dlq_pack_stem_weights_f8": ([_vp, _vp, _vp, _vp], _i),
    "dlq_stem_fused_f8": ([_vp, _i, _vp, _vp, _vp, _f, _vp, _vp], _i),
    "dlq_conv2d_s2_ds_nhwc_f8": ([C.POINTER(ConvDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "dlq_block_l1_nhwc_f8": ([_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, C.c_float, _vp, _vp], _i),
}

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()). "
        "There is no fallback path.")
lib = C.CDLL(LIB_PATH)
for _name, (_args, _res) in _SIGS.items():
    _fn = getattr(lib, _name)
    _fn.argtypes = _args
    _fn.restype = _res


def exported_symbols():
    return list(_SIGS)


def last_error() -> str:
    return lib.dlq_last_error().decode()


def check(rc: int, what: str = "dlq") -> None:
    if rc != DLQ_OK:
        raise DLQError(f"{what} failed (code {rc}): {last_error()}")


def get_knob(name: str) -> int:
    v = C.c_int(0)
    check(lib.dlq_get_knob(name.encode(), C.byref(v)), f"get_knob({name})")
    return v.value


def set_knob(name: str, value: int) -> int:
    """Set a process-wide knob (include/dlq.h dlq_set_knob); returns the old value."""
    old = get_knob(name)
    check(lib.dlq_set_knob(name.encode(), int(value)), f"set_knob({name})")
    return old


def ptr(t) -> int | None:
    """Device (or host numpy) address of a tensor/array, None for None."""
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        return t.data_ptr()
    return t.ctypes.data  # numpy


def stream_handle(stream=None) -> int | None:
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream
