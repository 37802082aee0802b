"""CPU: libdlq.so loads, exports every symbol include/dlq.h declares, its
host-side weight preparation is bit-identical to the oracle, and it reports
errors (never exits) -- all without touching a GPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import rand_conv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dlq.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dlq_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from dlq_amd import lib as L
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L.lib, s)]
    assert not missing, missing
    assert set(L.exported_symbols()) == set(syms), set(syms) ^ set(L.exported_symbols())
    assert b"gfx950" in L.lib.dlq_version()


def test_launcher_links_library():
    exe = os.path.join(ROOT, "bin", "dlq_e2e")
    if not os.path.exists(exe):
        pytest.skip("bin/dlq_e2e not built")
    import subprocess
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 1 and "--manifest" in r.stdout  # usage, like infer_e2e.cu:221-240


def test_step_driver_links_library():
    exe = os.path.join(ROOT, "bin", "dlq_step")
    if not os.path.exists(exe):
        pytest.skip("bin/dlq_step not built")
    import subprocess
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 1 and "--step head" in r.stdout  # usage, like infer_head.cu:12-14


def test_host_quantize_and_fold_match_oracle():
    from dlq_amd import ops
    rng = np.random.default_rng(0)
    for (oc, ic, k) in [(64, 3, 7), (128, 64, 3), (512, 256, 1), (1000, 512, 1)]:
        w, bn = rand_conv(rng, oc, ic, k)
        q_lib, s_lib = ops.quantize_weights(w)
        q_ora, s_ora = O.quantize_weights_s8(w)
        assert np.array_equal(q_lib, q_ora) and np.array_equal(s_lib, s_ora)
        a_lib, b_lib = ops.fold_bn(0.0123, s_lib, *bn, 0.047)
        a_ora, b_ora = O.fold_bn(0.0123, s_ora, bn, 0.047)
        assert np.array_equal(a_lib, a_ora) and np.array_equal(b_lib, b_ora)
        assert np.float32(ops.res_scale(0.052, 0.047)) == O.res_scale(0.052, 0.047)


def test_pack_layout():
    """Packed image is [OCp][kh][kw][C] (K contiguous, zero padded); the stem
    pads 7x7 taps to 8x8 and 3 channels to 4."""
    from dlq_amd import ops
    rng = np.random.default_rng(1)
    q = rng.integers(-127, 128, size=(100, 128, 3, 3), dtype=np.int8)
    ocp = ops.packed_oc(100)
    # [C/64][OCp/64][64 oc][9 taps][4 chunks of 16, stored at chunk ^ ((oc%64>>2)&3)]
    p = ops.pack_conv_weights(q, 128, 56, 1, 1).reshape(2, ocp // 64, 64, 9, 4, 16)
    oc = np.arange(ocp).reshape(ocp // 64, 64)
    perm = (np.arange(4)[None, :] ^ ((np.arange(64)[:, None] >> 2) & 3))  # [ol][logical chunk] -> stored pos
    logical = np.empty_like(p)
    for ol in range(64):
        for lc in range(4):
            logical[:, :, ol, :, lc, :] = p[:, :, ol, :, perm[ol, lc], :]
    dense = logical.transpose(1, 2, 3, 0, 4, 5).reshape(ocp, 3, 3, 128)  # [OCp][kh][kw][c]
    assert np.array_equal(dense[:100], np.transpose(q, (0, 2, 3, 1)))
    assert not dense[100:].any() and oc.size == ocp
    qs = rng.integers(-127, 128, size=(64, 3, 7, 7), dtype=np.int8)
    ps = ops.pack_conv_weights(qs, 4, 224, 2, 3).reshape(64, 8, 8, 4)
    assert np.array_equal(ps[:, :7, :7, :3], np.transpose(qs, (0, 2, 3, 1)))
    assert not ps[:, 7].any() and not ps[:, :, 7].any() and not ps[..., 3].any()


@pytest.mark.parametrize("C,H", [(128, 28), (256, 14), (512, 7)])
def test_pack_layout_wide_s1(C, H):
    """Wide stride-1 3x3 convs: [OC/128][C/32][128 oc][9 taps x 32 ch + 16 zero]."""
    from dlq_amd import ops
    rng = np.random.default_rng(C)
    q = rng.integers(-127, 128, size=(C, C, 3, 3), dtype=np.int8)
    p = ops.pack_conv_weights(q, C, H, 1, 1).reshape(C // 128, C // 32, 128, 304)
    assert not p[..., 288:].any()
    taps = p[..., :288].reshape(C // 128, C // 32, 128, 9, 32)      # [ot][j][ol][tap][cc]
    dense = taps.transpose(0, 2, 3, 1, 4).reshape(C, 3, 3, C)        # [oc][kh][kw][c]
    assert np.array_equal(dense, np.transpose(q, (0, 2, 3, 1)))
    # the same weights for a stride-2 conv or another resolution keep the generic layout
    assert ops.pack_conv_weights(q, C, 2 * H, 1, 1).size == C * 9 * C


def test_errors_are_returned_not_exited():
    from dlq_amd.lib import ConvDesc, lib
    d = ConvDesc(1, 8, 8, 3, 8, 3, 3, 1, 1, 1, 1)  # C=3 with a 3x3 kernel: unsupported
    rc = lib.dlq_conv2d_nhwc_s8(C.byref(d), 1, 1, 1, 1, None, 0.0, 1, 0, 1, None)
    assert rc == 1 and b"unsupported" in lib.dlq_last_error()
    assert lib.dlq_conv_packed_bytes(C.byref(d)) == 0
    h = C.c_void_p()
    assert lib.dlq_resnet18_create(C.byref(h)) == 0
    try:
        assert lib.dlq_resnet18_set_tensor(h, b"nope.weight", np.zeros(1, np.float32).ctypes.data, 1) == 1
        assert lib.dlq_resnet18_set_scale(h, b"conv1", -1.0) == 1
        assert lib.dlq_resnet18_prepare(h, 4, None) == 5  # missing tensors -> DLQ_ERR_STATE
        assert b"missing tensor" in lib.dlq_last_error()
        assert lib.dlq_resnet18_load_manifest(h, b"/nonexistent_dir") == 4
        assert lib.dlq_resnet18_forward(h, 1, 1, 1, None) == 5  # not prepared
    finally:
        lib.dlq_resnet18_destroy(h)


def test_scales_roundtrip(tmp_path):
    from dlq_amd.quant import load_scales, save_scales
    from tests.helpers import model_and_scales
    _, scales = model_and_scales()
    p = tmp_path / "scales.txt"
    save_scales(scales, str(p))
    back = load_scales(str(p))
    assert all(np.float32(back[k]) == np.float32(v) for k, v in scales.items())
