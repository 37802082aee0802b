"""GPU parity: every HIP kernel through the C ABI vs the CPU oracle.

Bar (BASELINE.json north_star): int32 accumulators bit-exact; the fp32
epilogue is a fixed IEEE op sequence, so int8 activations and fp32 logits
are required bit-exact too (stricter than the 1e-6 rel the north star allows).
The oracle works in the reference's layout (NCHW, im2col row order
c*kH*kW+kh*kW+kw, kernels/im2col.cu:37-54); the GPU works in NHWC with K
ordered (kh,kw,c) -- equal int32 sums prove the implicit im2col.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import model_and_scales, nchw_to_nhwc, nhwc_to_nchw, rand_conv, rand_s8

pytestmark = pytest.mark.gpu

# Every conv shape of ResNet-18 (infer_e2e.cu:259-407): (name, IC, OC, k, s, p, H)
CONV_SHAPES = [
    ("stem", 3, 64, 7, 2, 3, 224),
    ("l1_3x3", 64, 64, 3, 1, 1, 56),
    ("l2_0_conv1", 64, 128, 3, 2, 1, 56),
    ("l2_3x3", 128, 128, 3, 1, 1, 28),
    ("l2_ds", 64, 128, 1, 2, 0, 56),
    ("l3_0_conv1", 128, 256, 3, 2, 1, 28),
    ("l3_3x3", 256, 256, 3, 1, 1, 14),
    ("l3_ds", 128, 256, 1, 2, 0, 28),
    ("l4_0_conv1", 256, 512, 3, 2, 1, 14),
    ("l4_3x3", 512, 512, 3, 1, 1, 7),
    ("l4_ds", 256, 512, 1, 2, 0, 14),
]


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _gpu_conv_inputs(x_nchw, wq, s, p):
    from dlq_amd import ops
    IC = wq.shape[1]
    c_store = 4 if IC == 3 else IC
    xh = nchw_to_nhwc(x_nchw)
    if c_store != IC:
        xh = np.concatenate([xh, np.zeros(xh.shape[:3] + (c_store - IC,), np.int8)], axis=3)
    packed = ops.pack_conv_weights(wq, c_store, x_nchw.shape[2], s, p)
    return _cuda(xh), _cuda(packed)


@pytest.mark.parametrize("shape", CONV_SHAPES, ids=[s[0] for s in CONV_SHAPES])
def test_conv_int32_accumulators_bitexact(gpu, shape):
    from dlq_amd import ops
    from dlq_amd.lib import DLQ_OUT_S32
    name, IC, OC, k, s, p, H = shape
    rng = np.random.default_rng(sum(map(ord, name)) * 7919)
    N = 2 if H >= 56 else 3  # ragged: 3*OH*OW is not a multiple of the pixel tile
    x = rand_s8(rng, (N, IC, H, H))
    w, _ = rand_conv(rng, OC, IC, k)
    wq, _ = O.quantize_weights_s8(w)
    ref = O.conv_s8_acc(x, wq, s, p)
    xd, wd = _gpu_conv_inputs(x, wq, s, p)
    acc = ops.conv2d_nhwc_s8(xd, wd, OC, k, s, p, out_kind=DLQ_OUT_S32)
    got = nhwc_to_nchw(acc.cpu().numpy())
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), f"{name}: {np.count_nonzero(got != ref)} int32 mismatches"


@pytest.mark.parametrize("shape", [CONV_SHAPES[i] for i in (0, 1, 2, 3, 4, 6, 9)],
                         ids=[CONV_SHAPES[i][0] for i in (0, 1, 2, 3, 4, 6, 9)])
@pytest.mark.parametrize("residual", [False, True])
def test_conv_fused_epilogue_bitexact(gpu, shape, residual):
    from dlq_amd import ops
    name, IC, OC, k, s, p, H = shape
    if residual and IC == 3:
        pytest.skip("the stem has no residual input")
    if residual and k == 3 and s == 2:
        pytest.skip("a stride-2 conv1 has no residual input (the API rejects one, see test_errors)")
    rng = np.random.default_rng(7 + sum(map(ord, name)))
    N = 3 if residual else 2  # 3: a half-empty last item at 14x14 / 7x7 (the LDS-staged residual's zero pieces)
    x = rand_s8(rng, (N, IC, H, H))
    w, bn = rand_conv(rng, OC, IC, k)
    wq, sw = O.quantize_weights_s8(w)
    s_x, s_y, s_r = 0.031, 0.047, 0.052
    alpha, beta = O.fold_bn(s_x, sw, bn, s_y)
    r_s = O.res_scale(s_r, s_y)
    acc = O.conv_s8_acc(x, wq, s, p)
    res = rand_s8(rng, acc.shape) if residual else None
    relu = (k != 1)  # downsample convs have no ReLU (infer_e2e.cu:187-196)
    ref = O.epilogue_s8(acc, alpha, beta, res, r_s, relu)
    xd, wd = _gpu_conv_inputs(x, wq, s, p)
    ocp = ops.packed_oc(OC)
    a_alpha, a_beta = ops.fold_bn(s_x, sw, *bn, s_y)
    assert np.array_equal(a_alpha, alpha) and np.array_equal(a_beta, beta)  # host prep == oracle
    y = ops.conv2d_nhwc_s8(xd, wd, OC, k, s, p, _cuda(ops.pad_vec(a_alpha, ocp)), _cuda(ops.pad_vec(a_beta, ocp)),
                           residual=_cuda(nchw_to_nhwc(res)) if residual else None, res_scale=r_s, relu=relu)
    got = nhwc_to_nchw(y.cpu().numpy())
    assert np.array_equal(got, ref), f"{name}: {np.count_nonzero(got != ref)} int8 mismatches"


@pytest.mark.parametrize("N", [1, 3, 37])
def test_stem_fused_bitexact(gpu, N):
    """quantise + conv1 7x7/s2 + BN/ReLU/requant + maxpool as ONE launch
    (infer_e2e.cu:259-301) == the oracle's four separate steps."""
    from dlq_amd import ops
    rng = np.random.default_rng(41 + N)
    x = (rng.standard_normal((N, 3, 224, 224), dtype=np.float32) * 1.7).astype(np.float32)
    x[0, :, 0, :6] = [[0.5, 1.5, -2.5, 1e9, -1e9, 0.0]] * 3  # ties, saturation, the padded border
    x[N - 1, 2, 223, 218:] = [-0.5, 2.5, 1e9, -1e9, 3.5, 0.0]
    w, bn = rand_conv(rng, 64, 3, 7)
    bn[0][::3] *= -1  # some negative BN gammas -> negative alpha (the packer's sign fold)
    wq, sw = O.quantize_weights_s8(w)
    s_in, s_y = 2.64 / 127, 0.043
    alpha, beta = O.fold_bn(s_in, sw, bn, s_y)
    assert (alpha < 0).any() and (alpha > 0).any()
    xq = O.quantize_f32_s8(x, s_in)
    ref = O.maxpool_s8(O.epilogue_s8(O.conv_s8_acc(xq, wq, 2, 3), alpha, beta, None, 0.0, True))
    wst, al_p = ops.pack_stem_weights(wq, alpha)
    y = ops.stem_fused_s8(_cuda(x), _cuda(wst), _cuda(al_p), _cuda(beta), s_in)
    got = nhwc_to_nchw(y.cpu().numpy())
    assert np.array_equal(got, ref), f"{np.count_nonzero(got != ref)} int8 mismatches"


@pytest.mark.parametrize("C,H,N", [(64, 56, 3), (128, 28, 5), (256, 14, 37)])
def test_s2_conv_with_fused_downsample_bitexact(gpu, C, H, N):
    """layerX.0: 3x3/s2 conv1 (+BN+ReLU) and the 1x1/s2 downsample (+BN, no
    ReLU) from ONE launch == the oracle's two convs (infer_e2e.cu:161-196)."""
    from dlq_amd import ops
    rng = np.random.default_rng(C * 7 + N)
    OC = 2 * C
    x = rand_s8(rng, (N, C, H, H))
    w, bn = rand_conv(rng, OC, C, 3)
    wd, bnd = rand_conv(rng, OC, C, 1)
    bnd[0][::5] *= -1
    wq, sw = O.quantize_weights_s8(w)
    wdq, swd = O.quantize_weights_s8(wd)
    s_x, s_y, s_d = 0.03, 0.045, 0.06
    alpha, beta = O.fold_bn(s_x, sw, bn, s_y)
    alpha_d, beta_d = O.fold_bn(s_x, swd, bnd, s_d)
    ref = O.epilogue_s8(O.conv_s8_acc(x, wq, 2, 1), alpha, beta, None, 0.0, True)
    ref_d = O.epilogue_s8(O.conv_s8_acc(x, wdq, 2, 0), alpha_d, beta_d, None, 0.0, False)
    xd, wdev = _gpu_conv_inputs(x, wq, 2, 1)
    wds = _cuda(ops.pack_downsample_weights(wdq.reshape(OC, C), C))
    y, y_ds = ops.conv2d_s2_ds_nhwc_s8(xd, wdev, _cuda(alpha), _cuda(beta), wds, _cuda(alpha_d), _cuda(beta_d))
    got, got_d = nhwc_to_nchw(y.cpu().numpy()), nhwc_to_nchw(y_ds.cpu().numpy())
    assert np.array_equal(got, ref), f"conv1: {np.count_nonzero(got != ref)} mismatches"
    assert np.array_equal(got_d, ref_d), f"downsample: {np.count_nonzero(got_d != ref_d)} mismatches"


def _dsres_case(C, H, N, seed):
    """A downsampling block's back half at conv2's resolution H (C channels):
    block input x (C/2 @ 2H), conv2 input h, weights, scales and the oracle's
    conv2 output with the downsample residual (infer_e2e.cu:177-202)."""
    rng = np.random.default_rng(seed)
    Ci = C // 2
    x = rand_s8(rng, (N, Ci, 2 * H, 2 * H))
    h = rand_s8(rng, (N, C, H, H))
    w2, bn2 = rand_conv(rng, C, C, 3)
    wd, bnd = rand_conv(rng, C, Ci, 1)
    bnd[0][::5] *= -1
    w2q, sw2 = O.quantize_weights_s8(w2)
    wdq, swd = O.quantize_weights_s8(wd)
    s_x, s_h, s_d, s_y = 0.03, 0.027, 0.06, 0.045  # a few % of both requantisations at a clamp
    alpha, beta = O.fold_bn(s_h, sw2, bn2, s_y)
    alpha_d, beta_d = O.fold_bn(s_x, swd, bnd, s_d)
    r_s = O.res_scale(s_d, s_y)
    return x, h, w2q, wdq, alpha, beta, alpha_d, beta_d, r_s


def _dsres_gpu(x, h, w2q, wdq, alpha, beta, alpha_d, beta_d, r_s):
    from dlq_amd import ops
    C = h.shape[1]
    hd, w2dev = _gpu_conv_inputs(h, w2q, 1, 1)
    wds = _cuda(ops.pack_downsample_weights(wdq.reshape(C, C // 2), C // 2))
    y = ops.conv2d_dsres_nhwc_s8(hd, w2dev, _cuda(alpha), _cuda(beta), _cuda(nchw_to_nhwc(x)), wds, _cuda(alpha_d),
                                 _cuda(beta_d), r_s)
    return nhwc_to_nchw(y.cpu().numpy())


@pytest.mark.parametrize("C,H,N", [(128, 28, 3), (256, 14, 5), (256, 14, 37), (128, 28, 1), (128, 28, 9)])
def test_conv2_with_downsample_residual_bitexact(gpu, C, H, N):
    """layerX.0 conv2 (+BN) + the block's 1x1/s2 downsample (+BN, requantised)
    computed in the same launch + ReLU == the oracle's downsample conv, its
    int8 epilogue, and conv2's residual epilogue (infer_e2e.cu:177-202); ragged
    batches (partial items, trash-line stores)."""
    x, h, w2q, wdq, alpha, beta, alpha_d, beta_d, r_s = _dsres_case(C, H, N, C * 11 + N)
    ref_d = O.epilogue_s8(O.conv_s8_acc(x, wdq, 2, 0), alpha_d, beta_d, None, 0.0, False)
    ref = O.epilogue_s8(O.conv_s8_acc(h, w2q, 1, 1), alpha, beta, ref_d, r_s, True)
    got = _dsres_gpu(x, h, w2q, wdq, alpha, beta, alpha_d, beta_d, r_s)
    assert np.array_equal(got, ref), f"{np.count_nonzero(got != ref)} int8 mismatches"


@pytest.mark.parametrize("C,H,N", [(128, 28, 90), (256, 14, 180)])
def test_conv2_with_downsample_residual_many_items(gpu, C, H, N):
    """The downsample-residual epilogue when every workgroup walks several
    items (the next item's DMA in flight during the epilogue's loads):
    sampled images against the oracle, and the whole batch against the fused
    stride-2 kernel's stored downsample fed to conv2 as a loaded residual."""
    from dlq_amd import ops
    x, h, w2q, wdq, alpha, beta, alpha_d, beta_d, r_s = _dsres_case(C, H, N, C + N)
    got = _dsres_gpu(x, h, w2q, wdq, alpha, beta, alpha_d, beta_d, r_s)
    for i in (0, 1, N // 2, N - 1):
        ref_d = O.epilogue_s8(O.conv_s8_acc(x[i:i + 1], wdq, 2, 0), alpha_d, beta_d, None, 0.0, False)
        ref = O.epilogue_s8(O.conv_s8_acc(h[i:i + 1], w2q, 1, 1), alpha, beta, ref_d, r_s, True)
        assert np.array_equal(got[i:i + 1], ref), f"image {i}: {np.count_nonzero(got[i:i + 1] != ref)} mismatches"
    # the two-launch form: downsample stored by the fused stride-2 kernel, read back as conv2's residual
    Ci = C // 2
    w1q, _ = O.quantize_weights_s8(rand_conv(np.random.default_rng(1), C, Ci, 3)[0])
    xd, w1dev = _gpu_conv_inputs(x, w1q, 2, 1)
    wds = _cuda(ops.pack_downsample_weights(wdq.reshape(C, Ci), Ci))
    ones, zeros = _cuda(np.ones(C, np.float32)), _cuda(np.zeros(C, np.float32))
    _, y_ds = ops.conv2d_s2_ds_nhwc_s8(xd, w1dev, ones, zeros, wds, _cuda(alpha_d), _cuda(beta_d))
    hd, w2dev = _gpu_conv_inputs(h, w2q, 1, 1)
    y2 = ops.conv2d_nhwc_s8(hd, w2dev, C, 3, 1, 1, _cuda(alpha), _cuda(beta), residual=y_ds, res_scale=r_s, relu=True)
    two = nhwc_to_nchw(y2.cpu().numpy())
    assert np.array_equal(got, two), f"{np.count_nonzero(got != two)} mismatches against the two-launch form"


def test_conv2_with_downsample_residual_rejects_bad_shapes(gpu):
    from dlq_amd import ops
    from dlq_amd.lib import DLQError
    h = torch.zeros((2, 28, 28, 128), dtype=torch.int8, device="cuda")
    v = torch.zeros(128, dtype=torch.float32, device="cuda")
    w = torch.zeros(1, dtype=torch.int8, device="cuda")
    with pytest.raises(ValueError):  # block input of the wrong resolution
        ops.conv2d_dsres_nhwc_s8(h, w, v, v, torch.zeros((2, 28, 28, 64), dtype=torch.int8, device="cuda"), w, v, v,
                                 1.0)
    h7 = torch.zeros((2, 7, 7, 256), dtype=torch.int8, device="cuda")  # not a wide stride-1 shape
    with pytest.raises(DLQError):
        ops.conv2d_dsres_nhwc_s8(h7, w, v, v, torch.zeros((2, 14, 14, 128), dtype=torch.int8, device="cuda"), w, v,
                                 v, 1.0)
    h7 = torch.zeros((2, 7, 7, 512), dtype=torch.int8, device="cuda")  # layer4.0: the fused stride-2 form only
    with pytest.raises(DLQError):
        ops.conv2d_dsres_nhwc_s8(h7, w, v, v, torch.zeros((2, 14, 14, 256), dtype=torch.int8, device="cuda"), w, v,
                                 v, 1.0)


def test_resnet18_downsample_residual_matches_fused_downsample(gpu, knobs):
    """B=256 forward with the layer2.0 / layer3.0 downsample computed in conv2's
    epilogue (the default) == knob ds_split = -1 (the stride-2 launch stores
    it, conv2 reads it) == 1 / 2 (in conv2 at layer3.0 / layer2.0 only)."""
    from dlq_amd.models import ResNet18Int8, synthetic_images
    sd, scales = model_and_scales()
    x = synthetic_images(256, seed=23).cuda()
    model = ResNet18Int8(sd, scales, max_batch=256)
    split = model(x).cpu().numpy()
    for v in (-1, 1, 2):
        knobs("ds_split", v)
        other = model(x).cpu().numpy()
        assert np.array_equal(split.view(np.int32), other.view(np.int32)), f"ds_split = {v}"


@pytest.mark.parametrize("C,H", [(128, 28), (256, 14), (512, 7)])
@pytest.mark.parametrize("residual", [False, True])
def test_wide_conv_no_relu_bitexact(gpu, C, H, residual):
    """The wide stride-1 kernel's signed requantisation (relu = 0: clamp
    [-127, 127]) with and without a residual, ragged batch -- the forward only
    runs the ReLU forms, the C-ABI takes either."""
    from dlq_amd import ops
    rng = np.random.default_rng(C + 3 * residual)
    N = 3
    x = rand_s8(rng, (N, C, H, H))
    w, bn = rand_conv(rng, C, C, 3)
    wq, sw = O.quantize_weights_s8(w)
    s_x, s_y, s_r = 0.023, 0.06, 0.031  # ~1-3 % of the outputs at a clamp
    alpha, beta = O.fold_bn(s_x, sw, bn, s_y)
    r_s = O.res_scale(s_r, s_y)
    res = rand_s8(rng, (N, C, H, H)) if residual else None
    ref = O.epilogue_s8(O.conv_s8_acc(x, wq, 1, 1), alpha, beta, res, r_s, False)
    assert ref.min() == -127 and ref.max() == 127  # both clamps exercised
    xd, wd = _gpu_conv_inputs(x, wq, 1, 1)
    y = ops.conv2d_nhwc_s8(xd, wd, C, 3, 1, 1, _cuda(alpha), _cuda(beta),
                           residual=_cuda(nchw_to_nhwc(res)) if residual else None, res_scale=r_s, relu=False)
    got = nhwc_to_nchw(y.cpu().numpy())
    assert np.array_equal(got, ref), f"{np.count_nonzero(got != ref)} int8 mismatches"


@pytest.mark.parametrize("C,H,N", [(128, 28, 90), (256, 14, 180), (512, 7, 360)])
def test_wide_conv_many_items_per_workgroup(gpu, C, H, N):
    """Batches large enough that every workgroup of the wide stride-1 kernel
    walks several items (ring wrap-around, item hand-over): sampled images
    against the oracle, each computed alone (a conv is per image)."""
    from dlq_amd import ops
    rng = np.random.default_rng(C + N)
    x = rand_s8(rng, (N, C, H, H))
    w, bn = rand_conv(rng, C, C, 3)
    wq, sw = O.quantize_weights_s8(w)
    s_x, s_y, s_r = 0.029, 0.051, 0.044
    alpha, beta = O.fold_bn(s_x, sw, bn, s_y)
    r_s = O.res_scale(s_r, s_y)
    res = rand_s8(rng, (N, C, H, H))
    xd, wd = _gpu_conv_inputs(x, wq, 1, 1)
    y = ops.conv2d_nhwc_s8(xd, wd, C, 3, 1, 1, _cuda(alpha), _cuda(beta), residual=_cuda(nchw_to_nhwc(res)),
                           res_scale=r_s, relu=True)
    got = nhwc_to_nchw(y.cpu().numpy())
    for i in (0, 1, N // 2, N - 2, N - 1):
        ref = O.epilogue_s8(O.conv_s8_acc(x[i:i + 1], wq, 1, 1), alpha, beta, res[i:i + 1], r_s, True)
        assert np.array_equal(got[i:i + 1], ref), f"image {i}: {np.count_nonzero(got[i:i + 1] != ref)} mismatches"


def test_fc_logits_bitexact(gpu):
    from dlq_amd import ops
    from dlq_amd.lib import DLQ_OUT_F32, DLQ_OUT_S32
    from tests.helpers import golden
    rng = np.random.default_rng(11)
    W = golden("fc.weight.bin", (1000, 512))  # the reference's real FC weights (tmp_e2e/)
    bias = golden("fc.bias.bin")
    wq, sw = O.quantize_weights_s8(W)
    for N in (1, 7, 256):
        x = rand_s8(rng, (N, 512), lo=0)
        alpha = O.fc_alpha(0.02, sw)
        ref, racc = O.fc_s8(x, wq, alpha, bias)
        packed = _cuda(ops.pack_linear_weights(wq))
        ocp = ops.packed_oc(1000)
        acc = ops.linear_s8(_cuda(x), packed, 1000, out_kind=DLQ_OUT_S32)
        assert np.array_equal(acc.cpu().numpy(), racc)
        out = ops.linear_s8(_cuda(x), packed, 1000, _cuda(ops.pad_vec(alpha, ocp)), _cuda(ops.pad_vec(bias, ocp)),
                            out_kind=DLQ_OUT_F32)
        assert np.array_equal(out.cpu().numpy().view(np.int32), ref.view(np.int32))


def test_quantize_input_bitexact(gpu):
    from dlq_amd import ops
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((3, 3, 224, 224), dtype=np.float32) * 1.3).astype(np.float32)
    x[0, 0, 0, :8] = [0.5, 1.5, 2.5, -0.5, -1.5, 1e9, -1e9, 0.0]  # ties and saturation
    s = 2.64 / 127
    ref = O.quantize_f32_s8(x, s)
    y = ops.quantize_nchw_to_nhwc(_cuda(x), s, 4).cpu().numpy()
    assert np.all(y[..., 3] == 0)
    assert np.array_equal(nhwc_to_nchw(y[..., :3]), ref)


def test_maxpool_and_gap_bitexact(gpu):
    from dlq_amd import ops
    rng = np.random.default_rng(5)
    x = rand_s8(rng, (3, 64, 112, 112), lo=-128)
    ref = O.maxpool_s8(x)
    got = nhwc_to_nchw(ops.maxpool2d_3x3_s2p1_nhwc_s8(_cuda(nchw_to_nhwc(x))).cpu().numpy())
    assert np.array_equal(got, ref)
    x4 = rand_s8(rng, (5, 512, 7, 7))
    k = O.gap_k(0.05, 49, 0.011)
    gref, _ = O.gap_s8(x4, k)
    ggot = ops.gap_nhwc_s8(_cuda(nchw_to_nhwc(x4)), float(k)).cpu().numpy()
    assert np.array_equal(ggot, gref)


@pytest.mark.parametrize("N,HW,OC,lo", [(1, 49, 1000, 0), (5, 49, 1000, 0), (256, 49, 1000, 0), (7, 1, 1000, 0),
                                        (6, 56, 64, 0), (3, 17, 10, 0), (5, 49, 1000, -128), (4, 1, 1000, -128)])
def test_gap_fc_fused_head_bitexact(gpu, N, HW, OC, lo):
    """gap_fc_kernel (one launch) == oracle GAP then FC, bit for bit, on ragged
    image groups (N % 4 != 0), HW from 1 to its 56 maximum and OC tails; lo =
    -128: signed bytes (every code, -128 included) and GAP codes saturating at
    -127 (HW = 1, where the mean is the byte itself)."""
    from dlq_amd import ops
    from tests.helpers import golden
    rng = np.random.default_rng(N * 131 + HW)
    W = golden("fc.weight.bin", (1000, 512))[:OC]  # the reference's real FC weights (tmp_e2e/)
    bias = golden("fc.bias.bin")[:OC]
    wq, sw = O.quantize_weights_s8(W)
    x = rand_s8(rng, (N, 512, 1, HW), lo=lo)  # int8 layer4 output (post-ReLU for lo = 0), NCHW
    k = O.gap_k(0.05, HW, 0.011 if lo == 0 else 0.04)
    g, _ = O.gap_s8(x, k)
    alpha = O.fc_alpha(0.011, sw)
    ref, _ = O.fc_s8(g, wq, alpha, bias)
    ocp = ops.packed_oc(OC)
    packed = _cuda(ops.pack_linear_weights(wq))
    a, b = _cuda(ops.pad_vec(alpha, ocp)), _cuda(ops.pad_vec(bias, ocp))
    xh = _cuda(nchw_to_nhwc(x))
    got = ops.gap_fc_s8(xh, float(k), packed, OC, a, b).cpu().numpy()
    assert np.array_equal(got.view(np.int32), ref.view(np.int32))
    split = ops.linear_s8(ops.gap_nhwc_s8(xh, float(k)), packed, OC, a, b).cpu().numpy()
    assert np.array_equal(got.view(np.int32), split.view(np.int32))


def test_gap_fc_rejects_unsupported_shapes(gpu):
    from dlq_amd import ops
    from dlq_amd.lib import DLQError
    x = torch.zeros((2, 8, 8, 512), dtype=torch.int8, device="cuda")  # HW 64 > 56
    w = torch.zeros(1024 * 512, dtype=torch.int8, device="cuda")
    v = torch.zeros(1024, dtype=torch.float32, device="cuda")
    with pytest.raises(DLQError):
        ops.gap_fc_s8(x, 0.1, w, 1000, v, v)
    with pytest.raises(DLQError):
        ops.gap_fc_s8(torch.zeros((2, 7, 7, 256), dtype=torch.int8, device="cuda"), 0.1, w, 1000, v, v)


def test_resnet18_fused_head_matches_split_head(gpu, knobs):
    """B=256 forward with the fused head (default) == knob head_split = 1."""
    from dlq_amd.models import ResNet18Int8, synthetic_images
    sd, scales = model_and_scales()
    x = synthetic_images(256, seed=21).cuda()
    model = ResNet18Int8(sd, scales, max_batch=256)
    fused = model(x).cpu().numpy()
    knobs("head_split", 1)
    split = model(x).cpu().numpy()
    assert np.array_equal(fused.view(np.int32), split.view(np.int32))


@pytest.mark.parametrize("B", [1, 3, 9, 256])
def test_resnet18_pooled_last_conv_matches_fused_head(gpu, knobs, B):
    """The last conv pooling its own output (default: conv3x3i GAP, then the
    FC alone) == knob gap_epi = -1 (the fused gap_fc_kernel head), bit for
    bit, at a ragged batch (items with absent images) and the bench batch."""
    from dlq_amd.models import ResNet18Int8, synthetic_images
    sd, scales = model_and_scales()
    x = synthetic_images(B, seed=31).cuda()
    model = ResNet18Int8(sd, scales, max_batch=256)
    pooled = model(x).cpu().numpy()
    knobs("gap_epi", -1)
    fused = model(x).cpu().numpy()
    assert np.array_equal(pooled.view(np.int32), fused.view(np.int32))


def test_im2col_reference_order_bitexact(gpu):
    from dlq_amd import ops
    rng = np.random.default_rng(9)
    for (C, H, k, s, p) in [(3, 224, 7, 2, 3), (64, 56, 3, 1, 1), (128, 28, 1, 2, 0)]:
        x = rand_s8(rng, (2, C, H, H))
        col = ops.im2col_nchw_s8(_cuda(x), k, s, p).cpu().numpy()
        for n in range(2):
            OH = O.out_dim(H, k, s, p)
            ref = np.empty(C * k * k * OH * OH, np.int8)
            O.lib().ora_im2col_nchw_s8(x[n].copy(), C, H, H, k, k, s, s, p, p, ref)
            assert np.array_equal(col[n].reshape(-1), ref)


def _stage_nchw(model, name, B):
    shapes = {"stem_pool": (56, 56, 64), "layer1": (56, 56, 64), "layer2": (28, 28, 128),
              "layer3": (14, 14, 256), "layer4": (7, 7, 512), "conv1": (112, 112, 64)}
    if name == "gap":
        return model.stage("gap", (B, 512)).cpu().numpy()
    h, w, c = shapes[name]
    return nhwc_to_nchw(model.stage(name, (B, h, w, c)).cpu().numpy())


def test_resnet18_end_to_end_bitexact(gpu):
    """Whole network, B=2: every stage's int8 activations and the fp32 logits."""
    from dlq_amd.models import ResNet18Int8, synthetic_images
    sd, scales = model_and_scales()
    x = synthetic_images(2, seed=77).numpy()
    ref_logits, dumps = O.resnet18_forward_s8(sd, scales, x)
    model = ResNet18Int8(sd, scales, max_batch=4, keep_stages=True)
    logits = model(_cuda(x)).cpu().numpy()
    torch.cuda.synchronize()
    for st in ("stem_pool", "layer1", "layer2", "layer3", "layer4", "gap"):
        got = _stage_nchw(model, st, 2)
        assert np.array_equal(got, dumps[st]), f"stage {st}: {np.count_nonzero(got != dumps[st])} mismatches"
    assert np.array_equal(logits.view(np.int32), ref_logits.view(np.int32))


def test_resnet18_batch_invariance_full_batch(gpu):
    """Batch 256 (the benchmark config): each image's logits are bit-identical
    to the same image run alone, and to the oracle on a sample."""
    from dlq_amd.models import ResNet18Int8, synthetic_images
    sd, scales = model_and_scales()
    x = synthetic_images(256, seed=99).cuda()
    model = ResNet18Int8(sd, scales, max_batch=256)
    big = model(x).cpu().numpy()
    again = model(x).cpu().numpy()
    assert np.array_equal(big.view(np.int32), again.view(np.int32))  # deterministic
    for i in (0, 1, 128, 255):
        one = model(x[i:i + 1].contiguous()).cpu().numpy()
        assert np.array_equal(one[0].view(np.int32), big[i].view(np.int32))
    ref, _ = O.resnet18_forward_s8(sd, scales, x[[0, 255]].cpu().numpy())
    assert np.array_equal(ref.view(np.int32), big[[0, 255]].view(np.int32))


def test_resnet18_graph_replay_matches_launches(gpu, knobs):
    """The forward is captured once per (x, B, logits) into a hipGraph and
    replayed (knob graph = 1, DLQ_GRAPH=1): a replay over NEW contents of the same input
    buffer, and a re-capture for another batch size, equal the kernel-by-
    kernel forward (the default) bit for bit."""
    from dlq_amd.models import ResNet18Int8, synthetic_images
    knobs("graph", 1)
    sd, scales = model_and_scales()
    model = ResNet18Int8(sd, scales, max_batch=64)
    x = synthetic_images(64, seed=3).cuda()
    out = torch.empty((64, 1000), dtype=torch.float32, device="cuda")
    got = []
    for seed in (3, 4):  # capture, then replay over new pixels in the same buffer
        x.copy_(synthetic_images(64, seed=seed).cuda())
        got.append(model(x, out=out).cpu().numpy())
    small = model(x[:5], out=out[:5]).cpu().numpy()  # another (x, B, logits): re-capture
    knobs("graph", 0)
    ref = model(x).cpu().numpy()
    x.copy_(synthetic_images(64, seed=3).cuda())
    ref0 = model(x).cpu().numpy()
    assert not np.array_equal(got[0], got[1])
    assert np.array_equal(got[0].view(np.int32), ref0.view(np.int32))
    assert np.array_equal(got[1].view(np.int32), ref.view(np.int32))
    assert np.array_equal(small.view(np.int32), ref[:5].view(np.int32))


def test_resnet18_half_batch_split_matches_single_stream(gpu, monkeypatch):
    """With DLQ_SPLIT=1, batches >= 64 run as two half-batches on two streams
    (separate halves of every workspace buffer); an odd batch must give the
    same logits as the single-stream pass (per-launch timing forces it).
    The switch is read once per process: this runs in a child process."""
    import subprocess
    import sys
    code = ("import numpy as np; from tests.test_gpu_parity import _split_case; _split_case()")
    env = dict(__import__("os").environ, DLQ_SPLIT="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr


def _split_case():
    from dlq_amd.models import ResNet18Int8, synthetic_images
    sd, scales = model_and_scales()
    x = synthetic_images(97, seed=7).cuda()
    model = ResNet18Int8(sd, scales, max_batch=128)
    split = model(x).cpu().numpy()
    model.set_timing(True)
    single = model(x).cpu().numpy()
    model.set_timing(False)
    assert np.array_equal(split.view(np.int32), single.view(np.int32))


def test_resnet18_empty_and_oversize_batch(gpu):
    from dlq_amd.lib import DLQError
    from dlq_amd.models import ResNet18Int8
    sd, scales = model_and_scales()
    model = ResNet18Int8(sd, scales, max_batch=2)
    out = model(torch.empty((0, 3, 224, 224), device="cuda"))
    assert out.shape == (0, 1000)
    with pytest.raises(DLQError):
        model(torch.zeros((3, 3, 224, 224), device="cuda"))


@pytest.mark.parametrize("hidden", [256, 128])
def test_mnist_mlp_bitexact(gpu, hidden):
    """MNIST FC path (v4.cu:255-302 / v5.cu:127-157) at batch 1024, int8."""
    from dlq_amd.models import MLPInt8, mlp_weights
    from dlq_amd.quant import calibrate_mlp
    W1, b1, W2, b2 = mlp_weights(784, hidden, 10)
    rng = np.random.default_rng(21)
    x = ((rng.random((1024, 784), dtype=np.float32) - np.float32(0.1307)) / np.float32(0.3081)).astype(np.float32)
    s_in, s_h = calibrate_mlp(W1, b1, x)
    # oracle: quantise, int32 GEMM in the reference [in][out] layout, epilogues
    xq = O.quantize_f32_s8(x, s_in)
    q1, sw1 = O.quantize_weights_s8(W1.T.copy())
    q2, sw2 = O.quantize_weights_s8(W2.T.copy())
    acc1 = np.empty((1024, hidden), np.int32)
    O.lib().ora_mlp_layer_s8_acc(xq, q1.T.copy(), 1024, 784, hidden, acc1)
    a1, bb1 = O.mlp_alpha_beta(s_in, sw1, b1, s_h)
    h = O.epilogue_s8(acc1[:, :, None], a1, bb1, relu=True)[:, :, 0]
    acc2 = np.empty((1024, 10), np.int32)
    O.lib().ora_mlp_layer_s8_acc(h, q2.T.copy(), 1024, hidden, 10, acc2)
    ref = np.empty((1024, 10), np.float32)
    O.lib().ora_epilogue_f32(acc2.reshape(-1), 1024, 10, 1, O.fc_alpha(s_h, sw2), b2, 0, ref)
    m = MLPInt8(W1, b1, W2, b2, s_in, s_h, max_batch=1024)
    out = m(_cuda(x)).cpu().numpy()
    assert np.array_equal(m.hidden_q(1024).cpu().numpy(), h)
    assert np.array_equal(out.view(np.int32), ref.view(np.int32))
    for B in (1, 3, 77):
        o2 = m(_cuda(x[:B])).cpu().numpy()
        assert np.array_equal(o2.view(np.int32), ref[:B].view(np.int32))


@pytest.mark.parametrize("inp,hidden,out,B", [(100, 64, 10, 50), (784, 192, 10, 1000), (257, 512, 37, 33),
                                              (784, 1024, 10, 64), (130, 128, 3, 17),
                                              (784, 8192, 10, 40), (16384, 256, 10, 9)])
def test_mlp_fused_shapes_bitexact(gpu, inp, hidden, out, B):
    """The one-launch MLP (head.hip mlp_fused_kernel) off the MNIST shape: `in`
    not a multiple of 4 or 64 (scalar loads, zero K tail), K split over waves
    (hidden < 256) or several tiles per wave (hidden > 256), more than one fc2
    tile, ragged row blocks -- int32 sums and epilogues bit-exact vs the oracle.
    The last two shapes need more than the fused kernel's 64 KiB of LDS
    (hidden 8192; in 16384): dlq_mlp_forward runs them as quantize_rows + two
    linear launches, with the same bits."""
    from dlq_amd.models import MLPInt8, mlp_weights
    from dlq_amd.quant import calibrate_mlp
    W1, b1, W2, b2 = mlp_weights(inp, hidden, out, seed=inp + hidden)
    b1 = (np.random.default_rng(3).standard_normal(hidden) * 0.1).astype(np.float32)
    b2 = (np.random.default_rng(4).standard_normal(out) * 0.1).astype(np.float32)
    rng = np.random.default_rng(inp * 7 + B)
    x = (rng.standard_normal((B, inp)) * 1.5).astype(np.float32)
    s_in, s_h = calibrate_mlp(W1, b1, x)
    xq = O.quantize_f32_s8(x, s_in)
    q1, sw1 = O.quantize_weights_s8(W1.T.copy())
    q2, sw2 = O.quantize_weights_s8(W2.T.copy())
    acc1 = np.empty((B, hidden), np.int32)
    O.lib().ora_mlp_layer_s8_acc(xq, q1.T.copy(), B, inp, hidden, acc1)
    a1, bb1 = O.mlp_alpha_beta(s_in, sw1, b1, s_h)
    h = O.epilogue_s8(acc1[:, :, None], a1, bb1, relu=True)[:, :, 0]
    acc2 = np.empty((B, out), np.int32)
    O.lib().ora_mlp_layer_s8_acc(h, q2.T.copy(), B, hidden, out, acc2)
    ref = np.empty((B, out), np.float32)
    O.lib().ora_epilogue_f32(acc2.reshape(-1), B, out, 1, O.fc_alpha(s_h, sw2), b2, 0, ref)
    m = MLPInt8(W1, b1, W2, b2, s_in, s_h, max_batch=B)
    got = m(_cuda(x)).cpu().numpy()
    assert np.array_equal(m.hidden_q(B).cpu().numpy(), h)
    assert np.array_equal(got.view(np.int32), ref.view(np.int32))
