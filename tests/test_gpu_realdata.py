"""The HIP path on the reference's own real data (tests/golden/, copied from
CUDA/resnet18-kernel-lab/tmp_e2e/ and tmp_e2e_full/ of the reference):

* l4.bin -- the real layer4 activations [512,7,7] of one ImageNet image --
  quantised at its amax scale, through the fused int8 head (dlq_gap_fc_s8)
  with the real FC weights: bit-exact with the oracle's int8 head, and scored
  against the reference's own fp32 logits out/step8_logits.bin with the
  metrics of tools/diag_e2e_compare.py:15-24 (top-1 must be 293, the
  reference's class; cosine floor 0.9999, measured 0.99992).
* input.bin -- the real preprocessed image [1,3,224,224] -- through the fused
  stem kernel (seeded conv1 weights: the reference ships no conv weights) and
  through the whole network, int8 engine and the GPU fp32 reference forward,
  each bit-exact against the oracle.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import golden, model_and_scales, nchw_to_nhwc, nhwc_to_nchw, rand_conv

pytestmark = pytest.mark.gpu


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _diag(a, b):
    """max_abs, mean_abs, cosine (diag_e2e_compare.py:15-24)."""
    a = a.astype(np.float64).ravel(); b = b.astype(np.float64).ravel()
    d = np.abs(a - b)
    return float(d.max()), float(d.mean()), float(np.dot(a, b) / (np.linalg.norm(a) * np.linalg.norm(b)))


def test_int8_head_on_reference_layer4(gpu):
    from dlq_amd import ops
    l4 = golden("l4.bin", (512, 7, 7))
    gap_ref = golden("gap.bin")
    W = golden("fc.weight.bin", (1000, 512))
    bias = golden("fc.bias.bin")
    ref_logits = golden("step8_logits.bin")
    s_l4 = np.float32(np.abs(l4).max() / 127)
    s_gap = np.float32(np.abs(gap_ref).max() / 127)
    q = O.quantize_f32_s8(l4[None], s_l4)  # [1,512,7,7] int8
    k = O.gap_k(s_l4, 49, s_gap)
    wq, sw = O.quantize_weights_s8(W)
    alpha = O.fc_alpha(s_gap, sw)
    g, _ = O.gap_s8(q, k)
    want, _ = O.fc_s8(g, wq, alpha, bias)
    ocp = ops.packed_oc(1000)
    got = ops.gap_fc_s8(_cuda(nchw_to_nhwc(q)), float(k), _cuda(ops.pack_linear_weights(wq)), 1000,
                        _cuda(ops.pad_vec(alpha, ocp)), _cuda(ops.pad_vec(bias, ocp))).cpu().numpy()
    assert np.array_equal(got.view(np.int32), want.view(np.int32))
    mx, mn, cs = _diag(got[0], ref_logits)
    assert int(np.argmax(got[0])) == int(np.argmax(ref_logits)) == 293
    assert cs >= 0.9999, (mx, mn, cs)


def test_stem_on_reference_input(gpu):
    from dlq_amd import ops
    x = golden("input.bin", (1, 3, 224, 224))
    rng = np.random.default_rng(77)
    w, bn = rand_conv(rng, 64, 3, 7)
    wq, sw = O.quantize_weights_s8(w)
    s_in = np.float32(np.abs(x).max() / 127)
    alpha, beta = O.fold_bn(s_in, sw, bn, 0.05)
    ref = O.maxpool_s8(O.epilogue_s8(O.conv_s8_acc(O.quantize_f32_s8(x, s_in), wq, 2, 3), alpha, beta, None, 0.0, True))
    wst, al_p = ops.pack_stem_weights(wq, alpha)
    got = nhwc_to_nchw(ops.stem_fused_s8(_cuda(x), _cuda(wst), _cuda(al_p), _cuda(beta), float(s_in)).cpu().numpy())
    assert np.array_equal(got, ref), f"{np.count_nonzero(got != ref)} int8 mismatches"
    assert np.count_nonzero(ref) > ref.size // 4  # a real, non-degenerate activation map


def test_network_on_reference_input(gpu):
    """The real image through the int8 engine (scales calibrated on it by the
    GPU fp32 reference forward) and through that fp32 forward itself: both
    bit-exact against the oracle."""
    from dlq_amd.models import ResNet18Int8
    x = golden("input.bin", (1, 3, 224, 224))
    sd, scales = model_and_scales()
    m = ResNet18Int8(sd, scales, max_batch=2)
    xd = _cuda(np.concatenate([x, x[:, :, ::-1].copy()]))  # the image and its vertical flip
    f32 = m.forward_f32(xd).cpu().numpy()
    for i in range(2):
        want, _ = O.resnet18_forward_f32(sd, xd[i].cpu().numpy())
        assert np.array_equal(f32[i].view(np.int32), want.view(np.int32)), i
    m.calibrate(xd)
    import tempfile, os
    from dlq_amd.quant import load_scales
    with tempfile.TemporaryDirectory() as d:
        m.scales(os.path.join(d, "s.txt"))
        cal = load_scales(os.path.join(d, "s.txt"))
    got = m(xd).cpu().numpy()
    want, _ = O.resnet18_forward_s8(sd, cal, xd.cpu().numpy())
    assert np.array_equal(got.view(np.int32), want.view(np.int32))
    # int8 tracks the fp32 reference on the real image
    for i in range(2):
        assert _diag(got[i], f32[i])[2] > 0.99
