"""GPU parity of the fp8 (e4m3) path through the C ABI vs the CPU oracle
(oracle.c ora_*_f8).

Bar, stated per kernel:
  * quantisation (fp32 -> e4m3), GAP, FC: bit-exact (the same IEEE ops; GAP
    sums exact integer units; FC accumulates exact products in fp64).
  * convs: the oracle's accumulator is the exact sum; the MFMA's is not
    IEEE fp32.  Its error is a random walk: tools/f8_err_stats.py measured
    |acc - exact| / sqrt(sum (w x)^2) with mean 0.9-1.2e-5 on every test
    shape (K = 64 .. 4608) and max 0.6-1.4e-4 (profiles/r05_f8_err_stats.json;
    tools/f8_acc_probe.py first bounded it by 2^-18 sum|w x| on large K, which
    small K exceeds up to 8.4x).  Per output, in output units (x |alpha|):
        e = max(2^-18 sum|w x|, ACC_MAXR sqrt(sum (w x)^2)),
        |dec(gpu) - dec(oracle)| <= step(e4m3 at that magnitude) + 8 e.
    How many outputs may change code follows from the same error model, not
    from a measured fraction: an output flips only if its exact value y lies
    within its error of a rounding boundary, which for a position uniform
    within its e4m3 step has probability p = min(1, 2 e / step(y)) for an
    error bounded by e, and p = E|err| / step(y) for an unbiased error of mean
    magnitude E|err| (it must also point at that boundary); 0 where the clamp
    decides (y < -e under ReLU, |y| > 448 + e).  With the TYPICAL error E|err|
    = ACC_TYP sqrt(sum (w x)^2) (ACC_TYP = 1.2e-5, the measured mean) the
    count must stay within 2 mu_t + 4 sqrt(mu_t) + 8, mu_t = sum p
    -- so lost accumulator precision or a wrong k order, which would double
    the count, fails -- and within the worst-case model's mu + 4 sqrt(mu) + 2
    (err = e).  A wrong tap, channel or scale moves far more outputs by far
    more than one step.
  * the whole network: a one-step flip of an input code moves each output
    it feeds by ~1/sqrt(taps) of its own value, a sizeable fraction of the
    coarse e4m3 step (12.5 %), so flips cascade through the 20 convs and
    code-level equality is not a meaningful bar past the first layer.  The
    first stage (stem_pool) keeps a code-level bound (<= 1 % differ); later
    stages are compared decoded (cosine >= 0.99 against the oracle's fp8
    forward) and the logits must track the fp32 reference as closely as the
    oracle's own fp8 logits do (cosine >= 0.995, test_oracle_f8.py).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import f8_sweep, model_and_scales_f8, nchw_to_nhwc, nhwc_to_nchw, rand_conv

pytestmark = pytest.mark.gpu

CONV_SHAPES = [
    ("stem", 3, 64, 7, 2, 3, 224),
    ("l1_3x3", 64, 64, 3, 1, 1, 56),
    ("l2_0_conv1", 64, 128, 3, 2, 1, 56),
    ("l2_3x3", 128, 128, 3, 1, 1, 28),
    ("l2_ds", 64, 128, 1, 2, 0, 56),
    ("l3_3x3", 256, 256, 3, 1, 1, 14),
    ("l4_0_conv1", 256, 512, 3, 2, 1, 14),
    ("l4_3x3", 512, 512, 3, 1, 1, 7),
    ("l4_ds", 256, 512, 1, 2, 0, 14),
]


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _step(v):
    """e4m3 spacing at magnitude v (2^-9 in the subnormal range)."""
    v = np.maximum(np.abs(v), 2.0 ** -6)
    return 2.0 ** (np.floor(np.log2(v)) - 3)


ACC_EPS = 2.0 ** -18  # measured |MFMA accumulator - exact| / sum|w x| (tools/f8_acc_probe.py)
# The accumulator error is a random walk: |acc - exact| / sqrt(sum (w x)^2)
# has mean 0.91-1.17e-5 on every test shape (K = 64 .. 4608) and max
# 0.6-1.4e-4 (tools/f8_err_stats.py, profiles/r05_f8_err_stats.json), while
# relative to sum|w x| it grows as K shrinks (up to 8.4 x 2^-18 at K = 64).
ACC_TYP = 1.2e-5  # the typical (mean) error, for the flip COUNT
ACC_MAXR = 2.0e-4  # above every measured per-output error, for the per-output bound


def _flip_mu(y, e, relu, sides=2):
    """Expected number of outputs whose e4m3 code can flip: sum over outputs
    of min(1, sides e / step(y)), 0 where the clamp decides regardless.  With
    e a BOUND on |err| (sides = 2) an output can flip if its exact value lies
    within e of the nearest boundary, either side; with e the MEAN |err| of
    an unbiased error (sides = 1) it flips if the error also points at that
    boundary: p = E|err| / step for a position uniform within the step."""
    y = np.asarray(y, np.float64)
    p = np.minimum(1.0, sides * e / _step(y))
    clamped = np.abs(y) > 448.0 + e
    if relu:
        clamped |= y < -e
    return float(np.sum(np.where(clamped, 0.0, p)))


def _conv_sq(x, wq, s, p):
    """sum over taps of (w x)^2 per output (float64, decoded e4m3 codes)."""
    xd = O.decode_f8(x).astype(np.float64) ** 2
    wd = O.decode_f8(wq).astype(np.float64) ** 2
    k = wd.shape[2]
    OH = (xd.shape[2] + 2 * p - k) // s + 1
    xp = np.pad(xd, ((0, 0), (0, 0), (p, p), (p, p)))
    out = np.zeros((xd.shape[0], wd.shape[0], OH, OH))
    for kh in range(k):
        for kw in range(k):
            out += np.einsum("nchw,oc->nohw", xp[:, :, kh:kh + s * OH:s, kw:kw + s * OH:s], wd[:, :, kh, kw],
                             optimize=True)
    return out


def _errs(alpha, s_abs, s_sq):
    """(per-output error bound e, typical error e_typ) in output units."""
    a = np.abs(alpha).astype(np.float64)[None, :, None, None]
    rms = np.sqrt(s_sq)
    return a * np.maximum(ACC_EPS * s_abs, ACC_MAXR * rms), a * ACC_TYP * rms


def _check_conv(got, ref, y, e, relu, what, e_typ):
    """got / ref: e4m3 codes; y: the exact pre-rounding outputs (float64); e:
    the per-output accumulator error bound, e_typ the typical error, both in
    output units (_errs).  Every output within one step + 8 e; the number of
    differing codes within the worst-case model (mu from e) AND within 2 mu_t
    + 4 sqrt(mu_t) + 8 of the typical-error model (mu_t from e_typ), which a
    doubling of the flip count (lost accumulator precision, a wrong k order)
    exceeds."""
    a, b = O.decode_f8(got).astype(np.float64), O.decode_f8(ref).astype(np.float64)
    lim = _step(np.maximum(np.abs(a), np.abs(b))) + 8 * e
    bad = np.abs(a - b) > lim
    n = np.count_nonzero(got != ref)
    assert not bad.any(), (f"{what}: {np.count_nonzero(bad)} outputs beyond one step + 2E, e.g. "
                           f"gpu={a[bad][:4]} ora={b[bad][:4]} E={4 * e[bad][:4]}")
    mu, mu_t = _flip_mu(y, e, relu), _flip_mu(y, e_typ, relu, sides=1)
    bar = 2 * mu_t + 4 * np.sqrt(mu_t) + 8
    print(f"[f8 bar] {what}: {n} of {got.size} codes differ, typical-error mu {mu_t:.1f} (bar {bar:.0f}, "
          f"{bar / max(n, 1):.1f}x the count), worst-case mu {mu:.1f}")
    assert n <= mu + 4 * np.sqrt(mu) + 2, f"{what}: {n} of {got.size} outputs differ (model mu = {mu:.1f})"
    assert n <= bar, f"{what}: {n} of {got.size} outputs differ (typical-error model mu = {mu_t:.1f}, bar {bar:.0f})"
    return n


def _close_codes(got, ref, frac, what):
    n = np.count_nonzero(got != ref)
    assert n <= frac * got.size, f"{what}: {n} of {got.size} codes differ (> {frac:%})"
    return n


def test_quantize_f32_f8_bitexact(gpu):
    from dlq_amd import ops
    rng = np.random.default_rng(11)
    x = f8_sweep(rng)
    x = np.concatenate([x, np.zeros((-len(x)) % 4 + 3, np.float32)])  # ragged tail (n % 4 == 3)
    for s in (1.0, 0.37):
        got = ops.quantize_f32_f8(_cuda(x), s).cpu().numpy()
        ref = O.quantize_f32_f8(x, s)
        bad = np.nonzero(got != ref)[0]
        assert bad.size == 0, f"{bad.size} mismatches, e.g. x={x[bad[:4]]} gpu={got[bad[:4]]} ora={ref[bad[:4]]}"


def test_quantize_input_nhwc4_bitexact(gpu):
    from dlq_amd import ops
    from dlq_amd.models import synthetic_images
    x = synthetic_images(2, seed=5).numpy()
    got = ops.quantize_nchw_to_nhwc_f8(_cuda(x), 0.0123).cpu().numpy()
    ref = nchw_to_nhwc(O.quantize_f32_f8(x, 0.0123))
    assert np.array_equal(got[..., :3], ref) and not got[..., 3].any()


def _conv_case(shape, residual, N):
    name, IC, OC, k, s, p, H = shape
    if residual and (IC == 3 or k == 1 or s == 2):
        pytest.skip("stem / downsample / stride-2 conv1 take no residual (the API rejects one)")
    _run_conv(shape, residual, N)


@pytest.mark.parametrize("shape", CONV_SHAPES, ids=[s[0] for s in CONV_SHAPES])
@pytest.mark.parametrize("residual", [False, True])
def test_conv_f8_within_one_step(gpu, shape, residual):
    _conv_case(shape, residual, 2)


@pytest.mark.parametrize("shape", [s for s in CONV_SHAPES if s[0] in ("l2_3x3", "l3_3x3", "l4_3x3")],
                         ids=["l2_3x3", "l3_3x3", "l4_3x3"])
@pytest.mark.parametrize("N", [1, 37])
def test_wide_conv_f8_batch_tails(gpu, shape, N):
    """The 392-px item kernel with e4m3 operands: partial items and one image."""
    _conv_case(shape, True, N)


def _run_conv(shape, residual, N):
    from dlq_amd import ops
    name, IC, OC, k, s, p, H = shape
    rng = np.random.default_rng(17 + sum(map(ord, name)) + N)
    x = O.quantize_f32_f8(np.abs(rng.standard_normal((N, IC, H, H))).astype(np.float32) * 40, 1.0)
    w, bn = rand_conv(rng, OC, IC, k)
    wq, sw = O.quantize_weights_f8(w)
    s_x, s_y, s_r = 0.011, 0.013, 0.017
    alpha, beta = O.fold_bn(s_x, sw, bn, s_y)
    r_s = O.res_scale(s_r, s_y)
    acc = O.conv_f8_acc(x, wq, s, p)
    res = O.quantize_f32_f8(rng.standard_normal(acc.shape).astype(np.float32) * 50, 1.0) if residual else None
    relu = k != 1
    ref = O.epilogue_f8(acc, alpha, beta, res, r_s, relu)
    c_store = 4 if IC == 3 else IC
    xh = nchw_to_nhwc(x)
    if c_store != IC:
        xh = np.concatenate([xh, np.zeros(xh.shape[:3] + (c_store - IC,), np.uint8)], axis=3)
    packed = ops.pack_conv_weights_f8(wq, c_store, H, s, p)
    ocp = ops.packed_oc(OC)
    y = ops.conv2d_nhwc_f8(_cuda(xh), _cuda(packed), OC, k, s, p, _cuda(ops.pad_vec(alpha, ocp)),
                           _cuda(ops.pad_vec(beta, ocp)), residual=_cuda(nchw_to_nhwc(res)) if residual else None,
                           res_scale=r_s, relu=relu)
    got = nhwc_to_nchw(y.cpu().numpy())
    assert got.shape == ref.shape
    assert len(np.unique(ref)) > 50  # a real spread of codes, not a saturated tensor
    s_abs = O.conv_f8_acc(x & 0x7F, wq & 0x7F, s, p)  # exact sum |w x|
    e, e_typ = _errs(alpha, s_abs, _conv_sq(x, wq, s, p))
    y = (alpha.astype(np.float64)[None, :, None, None] * acc + beta.astype(np.float64)[None, :, None, None]
         + (np.float64(r_s) * O.decode_f8(res).astype(np.float64) if residual else 0.0))
    _check_conv(got, ref, y, e, relu, name, e_typ)


def _maxpool_f64(a):
    """3x3/s2/p1 max over NCHW float64 (-inf padding)."""
    N, Cc, H, W = a.shape
    ap = np.pad(a, ((0, 0), (0, 0), (1, 1), (1, 1)), constant_values=-np.inf)
    OH = (H + 2 - 3) // 2 + 1
    out = np.full((N, Cc, OH, OH), -np.inf)
    for kh in range(3):
        for kw in range(3):
            out = np.maximum(out, ap[:, :, kh:kh + 2 * OH:2, kw:kw + 2 * OH:2])
    return out


def _pool_at_argmax(y, v):
    """3x3/s2/p1 max pool of y; returns v at each window's argmax (NCHW)."""
    N, Cc, H, W = y.shape
    yp = np.pad(y, ((0, 0), (0, 0), (1, 1), (1, 1)), constant_values=-np.inf)
    vp = np.pad(v, ((0, 0), (0, 0), (1, 1), (1, 1)))
    OH = (H + 2 - 3) // 2 + 1
    best = np.full((N, Cc, OH, OH), -np.inf)
    out = np.zeros((N, Cc, OH, OH))
    for kh in range(3):
        for kw in range(3):
            yy = yp[:, :, kh:kh + 2 * OH:2, kw:kw + 2 * OH:2]
            take = yy > best
            best = np.where(take, yy, best)
            out = np.where(take, vp[:, :, kh:kh + 2 * OH:2, kw:kw + 2 * OH:2], out)
    return out


@pytest.mark.parametrize("N", [1, 3])
def test_stem_fused_f8_within_bound(gpu, N):
    """quantise + conv1 + BN/ReLU + maxpool in one launch vs the oracle's
    separate steps; the pooled bound is the window max of the conv bound."""
    from dlq_amd import ops
    from dlq_amd.models import synthetic_images
    rng = np.random.default_rng(41 + N)
    x = synthetic_images(N, seed=100 + N).numpy()
    w, bn = rand_conv(rng, 64, 3, 7)
    wq, sw = O.quantize_weights_f8(w)
    s_in, s_y = 0.0061, 0.0123
    alpha, beta = O.fold_bn(s_in, sw, bn, s_y)
    alpha[5] = -abs(alpha[5])  # a negative-alpha channel: the sign-flip packing path
    xq = O.quantize_f32_f8(x, s_in)
    acc = O.conv_f8_acc(xq, wq, 2, 3)
    ref = O.maxpool_s8(O.epilogue_f8(acc, alpha, beta, relu=True).view(np.int8)).view(np.uint8)
    s_abs = O.conv_f8_acc(xq & 0x7F, wq & 0x7F, 2, 3)
    # pooled: a window's max can flip through any of its 9 outputs -> 9x the
    # window-max bound; the typical flip is the max's own (its error, taken
    # at the window's argmax)
    e_all, e_typ_all = _errs(alpha, s_abs, _conv_sq(xq, wq, 2, 3))
    y_all = alpha.astype(np.float64)[None, :, None, None] * acc + beta.astype(np.float64)[None, :, None, None]
    e, e_typ = _maxpool_f64(e_all), _pool_at_argmax(y_all, e_typ_all)
    y_ex = _maxpool_f64(alpha.astype(np.float64)[None, :, None, None] * acc + beta.astype(np.float64)[None, :, None, None])
    ws, ap = ops.pack_stem_weights_f8(wq, alpha)
    y = ops.stem_fused_f8(_cuda(x), _cuda(ws), _cuda(ap), _cuda(beta), s_in)
    got = nhwc_to_nchw(y.cpu().numpy())
    assert got.shape == ref.shape
    assert len(np.unique(ref)) > 50
    a_, b_ = O.decode_f8(got).astype(np.float64), O.decode_f8(ref).astype(np.float64)
    assert not (np.abs(a_ - b_) > _step(np.maximum(np.abs(a_), np.abs(b_))) + 8 * e).any(), "stem: beyond one step + 2E"
    n = np.count_nonzero(got != ref)
    mu, mu_t = _flip_mu(y_ex, 9 * e, True), _flip_mu(y_ex, e_typ, True, sides=1)
    bar = 2 * mu_t + 4 * np.sqrt(mu_t) + 8
    print(f"[f8 bar] stem: {n} of {got.size} codes differ, typical-error mu {mu_t:.1f} (bar {bar:.0f}, "
          f"{bar / max(n, 1):.1f}x the count), worst-case mu {mu:.1f}")
    assert n <= mu + 4 * np.sqrt(mu) + 2, f"stem: {n} of {got.size} outputs differ (model mu = {mu:.1f})"
    assert n <= bar, f"stem: {n} of {got.size} outputs differ (typical-error model mu = {mu_t:.1f})"


@pytest.mark.parametrize("N,grid", [(3, None), (5, "2")])
def test_block_l1_f8_equals_two_convs(gpu, N, grid, knobs):
    """The fused layer1 block groups each tap's 64 channels into one MFMA in
    the same lane order and tap order as the generic conv kernel, so it is
    bit-identical to two dlq_conv2d_nhwc_f8 calls (which the oracle checks);
    grid "2" puts several images in one workgroup (the "l1_grid" knob)."""
    from dlq_amd import ops
    if grid:
        knobs("l1_grid", int(grid))
    rng = np.random.default_rng(53 + N)
    x = O.quantize_f32_f8(np.abs(rng.standard_normal((N, 56, 56, 64))).astype(np.float32) * 30, 1.0)
    ws, al, be = [], [], []
    for _ in range(2):
        w, bn = rand_conv(rng, 64, 64, 3)
        wq, sw = O.quantize_weights_f8(w)
        a_, b_ = O.fold_bn(0.02, sw, bn, 0.021)
        ws.append(_cuda(ops.pack_conv_weights_f8(wq, 64, 56, 1, 1)))
        al.append(_cuda(a_))
        be.append(_cuda(b_))
    r_s = float(O.res_scale(0.02, 0.021))
    xd = _cuda(x)
    y = ops.block_l1_f8(xd, ws[0], al[0], be[0], ws[1], al[1], be[1], r_s).cpu().numpy()
    h = ops.conv2d_nhwc_f8(xd, ws[0], 64, 3, 1, 1, al[0], be[0], relu=True)
    y2 = ops.conv2d_nhwc_f8(h, ws[1], 64, 3, 1, 1, al[1], be[1], residual=xd, res_scale=r_s, relu=True).cpu().numpy()
    assert len(np.unique(y2)) > 50
    assert np.array_equal(y, y2), f"{np.count_nonzero(y != y2)} of {y.size} codes differ"


@pytest.mark.parametrize("C,H,N", [(64, 56, 3), (128, 28, 5), (256, 14, 37)])
def test_s2_conv_with_fused_downsample_f8(gpu, C, H, N):
    """layerX.0 with e4m3 operands: 3x3/s2 conv1 (+BN+ReLU) and the 1x1/s2
    downsample (+BN) from ONE launch.  Both outputs within the conv bound of
    the oracle; conv1's equals the standalone dlq_conv2d_nhwc_f8 call (the
    same kernel without the downsample) code for code."""
    from dlq_amd import ops
    rng = np.random.default_rng(C * 11 + N)
    OC = 2 * C
    x = O.quantize_f32_f8(np.abs(rng.standard_normal((N, C, H, H))).astype(np.float32) * 40, 1.0)
    w, bn = rand_conv(rng, OC, C, 3)
    wd, bnd = rand_conv(rng, OC, C, 1)
    bnd[0][::5] *= -1
    wq, sw = O.quantize_weights_f8(w)
    wdq, swd = O.quantize_weights_f8(wd)
    s_x, s_y, s_d = 0.011, 0.013, 0.015
    alpha, beta = O.fold_bn(s_x, sw, bn, s_y)
    alpha_d, beta_d = O.fold_bn(s_x, swd, bnd, s_d)
    acc, acc_d = O.conv_f8_acc(x, wq, 2, 1), O.conv_f8_acc(x, wdq, 2, 0)
    ref = O.epilogue_f8(acc, alpha, beta, None, 0.0, True)
    ref_d = O.epilogue_f8(acc_d, alpha_d, beta_d, None, 0.0, False)
    xd = _cuda(nchw_to_nhwc(x))
    wdev = _cuda(ops.pack_conv_weights_f8(wq, C, H, 2, 1))
    wds = _cuda(ops.pack_downsample_weights(wdq.reshape(OC, C).view(np.int8), C))
    y, y_ds = ops.conv2d_s2_ds_nhwc_f8(xd, wdev, _cuda(alpha), _cuda(beta), wds, _cuda(alpha_d), _cuda(beta_d))
    got, got_d = nhwc_to_nchw(y.cpu().numpy()), nhwc_to_nchw(y_ds.cpu().numpy())
    for g, r, ac, wqq, al, be_, s_, p_, relu, what in ((got, ref, acc, wq, alpha, beta, 2, 1, True, "conv1"),
                                                         (got_d, ref_d, acc_d, wdq, alpha_d, beta_d, 2, 0, False, "ds")):
        assert len(np.unique(r)) > 50
        s_abs = O.conv_f8_acc(x & 0x7F, wqq & 0x7F, s_, p_)
        e, e_typ = _errs(al, s_abs, _conv_sq(x, wqq, s_, p_))
        yv = al.astype(np.float64)[None, :, None, None] * ac + be_.astype(np.float64)[None, :, None, None]
        _check_conv(g, r, yv, e, relu, what, e_typ)
    alone = ops.conv2d_nhwc_f8(xd, wdev, OC, 3, 2, 1, _cuda(alpha), _cuda(beta), relu=True).cpu().numpy()
    assert np.array_equal(y.cpu().numpy(), alone)


@pytest.mark.parametrize("N", [5, 37])
def test_gap_and_fc_f8_bitexact(gpu, N):
    """GAP (16-channel shuffle kernel) and FC (f64 MFMA kernel, exact sums):
    bit-exact; N = 37 leaves partial 16-row FC tiles."""
    from dlq_amd import ops
    rng = np.random.default_rng(23 + N)
    x = O.quantize_f32_f8(np.abs(rng.standard_normal((N, 512, 7, 7))).astype(np.float32) * 30, 1.0)
    k = O.gap_k_f8(0.02, 49, 0.015)
    g_ref, _ = O.gap_f8(x, k)
    g = ops.gap_nhwc_f8(_cuda(nchw_to_nhwc(x)), float(k)).cpu().numpy()
    assert np.array_equal(g, g_ref)
    w = rng.standard_normal((1000, 512)).astype(np.float32)
    wq, sw = O.quantize_weights_f8(w)
    bias = rng.standard_normal(1000).astype(np.float32)
    al = O.fc_alpha(0.015, sw)
    ref, _ = O.fc_f8(g_ref, wq, al, bias)
    out = ops.linear_f8(_cuda(g_ref), _cuda(wq), _cuda(al), _cuda(bias)).cpu().numpy()
    assert np.array_equal(out.view(np.int32), ref.view(np.int32))


def test_resnet18_fp8_end_to_end(gpu):
    from dlq_amd.models import ResNet18Int8, synthetic_images
    sd, scales = model_and_scales_f8()
    x = synthetic_images(2, seed=77).numpy()
    ref_logits, dumps = O.resnet18_forward_f8(sd, scales, x)
    model = ResNet18Int8(sd, scales, max_batch=4, keep_stages=True, precision="fp8")
    logits = model(_cuda(x)).cpu().numpy()
    torch.cuda.synchronize()
    shapes = {"stem_pool": (56, 56, 64), "layer1": (56, 56, 64), "layer2": (28, 28, 128),
              "layer3": (14, 14, 256), "layer4": (7, 7, 512)}
    cosine = lambda a, b: float(np.dot(a.ravel(), b.ravel()) / np.linalg.norm(a) / np.linalg.norm(b))  # noqa: E731
    worst = {}
    for st, (h, w, c) in shapes.items():
        got = nhwc_to_nchw(model.stage(st, (2, h, w, c)).cpu().numpy().view(np.uint8))
        n = np.count_nonzero(got != dumps[st])
        cs = cosine(O.decode_f8(got).astype(np.float64), O.decode_f8(dumps[st]).astype(np.float64))
        print(f"{st}: {n / got.size:.4%} codes differ, decoded cosine vs oracle {cs:.6f}")
        worst[st] = (n / got.size, cs)
    for i in range(2):
        f, _ = O.resnet18_forward_f32(sd, x[i])
        cg = cosine(logits[i].astype(np.float64), f.astype(np.float64))
        co = cosine(logits[i].astype(np.float64), ref_logits[i].astype(np.float64))
        print(f"logits[{i}]: cosine vs fp32 reference {cg:.6f}, vs oracle fp8 {co:.6f}")
        worst[f"logits{i}"] = (cg, co)
    assert worst["stem_pool"][0] <= 0.01, worst
    assert all(v[1] >= 0.99 for k, v in worst.items() if not k.startswith("logits")), worst
    assert all(worst[f"logits{i}"][0] >= 0.995 for i in range(2)), worst


def test_resnet18_fp8_batch_256_rows_independent(gpu):
    """Full bench batch: rows 0 and 255 equal the same images run alone."""
    from dlq_amd.models import ResNet18Int8, synthetic_images
    sd, scales = model_and_scales_f8()
    x = synthetic_images(256, seed=9).cuda()
    model = ResNet18Int8(sd, scales, max_batch=256, precision="fp8")
    full = model(x).cpu().numpy()
    pair = model(x[[0, 255]].contiguous()).cpu().numpy()
    assert np.array_equal(full[[0, 255]], pair)
    assert np.isfinite(full).all()
