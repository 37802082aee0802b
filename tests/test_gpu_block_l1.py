"""GPU parity of the fused layer1 basic block (block_l1.hip,
dlq_block_l1_nhwc_s8) against the CPU oracle: conv1 + BN + ReLU requant,
conv2 + BN + residual + ReLU requant (oracle.c ora_conv2d_nchw_s8_acc +
ora_epilogue_s8, the restatement of RK/runtime/infer_e2e.cu:156-203)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import nchw_to_nhwc, nhwc_to_nchw, rand_conv, rand_s8

pytestmark = pytest.mark.gpu


def _layer(rng, s_x, s_y):
    from dlq_amd import ops
    w, bn = rand_conv(rng, 64, 64, 3)
    wq, sw = O.quantize_weights_s8(w)
    alpha, beta = O.fold_bn(s_x, sw, bn, s_y)
    packed = ops.pack_conv_weights(wq, 64, 56, 1, 1)
    return wq, alpha, beta, packed


def _run(N, seed, lo, grid=None, knobs=None):
    from dlq_amd import ops
    rng = np.random.default_rng(seed)
    s_x, s_h, s_y = np.float32(0.03), np.float32(0.05), np.float32(0.06)
    wq1, a1, b1, p1 = _layer(rng, s_x, s_h)
    wq2, a2, b2, p2 = _layer(rng, s_h, s_y)
    r_s = O.res_scale(s_x, s_y)
    x = rand_s8(rng, (N, 64, 56, 56), lo=lo)
    h = O.epilogue_s8(O.conv_s8_acc(x, wq1, 1, 1), a1, b1, relu=True)
    ref = O.epilogue_s8(O.conv_s8_acc(h, wq2, 1, 1), a2, b2, res=x, r_s=r_s, relu=True)
    if grid is not None:
        knobs("l1_grid", grid)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    y = ops.block_l1_s8(cu(nchw_to_nhwc(x)), cu(p1), cu(a1), cu(b1), cu(p2), cu(a2), cu(b2), float(r_s))
    torch.cuda.synchronize()
    return nhwc_to_nchw(y.cpu().numpy()), ref


@pytest.mark.parametrize("N,lo", [(1, 0), (3, -127)])
def test_block_l1_bitexact(gpu, N, lo):
    got, ref = _run(N, 100 + N, lo)
    assert np.array_equal(got, ref)


def test_block_l1_several_images_per_workgroup(gpu, knobs):
    """Grid capped at 2 workgroups: images 0,2,4 and 1,3 each run as one
    stream of rows through the LDS rings (image boundaries inside a phase)."""
    got, ref = _run(5, 7, 0, grid=2, knobs=knobs)
    assert np.array_equal(got, ref)


def test_block_l1_matches_two_conv_launches(gpu):
    """The fused launch equals the engine's two-launch path on the same data."""
    from dlq_amd import ops
    rng = np.random.default_rng(11)
    s_x, s_h, s_y = np.float32(0.02), np.float32(0.04), np.float32(0.05)
    _, a1, b1, p1 = _layer(rng, s_x, s_h)
    _, a2, b2, p2 = _layer(rng, s_h, s_y)
    r_s = float(O.res_scale(s_x, s_y))
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    x = cu(rand_s8(rng, (4, 56, 56, 64), lo=0))
    P1, P2, A1, B1, A2, B2 = cu(p1), cu(p2), cu(a1), cu(b1), cu(a2), cu(b2)
    h = ops.conv2d_nhwc_s8(x, P1, 64, 3, 1, 1, A1, B1, relu=True)
    two = ops.conv2d_nhwc_s8(h, P2, 64, 3, 1, 1, A2, B2, residual=x, res_scale=r_s, relu=True)
    one = ops.block_l1_s8(x, P1, A1, B1, P2, A2, B2, r_s)
    torch.cuda.synchronize()
    assert torch.equal(one, two)
