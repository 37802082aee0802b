"""GPU parity of the per-layer C-ABI in the reference's layout (NCHW / OIHW /
row-major, layerops.hip) against the CPU oracle."""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import model_and_scales, nchw_to_nhwc, nhwc_to_nchw, rand_conv, rand_s8

pytestmark = pytest.mark.gpu


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


_KEEP = []  # device copies stay alive until the test's calls are done (a temporary's memory can be reused)


def _p(t):
    _KEEP.append(t)
    return C.c_void_p(t.data_ptr())


@pytest.fixture(autouse=True)
def _release():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


def _ok(rc):
    from dlq_amd.lib import lib
    assert rc == 0, lib.dlq_last_error()


def test_init_finalize(gpu):
    from dlq_amd.lib import lib
    _ok(lib.dlq_init(0))
    _ok(lib.dlq_finalize())


def test_quantize_f32_s8(gpu):
    from dlq_amd.lib import lib
    rng = np.random.default_rng(1)
    x = (rng.standard_normal(100003, dtype=np.float32) * 3).astype(np.float32)
    x[:6] = [0.5, 1.5, -2.5, 1e9, -1e9, 0.0]
    s = np.float32(0.021)
    q = torch.empty(x.size, dtype=torch.int8, device="cuda")
    _ok(lib.dlq_quantize_f32_s8(_p(_cuda(x)), x.size, float(O.inv_scale(s)), _p(q), None))
    torch.cuda.synchronize()
    assert np.array_equal(q.cpu().numpy(), O.quantize_f32_s8(x, s))


@pytest.mark.parametrize("M,N,K", [(100, 77, 61), (1000, 1, 512), (64, 3136, 576), (33, 65, 1), (256, 256, 64),
                                   (512, 768, 1152), (257, 263, 2304), (300, 520, 72), (128, 196, 4608),
                                   (1, 5000, 3), (513, 255, 65), (257, 272, 2304), (300, 528, 80), (33, 16, 16),
                                   (1024, 512, 192)])
def test_gemm_s8s8s32_reference_layout(gpu, M, N, K):
    """sgemm_tiled's layout and contract (any M, N, K) in int8 -> int32:
    whole 256 x 256 tiles, M / N / K tails inside a tile and a stage, both
    kernels (K % 16 == N % 16 == 0: the LDS-DMA ring with transposed B reads;
    otherwise the register-staged kernel, byte loads for unaligned rows) and
    the extremes -128 / 127, bit-exact with the oracle."""
    from dlq_amd.lib import lib
    rng = np.random.default_rng(M + N + K)
    A = rand_s8(rng, (M, K), lo=-128)
    B = rand_s8(rng, (K, N), lo=-128)
    A.flat[:3] = -128
    B.flat[:3] = -128
    ref = np.empty((M, N), np.int32)
    O.lib().ora_gemm_s8s8s32(A, B, ref, M, N, K)
    Cd = torch.empty((M, N), dtype=torch.int32, device="cuda")
    _ok(lib.dlq_gemm_s8s8s32(_p(_cuda(A)), _p(_cuda(B)), _p(Cd), M, N, K, None))
    torch.cuda.synchronize()
    assert np.array_equal(Cd.cpu().numpy(), ref)


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 528, 2304), (257, 400, 80), (130, 1040, 4608),
                                   (513, 144, 16), (2304, 4096, 144), (448, 672, 384), (225, 225, 272)])
def test_gemm_s8s8s32_every_tile_shape(gpu, knobs, tile, M, N, K):
    """Each tile of the LDS-DMA kernel (knob gemm_tile: 1 = 256 x 256, 2 = 256 x
    128, 3 = 128 x 128, 4 = 256 x 224, 5 = 224 x 128, 6 = 224 x 256; by
    default chosen by shape) on whole tiles, M / N / K
    tails and K below one stage, and a grid of several tiles per CU in the
    grouped raster (2304 x 4096: 9 row blocks = two full groups of 4 and a
    group of 1) -- bit-exact with the oracle."""
    from dlq_amd.lib import lib
    knobs("gemm_tile", tile)
    rng = np.random.default_rng(M + 3 * N + 7 * K + tile)
    A = rand_s8(rng, (M, K), lo=-128)
    B = rand_s8(rng, (K, N), lo=-128)
    A.flat[-3:] = -128
    B.flat[:3] = -128
    ref = np.empty((M, N), np.int32)
    O.lib().ora_gemm_s8s8s32(A, B, ref, M, N, K)
    Cd = torch.full((M, N), 7, dtype=torch.int32, device="cuda")
    _ok(lib.dlq_gemm_s8s8s32(_p(_cuda(A)), _p(_cuda(B)), _p(Cd), M, N, K, None))
    torch.cuda.synchronize()
    assert np.array_equal(Cd.cpu().numpy(), ref)


@pytest.mark.parametrize("M,N,K,a_off,b_off", [(300, 520, 128, 0, 0), (257, 264, 2304, 0, 0), (256, 256, 64, 1, 0),
                                               (300, 520, 128, 0, 8), (200, 512, 256, 16, 24),
                                               (130, 264, 96, 3, 5)])
def test_gemm_s8s8s32_kernel_selection(gpu, M, N, K, a_off, b_off):
    """The alignment-based kernel choice of dlq_gemm_s8s8s32: K % 16 == 0 with
    N % 8 == 0 but N % 16 != 0 (or B only 8-byte aligned) takes the
    register-staged kernel's vector loads (uint2 B rows, 16-byte A rows);
    offset base pointers (A = buf[a_off:], B = buf[b_off:]) move a shape
    between the LDS-DMA kernel, the vector-load path and the byte-load path.
    Bit-exact with the oracle in every case."""
    from dlq_amd.lib import lib
    rng = np.random.default_rng(M * 7 + N + K + a_off + b_off)
    A = rand_s8(rng, (M, K), lo=-128)
    B = rand_s8(rng, (K, N), lo=-128)
    A.flat[:3] = -128
    B.flat[-3:] = -128
    ref = np.empty((M, N), np.int32)
    O.lib().ora_gemm_s8s8s32(A, B, ref, M, N, K)
    abuf = torch.zeros(M * K + 64, dtype=torch.int8, device="cuda")
    bbuf = torch.zeros(K * N + 64, dtype=torch.int8, device="cuda")
    abuf[a_off:a_off + M * K] = torch.from_numpy(A.reshape(-1)).cuda()
    bbuf[b_off:b_off + K * N] = torch.from_numpy(B.reshape(-1)).cuda()
    Cd = torch.empty((M, N), dtype=torch.int32, device="cuda")
    _ok(lib.dlq_gemm_s8s8s32(abuf.data_ptr() + a_off, bbuf.data_ptr() + b_off, _p(Cd), M, N, K, None))
    torch.cuda.synchronize()
    assert np.array_equal(Cd.cpu().numpy(), ref)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("M,N,K,a_off,b_off", [(256, 256, 128, 0, 0), (300, 521, 2304, 0, 0), (257, 400, 80, 0, 0),
                                               (130, 1040, 4608, 0, 0), (513, 7, 16, 0, 0), (100, 77, 61, 0, 0),
                                               (33, 65, 1, 0, 0), (300, 520, 128, 0, 8), (130, 264, 96, 3, 5)])
def test_gemm_s8s8s32_nt(gpu, knobs, tile, M, N, K, a_off, b_off):
    """dlq_gemm_s8s8s32_nt (B supplied as Bt[N][K]): every LDS-DMA tile on
    whole tiles, M / N / K tails and any N (no N % 16 condition), and the
    register-staged kernel for K % 16 != 0 or unaligned bases (a_off /
    b_off), bit-exact with the oracle's NN GEMM of B = Bt^T."""
    from dlq_amd.lib import lib
    knobs("gemm_tile", tile)
    rng = np.random.default_rng(M + 5 * N + 11 * K + tile + a_off)
    A = rand_s8(rng, (M, K), lo=-128)
    Bt = rand_s8(rng, (N, K), lo=-128)
    A.flat[:3] = -128
    Bt.flat[-3:] = -128
    B = np.ascontiguousarray(Bt.T)
    ref = np.empty((M, N), np.int32)
    O.lib().ora_gemm_s8s8s32(A, B, ref, M, N, K)
    abuf = torch.zeros(M * K + 64, dtype=torch.int8, device="cuda")
    bbuf = torch.zeros(K * N + 64, dtype=torch.int8, device="cuda")
    abuf[a_off:a_off + M * K] = torch.from_numpy(A.reshape(-1)).cuda()
    bbuf[b_off:b_off + K * N] = torch.from_numpy(Bt.reshape(-1)).cuda()
    Cd = torch.full((M, N), 7, dtype=torch.int32, device="cuda")
    _ok(lib.dlq_gemm_s8s8s32_nt(abuf.data_ptr() + a_off, bbuf.data_ptr() + b_off, _p(Cd), M, N, K, None))
    torch.cuda.synchronize()
    assert np.array_equal(Cd.cpu().numpy(), ref)


@pytest.mark.parametrize("IC,OC,k,s,p,H,N", [(3, 64, 7, 2, 3, 224, 1), (64, 64, 3, 1, 1, 56, 2),
                                             (64, 128, 1, 2, 0, 56, 2), (128, 128, 3, 1, 1, 28, 3),
                                             (256, 512, 3, 2, 1, 14, 2)])
@pytest.mark.parametrize("out_kind", [0, 2])
def test_conv2d_nchw_reference_signature(gpu, IC, OC, k, s, p, H, N, out_kind):
    """conv2d_nchw_im2col_gemm's argument order (infer_e2e.cu:102-107): NCHW
    in/out, OIHW weights, (OH, OW) returned."""
    from dlq_amd.lib import lib
    rng = np.random.default_rng(IC * 3 + OC + k)
    x = rand_s8(rng, (N, IC, H, H))
    w, bn = rand_conv(rng, OC, IC, k)
    wq, sw = O.quantize_weights_s8(w)
    alpha, beta = O.fold_bn(0.03, sw, bn, 0.05)
    acc = O.conv_s8_acc(x, wq, s, p)
    ref = acc if out_kind == 2 else O.epilogue_s8(acc, alpha, beta, None, 0.0, True)
    ocp = lib.dlq_conv_packed_oc(OC)
    from dlq_amd.ops import pad_vec
    ws_n = lib.dlq_conv2d_nchw_workspace_bytes(N, IC, H, H, OC, k, k, s, s, p, p)
    assert ws_n > 0
    ws = torch.empty(ws_n, dtype=torch.int8, device="cuda")
    y = torch.empty(ref.shape, dtype=torch.int32 if out_kind == 2 else torch.int8, device="cuda")
    oh, ow = C.c_int(), C.c_int()
    _ok(lib.dlq_conv2d_nchw_s8(_p(_cuda(x)), N, IC, H, H, wq.ctypes.data, OC, k, k, s, s, p, p,
                               _p(_cuda(pad_vec(alpha, ocp))), _p(_cuda(pad_vec(beta, ocp))), 1, out_kind, _p(y),
                               _p(ws), ws_n, None, C.byref(oh), C.byref(ow)))
    torch.cuda.synchronize()
    assert (oh.value, ow.value) == ref.shape[2:]
    assert np.array_equal(y.cpu().numpy(), ref)


def test_bn_relu_add_requant_dequant(gpu):
    from dlq_amd.lib import lib
    rng = np.random.default_rng(5)
    N, Cc, HW = 3, 64, 49
    acc = rng.integers(-40000, 40000, size=(N, Cc, HW), dtype=np.int32)
    alpha = (rng.random(Cc, dtype=np.float32) * 2e-3).astype(np.float32)
    beta = (rng.standard_normal(Cc, dtype=np.float32) * 3).astype(np.float32)
    for relu in (0, 1):
        ref = O.epilogue_s8(acc, alpha, beta, None, 0.0, bool(relu))
        y = torch.empty((N, Cc, HW), dtype=torch.int8, device="cuda")
        _ok(lib.dlq_bn_relu_requant_s8(_p(_cuda(acc)), N, Cc, HW, _p(_cuda(alpha)), _p(_cuda(beta)), relu, _p(y), None))
        torch.cuda.synchronize()
        assert np.array_equal(y.cpu().numpy(), ref)
    a = rand_s8(rng, (N, Cc, HW), lo=-127)
    r = rand_s8(rng, (N, Cc, HW), lo=-127)
    for relu in (0, 1):
        ref = O.add_requant_s8(a, r, 0.7, 1.3, bool(relu))
        y = torch.empty(a.shape, dtype=torch.int8, device="cuda")
        _ok(lib.dlq_add_relu_requant_s8(_p(_cuda(a)), _p(_cuda(r)), a.size, 0.7, 1.3, relu, _p(y), None))
        torch.cuda.synchronize()
        assert np.array_equal(y.cpu().numpy(), ref)
    scale = (rng.random(Cc, dtype=np.float32) * 1e-2).astype(np.float32)
    yf = torch.empty(acc.shape, dtype=torch.float32, device="cuda")
    _ok(lib.dlq_dequant_s32_f32(_p(_cuda(acc)), N, Cc, HW, _p(_cuda(scale)), _p(yf), None))
    torch.cuda.synchronize()
    ref = acc.astype(np.float32) * scale[None, :, None]
    assert np.array_equal(yf.cpu().numpy().view(np.int32), ref.view(np.int32))


@pytest.mark.parametrize("n,off", [(1023, 0), (1024, 0), (100003, 0), (100003, 4), (100003, 1), (3 * 224 * 224 * 9, 0)])
def test_quantize_f32_s8_streaming(gpu, n, off):
    """The 16-byte streaming form of dlq_quantize_f32_s8 (16-byte aligned x,
    n >= 1024: the vector body + a scalar tail) and the scalar kernel
    (misaligned x: off floats into the buffer), bit-exact with the oracle
    (ties, saturation, signed zero)."""
    from dlq_amd.lib import lib
    rng = np.random.default_rng(n + off)
    x = (rng.standard_normal(n, dtype=np.float32) * 3).astype(np.float32)
    x[:8] = [0.5, 1.5, -2.5, 1e9, -1e9, 0.0, -0.0, 126.5 * 0.021]
    s = np.float32(0.021)
    xb = torch.zeros(n + 8, dtype=torch.float32, device="cuda")
    xb[off:off + n] = torch.from_numpy(x).cuda()
    q = torch.empty(n, dtype=torch.int8, device="cuda")
    _ok(lib.dlq_quantize_f32_s8(xb.data_ptr() + 4 * off, n, float(O.inv_scale(s)), _p(q), None))
    torch.cuda.synchronize()
    assert np.array_equal(q.cpu().numpy(), O.quantize_f32_s8(x, s))


@pytest.mark.parametrize("N,Cc,HW", [(3, 5, 12), (2, 64, 3136), (4, 512, 49), (256, 1000, 1), (1, 7, 4)])
def test_dequant_s32_f32_streaming(gpu, N, Cc, HW):
    """dlq_dequant_s32_f32: the 16-byte streaming kernel (HW % 4 == 0, >= 1024
    elements, 32-bit index math) and the scalar kernel otherwise; y =
    float(acc) * scale[c] bit for bit."""
    from dlq_amd.lib import lib
    rng = np.random.default_rng(N * Cc + HW)
    acc = rng.integers(-(1 << 24), 1 << 24, size=(N, Cc, HW), dtype=np.int32)
    acc.flat[:2] = [2**31 - 1, -2**31]
    scale = (rng.random(Cc, dtype=np.float32) * 1e-2).astype(np.float32)
    yf = torch.empty(acc.shape, dtype=torch.float32, device="cuda")
    _ok(lib.dlq_dequant_s32_f32(_p(_cuda(acc)), N, Cc, HW, _p(_cuda(scale)), _p(yf), None))
    torch.cuda.synchronize()
    ref = acc.astype(np.float32) * scale[None, :, None]
    assert np.array_equal(yf.cpu().numpy().view(np.int32), ref.view(np.int32))


def test_maxpool_gap_fc_nchw(gpu):
    from dlq_amd import ops
    from dlq_amd.lib import lib
    from tests.helpers import golden
    rng = np.random.default_rng(6)
    x = rand_s8(rng, (2, 64, 112, 112), lo=-128)
    y = torch.empty((2, 64, 56, 56), dtype=torch.int8, device="cuda")
    _ok(lib.dlq_maxpool2d_3x3_s2p1_nchw_s8(_p(_cuda(x)), 2, 64, 112, 112, _p(y), None))
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), O.maxpool_s8(x))
    x4 = rand_s8(rng, (3, 512, 7, 7))
    k = O.gap_k(0.05, 49, 0.011)
    g = torch.empty((3, 512), dtype=torch.int8, device="cuda")
    _ok(lib.dlq_gap_s8(_p(_cuda(x4)), 3, 512, 49, float(k), _p(g), None))
    torch.cuda.synchronize()
    gref, _ = O.gap_s8(x4, k)
    assert np.array_equal(g.cpu().numpy(), gref)
    W = golden("fc.weight.bin", (1000, 512))
    bias = golden("fc.bias.bin")
    wq, sw = O.quantize_weights_s8(W)
    alpha = O.fc_alpha(0.02, sw)
    ref, _ = O.fc_s8(gref, wq, alpha, bias)
    ocp = ops.packed_oc(1000)
    out = torch.empty((3, 1000), dtype=torch.float32, device="cuda")
    _ok(lib.dlq_fc_s8(_p(g), 3, 512, _p(_cuda(ops.pack_linear_weights(wq))), 1000, _p(_cuda(ops.pad_vec(alpha, ocp))),
                      _p(_cuda(ops.pad_vec(bias, ocp))), _p(out), None))
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.int32), ref.view(np.int32))


def test_basic_block_api_matches_oracle_stages(gpu):
    """dlq_basic_block_s8 on blocks 0..3 (layer1.0 .. layer2.1, incl. the
    fused stride-2 + downsample block) reproduces the oracle's stage dumps."""
    from dlq_amd.lib import lib
    from dlq_amd.models import ResNet18Int8, synthetic_images
    sd, scales = model_and_scales()
    x = synthetic_images(2, seed=5).numpy()
    _, dumps = O.resnet18_forward_s8(sd, scales, x)
    model = ResNet18Int8(sd, scales, max_batch=4)
    h = model.h
    cur = _cuda(nchw_to_nhwc(dumps["stem_pool"]))
    outs = []
    for b, (Hh, Cc) in enumerate([(56, 64), (56, 64), (28, 128), (28, 128)]):
        y = torch.empty((2, Hh, Hh, Cc), dtype=torch.int8, device="cuda")
        _ok(lib.dlq_basic_block_s8(h, b, _p(cur), 2, _p(y), None))
        cur = y
        outs.append(y)
    torch.cuda.synchronize()
    assert np.array_equal(nhwc_to_nchw(outs[1].cpu().numpy()), dumps["layer1"])
    assert np.array_equal(nhwc_to_nchw(outs[3].cpu().numpy()), dumps["layer2"])
