"""The host DMA-plan checker (tools/check/dma_plan.py) pinned to the compiled
kernels: tools/check/libplancap.so builds conv3x3i.hip and conv3x3s2i.hip
with DLQ_PLAN_CAPTURE (device_common.h), so their launchers run the real
kernels and every LDS-DMA piece is recorded -- LDS address and 64 lane
sources, in issue order per workgroup and wave -- instead of issued.  Each
recorded piece must equal the piece dma_plan.py derives (which in turn is
proven to stage the reference im2col's bytes, tests/test_dma_plan.py): an
edit of a kernel's piece plan that the checker does not follow fails here.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "check"))
import dma_plan as D  # noqa: E402

pytestmark = pytest.mark.gpu
LIB = os.path.join(ROOT, "tools", "check", "libplancap.so")
MAXREC = 160  # pieces per wave (the largest plans: about 80, conv3x3i W = 7: 8 stages x 10)


def _capture(kind, W, N):
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: build it with `make` (Makefile target tools/check/libplancap.so)")
    lib = C.CDLL(LIB)
    grid = 256
    nw = grid * 8
    cnt = np.zeros(nw, np.uint32)
    lds = np.zeros(nw * MAXREC, np.uint32)
    src = np.zeros(nw * MAXREC * 64, np.uint64)
    bases = np.zeros(4, np.uint64)
    f = lib.plancap_run_wide if kind == 0 else lib.plancap_run_s2i
    f.restype = C.c_int
    n = f(C.c_int(kind), C.c_int(W), C.c_int(N), C.c_uint(MAXREC), cnt.ctypes.data_as(C.c_void_p),
          lds.ctypes.data_as(C.c_void_p), src.ctypes.data_as(C.c_void_p), bases.ctypes.data_as(C.c_void_p),
          C.c_int(nw))
    assert n != -2, "plan capture dropped pieces (a wave past the capture buffers, or more than MAXREC pieces)"
    assert n != -3, "the launch has more waves than the capture arrays hold"
    assert n > 0, "plan capture launch failed"
    return n, cnt[:n], lds[:n * MAXREC].reshape(n, MAXREC), src[:n * MAXREC * 64].reshape(n, MAXREC, 64), bases


def _classify(src, bases, sizes):
    """source addresses -> code(kind, offset), -1 outside every buffer"""
    out = np.full(src.shape, -1, np.int64)
    for kind, base, size in ((D.KX, bases[0], sizes[0]), (D.KW, bases[1], sizes[1]), (D.KD, bases[2], sizes[2]),
                             (D.KZ, bases[3], 1024)):
        if size == 0:
            continue
        rel = src.astype(np.int64) - np.int64(base)
        hit = (rel >= 0) & (rel < size)
        out = np.where(hit, D.code(kind, np.where(hit, rel, 0)), out)
    return out


def _compare(emit, n, cnt, lds, src, bases, sizes, what):
    # the workgroup's LDS base (M0 = lds32 + offset): one constant for all pieces
    delta = None
    for (b, wv), pieces in emit.items():
        w = b * 8 + wv
        assert w < n, f"{what}: workgroup {b} not launched"
        assert cnt[w] == len(pieces), f"{what}: wave {w} recorded {cnt[w]} pieces, the checker plans {len(pieces)}"
        got = _classify(src[w, :len(pieces)], bases, sizes)
        for i, (dst, codes) in enumerate(pieces):
            d = int(lds[w, i]) - int(dst)
            if delta is None:
                delta = d
            assert d == delta, f"{what}: wave {w} piece {i}: LDS address {lds[w, i]} vs planned {dst} (+{delta})"
            bad = np.nonzero(got[i] != codes)[0]
            assert bad.size == 0, (f"{what}: wave {w} piece {i} lane {bad[0]}: source code {got[i][bad[0]]:#x} "
                                   f"vs planned {int(codes[bad[0]]):#x}")
    waves = {b * 8 + wv for (b, wv) in emit}
    extra = [w for w in range(n) if w not in waves and cnt[w]]
    assert not extra, f"{what}: waves {extra[:4]} issued pieces the checker does not plan"


@pytest.mark.parametrize("W,N", [(28, 256), (28, 3), (14, 256), (14, 5), (7, 256), (7, 17)])
def test_wide_conv_plan_is_the_kernels(gpu, W, N):
    C_ = {28: 128, 14: 256, 7: 512}[W]
    emit = {}
    D.check_conv3x3i(W, N, emit)
    n, cnt, lds, src, bases = _capture(0, W, N)
    sizes = (N * W * W * C_, (C_ // 32) * max(C_, 128) * 304, 0)
    _compare(emit, n, cnt, lds, src, bases, sizes, f"conv3x3i W={W} N={N}")


@pytest.mark.parametrize("OW,N", [(28, 256), (28, 3), (14, 256), (14, 5), (7, 256), (7, 17)])
def test_stride2_conv_plan_is_the_kernels(gpu, OW, N):
    C_ = {28: 64, 14: 128, 7: 256}[OW]
    emit = {}
    D.check_s2i(OW, N, emit)
    n, cnt, lds, src, bases = _capture(1, 2 * OW, N)
    sizes = (N * 4 * OW * OW * C_, (C_ // 32) * 2 * C_ * 304, (C_ // 32) * 2 * C_ * 48)
    _compare(emit, n, cnt, lds, src, bases, sizes, f"conv3x3s2i OW={OW} N={N}")


def test_masked_lds_dma(gpu):
    """The masked LDS-DMA issues the kernels' shared piece plans use for empty
    slots (device_common.h glds16_asm_m / glds16_saddr_m), run for real
    (tools/check/dma_mask_check.hip, compiled without DLQ_PLAN_CAPTURE): with
    valid = false neither form writes its LDS piece (the poison stays), with
    valid = true both land their 1 KiB, and every lane stores after each
    (EXEC restored).  The conv tests cannot see this: an empty slot re-issues
    another wave's piece, identical bytes to the same address."""
    import torch
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: build it with `make` (Makefile target tools/check/libplancap.so)")
    lib = C.CDLL(LIB)
    lib.dmamask_run.restype = C.c_int
    src = torch.arange(4096, dtype=torch.int32, device="cuda").remainder(251).to(torch.int8)
    out = torch.zeros(4096, dtype=torch.int8, device="cuda")
    lanes = torch.zeros(256, dtype=torch.int32, device="cuda")
    assert lib.dmamask_run(C.c_void_p(src.data_ptr()), C.c_void_p(out.data_ptr()), C.c_void_p(lanes.data_ptr())) == 0
    o, s = out.cpu().numpy(), src.cpu().numpy()
    assert (o[:2048].view(np.uint8) == 0xA5).all(), "a masked (valid = false) piece wrote LDS"
    assert np.array_equal(o[2048:], s[2048:]), "an unmasked piece did not land"
    assert np.array_equal(lanes.cpu().numpy(), np.tile(np.arange(1, 65, dtype=np.int32), 4)), "EXEC not restored"
