"""GPU parity of the path's ends through the C ABI: preprocessing
(dlq_preprocess_u8: bit-exact vs the oracle, which the reference's goldens
pin) and the head (dlq_softmax_f32 within 2e-6 + 2e-7*|z| relative of
an exact softmax, z = x - max: fp32 rounding of z grows the relative error
of exp(z) with |z|; softmax_1d itself uses __expf, so there is no bit
pattern to match; dlq_top1_f32 exact)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import preprocess_cases, synth_image

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", preprocess_cases(), ids=lambda c: f"{c[0]}x{c[1]}")
def test_preprocess_bitexact(gpu, case):
    from dlq_amd import ops
    h, w, seed = case[:3]
    imgs = np.stack([synth_image(h, w, seed), synth_image(h, w, seed + 100)])
    got = ops.preprocess_u8(torch.from_numpy(imgs).cuda()).cpu().numpy()
    for n in range(2):
        ref = O.preprocess_u8(imgs[n])
        assert np.array_equal(got[n].view(np.int32), ref.view(np.int32)), \
            f"image {n}: {np.count_nonzero(got[n] != ref)} mismatches, max |d| {np.abs(got[n] - ref).max()}"


def test_preprocess_sizes_and_errors(gpu):
    from dlq_amd import ops
    from dlq_amd.lib import lib
    assert ops.preprocess_size(300, 400) == O.preprocess_size(300, 400)
    assert ops.preprocess_size(641, 333) == O.preprocess_size(641, 333)
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, size=(1, 700, 900, 3), dtype=np.uint8)  # downscale 2.7x: 6-tap filters
    got = ops.preprocess_u8(torch.from_numpy(img).cuda()).cpu().numpy()[0]
    assert np.array_equal(got.view(np.int32), O.preprocess_u8(img[0]).view(np.int32))
    with pytest.raises(RuntimeError):
        ops.preprocess_u8(torch.zeros((1, 4000, 4000, 3), dtype=torch.uint8, device="cuda"))  # > 7x
    assert lib.dlq_preprocess_u8(None, 0, 10, 10, None, None) == 0  # empty batch


def test_softmax_within_tolerance(gpu):
    from dlq_amd import ops
    rng = np.random.default_rng(7)
    x = (rng.standard_normal((37, 1000)) * 6).astype(np.float32)
    x[3, 17] = 80.0  # one dominant logit
    got = ops.softmax(torch.from_numpy(x).cuda()).cpu().numpy()
    ref = O.softmax_f64(x)
    z = np.abs(x.astype(np.float64) - x.max(1, keepdims=True))
    tol = ref * (2e-6 + 2e-7 * z) + 1e-30
    assert np.all(np.abs(got - ref) <= tol), np.max(np.abs(got - ref) / tol)
    assert np.allclose(got.astype(np.float64).sum(1), 1.0, atol=1e-6)


def test_top1_matches_launcher_rule(gpu):
    from dlq_amd import ops
    rng = np.random.default_rng(9)
    x = rng.standard_normal((70, 1000)).astype(np.float32)
    x[5, [10, 700]] = 9.0                   # tie: the first index wins
    x[6, :] = -np.inf                        # nothing beats -1e30
    x[7, ::2] = np.nan                       # NaNs never win
    x[8, :] = -2e30                          # below the -1e30 floor
    idx, val = ops.top1(torch.from_numpy(x).cuda())
    ridx, rval = O.top1(x)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    assert np.array_equal(val.cpu().numpy(), rval)
