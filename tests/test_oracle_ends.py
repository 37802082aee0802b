"""The oracle's restatement of the path's ends, pinned before it is trusted:
preprocessing (RK/tools/preprocess_to_bin.py:8-33 driving Pillow's 8-bit
BILINEAR resampler) against tests/golden/preprocess_golden.npz, which
tools/make_preprocess_golden.py wrote from the reference's own functions;
and the launcher's top-1 rule (RK/runtime/infer_e2e.cu:436-438)."""
import hashlib

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import preprocess_cases, synth_image


@pytest.mark.parametrize("case", preprocess_cases(), ids=lambda c: f"{c[0]}x{c[1]}")
def test_preprocess_oracle_matches_reference_goldens(case):
    h, w, seed, crop_sha, out_sha = case
    img = synth_image(h, w, seed)
    crop = O.preprocess_resize_crop_u8(img)
    assert crop.shape == (224, 224, 3)
    assert hashlib.sha256(crop.tobytes()).digest() == crop_sha, "u8 resize+crop differs from Pillow via the reference"
    x = O.preprocess_u8(img)[None]
    assert x.dtype == np.float32 and x.shape == (1, 3, 224, 224)
    assert hashlib.sha256(x.tobytes()).digest() == out_sha, "fp32 normalisation differs from to_nchw_float32"


def test_preprocess_size_rounds_half_even():
    assert O.preprocess_size(300, 400) == (256, 341)   # 341.33
    assert O.preprocess_size(400, 300) == (341, 256)
    assert O.preprocess_size(256, 256) == (256, 256)
    assert O.preprocess_size(512, 640) == (256, 320)   # exact
    # Python round() is half-to-even: 160*256/128 -> 320 exactly; 2.5-style ties
    assert O.preprocess_size(128, 161) == (256, 322)   # 322.0


def test_top1_first_max_and_floor():
    x = np.array([[1.0, 3.0, 3.0, -2.0],
                  [-np.inf, -np.inf, -np.inf, -np.inf],
                  [np.nan, 0.5, np.nan, 0.5],
                  [-2e30, -1e31, -5e30, -3e30]], dtype=np.float32)
    idx, val = O.top1(x)
    assert idx.tolist() == [1, -1, 1, -1]
    assert val[0] == 3.0 and val[2] == 0.5 and val[1] == np.float32(-1e30)


def test_softmax_reference_is_normalised():
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((4, 1000)) * 5).astype(np.float32)
    p = O.softmax_f64(x)
    assert np.allclose(p.sum(1), 1.0) and (p > 0).all()
