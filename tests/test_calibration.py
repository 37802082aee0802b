"""Activation-scale calibration as bench.py runs it: the 22
sites of the int8 scheme, and the engine's GPU calibration
(dlq_resnet18_calibrate: the reference's fp32 forward op for op, scale =
amax / qmax per site) read back through ResNet18Int8.scale_dict, against
the torch fp32 calibration of the same images (different summation orders:
a stated relative bound, 1e-4)."""
import pytest
import torch

from dlq_amd.models import resnet18_state_dict, site_names, synthetic_images
from dlq_amd.quant import calibrate_resnet18

SEED = 0x20260306


def test_site_names_are_the_calibrated_sites():
    sd = resnet18_state_dict(SEED)
    scales = calibrate_resnet18(sd, synthetic_images(1, seed=SEED + 1), device="cpu")
    names = site_names()
    assert len(names) == 22 and len(set(names)) == 22
    assert set(names) == set(scales)


@pytest.mark.gpu
@pytest.mark.parametrize("qmax", [127.0, 448.0])
def test_gpu_calibration_matches_torch_fp32(gpu, qmax):
    from dlq_amd.models import ResNet18Int8
    sd = resnet18_state_dict(SEED)
    x = synthetic_images(4, seed=SEED + 1)
    ref = calibrate_resnet18(sd, x, device="cpu", qmax=qmax)
    m = ResNet18Int8(sd, {s: 1.0 for s in site_names()}, max_batch=8,
                     precision="fp8" if qmax == 448.0 else "int8")
    m.calibrate(x.cuda().contiguous(), qmax)
    got = m.scale_dict()
    assert set(got) == set(ref)
    for s in ref:
        assert got[s] == pytest.approx(ref[s], rel=1e-4), s
    # the engine runs with them: a forward after calibrate gives finite logits
    out = m.forward(x.cuda().contiguous())
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
