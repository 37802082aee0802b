"""bin/dlq_step, the per-step drivers (the reference's infer_conv1_bn1_relu /
infer_layerN / infer_head, RK/runtime/*.cu): the head step on the
reference's own after-layer4 fixture and logits (tests/golden: l4.bin,
step8_logits.bin, fc.weight/bias.bin), bit-exact with the oracle's int8 head
on the same grid and within the driver's int8 bar of the fp32 logits; the
engine steps on an exported manifest, bit-exact with the oracle's int8
forward (as --expect fixtures: max_abs 0) and within the bar of the
reference-semantics fp32 forward."""
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from tools.export_manifest import export

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
EXE = os.path.join(ROOT, "bin", "dlq_step")
DIFF_RE = re.compile(r"max_abs=(\S+) mean_abs=(\S+)")


def _step(args):
    r = subprocess.run([EXE] + args, capture_output=True, text=True, timeout=120)
    return r.returncode, r.stdout + r.stderr


def test_step_head_reference_fixture(gpu, tmp_path):
    out = str(tmp_path / "logits.bin")
    rc, log = _step(["--step", "head", "--manifest", GOLD, "--input", os.path.join(GOLD, "l4.bin"),
                     "--expect", os.path.join(GOLD, "step8_logits.bin"), "--out", out])
    assert rc == 0, log
    assert "Head done" in log and "[OK]" in log
    # the same int8 head in the oracle: grid max|x|/127, GAP k = 1/49, per-row FC weights
    l4 = np.fromfile(os.path.join(GOLD, "l4.bin"), np.float32).reshape(1, 512, 7, 7)
    s = np.float32(np.abs(l4).max()) / np.float32(127.0)
    q = O.quantize_f32_s8(l4, s)
    g, _ = O.gap_s8(q, np.float32(1.0) / np.float32(49.0))
    w = np.fromfile(os.path.join(GOLD, "fc.weight.bin"), np.float32).reshape(1000, 512)
    b = np.fromfile(os.path.join(GOLD, "fc.bias.bin"), np.float32)
    wq, sw = O.quantize_weights_s8(w)
    ref, _ = O.fc_s8(g, wq, O.fc_alpha(s, sw), b)
    got = np.fromfile(out, np.float32)
    assert np.array_equal(got.view(np.int32), ref[0].view(np.int32))
    # and the fp32 fixture's top-1
    fix = np.fromfile(os.path.join(GOLD, "step8_logits.bin"), np.float32)
    assert int(np.argmax(got)) == int(np.argmax(fix))


def test_step_head_fails_loudly_on_a_wrong_fixture(gpu, tmp_path):
    bad = tmp_path / "bad.bin"
    (-np.fromfile(os.path.join(GOLD, "step8_logits.bin"), np.float32)).tofile(bad)
    rc, log = _step(["--step", "head", "--manifest", GOLD, "--input", os.path.join(GOLD, "l4.bin"),
                     "--expect", str(bad)])
    assert rc == 2 and "[FAIL]" in log


SITES = {"stem": ("stem_pool", "conv1"), "layer1": ("layer1", "layer1.1.conv2"),
         "layer2": ("layer2", "layer2.1.conv2"), "layer3": ("layer3", "layer3.1.conv2"),
         "layer4": ("layer4", "layer4.1.conv2"), "gap": ("gap", "gap")}


@pytest.fixture(scope="module")
def manifest(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("mani"))
    sd, scales, x = export(d)
    _, dumps = O.resnet18_forward_s8(sd, scales, x)
    return d, scales, dumps


@pytest.mark.parametrize("step", list(SITES))
def test_step_engine_stage(gpu, manifest, tmp_path, step):
    d, scales, dumps = manifest
    stage, site = SITES[step]
    ref = (dumps[stage][0].astype(np.float32) * np.float32(scales[site])).reshape(-1)
    fix = tmp_path / "expect.bin"
    ref.astype(np.float32).tofile(fix)
    out = str(tmp_path / "out.bin")
    args = ["--step", step, "--manifest", d, "--input", os.path.join(d, "input.bin")]
    rc, log = _step(args + ["--expect", str(fix), "--out", out])
    assert rc == 0, log
    m = DIFF_RE.search(log)
    assert m and float(m.group(1)) == 0.0, log  # the oracle's int8 stage as the fixture: exact
    assert np.array_equal(np.fromfile(out, np.float32).view(np.int32), ref.view(np.int32))
    # without --expect: against the reference-semantics fp32 forward on the GPU
    rc, log = _step(args)
    assert rc == 0 and "fp32 reference forward" in log and "[OK]" in log, log
