"""The C++ launcher (bin/dlq_e2e, the reference's step8_e2e main,
RK/runtime/infer_e2e.cu:230-441) end to end on the GPU: manifest directory in
the reference's export format (fp32, and the int8 variant) -> forward ->
stdout top-1 line (:436-438) and the seven --dump_dir checkpoints
(:243-248), compared with the oracle: int8 stages dequantised exactly as the
launcher does (float(q) * scale), logits bit-exact; tools/diag_compare.py
(diag_e2e_compare.py's metrics) reports zero difference."""
import os
import re
import subprocess

import numpy as np
import pytest

from dlq_amd.manifest import Manifest
from oracle import oracle as O
from tools.diag_compare import CKPTS, compare
from tools.export_manifest import export

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SITES = {"stem_pool": "conv1", "layer1": "layer1.1.conv2", "layer2": "layer2.1.conv2",
         "layer3": "layer3.1.conv2", "layer4": "layer4.1.conv2", "gap": "gap"}


def _run(d, dump):
    exe = os.path.join(ROOT, "bin", "dlq_e2e")
    r = subprocess.run([exe, "--manifest", d, "--input", os.path.join(d, "input.bin"),
                        "--scales", os.path.join(d, "scales.txt"), "--dump_dir", dump],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"\[E2E\] top-1 class index = (-?\d+), logit=(\S+)", r.stdout)
    assert m, r.stdout
    return int(m.group(1)), float(m.group(2))


@pytest.mark.parametrize("int8", [False, True], ids=["fp32_manifest", "int8_manifest"])
def test_launcher_dumps_match_oracle(gpu, tmp_path, int8):
    d = str(tmp_path / "mani")
    sd, scales, x = export(d)
    if int8:  # re-write the same weights as an int8 manifest (+ the same scales and input)
        q8 = str(tmp_path / "mani8")
        Manifest.load(d).save(q8, int8=True)
        for f in ("scales.txt", "input.bin"):
            os.replace(os.path.join(d, f), os.path.join(q8, f))
        d = q8
    dump = str(tmp_path / "dump")
    top, logit = _run(d, dump)
    ref_logits, dumps = O.resnet18_forward_s8(sd, scales, x)
    for stage, site in SITES.items():
        got = np.fromfile(os.path.join(dump, stage + ".bin"), np.float32)
        ref = (dumps[stage][0].astype(np.float32) * np.float32(scales[site])).reshape(-1)
        assert np.array_equal(got.view(np.int32), ref.view(np.int32)), stage
    got = np.fromfile(os.path.join(dump, "logits.bin"), np.float32)
    assert np.array_equal(got.view(np.int32), ref_logits[0].view(np.int32))
    idx, val = O.top1(ref_logits[:1])
    assert top == idx[0] and logit == pytest.approx(float(val[0]), rel=1e-5)  # printed %g (6 digits), as the reference
    # the reference's comparison tool over the launcher's dumps and the oracle's
    ref_dir = tmp_path / "ref"
    ref_dir.mkdir()
    for stage, site in SITES.items():
        (dumps[stage][0].astype(np.float32) * np.float32(scales[site])).astype(np.float32).tofile(ref_dir / (stage + ".bin"))
    ref_logits[0].astype(np.float32).tofile(ref_dir / "logits.bin")
    for name, (mx, mn, cs) in compare(str(ref_dir), dump).items():
        assert mx == 0.0 and mn == 0.0, name


# The reference harness's call and parse (RKT/bench_fp32_vs_torch_e2e.py:51,105)
TOP1_RE = re.compile(r"top-1 class index\s*=\s*(\d+)")


def _exe(args, tmp_path=None):
    r = subprocess.run([os.path.join(ROOT, "bin", "dlq_e2e")] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r


def test_launcher_reference_argv(gpu, tmp_path):
    """Exactly the argv the reference harness builds: --manifest DIR --input X
    (no --scales): the launcher reads DIR/scales.txt, the harness's TOP1_RE
    parses its stdout, and top-1 equals the oracle's."""
    d = str(tmp_path / "mani")
    sd, scales, x = export(d)
    r = _exe(["--manifest", d, "--input", os.path.join(d, "input.bin")])
    m = TOP1_RE.search(r.stdout)
    assert m, r.stdout
    ref_logits, _ = O.resnet18_forward_s8(sd, scales, x)
    assert int(m.group(1)) == O.top1(ref_logits[:1])[0][0]


def test_launcher_calibrates_without_scales(gpu, tmp_path):
    """No --scales and no scales.txt: the launcher calibrates on the input with
    the reference-semantics fp32 forward on the GPU.  The scales equal the
    oracle's fp32 forward (resnet18_forward_f32, record hook) amax / 127 bit
    for bit, and the int8 logits equal the oracle's int8 forward with them."""
    d = str(tmp_path / "mani")
    sd, _, x = export(d)
    os.remove(os.path.join(d, "scales.txt"))
    dump, sc_path = str(tmp_path / "dump"), str(tmp_path / "cal.txt")
    r = _exe(["--manifest", d, "--input", os.path.join(d, "input.bin"), "--dump_dir", dump, "--save_scales", sc_path])
    assert "calibrated" in r.stderr
    amax = {"input": float(np.abs(x).max())}

    def rec(name, t):
        amax[name] = max(amax.get(name, 0.0), float(np.abs(t).max()))
    O.resnet18_forward_f32(sd, x[0], record=rec)
    want = {k: float(np.float32(max(v, 1e-8) / 127.0)) for k, v in amax.items()}
    from dlq_amd.quant import load_scales
    got = load_scales(sc_path)
    assert set(got) == set(want)
    for k in want:
        assert np.float32(got[k]) == np.float32(want[k]), k
    ref_logits, _ = O.resnet18_forward_s8(sd, got, x)
    lg = np.fromfile(os.path.join(dump, "logits.bin"), np.float32)
    assert np.array_equal(lg.view(np.int32), ref_logits[0].view(np.int32))


def test_launcher_fp32_reference_semantics(gpu, tmp_path):
    """--fp32: the reference's own fp32 forward (im2col-ordered fmaf GEMM, BN,
    pool, GAP tree, FC + host bias) on the GPU: every dump and the logits are
    bit-identical to the oracle's fp32 restatement, which the reference's
    golden out/step8_logits.bin pins (tests/test_oracle.py)."""
    d = str(tmp_path / "mani")
    sd, _, x = export(d)
    dump = str(tmp_path / "dump")
    r = _exe(["--manifest", d, "--input", os.path.join(d, "input.bin"), "--dump_dir", dump, "--fp32"])
    ref_logits, dumps = O.resnet18_forward_f32(sd, x[0])
    for stage in ("stem_pool", "layer1", "layer2", "layer3", "layer4", "gap", "logits"):
        got = np.fromfile(os.path.join(dump, stage + ".bin"), np.float32)
        assert np.array_equal(got.view(np.int32), np.ascontiguousarray(dumps[stage], np.float32).reshape(-1).view(np.int32)), stage
    top = int(TOP1_RE.search(r.stdout).group(1))
    assert top == int(np.argmax(ref_logits))
