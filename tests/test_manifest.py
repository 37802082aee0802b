"""Weight manifest I/O and the stage-dump comparison
tool (row 2), host side: the engine's reader / writer through the C ABI in
the reference's export format (tools/export_resnet18.py:57-113; read back by
load_bin_f32, RK/include/utils.hpp:48-60), its int8 variant, and the
diag_e2e_compare.py:5-40 metrics.  No GPU needed (nothing is prepared)."""
import filecmp
import json
import os

import numpy as np
import pytest

from dlq_amd.manifest import Manifest
from oracle import oracle as O
from tools.diag_compare import CKPTS, compare, metrics
from tools.export_manifest import export


@pytest.fixture(scope="module")
def exported(tmp_path_factory):
    d = tmp_path_factory.mktemp("mani_fp32")
    sd, scales, x = export(str(d))
    return str(d), sd, scales, x


def _same_dirs(a, b, names):
    for n in names:
        assert filecmp.cmp(os.path.join(a, n), os.path.join(b, n), shallow=False), n


def test_fp32_manifest_reference_layout(exported):
    d, sd, _, x = exported
    j = json.load(open(os.path.join(d, "manifest.json")))
    assert j["dtype"] == "fp32" and j["layout"] == "NCHW" and j["model"] == "resnet18"
    t = j["tensors"]
    assert t["conv1.weight"] == {"shape": [64, 3, 7, 7], "layout": "OIHW", "kind": "conv_weight",
                                 "path": "conv1.weight.bin"}
    assert t["fc.weight"]["layout"] == "OI" and t["bn1.running_var"]["kind"] == "bn_buffer"
    for name, meta in t.items():  # raw fp32, C order, exactly the state_dict tensor
        a = np.fromfile(os.path.join(d, meta["path"]), np.float32)
        assert np.array_equal(a, np.ascontiguousarray(sd[name], np.float32).reshape(-1)), name
    assert np.fromfile(os.path.join(d, "input.bin"), np.float32).size == 3 * 224 * 224


def test_fp32_roundtrip_and_bare_directory(exported, tmp_path):
    d, sd, _, _ = exported
    m = Manifest.load(d, os.path.join(d, "scales.txt"))
    m.save(str(tmp_path / "again"))
    names = [f for f in os.listdir(d) if f.endswith(".bin") and f != "input.bin"] + ["manifest.json"]
    _same_dirs(d, str(tmp_path / "again"), names)
    os.remove(tmp_path / "again" / "manifest.json")  # a bare directory of .bin files reads as fp32
    Manifest.load(str(tmp_path / "again")).save(str(tmp_path / "third"))
    _same_dirs(d, str(tmp_path / "third"), names)


def test_int8_manifest_equals_quantising_fp32(exported, tmp_path):
    d, sd, _, _ = exported
    q8 = str(tmp_path / "int8")
    Manifest.load(d).save(q8, int8=True)
    j = json.load(open(os.path.join(q8, "manifest.json")))
    assert j["dtype"] == "int8"
    for name in ("conv1.weight", "layer3.0.downsample.0.weight", "fc.weight"):
        meta = j["tensors"][name]
        assert meta["dtype"] == "int8" and meta["scale_path"] == name + ".scale.bin"
        q = np.fromfile(os.path.join(q8, name + ".bin"), np.int8)
        s = np.fromfile(os.path.join(q8, name + ".scale.bin"), np.float32)
        rq, rs = O.quantize_weights_s8(sd[name])
        assert np.array_equal(q, rq.reshape(-1)) and np.array_equal(s, rs), name
    assert np.array_equal(np.fromfile(os.path.join(q8, "bn1.weight.bin"), np.float32), sd["bn1.weight"])
    # int8 manifest -> engine -> int8 manifest: byte-identical
    Manifest.load(q8).save(str(tmp_path / "int8b"), int8=True)
    _same_dirs(q8, str(tmp_path / "int8b"), os.listdir(q8))
    # weights held only as int8 cannot be written back as fp32
    with pytest.raises(RuntimeError, match="only held as int8"):
        Manifest.load(q8).save(str(tmp_path / "fp32b"))


def test_int8_manifest_rejects_bad_weights(exported, tmp_path):
    d, sd, _, _ = exported
    q8 = str(tmp_path / "int8")
    Manifest.load(d).save(q8, int8=True)
    q = np.fromfile(os.path.join(q8, "conv1.weight.bin"), np.int8)
    q[5] = -128
    q.tofile(os.path.join(q8, "conv1.weight.bin"))
    with pytest.raises(RuntimeError, match="-128"):
        Manifest.load(q8)
    q[5] = 0
    q.tofile(os.path.join(q8, "conv1.weight.bin"))
    os.remove(os.path.join(q8, "fc.weight.scale.bin"))
    with pytest.raises(RuntimeError, match="open fail"):
        Manifest.load(q8)


def test_diag_metrics_match_reference_definitions(tmp_path):
    rng = np.random.default_rng(1)
    a, b = (tmp_path / "a"), (tmp_path / "b")
    a.mkdir(); b.mkdir()
    for name, shape in CKPTS:
        x = rng.standard_normal(shape).astype(np.float32)
        x.tofile(a / name)
        (x + np.float32(0.25) * (name == "layer2.bin")).astype(np.float32).tofile(b / name)
    res = compare(str(a), str(b))
    for name, (mx, mn, cs) in res.items():
        if name == "layer2.bin":
            assert mx == pytest.approx(0.25) and mn == pytest.approx(0.25) and cs < 1.0
        else:
            assert (mx, mn) == (0.0, 0.0) and cs == pytest.approx(1.0)
    z = np.zeros(4, np.float32)
    assert metrics(z, z) == (0.0, 0.0, 0.0)  # diag_e2e_compare.py:19: cosine 0 for a zero vector
