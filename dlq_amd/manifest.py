"""Weight manifests in the reference's export format, host side only.

The reference exports a state_dict as <dir>/<name>.bin raw fp32 tensors plus
manifest.json (CUDA/resnet18-kernel-lab/tools/export_resnet18.py:57-113) and
its launcher reads them back with load_bin_f32 (RK/include/utils.hpp:48-60,
RK/runtime/infer_e2e.cu:262,304-334).  ``Manifest`` drives the engine's own
reader/writer through the C ABI (dlq_resnet18_load_manifest /
dlq_resnet18_save_manifest), including the int8 variant ("dtype": "int8":
conv / fc weights as int8 <name>.bin + fp32 per-output-channel
<name>.scale.bin) that ships pre-quantised weights.  No GPU is touched: the
engine is only created, filled and written (no dlq_resnet18_prepare).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .lib import check, lib


class Manifest:
    def __init__(self):
        h = C.c_void_p()
        check(lib.dlq_resnet18_create(C.byref(h)), "resnet18_create")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            lib.dlq_resnet18_destroy(self.h)
            self.h = None

    @classmethod
    def from_state_dict(cls, sd: dict[str, np.ndarray], scales: dict[str, float] | None = None) -> "Manifest":
        m = cls()
        for name, arr in sd.items():
            a = np.ascontiguousarray(arr, np.float32)
            check(lib.dlq_resnet18_set_tensor(m.h, name.encode(), a.ctypes.data, a.size), f"set_tensor {name}")
        for site, s in (scales or {}).items():
            check(lib.dlq_resnet18_set_scale(m.h, site.encode(), float(s)), f"set_scale {site}")
        return m

    @classmethod
    def load(cls, directory: str, scales_path: str | None = None) -> "Manifest":
        m = cls()
        check(lib.dlq_resnet18_load_manifest(m.h, os.fspath(directory).encode()), "load_manifest")
        if scales_path:
            check(lib.dlq_resnet18_load_scales(m.h, os.fspath(scales_path).encode()), "load_scales")
        return m

    def save(self, directory: str, int8: bool = False) -> None:
        check(lib.dlq_resnet18_save_manifest(self.h, os.fspath(directory).encode(), int(int8)), "save_manifest")

    def save_scales(self, path: str) -> None:
        check(lib.dlq_resnet18_save_scales(self.h, os.fspath(path).encode()), "save_scales")
