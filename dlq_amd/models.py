"""Model-level host code: synthetic weights, the fp32 torch definitions used for
calibration and the CPU baseline, and the int8 engines over the C ABI.

ResNet-18 topology = torchvision BasicBlock ResNet-18, as loaded by the
reference (tools/export_resnet18.py:62, DeepLearning/CheckFeaturemap/
resnet18_feat.py:95-103) and wired by runtime/infer_e2e.cu:259-433.
torchvision is not installed and pretrained weights cannot be fetched, so the
fp32 network is defined here with plain torch.nn and seeded weights.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# (name, in_c, out_c, stride, downsample) -- infer_e2e.cu:336-407
BLOCKS = [
    ("layer1.0", 64, 64, 1, False), ("layer1.1", 64, 64, 1, False),
    ("layer2.0", 64, 128, 2, True), ("layer2.1", 128, 128, 1, False),
    ("layer3.0", 128, 256, 2, True), ("layer3.1", 256, 256, 1, False),
    ("layer4.0", 256, 512, 2, True), ("layer4.1", 512, 512, 1, False),
]
IMAGENET_MEAN = (0.485, 0.456, 0.406)  # tools/export_resnet18.py:73-78
IMAGENET_STD = (0.229, 0.224, 0.225)


def conv_sites():
    """Activation-scale sites of the int8 net, in forward order."""
    s = ["input", "conv1"]
    for name, _, _, _, ds in BLOCKS:
        s.append(f"{name}.conv1")
        if ds:
            s.append(f"{name}.downsample")
        s.append(f"{name}.conv2")
    s.append("gap")
    return s


def _bn_params(g: torch.Generator, c: int):
    return {
        "weight": torch.rand(c, generator=g) + 0.5,             # gamma ~ U(0.5, 1.5)
        "bias": (torch.rand(c, generator=g) - 0.5) * 0.2,      # beta  ~ U(-0.1, 0.1)
        "running_mean": torch.randn(c, generator=g) * 0.1,     # mu    ~ N(0, 0.1)
        "running_var": torch.rand(c, generator=g) + 0.5,       # var   ~ U(0.5, 1.5)
    }


def resnet18_state_dict(seed: int = 0x20260306) -> dict[str, np.ndarray]:
    """Seeded synthetic ResNet-18 weights with torchvision's state_dict names
    (Kaiming-normal fan_out convs as torchvision initialises them; BN
    parameters drawn so every per-channel epilogue is non-trivial)."""
    g = torch.Generator().manual_seed(seed)
    sd: dict[str, torch.Tensor] = {}

    def conv(name, oc, ic, k):
        std = (2.0 / (oc * k * k)) ** 0.5
        sd[name] = torch.randn(oc, ic, k, k, generator=g) * std

    def bn(prefix, c):
        for k, v in _bn_params(g, c).items():
            sd[f"{prefix}.{k}"] = v

    conv("conv1.weight", 64, 3, 7)
    bn("bn1", 64)
    for name, ic, oc, _, ds in BLOCKS:
        conv(f"{name}.conv1.weight", oc, ic, 3)
        bn(f"{name}.bn1", oc)
        conv(f"{name}.conv2.weight", oc, oc, 3)
        bn(f"{name}.bn2", oc)
        if ds:
            conv(f"{name}.downsample.0.weight", oc, ic, 1)
            bn(f"{name}.downsample.1", oc)
    bound = 1.0 / 512 ** 0.5
    sd["fc.weight"] = (torch.rand(1000, 512, generator=g) * 2 - 1) * bound
    sd["fc.bias"] = (torch.rand(1000, generator=g) * 2 - 1) * bound
    return {k: v.float().numpy() for k, v in sd.items()}


def site_names() -> list[str]:
    """The 22 activation-scale sites of the int8 scheme, in
    forward order: input, conv1, each block's conv1 / downsample / conv2, gap."""
    out = ["input", "conv1"]
    for name, _, _, _, ds in BLOCKS:
        out += [f"{name}.conv1"] + ([f"{name}.downsample"] if ds else []) + [f"{name}.conv2"]
    return out + ["gap"]


def synthetic_images(n: int, seed: int = 0x20260306, device="cpu") -> torch.Tensor:
    """Seeded u8 pixels ~ U{0..255} normalised like tools/preprocess_to_bin.py:24-33
    ((p/255 - mean)/std) -> fp32 NCHW [n,3,224,224]."""
    g = torch.Generator().manual_seed(seed)
    p = torch.randint(0, 256, (n, 3, 224, 224), generator=g, dtype=torch.uint8).float() / 255.0
    mean = torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
    return ((p - mean) / std).to(device)


# ---------------------------------------------------------------- fp32 torch

class BasicBlock(nn.Module):
    def __init__(self, ic, oc, stride, down):
        super().__init__()
        self.conv1 = nn.Conv2d(ic, oc, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(oc)
        self.conv2 = nn.Conv2d(oc, oc, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(oc)
        self.downsample = (nn.Sequential(nn.Conv2d(ic, oc, 1, stride, bias=False), nn.BatchNorm2d(oc))
                           if down else None)

    def forward(self, x):
        h = F.relu(self.bn1(self.conv1(x)))
        o = self.bn2(self.conv2(h))
        skip = self.downsample(x) if self.downsample is not None else x
        return F.relu(o + skip)


class TorchResNet18(nn.Module):
    """fp32 ResNet-18 (torchvision topology) -- calibration + CPU baseline."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        layers = {}
        for name, ic, oc, s, ds in BLOCKS:
            layers.setdefault(name.split(".")[0], []).append(BasicBlock(ic, oc, s, ds))
        for k, v in layers.items():
            setattr(self, k, nn.Sequential(*v))
        self.fc = nn.Linear(512, 1000)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def torch_resnet18(sd: dict[str, np.ndarray], device="cpu") -> TorchResNet18:
    m = TorchResNet18()
    tsd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}
    missing, unexpected = m.load_state_dict(tsd, strict=False)
    if unexpected or any(not k.endswith("num_batches_tracked") for k in missing):
        raise KeyError(f"state_dict mismatch: missing={missing} unexpected={unexpected}")
    return m.eval().to(device)


# ---------------------------------------------------------------- int8 engines

class ResNet18Int8:
    """dlq_resnet18 engine (C ABI): weights quantised/folded/resident once,
    forward = 16 launches on the current stream (stem, 2 fused layer1 blocks, 3 stride-2 + downsample, 9 wide convs, fused GAP+FC), no host sync."""

    def __init__(self, sd: dict[str, np.ndarray], scales: dict[str, float], max_batch: int,
                 keep_stages: bool = False, precision: str = "int8"):
        from .lib import check, lib
        self._lib, self._check = lib, check
        h = C.c_void_p()
        check(lib.dlq_resnet18_create(C.byref(h)), "resnet18_create")
        self.h = h
        for name, arr in sd.items():
            a = np.ascontiguousarray(arr, np.float32)
            check(lib.dlq_resnet18_set_tensor(h, name.encode(), a.ctypes.data, a.size), f"set_tensor {name}")
        for site, s in scales.items():
            check(lib.dlq_resnet18_set_scale(h, site.encode(), float(s)), f"set_scale {site}")
        check(lib.dlq_resnet18_set_keep_stages(h, int(keep_stages)), "keep_stages")
        if precision not in ("int8", "fp8"):
            raise ValueError("precision must be 'int8' or 'fp8'")
        self.precision = precision
        check(lib.dlq_resnet18_set_precision(h, 1 if precision == "fp8" else 0), "set_precision")
        check(lib.dlq_resnet18_prepare(h, max_batch, None), "resnet18_prepare")
        self.max_batch = max_batch

    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        from .lib import stream_handle
        if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.shape[1:] == (3, 224, 224)):
            raise TypeError("x must be a contiguous CUDA fp32 [B,3,224,224] tensor")
        B = x.shape[0]
        if out is None:
            out = torch.empty((B, 1000), dtype=torch.float32, device=x.device)
        self._check(self._lib.dlq_resnet18_forward(self.h, x.data_ptr(), B, out.data_ptr(), stream_handle()),
                    "resnet18_forward")
        return out

    __call__ = forward

    def stage(self, name: str, shape) -> torch.Tensor:
        from .lib import stream_handle
        nb = C.c_size_t()
        self._check(self._lib.dlq_resnet18_stage(self.h, name.encode(), None, 0, C.byref(nb), None), "stage")
        t = torch.empty(int(nb.value), dtype=torch.int8, device="cuda")
        self._check(self._lib.dlq_resnet18_stage(self.h, name.encode(), t.data_ptr(), t.numel(), C.byref(nb),
                                                 stream_handle()), "stage")
        return t.view(*shape)

    def forward_f32(self, x: torch.Tensor) -> torch.Tensor:
        """The reference's fp32 forward op for op on the GPU
        (dlq_resnet18_forward_f32): logits [B,1000] fp32."""
        from .lib import stream_handle
        if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.shape[1:] == (3, 224, 224)):
            raise TypeError("x must be a contiguous CUDA fp32 [B,3,224,224] tensor")
        out = torch.empty((x.shape[0], 1000), dtype=torch.float32, device=x.device)
        self._check(self._lib.dlq_resnet18_forward_f32(self.h, x.data_ptr(), x.shape[0], out.data_ptr(),
                                                       stream_handle()), "resnet18_forward_f32")
        return out

    def stage_f32(self, name: str) -> torch.Tensor:
        """fp32 NCHW stage of the last forward_f32 (flat)."""
        nb = C.c_size_t()
        self._check(self._lib.dlq_resnet18_stage_f32(self.h, name.encode(), None, 0, C.byref(nb), None), "stage_f32")
        t = torch.empty(int(nb.value) // 4, dtype=torch.float32, device="cuda")
        self._check(self._lib.dlq_resnet18_stage_f32(self.h, name.encode(), t.data_ptr(), int(nb.value), C.byref(nb),
                                                     None), "stage_f32")
        torch.cuda.synchronize()
        return t

    def calibrate(self, x: torch.Tensor, qmax: float = 127.0) -> None:
        """Set every activation scale from the GPU fp32 reference forward over
        x (dlq_resnet18_calibrate) and prepare again."""
        from .lib import stream_handle
        if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.shape[1:] == (3, 224, 224)):
            raise TypeError("x must be a contiguous CUDA fp32 [B,3,224,224] tensor")
        self._check(self._lib.dlq_resnet18_calibrate(self.h, x.data_ptr(), x.shape[0], float(qmax), stream_handle()),
                    "resnet18_calibrate")
        self._check(self._lib.dlq_resnet18_prepare(self.h, self.max_batch, None), "resnet18_prepare")

    def scales(self, path: str) -> None:
        """Write the current activation scales (dlq_resnet18_load_scales format)."""
        self._check(self._lib.dlq_resnet18_save_scales(self.h, path.encode()), "save_scales")

    def scale_dict(self) -> dict[str, float]:
        """The current activation scales as {site: scale} (through save_scales' text)."""
        import os
        import tempfile
        fd, path = tempfile.mkstemp(suffix=".txt")
        os.close(fd)
        try:
            self.scales(path)
            out = {}
            for line in open(path):
                parts = line.split()
                if len(parts) == 2 and not line.startswith("#"):
                    out[parts[0]] = float(parts[1])
            return out
        finally:
            os.unlink(path)

    def set_timing(self, on: bool):
        self._check(self._lib.dlq_resnet18_set_timing(self.h, int(on)), "set_timing")

    def timing(self):
        """Per kernel family (lib.FAMILIES): (summed ms, launches), and the
        forwards covered since set_timing / the last call."""
        ms = (C.c_double * 8)()
        nl = (C.c_int * 8)()
        nf = C.c_int()
        self._check(self._lib.dlq_resnet18_timing(self.h, ms, nl, C.byref(nf)), "timing")
        return list(ms), list(nl), nf.value

    def family_work(self):
        """Per kernel family: (algorithmic MACs, activation bytes) per image and forward."""
        macs = (C.c_double * 8)()
        nbytes = (C.c_double * 8)()
        self._check(self._lib.dlq_resnet18_family_work(self.h, macs, nbytes), "family_work")
        return list(macs), list(nbytes)

    def macs_per_image(self):
        cm, fm = C.c_double(), C.c_double()
        self._check(self._lib.dlq_resnet18_macs_per_image(self.h, C.byref(cm), C.byref(fm)), "macs")
        return cm.value, fm.value

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self._lib.dlq_resnet18_destroy(h)
            self.h = None


class MLPInt8:
    """dlq_mlp engine: X[B,in] fp32 -> int8 -> FC+bias+ReLU -> int8 -> FC+bias -> fp32."""

    def __init__(self, W1, b1, W2, b2, s_in: float, s_hidden: float, max_batch: int):
        from .lib import check, lib
        self._lib, self._check = lib, check
        W1 = np.ascontiguousarray(W1, np.float32); W2 = np.ascontiguousarray(W2, np.float32)
        b1 = np.ascontiguousarray(b1, np.float32); b2 = np.ascontiguousarray(b2, np.float32)
        self.inp, self.hidden = W1.shape
        self.out = W2.shape[1]
        h = C.c_void_p()
        check(lib.dlq_mlp_create(self.inp, self.hidden, self.out, W1.ctypes.data, b1.ctypes.data,
                                 W2.ctypes.data, b2.ctypes.data, float(s_in), float(s_hidden), max_batch,
                                 None, C.byref(h)), "mlp_create")
        self.h = h

    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        from .lib import stream_handle
        if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()):
            raise TypeError("x must be a contiguous CUDA fp32 tensor")
        B = x.shape[0]
        if out is None:
            out = torch.empty((B, self.out), dtype=torch.float32, device=x.device)
        self._check(self._lib.dlq_mlp_forward(self.h, x.data_ptr(), B, out.data_ptr(), stream_handle()),
                    "mlp_forward")
        return out

    __call__ = forward

    def hidden_q(self, B: int) -> torch.Tensor:
        """int8 hidden activations [B, hidden] of the last forward (copied)."""
        from .lib import stream_handle
        t = torch.empty((B, self.hidden), dtype=torch.int8, device="cuda")
        self._check(self._lib.dlq_mlp_copy_hidden(self.h, B, t.data_ptr(), t.numel(), stream_handle()),
                    "mlp_copy_hidden")
        return t

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self._lib.dlq_mlp_destroy(h)
            self.h = None


def mlp_weights(inp=784, hidden=256, out=10, seed=12345):
    """He-uniform weights as v5.cu:85-90 / v4.cu:95-100 draw them
    (scale = sqrt(2/fan_in), U(-scale, scale)), [in][out] layout, zero bias
    (v4.cu:102-107); seeded numpy instead of glibc rand()."""
    rng = np.random.default_rng(seed)
    s1 = np.float32(np.sqrt(2.0 / inp)); s2 = np.float32(np.sqrt(2.0 / hidden))
    W1 = (rng.random((inp, hidden), dtype=np.float32) * 2 * s1 - s1).astype(np.float32)
    W2 = (rng.random((hidden, out), dtype=np.float32) * 2 * s2 - s2).astype(np.float32)
    b1 = (rng.random(hidden, dtype=np.float32) * 0.02 - 0.01).astype(np.float32)
    b2 = (rng.random(out, dtype=np.float32) * 0.02 - 0.01).astype(np.float32)
    return W1, b1, W2, b2


# ------------------------------------------------------- MNIST fp32 CPU path

class MNISTMLP(nn.Module):
    """BASELINE configs[0]: the reference's 2-layer MLP in PyTorch on the CPU
    (CUDA/MNIST_on_GPU/v1.py:35-47: fc1 -> ReLU -> fc2, 784 -> hidden -> 10),
    built from [in][out] weights as the reference's C/CUDA versions store
    them (v4.cu:95-107; nn.Linear keeps [out][in], hence the transposes).
    The plumbing baseline beside the int8 MLP on the GPU (MLPInt8); not part
    of the int8 engine."""

    def __init__(self, W1, b1, W2, b2):
        super().__init__()
        inp, hidden = W1.shape
        out = W2.shape[1]
        self.fc1 = nn.Linear(inp, hidden)
        self.relu = nn.ReLU()
        self.fc2 = nn.Linear(hidden, out)
        with torch.no_grad():
            self.fc1.weight.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(W1, np.float32).T)))
            self.fc1.bias.copy_(torch.from_numpy(np.asarray(b1, np.float32)))
            self.fc2.weight.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(W2, np.float32).T)))
            self.fc2.bias.copy_(torch.from_numpy(np.asarray(b2, np.float32)))

    def forward(self, x):
        x = x.reshape(x.shape[0], -1)  # v1.py:43 (x.reshape(batch_size, 28 * 28))
        return self.fc2(self.relu(self.fc1(x)))


def mnist_inputs(B: int, seed: int = 7) -> np.ndarray:
    """Synthetic MNIST-shaped batch [B,784]: seeded u8 pixels /255, normalised
    with the reference's mean/std (v1.py:21-24); the data files are absent."""
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 256, size=(B, 784), dtype=np.uint8).astype(np.float32) / np.float32(255.0)
    return ((x - np.float32(0.1307)) / np.float32(0.3081)).astype(np.float32)
