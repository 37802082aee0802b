"""Probe (measurement tooling): per-forward device time of the int8 ResNet-18
forward (B=256) from an idle GPU -- 60 forwards back to back, hipEvents
around each -- after a given pre-phase: none, the GPU fp32 calibration over
32 images, or 100 ms of sleep.  Shows how many forwards the clock needs.
python tools/ramp_probe.py [pre]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dlq_amd.models import ResNet18Int8, resnet18_state_dict, site_names, synthetic_images  # noqa: E402

pre = sys.argv[1] if len(sys.argv) > 1 else "none"
sd = resnet18_state_dict(0x20260306)
m = ResNet18Int8(sd, {s: 1.0 for s in site_names()}, max_batch=256)
dev = torch.device("cuda")
x = synthetic_images(256).to(dev).contiguous()
out = torch.empty((256, 1000), device=dev)
m.calibrate(x[:32].contiguous())
m.forward(x, out)
torch.cuda.synchronize()
time.sleep(2.0)  # idle, like the bench's setup before its warmup
if pre == "cal":
    m.calibrate(x[:32].contiguous())
    torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(61)]
ev[0].record()
for i in range(60):
    m.forward(x, out)
    ev[i + 1].record()
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(60)]
print(pre, "per-forward ms:", " ".join(f"{v:.3f}" for v in ms))
print(pre, "mean of 1-5: %.3f  6-25: %.3f  26-60: %.3f" % (sum(ms[:5]) / 5, sum(ms[5:25]) / 20, sum(ms[25:]) / 35))
