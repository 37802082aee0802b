"""A/B timing of libdlq.so builds on one GPU box (kernel work, not product).

usage: python tools/ab.py [--rounds 3] [--steps 20] LIB [LIB ...]
Each LIB is a libdlq.so path (tools/build_variant.sh); 'base' = the in-tree
dlq_amd/libdlq.so; LIB@VAR=VAL runs it with VAR=VAL in the environment (a
knob's variable, e.g. base@DLQ_DS_SPLIT=1 or base@DLQ_HEAD_SPLIT=1).  Every round runs each build in its own process (the
library is chosen with DLQ_LIB_PATH), in rotating order, and prints the
forward time and the per-family launch averages (hipEvents, rescaled to the
timed forward as bench.py does).  With --check the first build's logits are
compared bit for bit against every other build's (same inputs).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# environment variables libdlq.so reads (capi.cpp knobs) or the child reads
KNOWN_VARS = {"DLQ_L1_GRID", "DLQ_HEAD_SPLIT", "DLQ_GRAPH", "DLQ_GEMM_TILE", "DLQ_DS_SPLIT", "DLQ_PREFETCH", "DLQ_GAP_EPI", "DLQ_LIB_PATH"}

CHILD = r"""
import json, os, sys, time, torch, numpy as np
sys.path.insert(0, ROOT)
from dlq_amd.lib import FAMILIES
from dlq_amd.models import ResNet18Int8, resnet18_state_dict, synthetic_images
from dlq_amd.quant import calibrate_resnet18
SEED = 0x20260306
B, steps = BATCH, STEPS
sd = resnet18_state_dict(SEED)
prec = PREC
scales = calibrate_resnet18(sd, synthetic_images(2, seed=SEED + 1), device="cpu", qmax=448.0 if prec == "fp8" else 127.0)
m = ResNet18Int8(sd, scales, max_batch=B, precision=prec)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(SEED + 1000)
pix = torch.randint(0, 256, (B, 3, 224, 224), generator=g, device=dev, dtype=torch.uint8)
mean = torch.tensor([0.485, 0.456, 0.406], device=dev).view(1, 3, 1, 1)
std = torch.tensor([0.229, 0.224, 0.225], device=dev).view(1, 3, 1, 1)
x = ((pix.float() / 255.0 - mean) / std).contiguous()
out = torch.empty((B, 1000), dtype=torch.float32, device=dev)
for _ in range(5):
    m.forward(x, out)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    m.forward(x, out)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
m.set_timing(True)
for _ in range(10):
    m.forward(x, out)
fam_ms, fam_n, n_fwd = m.timing()
m.set_timing(False)
ev = sum(fam_ms) / max(n_fwd, 1)
sc = min(1.0, dt * 1e3 / ev) if ev > 0 else 1.0
fam = {FAMILIES[f].split(" ")[0]: round(fam_ms[f] * sc * 1e3 / fam_n[f], 2) for f in range(len(FAMILIES)) if fam_n[f]}
digest = None
if CHECK:
    import hashlib
    m.forward(x, out); torch.cuda.synchronize()
    digest = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
print("ABJSON " + json.dumps({"ms": round(dt * 1e3, 4), "img_s": round(B / dt, 1), "fam_us": fam, "digest": digest}), flush=True)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--precision", default="int8")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("libs", nargs="+")
    args = ap.parse_args()
    code = (CHILD.replace("ROOT", repr(ROOT)).replace("BATCH", str(args.batch)).replace("STEPS", str(args.steps))
            .replace("PREC", repr(args.precision)).replace("CHECK", str(bool(args.check))))
    res = {l: [] for l in args.libs}
    for r in range(args.rounds):
        order = args.libs[r % len(args.libs):] + args.libs[:r % len(args.libs)]
        for lib in order:
            env = dict(os.environ)
            path, _, kv = lib.partition("@")
            if kv:
                k, _, v = kv.partition("=")
                if k not in KNOWN_VARS:
                    print(f"warning: {k} is not a libdlq knob variable ({', '.join(sorted(KNOWN_VARS))}): "
                          f"{lib} runs with it set but nothing reads it", flush=True)
                env[k] = v
            if path != "base":
                env["DLQ_LIB_PATH"] = os.path.abspath(path)
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            line = [l for l in p.stdout.splitlines() if l.startswith("ABJSON ")]
            if p.returncode != 0 or not line:
                print(f"{lib}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            d = json.loads(line[0][7:])
            res[lib].append(d)
            print(f"round {r} {lib:40s} {d['ms']:.4f} ms {d['img_s']:9.1f} img/s {d['fam_us']} {d['digest'] or ''}",
                  flush=True)
    print("---- best of rounds (min ms) ----")
    for lib, ds in res.items():
        best = min(ds, key=lambda d: d["ms"])
        fams = {}
        for k in best["fam_us"]:
            fams[k] = min(d["fam_us"][k] for d in ds)
        print(f"{lib:40s} {best['ms']:.4f} ms {best['img_s']:9.1f} img/s  fam(min) {fams}")
    if args.check:
        dg = {lib: {d["digest"] for d in ds} for lib, ds in res.items()}
        ref = dg[args.libs[0]]
        for lib, s in dg.items():
            print(f"digest {lib}: {sorted(s)} {'SAME' if s == ref and len(s) == 1 else 'DIFFERENT'}")


if __name__ == "__main__":
    main()
