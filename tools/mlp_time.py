"""configs[1] timing only (MNIST int8 784x128x10, B = 1024, dlq_mlp_*): the
bench's graph-replay device time per forward and bit-exactness against the
first library given (A/B of libdlq.so builds: each in its own process,
DLQ_LIB_PATH).  python tools/mlp_time.py [LIB ...]   ('base' = in-tree)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import hashlib, json, sys, torch
sys.path.insert(0, ROOT)
import bench
from dlq_amd.models import MLPInt8, mlp_weights, mnist_inputs
from dlq_amd.quant import calibrate_mlp
dev = torch.device("cuda")
W1, b1, W2, b2 = mlp_weights(hidden=128)
xs = mnist_inputs(1024)
s_in, s_h = calibrate_mlp(W1, b1, xs)
mlp = MLPInt8(W1, b1, W2, b2, s_in, s_h, max_batch=1024)
xd = torch.from_numpy(xs).to(dev)
yd = torch.empty((1024, 10), dtype=torch.float32, device=dev)
for _ in range(20):
    mlp.forward(xd, yd)
g, reps = torch.cuda.CUDAGraph(), 50
with torch.cuda.graph(g):
    for _ in range(reps):
        mlp.forward(xd, yd)
best = min(bench.timed_cuda(g.replay, 20) / reps for _ in range(5))
mlp.forward(xd, yd); torch.cuda.synchronize()
print("MLPJSON " + json.dumps({"us_per_forward": round(best * 1e3, 3),
      "digest": hashlib.sha256(yd.cpu().numpy().tobytes()).hexdigest()[:16]}), flush=True)
"""


def main():
    libs = sys.argv[1:] or ["base"]
    code = CHILD.replace("ROOT", repr(ROOT))
    for r in range(3):
        for lib in libs:
            env = dict(os.environ)
            if lib != "base":
                env["DLQ_LIB_PATH"] = os.path.abspath(lib)
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            line = [l for l in p.stdout.splitlines() if l.startswith("MLPJSON ")]
            if p.returncode != 0 or not line:
                print(f"{lib}: FAILED\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            print(f"round {r} {lib:30s} {line[0][8:]}", flush=True)


if __name__ == "__main__":
    main()
