"""Graph-replay floor for a one-launch forward: device time per replayed
launch of a near-empty kernel (zero-fill of configs[1]'s 1024 x 10 logits),
beside the MNIST forward (tools/mlp_time.py's measurement).
python tools/graph_floor.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

dev = torch.device("cuda")
yd = torch.empty((1024, 10), dtype=torch.float32, device=dev)
for _ in range(20):
    yd.zero_()
g, reps = torch.cuda.CUDAGraph(), 50
with torch.cuda.graph(g):
    for _ in range(reps):
        yd.zero_()
best = min(bench.timed_cuda(g.replay, 20) / reps for _ in range(5))
print(json.dumps({"graph_replay_us_per_empty_launch": round(best * 1e3, 3)}), flush=True)
