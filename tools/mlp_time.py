import sys, json, torch
sys.path.insert(0, '.')
import bench
print(json.dumps(bench.extra_configs(torch.device('cuda'))["configs[1] mnist_fc_int8_gpu"]))
