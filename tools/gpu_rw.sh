# layer2.0 resident-weight s2 kernel: s2 parity (int8 + fp8), e2e, bench A/B, torchrun world 1.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_f8.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/rw_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/rw_tests.log
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --cpu-baseline-images 0 --torch-cpu-images 0"
timeout -k 10 300 $B > gpurun_out/rw_bench.log 2>&1; rc=$?; echo "rw rc=$rc"; grep '^{"metric"' gpurun_out/rw_bench.log > gpurun_out/rw_bench.json; cut -c 1-200 gpurun_out/rw_bench.json
[ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/rw_bench.json'));[print(k,v) for k,v in d['kernels'].items()]"
DLQ_S2_RING=1 timeout -k 10 300 $B > gpurun_out/rw_bench0.log 2>&1; rc=$?; echo "ring rc=$rc"; grep '^{"metric"' gpurun_out/rw_bench0.log > gpurun_out/rw_bench0.json; cut -c 1-200 gpurun_out/rw_bench0.json
[ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/rw_bench0.json'));[print(k,v) for k,v in d['kernels'].items() if 's2' in k]"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 3 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/rw_torchrun.log 2>&1; rc=$?; echo "torchrun rc=$rc"; grep '^{"metric"' gpurun_out/rw_torchrun.log | cut -c 1-200
exit $rc
