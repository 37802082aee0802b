# fp8 stride-2 + downsample kernel: fp8 GPU tests, fp8 bench, int8 s2 parity.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_f8.py tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/f8s2_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/f8s2_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --precision fp8 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/f8s2_bench.log 2>&1; rc=$?; echo "f8 rc=$rc"; grep '^{"metric"' gpurun_out/f8s2_bench.log > gpurun_out/f8s2_bench.json; cut -c 1-300 gpurun_out/f8s2_bench.json
python3 -c "import json;d=json.load(open('gpurun_out/f8s2_bench.json'));[print(k,v) for k,v in d['kernels'].items()]"
exit $rc
