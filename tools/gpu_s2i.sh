cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layerops.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/s2_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/s2_tests.log
[ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 40 --warmup 5 --prof-steps 0 --cpu-baseline-images 0 --torch-cpu-images 0"
timeout -k 10 200 $B > gpurun_out/b0.log 2>&1 || exit 1; tail -1 gpurun_out/b0.log | cut -c100-200
DLQ_S2_128=1 timeout -k 10 200 $B > gpurun_out/b1.log 2>&1 || exit 1; tail -1 gpurun_out/b1.log | cut -c100-200
rm -rf gpurun_out/kt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -o run -- python3 bench.py --steps 20 --warmup 3 --prof-steps 0 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/kt.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/fwdstats.py $(find gpurun_out/kt -name '*kernel_trace.csv' | head -1) | tail -19
