# hipGraph forward: parity tests + int8 bench (graph on, then DLQ_GRAPH=0 for A/B).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_launcher.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/g_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g_tests.log
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --cpu-baseline-images 0 --torch-cpu-images 0"
timeout -k 10 300 $B > gpurun_out/g_bench.log 2>&1; rc=$?; echo "graph rc=$rc"; grep '^{"metric"' gpurun_out/g_bench.log | cut -c 1-260
[ $rc -eq 0 ] || exit $rc
DLQ_GRAPH=0 timeout -k 10 300 $B > gpurun_out/g_bench0.log 2>&1; rc=$?; echo "nograph rc=$rc"; grep '^{"metric"' gpurun_out/g_bench0.log | cut -c 1-260
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B > gpurun_out/g_bench2.log 2>&1; rc=$?; echo "graph rc=$rc"; grep '^{"metric"' gpurun_out/g_bench2.log | cut -c 1-260
exit $rc
