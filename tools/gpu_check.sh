# Quick validation: GPU tests, default bench, fp8 bench.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/chk_gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/chk_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/chk_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{"metric"' gpurun_out/chk_bench.log | cut -c 1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --precision fp8 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/chk_f8.log 2>&1; rc=$?; echo "f8 rc=$rc"; grep '^{"metric"' gpurun_out/chk_f8.log | cut -c 1-300
exit $rc
