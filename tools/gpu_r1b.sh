# Re-entry check: GPU tests, bench line, per-position kernel trace.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/kt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -o run -- python3 bench.py --steps 20 --warmup 3 --prof-steps 0 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/kt.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/fwdstats.py $(find gpurun_out/kt -name '*kernel_trace.csv' | head -1)
