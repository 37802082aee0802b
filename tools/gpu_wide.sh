# 392-px wide conv: parity first, then A/B per-layer timing and the bench.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread -k "conv or wide" > gpurun_out/wide_tests.log 2>&1; rc=$?; echo "wide tests rc=$rc"; tail -15 gpurun_out/wide_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/convbench.py --only l2,l3,l4 2>&1 | grep -v amdgpu.ids; [ $? -eq 0 ] || exit 1
DLQ_WIDE_256=1 timeout -k 10 120 python tools/convbench.py --only l2,l3,l4 2>&1 | grep -v amdgpu.ids; [ $? -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-250
