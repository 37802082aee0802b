cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 4 --torch-cpu-images 2 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
