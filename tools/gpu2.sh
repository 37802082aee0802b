# GPU round: parity tests, bench, kernel-trace profile.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-900
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/prof_bench.log 2>&1; echo "prof rc=$?"
