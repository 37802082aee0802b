cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k stem_fused > gpurun_out/gpu_stem.log 2>&1; rc=$?; echo "stem tests rc=$rc"; tail -15 gpurun_out/gpu_stem.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
DLQ_STEM_UNFUSED=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench_unf.log 2>&1; rc=$?; echo "bench unfused rc=$rc"; tail -1 gpurun_out/bench_unf.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/prof5.log 2>&1; rc=$?; echo "prof rc=$rc"
f=$(find gpurun_out/prof5 -name '*kernel_trace.csv' | head -1); python3 tools/kstats.py $f
