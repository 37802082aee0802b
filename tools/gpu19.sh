cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "s2 or l2_0 or l3_0 or l4_0" > gpurun_out/gpu_s2.log 2>&1; rc=$?; echo "s2 tests rc=$rc"; tail -25 gpurun_out/gpu_s2.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench19.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench19.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof19 -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/prof19.log 2>&1; rc=$?; echo "prof rc=$rc"
python3 tools/fwdstats.py $(find gpurun_out/prof19 -name '*kernel_trace.csv' | head -1)
