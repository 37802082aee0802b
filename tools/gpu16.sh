cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench16.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench16.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof16 -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/prof16.log 2>&1; rc=$?; echo "prof rc=$rc"
python3 tools/kstats.py $(find gpurun_out/prof16 -name '*kernel_trace.csv' | head -1)
