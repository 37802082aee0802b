cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "l2_3x3 or l3_3x3 or l4_3x3" > gpurun_out/gpu_w.log 2>&1; rc=$?; echo "wide tests rc=$rc"; tail -25 gpurun_out/gpu_w.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/convbench.py --only l2,l3,l4 > gpurun_out/cb7.log 2>&1 || exit $?
DLQ_DBG=1 timeout -k 10 120 python tools/convbench.py --only l2,l3,l4 >> gpurun_out/cb7.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/cb7.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
