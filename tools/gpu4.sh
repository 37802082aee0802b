cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L=l1,l2,l3,l4
timeout -k 10 120 python tools/convbench.py --only $L > gpurun_out/cb.log 2>&1 || exit $?
for d in 1 2 3 5; do DLQ_DBG=$d timeout -k 10 120 python tools/convbench.py --only $L >> gpurun_out/cb.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/cb.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400
