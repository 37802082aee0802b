cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_block_l1.py -q -x > gpurun_out/gpu_l1.log 2>&1; rc=$?; echo "l1 tests rc=$rc"; tail -15 gpurun_out/gpu_l1.log
grep -q "HSA_STATUS_ERROR\|Memory access fault" gpurun_out/gpu_l1.log && exit 3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"
python3 -c "
import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step']); [print(k, v) for k,v in d['kernels'].items()]"
