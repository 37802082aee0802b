cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for sp in 1 0 1 0; do
DLQ_SPLIT=$sp timeout -k 10 300 python bench.py --steps 30 --warmup 5 --prof-steps 0 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench_sp$sp.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_sp$sp.log').read().strip().splitlines()[-1]); print('split=$sp', d['value'], d['ms_per_step'])"
done
