# prep_issue without scratch spills: parity, convbench, s2 probe, bench.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_f8.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/sp_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/sp_tests.log
[ $rc -eq 0 ] || exit $rc
for d in 0 4; do DLQ_DBG=$d timeout -k 5 120 python3 tools/convbench.py --only l2,l3,l4 2>&1 | grep -v amdgpu.ids || exit 1; done
for ow in 28 14 7; do for d in 0 4 6; do timeout -k 5 60 ./tools/probe/conv3x3s2i_probe $ow $d || exit 1; done; done
B="python3 bench.py --cpu-baseline-images 0 --torch-cpu-images 0"
timeout -k 10 300 $B > gpurun_out/sp_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{"metric"' gpurun_out/sp_bench.log > gpurun_out/sp_bench.json; cut -c 1-200 gpurun_out/sp_bench.json
python3 -c "import json;d=json.load(open('gpurun_out/sp_bench.json'));[print(k,v) for k,v in d['kernels'].items()]"
exit $rc
