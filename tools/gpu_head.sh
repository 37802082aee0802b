# Fused GAP+FC head: parity, then bench A/B (fused default vs DLQ_HEAD_SPLIT=1).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/hd_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/hd_tests.log
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --cpu-baseline-images 0 --torch-cpu-images 0"
for v in 0 1 0 1; do
  DLQ_HEAD_SPLIT=$v timeout -k 10 300 $B > gpurun_out/hd_bench$v.log 2>&1 || exit 1
  echo "split=$v $(grep '^{"metric"' gpurun_out/hd_bench$v.log | python3 -c 'import json,sys;d=json.load(sys.stdin);print(d["value"], d["ms_per_step"], {k:v["avg_launch_us"] for k,v in d["kernels"].items()})')"
done
