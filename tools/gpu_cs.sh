# wide conv chunk pitch: parity, bench, LDS conflicts.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_f8.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/cs_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/cs_tests.log
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --cpu-baseline-images 0 --torch-cpu-images 0"
timeout -k 10 300 $B > gpurun_out/cs_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{"metric"' gpurun_out/cs_bench.log > gpurun_out/cs_bench.json; cut -c 1-200 gpurun_out/cs_bench.json
[ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/cs_bench.json'));[print(k,v) for k,v in d['kernels'].items()]"
bash tools/gpu_ldspmc.sh > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/ldspmc/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].replace('void dlq::(anonymous namespace)::','')[:60]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    a = d.get('SQ_LDS_IDX_ACTIVE', 0)
    if a: print(f"{k:60s} conflict/active = {d.get('SQ_LDS_BANK_CONFLICT', 0) / a:.3f}")
PY
