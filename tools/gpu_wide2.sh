cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread -k "conv or wide or end_to_end" > gpurun_out/wide_tests.log 2>&1; rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/wide_tests.log
[ $rc -eq 0 ] || exit $rc
for W in 7 14 28; do timeout -k 5 60 tools/probe/conv3x3i_nostamp $W || exit 1; done
timeout -k 5 60 tools/probe/conv3x3i_stamps 14 || exit 1
timeout -k 10 120 python tools/convbench.py --only l2,l3,l4 2>&1 | grep -v amdgpu.ids; [ $? -eq 0 ] || exit 1
rm -rf gpurun_out/pmci; mkdir -p gpurun_out/pmci
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmci/a14 -o run -- tools/probe/conv3x3i_nostamp 14 > gpurun_out/pmci/a14.log 2>&1 || exit 1
python3 - <<'PY'
import csv,glob,collections
for f in sorted(glob.glob('gpurun_out/pmci/*/**/*counter_collection.csv',recursive=True)):
    acc=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'conv3x3i' not in r['Kernel_Name']: continue
        acc[(r['Dispatch_Id'],r['Counter_Name'])].append(float(r['Counter_Value']))
    per=collections.defaultdict(list)
    for (d,c),v in acc.items(): per[c].append(sum(v))
    print(f)
    for c,v in sorted(per.items()): print(f"  {c:28s} {sum(v)/len(v):.4g}")
PY
