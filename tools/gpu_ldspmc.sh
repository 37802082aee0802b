# LDS bank-conflict share per kernel of the default forward (one PMC pass).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
rm -rf gpurun_out/ldspmc
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/ldspmc -o run -- python3 bench.py --steps 3 --warmup 1 --prof-steps 0 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/ldspmc.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/ldspmc/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0][-60:]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    a = d.get('SQ_LDS_IDX_ACTIVE', 0)
    if a: print(f"{k:60s} conflict/active = {d.get('SQ_LDS_BANK_CONFLICT', 0) / a:.3f}")
PY
