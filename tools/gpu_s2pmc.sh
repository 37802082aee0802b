# LDS counters of the stride-2 kernel (timing probe, no DMA / epilogue variants).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
for ow in 28 7; do for d in 0 6; do
rm -rf gpurun_out/s2pmc_${ow}_${d}
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/s2pmc_${ow}_${d} -o run -- ./tools/probe/conv3x3s2i_probe $ow $d > gpurun_out/s2pmc_${ow}_${d}.log 2>&1 || exit 1
done; done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/s2pmc_*/**/*counter_collection.csv', recursive=True)):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if 'conv3x3s2i' not in r['Kernel_Name']: continue
        agg[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
    print(f.split('/')[1], {k: round(v / max(n[k], 1) / 1, 0) for k, v in agg.items()})
PY
