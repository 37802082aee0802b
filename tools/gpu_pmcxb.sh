# LDS / issue counters for the wide conv probe (one SQ pass per command).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
rm -rf gpurun_out/pmcxb; mkdir -p gpurun_out/pmcxb
for W in 7 28; do
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmcxb/a$W -o run -- tools/probe/conv3x3w_nostamp $W 0 > gpurun_out/pmcxb/a$W.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL SQ_INSTS_SALU --output-format csv -d gpurun_out/pmcxb/b$W -o run -- tools/probe/conv3x3w_nostamp $W 0 > gpurun_out/pmcxb/b$W.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv,glob,collections
for f in sorted(glob.glob('gpurun_out/pmcxb/*/**/*counter_collection.csv',recursive=True)):
    acc=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'conv3x3w' not in r['Kernel_Name']: continue
        acc[(r['Dispatch_Id'],r['Counter_Name'])].append(float(r['Counter_Value']))
    per=collections.defaultdict(list)
    for (d,c),v in acc.items(): per[c].append(sum(v))
    print(f)
    for c,v in sorted(per.items()): print(f"  {c:28s} {sum(v)/len(v):.4g}")
PY
