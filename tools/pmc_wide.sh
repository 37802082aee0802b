#!/bin/bash
# PMC passes over the wide-conv probe (tools/probe/conv3x3i_time W dbg), one
# rocprofv3 run per counter set, summaries to gpurun_out/pmc_wide_*.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA"
for W in ${WS:-14}; do for d in ${DBGS:-0}; do
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  rm -rf gpurun_out/pw$i
  timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pw$i -o run -- tools/probe/conv3x3i_time $W $d > gpurun_out/pw$i.log 2>&1 || exit 1
  python3 - "$W" "$d" "$i" <<'PY'
import csv, glob, sys, collections
W, d, i = sys.argv[1:4]
f = glob.glob(f"gpurun_out/pw{i}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if "conv3x3i" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(f"W={W} dbg={d} " + " ".join(f"{k}={acc[k]/max(n[k],1):.4g}" for k in sorted(acc)))
PY
done; done; done
