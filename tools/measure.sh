#!/bin/bash
# Round measurement recipe (run on the GPU box through gpurun; writes
# gpurun_out/${ROUND}_*, copied into profiles/ afterwards):
#   smoke + GPU tests; PMC passes, each its own rocprofv3 run with no trace
#   domains (FETCH_SIZE, WRITE_SIZE: HBM traffic, tools/pmc_traffic.py;
#   SQ MFMA/wave counters: MFMA utilisation, tools/pmc_summary.py); the
#   default bench command under rocprofv3 --kernel-trace --stats (its JSON
#   line and the kernel stats from one process); a plain bench run; the
#   MFMA power probe (the chip's loaded-clock MFMA ceiling on random data).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
R=${ROUND:-r02}
set -o pipefail
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || exit 1; tail -1 gpurun_out/${R}_smoke.log
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${R}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
fi
B="python3 bench.py --steps 6 --warmup 2 --prof-steps 0 --cpu-baseline-images 0 --oracle-images 0 --extras 0"
rm -rf gpurun_out/pf gpurun_out/pw gpurun_out/pm gpurun_out/kt gpurun_out/kt0
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf -o run -- $B > gpurun_out/pf.log 2>&1; rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw -o run -- $B > gpurun_out/pw.log 2>&1; rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pm -o run -- $B > gpurun_out/pm.log 2>&1; rc=$?; echo "mfma pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt0 -o run -- $B > gpurun_out/kt0.log 2>&1; rc=$?; echo "trace(short) rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_traffic.py --fetch gpurun_out/pf --write gpurun_out/pw --trace gpurun_out/kt0 --cmd "$B" -o gpurun_out/${R}_pmc_traffic.json > /dev/null || exit 1
python3 tools/pmc_summary.py gpurun_out/pm -o gpurun_out/${R}_pmc_mfma.json > /dev/null || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- python3 bench.py --extras 0 > gpurun_out/${R}_bench_under_rocprof.log 2>&1; rc=$?; echo "bench(rocprof) rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{"metric"' gpurun_out/${R}_bench_under_rocprof.log > gpurun_out/${R}_bench_under_rocprof.json
cp $(find gpurun_out/kt -name '*kernel_stats.csv' | head -1) gpurun_out/${R}_kernel_stats.csv
python3 tools/fwdstats.py $(find gpurun_out/kt -name '*kernel_trace.csv' | head -1) > gpurun_out/${R}_per_position.txt
timeout -k 10 400 python3 bench.py > gpurun_out/${R}_bench_plain.log 2>&1; rc=$?; echo "bench(plain) rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{"metric"' gpurun_out/${R}_bench_plain.log > gpurun_out/${R}_bench.json; cut -c 1-160 gpurun_out/${R}_bench.json
if [ -x tools/probe/mfma_power_probe ]; then timeout -k 5 120 tools/probe/mfma_power_probe > gpurun_out/${R}_mfma_power_probe.txt 2>&1 || exit 1; fi
exit 0
