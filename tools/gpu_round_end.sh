# Round-end measurement (profiles/): GPU tests; the PMC traffic passes
# (FETCH_SIZE, WRITE_SIZE: separate passes, no trace domains) summarised by
# tools/pmc_traffic.py into profiles/; then the default bench command run
# under rocprofv3 --kernel-trace --stats, so its JSON line (which reads the
# traffic summary) and the kernel stats come from the same process and the
# per-kernel averages agree; finally a plain bench run.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${ROUND:-r01}_smoke.log 2>&1 || exit 1; tail -1 gpurun_out/${ROUND:-r01}_smoke.log
R=${ROUND:-r01}
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${R}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 6 --warmup 2 --prof-steps 0 --cpu-baseline-images 0 --torch-cpu-images 0"
rm -rf gpurun_out/pf gpurun_out/pw gpurun_out/kt gpurun_out/kt0
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf -o run -- $B > gpurun_out/pf.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw -o run -- $B > gpurun_out/pw.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt0 -o run -- $B > gpurun_out/kt0.log 2>&1; rc=$?; echo "trace(short) rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/pmc_traffic.py --fetch gpurun_out/pf --write gpurun_out/pw --trace gpurun_out/kt0 --cmd "$B" -o gpurun_out/${R}_pmc_traffic.json
cp gpurun_out/${R}_pmc_traffic.json profiles/${R}_pmc_traffic.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- python3 bench.py > gpurun_out/${R}_bench_under_rocprof.log 2>&1; rc=$?; echo "bench(rocprof) rc=$rc"
[ $rc -eq 0 ] || exit $rc
grep '^{"metric"' gpurun_out/${R}_bench_under_rocprof.log > gpurun_out/${R}_bench_under_rocprof.json
cp $(find gpurun_out/kt -name '*kernel_stats.csv' | head -1) gpurun_out/${R}_kernel_stats.csv
python3 tools/fwdstats.py $(find gpurun_out/kt -name '*kernel_trace.csv' | head -1) > gpurun_out/${R}_per_position.txt
tail -19 gpurun_out/${R}_per_position.txt
timeout -k 10 300 python3 bench.py > gpurun_out/${R}_bench_plain.log 2>&1; rc=$?; echo "bench(plain) rc=$rc"
grep '^{"metric"' gpurun_out/${R}_bench_plain.log > gpurun_out/${R}_bench.json; cut -c 1-200 gpurun_out/${R}_bench.json
# fp8 (configs[4]): kernel stats of the same bench command under rocprofv3, then a plain run
rm -rf gpurun_out/kt8
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt8 -o run -- python3 bench.py --precision fp8 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/${R}_f8_bench_under_rocprof.log 2>&1; rc=$?; echo "f8 bench(rocprof) rc=$rc"
[ $rc -eq 0 ] || exit $rc
cp $(find gpurun_out/kt8 -name '*kernel_stats.csv' | head -1) gpurun_out/${R}_f8_kernel_stats.csv
timeout -k 10 300 python3 bench.py --precision fp8 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/${R}_f8_bench_plain.log 2>&1; rc=$?; echo "f8 bench(plain) rc=$rc"
grep '^{"metric"' gpurun_out/${R}_f8_bench_plain.log > gpurun_out/${R}_f8_bench.json; cut -c 1-200 gpurun_out/${R}_f8_bench.json
exit $rc
