# Round-end measurement: GPU tests, bench line, rocprofv3 kernel-trace stats and
# the two PMC traffic passes (FETCH_SIZE, WRITE_SIZE: separate passes, no trace
# domains), summarised into profiles/ by tools/pmc_traffic.py.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
R=${ROUND:-r01}
B="python3 bench.py --steps 6 --warmup 2 --prof-steps 0 --cpu-baseline-images 0 --torch-cpu-images 0"
set -o pipefail
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/kt gpurun_out/pf gpurun_out/pw
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- $B > gpurun_out/kt.log 2>&1; rc=$?; echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf -o run -- $B > gpurun_out/pf.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw -o run -- $B > gpurun_out/pw.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/pmc_traffic.py --fetch gpurun_out/pf --write gpurun_out/pw --trace gpurun_out/kt --cmd "$B" -o gpurun_out/${R}_pmc_traffic.json
cp $(find gpurun_out/kt -name '*kernel_stats.csv' | head -1) gpurun_out/${R}_kernel_stats.csv
