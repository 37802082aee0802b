# Kernel-trace profile of bench.py (rocprofv3 --kernel-trace --stats).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/prof_bench.log 2>&1; rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/prof_bench.log
find $OUT -name "*stats*" | head; 
