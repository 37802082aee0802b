cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof18 -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/prof18.log 2>&1; rc=$?; echo "prof rc=$rc"
python3 tools/fwdstats.py $(find gpurun_out/prof18 -name '*kernel_trace.csv' | head -1)
