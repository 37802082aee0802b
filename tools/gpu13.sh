cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for d in 0 64 128 35 291; do DLQ_DBG=$d timeout -k 10 120 python tools/convbench.py --only l2,l4 >> gpurun_out/cb13.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/cb13.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof13 -o run -- python3 tools/convbench.py --only l2,l4 --iters 20 > gpurun_out/prof13.log 2>&1 || exit $?
python3 tools/kstats.py $(find gpurun_out/prof13 -name '*kernel_trace.csv' | head -1)
