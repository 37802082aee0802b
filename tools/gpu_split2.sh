cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
B="python bench.py --steps 40 --warmup 5 --prof-steps 0 --cpu-baseline-images 0 --torch-cpu-images 0"
timeout -k 10 200 $B > gpurun_out/b0.log 2>&1 || exit 1; tail -1 gpurun_out/b0.log | cut -c100-200
DLQ_SPLIT=1 timeout -k 10 200 $B > gpurun_out/b1.log 2>&1 || exit 1; tail -1 gpurun_out/b1.log | cut -c100-200
timeout -k 10 200 $B > gpurun_out/b2.log 2>&1 || exit 1; tail -1 gpurun_out/b2.log | cut -c100-200
DLQ_SPLIT=1 timeout -k 10 200 $B > gpurun_out/b3.log 2>&1 || exit 1; tail -1 gpurun_out/b3.log | cut -c100-200
