cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
L=l1,l2,l3,l4
timeout -k 10 120 python tools/convbench.py --only $L > gpurun_out/cb.log 2>&1 || exit $?
DLQ_CONV_V1=1 timeout -k 10 120 python tools/convbench.py --only $L >> gpurun_out/cb.log 2>&1 || exit $?
for d in 1 2 4 6 3 5; do DLQ_DBG=$d timeout -k 10 120 python tools/convbench.py --only $L >> gpurun_out/cb.log 2>&1 || exit $?; done
cat gpurun_out/cb.log
