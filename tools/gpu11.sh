cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for d in 0 1 2 3 32 33 34 35; do DLQ_DBG=$d timeout -k 10 120 python tools/convbench.py --only l2,l3,l4 >> gpurun_out/cb11.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/cb11.log
