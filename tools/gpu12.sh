cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for d in 0 1 2 3 32 35; do DLQ_DBG=$d timeout -k 10 120 python tools/convbench.py --only l1,l2,l3,l4,l2_0c1,l2_ds,l3_0c1,l4_0c1,stemf >> gpurun_out/cb12.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/cb12.log
