cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for d in 0 1 2 4 8 3 6 9 10 12 14 11 13; do DLQ_DBG=$d timeout -k 10 120 python tools/convbench.py --only stemf >> gpurun_out/cb6.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/cb6.log
