cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "l2_3x3 or l3_3x3 or l4_3x3 or wide" > gpurun_out/gpu_w.log 2>&1; rc=$?; echo "wide tests rc=$rc"; tail -5 gpurun_out/gpu_w.log
if [ $rc -ne 0 ]; then exit $rc; fi
for d in 0 1; do DLQ_DBG=$d timeout -k 10 120 python tools/convbench.py --only l2,l3,l4 >> gpurun_out/cb10.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/cb10.log
