cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_block_l1.py -q -x > gpurun_out/gpu_l1.log 2>&1; rc=$?; echo "l1 tests rc=$rc"; tail -3 gpurun_out/gpu_l1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/probe/block_l1_nostamp 256 || exit 1
for v in 0 1; do timeout -k 10 60 tools/probe/block_l1_p$v 256 > gpurun_out/l1p$v.log || exit 1; head -9 gpurun_out/l1p$v.log; done
