cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for v in 7 9; do timeout -k 10 60 tools/probe/block_l1_p$v 256 > gpurun_out/l1p$v.log || exit 1; head -9 gpurun_out/l1p$v.log; done
