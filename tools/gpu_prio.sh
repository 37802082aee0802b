cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for W in 7 14 28; do for d in 0 2 16 18; do timeout -k 5 60 tools/probe/conv3x3i_nostamp $W $d || exit 1; done; done
timeout -k 5 60 tools/probe/conv3x3i_stamps 14 18 || exit 1
