cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for W in 7 14 28; do for d in 0 4 8 12 2; do timeout -k 5 60 tools/probe/conv3x3i_nostamp $W $d || exit 1; done; done
