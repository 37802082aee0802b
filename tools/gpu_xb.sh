cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for W in 7 14 28; do for xb in 0 64 96 0 64; do
timeout -k 10 60 tools/probe/conv3x3w_nostamp $W $xb || exit 1
done; done
