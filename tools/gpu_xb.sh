cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for a in "7 0" "7 17" "7 1" "7 16" "28 0" "28 17"; do
timeout -k 10 60 tools/probe/conv3x3w_stamps $a || exit 1
done
