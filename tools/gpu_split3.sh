cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread -k "conv or wide or end_to_end" > gpurun_out/t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
for W in 7 14 28; do for i in 1 2; do timeout -k 5 60 tools/probe/conv3x3i_nostamp $W 0 || exit 1; timeout -k 5 60 tools/probe/conv3x3i_nostamp12 $W 0 || exit 1; done; done
