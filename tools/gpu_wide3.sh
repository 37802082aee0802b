cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread -k "conv or wide or end_to_end" > gpurun_out/wide_tests.log 2>&1; rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/wide_tests.log
[ $rc -eq 0 ] || exit $rc
for W in 7 14 28; do for d in 0 2; do timeout -k 5 60 tools/probe/conv3x3i_nostamp $W $d || exit 1; done; done
timeout -k 5 60 tools/probe/conv3x3i_stamps 14 || exit 1
timeout -k 10 120 python tools/convbench.py --only l2,l3,l4 2>&1 | grep -v amdgpu.ids; [ $? -eq 0 ] || exit 1
