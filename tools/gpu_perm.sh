# s2 pixel permutation: parity, probe timings, bench, LDS conflicts.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_f8.py tests/test_gpu_layerops.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/perm_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/perm_tests.log
[ $rc -eq 0 ] || exit $rc
for ow in 28 14 7; do for d in 0 6; do timeout -k 5 60 ./tools/probe/conv3x3s2i_probe $ow $d || exit 1; done; done
bash tools/gpu_cs.sh 2>&1 | grep -v "^tests\|passed\|\.\.\.\."
