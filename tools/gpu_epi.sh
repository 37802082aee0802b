cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layerops.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
for W in 7 14 28; do timeout -k 5 60 tools/probe/conv3x3i_nostamp $W 0 || exit 1; timeout -k 5 60 tools/probe/conv3x3s2i_probe $W 0 || exit 1; done
B="python bench.py --steps 40 --warmup 5 --prof-steps 0 --cpu-baseline-images 0 --torch-cpu-images 0"
timeout -k 10 200 $B > gpurun_out/b0.log 2>&1 || exit 1; tail -1 gpurun_out/b0.log | cut -c100-200
