#!/bin/bash
# A/B of the GEMM drop-in on one GPU box (run through gpurun):
#   bash tools/gemm_ab.sh abvar/VARIANT/libdlq.so
# GEMM parity tests on the in-tree library, then three alternating rounds of
# tools/gemm_run.py (in-tree vs VARIANT, lines of the latter prefixed OLD).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
ALT=${1:?usage: tools/gemm_ab.sh abvar/VARIANT/libdlq.so}
timeout -k 10 300 python -u -m pytest tests/test_gpu_layerops.py -x -q -m gpu -k gemm --timeout 120 --timeout-method thread > gpurun_out/t_gemm.log 2>&1 || { tail -5 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
for r in 1 2 3; do
for shp in "8192 8192 8192 10" "4096 4096 4096 20" "50176 256 2304 20"; do
  timeout -k 5 120 python3 tools/gemm_run.py $shp || exit 1
  DLQ_LIB_PATH=$PWD/$ALT timeout -k 5 120 python3 tools/gemm_run.py $shp | sed 's/^/OLD /' || exit 1
done; done
