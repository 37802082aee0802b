cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_layerops.py -x -q -m gpu -k gemm --timeout 120 --timeout-method thread > gpurun_out/t_gemm.log 2>&1 || { tail -5 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
for r in 1 2 3; do
for shp in "8192 8192 8192 10" "4096 4096 4096 20" "50176 256 2304 20"; do
  timeout -k 5 120 python3 tools/gemm_run.py $shp || exit 1
  DLQ_LIB_PATH=$PWD/scratch/gold/libdlq.so timeout -k 5 120 python3 tools/gemm_run.py $shp | sed 's/^/OLD /' || exit 1
done; done
