cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
B="python3 bench.py --steps 30 --warmup 5 --prof-steps 0 --cpu-baseline-images 0 --oracle-images 0 --extras 0"
for r in 1 2; do
for v in new old; do
  rm -rf gpurun_out/kt_$v
  if [ $v = old ]; then export DLQ_LIB_PATH=$PWD/abvar/oldwide/libdlq.so; else unset DLQ_LIB_PATH; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_$v -o run -- $B > gpurun_out/kt_$v.log 2>&1 || exit 1
  echo "== $v round $r"; python3 tools/fwdstats.py $(find gpurun_out/kt_$v -name '*kernel_trace.csv' | head -1)
done
done
