cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
true; rc=0
if [ $rc -ne 0 ]; then exit $rc; fi
true
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/convbench.py --only stemf > gpurun_out/cb17.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/cb17.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --torch-cpu-images 0 > gpurun_out/bench17.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench17.log | cut -c1-200
