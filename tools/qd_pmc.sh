#!/bin/bash
# rocprofv3 counter evidence for the standalone quantise / dequant passes
# (run on the GPU box; three separate runs, program directly after --):
#   bash tools/qd_pmc.sh OUT.json
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -rf gpurun_out/qf gpurun_out/qw gpurun_out/qt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/qf -o run -- python3 tools/qd_time.py > gpurun_out/qf.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/qw -o run -- python3 tools/qd_time.py > gpurun_out/qw.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qt -o run -- python3 tools/qd_time.py > gpurun_out/qt.log 2>&1 || exit 1
python3 tools/qd_pmc.py --fetch gpurun_out/qf --write gpurun_out/qw --trace gpurun_out/qt -o "${1:-gpurun_out/qd_pmc.json}"
