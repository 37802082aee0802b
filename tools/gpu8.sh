cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for L in l2 l3 l4; do
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc8_$L -o run -- python3 tools/convbench.py --only $L --iters 5 > gpurun_out/pmc8_$L.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc8b_$L -o run -- python3 tools/convbench.py --only $L --iters 5 >> gpurun_out/pmc8_$L.log 2>&1 || exit $?
done
ls -R gpurun_out/pmc8_l4 | head
