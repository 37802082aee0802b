# Wide-conv limiter experiments: xb bits = 1 no MFMA, 8 no epilogue, 16 no LDS-DMA, 4 weights from one block
cd $GRAFT_REPO_ROOT
for W in 7 14 28; do for xb in 0 1 16 17 8 4; do
timeout -k 10 60 tools/probe/conv3x3w_nostamp $W $xb || exit 1
done; done
