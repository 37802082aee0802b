#!/bin/bash
# Build a variant of libdlq.so for A/B timing (tools/ab.py):
#   tools/build_variant.sh NAME "-DFLAG=1 ..."
# -> abvar/NAME/libdlq_ab.so (git-ignored but not gpurun-ignored, so it travels
# to the GPU box for tools/ab.py; delete abvar/ once the A/B is recorded so no
# stale library rides along; not named libdlq.so so it is never mistaken for
# the product library).  Objects go to scratch/ (gpurun-ignored).
# SRC=dir builds the sources of another tree (default dlq_amd/csrc).
set -e
cd "$(dirname "$0")/.."
NAME=$1
shift
FLAGS="$*"
OUT=abvar/$NAME
OBJ=scratch/abobj/$NAME
mkdir -p $OUT $OBJ
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result $FLAGS"
pids=()
objs=()
SRC=${SRC:-dlq_amd/csrc}
for f in $SRC/*.hip $SRC/*.cpp; do
  b=$(basename $f)
  [ "$b" = main_e2e.cpp ] || [ "$b" = main_step.cpp ] && continue
  o=$OBJ/${b%.*}.o
  objs+=($o)
  if [[ $f == *.cpp ]]; then x="-x hip"; else x=""; fi
  # as the Makefile (block_l1.hip), plus any file named in $NOSLP
  for n in block_l1.hip conv3x3i.hip conv3x3s2i.hip $NOSLP; do [ "$b" = $n ] && x="$x -fno-slp-vectorize"; done
  /opt/rocm/bin/hipcc $HIPFLAGS $x -c -o $o $f &
  pids+=($!)
  if [ ${#pids[@]} -ge 8 ]; then wait ${pids[0]}; pids=("${pids[@]:1}"); fi
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libdlq_ab.so "${objs[@]}"
echo "built $OUT/libdlq_ab.so from $SRC ($FLAGS)"
