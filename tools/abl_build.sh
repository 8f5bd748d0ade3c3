#!/bin/bash
# Build an ablation variant of libebert.so: tools/abl_build.sh NAME "-DFLAG ..." -> _abl/libebert_NAME.so
# (git-ignored, but shipped to the GPU box by gpurun; load it with EBERT_LIB=_abl/libebert_NAME.so).
set -e
NAME=$1; FLAGS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/robot_ebert_amd/csrc
B=$R/_abl/build_$NAME
mkdir -p $B
CXX="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $FLAGS"
pids=()
for f in $(cd $S && ls *.hip | sed "s/\.hip$//"); do
  $CXX -c $S/$f.hip -o $B/$f.o & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $R/_abl/libebert_$NAME.so $B/*.o -Wl,-rpath,/opt/rocm/lib
echo "built _abl/libebert_$NAME.so"
