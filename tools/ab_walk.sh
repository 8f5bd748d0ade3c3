#!/bin/bash
# The tile walk's divisions as shifts (gpurun -- bash tools/ab_walk.sh): the -m gpu suite,
# per-phase epilogue cycles of the previous and new build, interleaved C2 / C3 bench lines of
# the new build and the previous commit (_abl/libebert_prev.so).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4w
bash tools/ab_epi.sh epi_prev epi
for i in 1 2; do
  bash tools/gpu.sh bench r4w_c3_new$i C3 --steps 20 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_prev.so bash tools/gpu.sh bench r4w_c3_prev$i C3 --steps 20 --no-cpu-baseline
done
for i in 1 2; do
  bash tools/gpu.sh bench r4w_c2_new$i C2 --steps 50 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_prev.so bash tools/gpu.sh bench r4w_c2_prev$i C2 --steps 50 --no-cpu-baseline
done
