#!/bin/bash
# Hit staging by query-half blocks vs by column (gpurun -- bash tools/ab_halfblock.sh): the -m gpu
# suite on the new build, per-phase epilogue cycles of both forms, interleaved C2 / C3 bench
# lines of the new build and the per-column form (_abl/libebert_bycol.so).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4b
bash tools/ab_epi.sh epi_bycol epi
for i in 1 2; do
  bash tools/gpu.sh bench r4b_c2_new$i C2 --steps 50 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_bycol.so bash tools/gpu.sh bench r4b_c2_bycol$i C2 --steps 50 --no-cpu-baseline
done
for i in 1 2; do
  bash tools/gpu.sh bench r4b_c3_new$i C3 --steps 20 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_bycol.so bash tools/gpu.sh bench r4b_c3_bycol$i C3 --steps 20 --no-cpu-baseline
done
