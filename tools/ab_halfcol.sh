#!/bin/bash
# Hit staging by half columns vs whole columns (gpurun -- bash tools/ab_halfcol.sh): the -m gpu
# suite on the new build, per-phase epilogue cycles of both forms, interleaved C2 / C3 bench
# lines of the new build and the whole-column form (_abl/libebert_whole.so, -DEBT_HIT_STAGE_WHOLE).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4h2
bash tools/ab_epi.sh epi_whole epi
for i in 1 2; do
  bash tools/gpu.sh bench r4h2_c2_new$i C2 --steps 50 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_whole.so bash tools/gpu.sh bench r4h2_c2_whole$i C2 --steps 50 --no-cpu-baseline
done
for i in 1 2; do
  bash tools/gpu.sh bench r4h2_c3_new$i C3 --steps 20 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_whole.so bash tools/gpu.sh bench r4h2_c3_whole$i C3 --steps 20 --no-cpu-baseline
done
