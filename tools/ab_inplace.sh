#!/bin/bash
# In-place hit processing vs the staged form (gpurun -- bash tools/ab_inplace.sh): the -m gpu
# suite on the new build, per-phase epilogue cycles of both forms, interleaved C2 / C3 bench
# lines of the new build and the staged form (_abl/libebert_staged.so, -DEBT_HIT_STAGED).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4i
bash tools/ab_epi.sh epi_staged epi
for i in 1 2; do
  bash tools/gpu.sh bench r4i_c2_new$i C2 --steps 50 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_staged.so bash tools/gpu.sh bench r4i_c2_staged$i C2 --steps 50 --no-cpu-baseline
done
for i in 1 2; do
  bash tools/gpu.sh bench r4i_c3_new$i C3 --steps 20 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_staged.so bash tools/gpu.sh bench r4i_c3_staged$i C3 --steps 20 --no-cpu-baseline
done
