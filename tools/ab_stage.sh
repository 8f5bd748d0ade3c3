#!/bin/bash
# Hit staging by per-lane passes with pre-scaled values (gpurun -- bash tools/ab_stage.sh):
# the -m gpu suite on the new build, per-phase epilogue cycles of the old and new staging
# (_abl/libebert_epi_old.so, _abl/libebert_epi.so), then interleaved C2 / C3 bench lines of the
# new build and the previous commit (_abl/libebert_head.so).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4g
bash tools/ab_epi.sh epi_old epi
for i in 1 2; do
  bash tools/gpu.sh bench r4g_c2_new$i C2 --steps 50 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_head.so bash tools/gpu.sh bench r4g_c2_head$i C2 --steps 50 --no-cpu-baseline
done
bash tools/gpu.sh bench r4g_c3_new C3 --steps 20 --no-cpu-baseline
EBERT_LIB=_abl/libebert_head.so bash tools/gpu.sh bench r4g_c3_head C3 --steps 20 --no-cpu-baseline
bash tools/gpu.sh bench r4g_c3_new2 C3 --steps 20 --no-cpu-baseline
