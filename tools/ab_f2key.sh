#!/bin/bash
# Branchless hit keys in the filter epilogue (gpurun -- bash tools/ab_f2key.sh): the -m gpu suite,
# interleaved C3 / C2 lines of the new build and the previous commit (_abl/libebert_prev.so),
# and C2's stages at half and twice its batch (how the merge scales with queries per SIMD).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4k2
for i in 1 2; do
  bash tools/gpu.sh bench r4k2_c3_new$i C3 --steps 20 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_prev.so bash tools/gpu.sh bench r4k2_c3_prev$i C3 --steps 20 --no-cpu-baseline
done
for i in 1 2; do
  bash tools/gpu.sh bench r4k2_c2_new$i C2 --steps 50 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_prev.so bash tools/gpu.sh bench r4k2_c2_prev$i C2 --steps 50 --no-cpu-baseline
done
bash tools/gpu.sh bench r4k2_c2_b512 C2 --steps 50 --no-cpu-baseline --b 512
bash tools/gpu.sh bench r4k2_c2_b2048 C2 --steps 50 --no-cpu-baseline --b 2048
