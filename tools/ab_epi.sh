#!/bin/bash
# Per-phase cycles of the filter launch's waves (gpurun -- bash tools/ab_epi.sh [LIBS...]):
# C2- and C3-shaped segments at their hit densities (tools/epi_stamp.py), per diagnostic build.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${*:-epi}; do
  bash tools/gpu.sh py r4e_c2_$v tools/epi_stamp.py --lib _abl/libebert_$v.so --n 100000 --b 1024 --d 768 --img bf16 --z 2.73 --cscale
  bash tools/gpu.sh py r4e_c3_$v tools/epi_stamp.py --lib _abl/libebert_$v.so
done
