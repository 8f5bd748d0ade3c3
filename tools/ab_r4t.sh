#!/bin/bash
# Round-4 A/B of the rescore and merge changes (gpurun -- bash tools/ab_r4t.sh): the suite, then
# interleaved C2 / C3 bench lines of the current build, the pre-change build (_abl/libebert_head.so),
# the LDS-query rescore form (EBT_RESCORE_REG=0) and one row per trip at 3..6 chunks per lane
# (_abl/libebert_nr1.so); then the filter epilogue's cost at C2's hit density (clock stamps).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4t
for i in 1 2; do
  bash tools/gpu.sh bench r4t_c2_new$i C2 --steps 50 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_head.so bash tools/gpu.sh bench r4t_c2_head$i C2 --steps 50 --no-cpu-baseline
  EBT_RESCORE_REG=0 bash tools/gpu.sh bench r4t_c2_ldsq$i C2 --steps 50 --no-cpu-baseline
done
bash tools/gpu.sh bench r4t_c3_new C3 --steps 20 --no-cpu-baseline
EBERT_LIB=_abl/libebert_head.so bash tools/gpu.sh bench r4t_c3_head C3 --steps 20 --no-cpu-baseline
EBERT_LIB=_abl/libebert_nr1.so bash tools/gpu.sh bench r4t_c3_nr1 C3 --steps 20 --no-cpu-baseline
bash tools/gpu.sh bench r4t_c2_streams2 C2 --steps 50 --no-cpu-baseline --streams 2
bash tools/gpu.sh py r4t_stamp tools/clock_stamp.py --n 100000 --b 1024 --d 768 --img bf16 --z 2.73 --secs 1.5
bash tools/gpu.sh py r4t_stamp_cs tools/clock_stamp.py --n 100000 --b 1024 --d 768 --img bf16 --z 2.73 --secs 1.5 --cscale
