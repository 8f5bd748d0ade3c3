#!/bin/bash
# Where the filter epilogue's hit path spends its time (gpurun -- bash tools/ab_hitpath.sh):
# clock-stamp launches of C2- and C3-shaped filter segments with the shipped epilogue, with the
# flagged columns staged but not processed, and with the column test alone (ablation builds,
# timing only: their results are wrong). tools/abl_build.sh stamp{,_stageonly,_hitnone}.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in stamp stamp_stageonly stamp_hitnone stamp; do
  bash tools/gpu.sh py r4h_$v tools/clock_stamp.py --lib _abl/libebert_$v.so --n 100000 --b 1024 \
    --d 768 --img bf16 --z 2.73 --cscale --secs 1.5
  bash tools/gpu.sh py r4h3_$v tools/clock_stamp.py --lib _abl/libebert_$v.so --secs 1.5
done
