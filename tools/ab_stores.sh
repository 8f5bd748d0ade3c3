#!/bin/bash
# The filter epilogue's global stores (hit slots, per-tile counts) against the counted LDS-DMA
# stream (gpurun -- bash tools/ab_stores.sh): clock-stamp launches of C2- and C3-shaped filter
# segments with ablation builds that drop the hit stores, the count stores, or both (timing
# only: those builds' results are wrong). tools/abl_build.sh stamp{,_nohit,_nocnt,_none}.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in stamp stamp_nohit stamp_nocnt stamp_none; do
  bash tools/gpu.sh py r4s_$v tools/clock_stamp.py --lib _abl/libebert_$v.so --n 100000 --b 1024 \
    --d 768 --img bf16 --z 2.73 --cscale --secs 1.5
  bash tools/gpu.sh py r4s3_$v tools/clock_stamp.py --lib _abl/libebert_$v.so --secs 1.5
done
