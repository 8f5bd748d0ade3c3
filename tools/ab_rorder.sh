#!/bin/bash
# Rescore ordering and s_min (gpurun -- bash tools/ab_rorder.sh): the rank count 8 rows per batch
# of LDS reads with two threads per row, s_min by wave count + DPP minimum (one LDS atomic per
# wave), one barrier fewer; against the previous commit (_abl/libebert_prev.so). The -m gpu suite,
# interleaved C2 / C3 lines, and the rescore phase cycles of the new build (-DEBT_RESCORE_STAMP).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4o
for i in 1 2; do
  bash tools/gpu.sh bench r4o_c2_new$i C2 --steps 50 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_prev.so bash tools/gpu.sh bench r4o_c2_prev$i C2 --steps 50 --no-cpu-baseline
done
for i in 1 2; do
  bash tools/gpu.sh bench r4o_c3_new$i C3 --steps 20 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_prev.so bash tools/gpu.sh bench r4o_c3_prev$i C3 --steps 20 --no-cpu-baseline
done
mkdir -p gpurun_out/r4o_stamp
for c in C2 C3; do
  EBERT_LIB=_abl/libebert_rst.so timeout -k 10 300 python -u tools/rescore_stamp.py --config $c >> gpurun_out/r4o_stamp/new.jsonl
done
