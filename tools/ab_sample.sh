#!/bin/bash
# Speculative sample size (gpurun -- bash tools/ab_sample.sh): EBT_SPEC_SAMPLE_DIV 200 (the
# default: C3 64 sample tiles, C4 192) against 40 (C3 96, C4 512) and 30 (C3 128, C4 512):
# a larger sample costs sample-GEMM rounds and buys fewer hits per query (filter hit path,
# merges). Interleaved C3 and C4 lines on one box (_abl/libebert_div40.so, div30.so).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  bash tools/gpu.sh bench r4s_c3_def$i C3 --steps 20 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_div40.so bash tools/gpu.sh bench r4s_c3_d40_$i C3 --steps 20 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_div30.so bash tools/gpu.sh bench r4s_c3_d30_$i C3 --steps 20 --no-cpu-baseline
done
for i in 1 2; do
  bash tools/gpu.sh bench r4s_c4_def$i C4 --steps 5 --warmup 1 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_div40.so bash tools/gpu.sh bench r4s_c4_d40_$i C4 --steps 5 --warmup 1 --no-cpu-baseline
done
