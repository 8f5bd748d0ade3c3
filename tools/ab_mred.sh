#!/bin/bash
# Wave merge (gpurun -- bash tools/ab_mred.sh): marker + DPP max-scan hit slots, DPP wave
# reductions, a 32-bit bisection and branchless write positions, against the previous commit
# (_abl/libebert_prev.so: per-lane slot loop, shuffle reductions). The -m gpu suite, interleaved
# C2 / C3 lines, and the merge phase cycles of both (-DEBT_MERGE_STAMP builds mst / mst0).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4n
for i in 1 2; do
  bash tools/gpu.sh bench r4n_c2_new$i C2 --steps 50 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_prev.so bash tools/gpu.sh bench r4n_c2_prev$i C2 --steps 50 --no-cpu-baseline
done
for i in 1 2; do
  bash tools/gpu.sh bench r4n_c3_new$i C3 --steps 20 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_prev.so bash tools/gpu.sh bench r4n_c3_prev$i C3 --steps 20 --no-cpu-baseline
done
mkdir -p gpurun_out/r4n_stamp
for c in C2 C3; do
  EBERT_LIB=_abl/libebert_mst.so timeout -k 10 300 python -u tools/merge_stamp.py --config $c >> gpurun_out/r4n_stamp/new.jsonl
  EBERT_LIB=_abl/libebert_mst0.so timeout -k 10 300 python -u tools/merge_stamp.py --config $c >> gpurun_out/r4n_stamp/prev.jsonl
done
