#!/bin/bash
# Stage-timer events without the system-scope fence (gpurun -- bash tools/ab_evfence.sh): the
# timed steps bracket the dominant kernel with hipEvents (roofline); created with
# hipEventDisableSystemFence they no longer write back + invalidate the caches around it. The
# -m gpu suite and interleaved C2 / C3 lines against the previous commit (_abl/libebert_prev.so),
# then a rocprofv3 kernel trace of the new C2 command (the stream gaps around the filter).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4v
for i in 1 2; do
  bash tools/gpu.sh bench r4v_c2_new$i C2 --steps 50 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_prev.so bash tools/gpu.sh bench r4v_c2_prev$i C2 --steps 50 --no-cpu-baseline
done
for i in 1 2; do
  bash tools/gpu.sh bench r4v_c3_new$i C3 --steps 20 --no-cpu-baseline
  EBERT_LIB=_abl/libebert_prev.so bash tools/gpu.sh bench r4v_c3_prev$i C3 --steps 20 --no-cpu-baseline
done
bash tools/gpu.sh trace r4v_trace python3 bench.py --config C2 --steps 10 --warmup 1 --no-cpu-baseline
