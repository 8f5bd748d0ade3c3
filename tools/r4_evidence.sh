#!/bin/bash
# Round-4 closing evidence (gpurun -- bash tools/r4_evidence.sh): the C3 and C2 bench lines with
# the CPU baseline and the host-oracle parity sample, rocprofv3 kernel stats + FETCH_SIZE /
# WRITE_SIZE passes of the C3 bench command, and the N = 2 rehearsal of the C-ABI sharded step
# (two ranks sharing GPU 0 over gloo) with its parity sample.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh bench r4z C3 --steps 20
bash tools/gpu.sh bench r4z C2 --steps 50
bash tools/gpu.sh prof r4z_prof C3 5
mkdir -p gpurun_out/r4z_share
timeout -k 10 600 python -u bench.py --gpus 2 --share-gpu --steps 10 --warmup 2 \
  > gpurun_out/r4z_share/bench_C3_n2_share.json 2> gpurun_out/r4z_share/bench.log
tail -1 gpurun_out/r4z_share/bench_C3_n2_share.json | cut -c1-400
