#!/bin/bash
# Round-4 final evidence on the final tree (gpurun -- bash tools/r4_final.sh): the -m gpu suite +
# smoke, the C3 and C2 lines with the CPU baseline and host-oracle parity, rocprofv3 kernel stats
# + FETCH_SIZE / WRITE_SIZE passes of the C3 command, C4 and C5 lines with 32 queries vs the host
# float64 oracle over the whole catalog, and the N = 2 share-GPU rehearsal of the C-ABI step.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh suite r4f
bash tools/gpu.sh bench r4f C3 --steps 20
bash tools/gpu.sh bench r4f C2 --steps 50
bash tools/gpu.sh prof r4f_prof C3 5
bash tools/gpu.sh bench r4f C4 --steps 5 --warmup 1 --parity 32
bash tools/gpu.sh bench r4f C5 --steps 3 --warmup 1 --parity 32
mkdir -p gpurun_out/r4f_share
timeout -k 10 600 python -u bench.py --gpus 2 --share-gpu --steps 10 --warmup 2 \
  > gpurun_out/r4f_share/bench_C3_n2_share.json 2> gpurun_out/r4f_share/bench.log
tail -1 gpurun_out/r4f_share/bench_C3_n2_share.json | cut -c1-300
