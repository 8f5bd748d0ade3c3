#!/bin/bash
# rocprofv3 kernel trace of rank 0's C3/8 step (tools/shard_sim.py --one-rank --only shared)
export TMPDIR=/tmp
O=gpurun_out/${1:-profsh}
mkdir -p $O
cd $O && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d . -o sh -- python3 ../../tools/shard_sim.py --config ${2:-C3} --one-rank --ranks 8 --only shared --steps 10 > sh.log 2>&1
