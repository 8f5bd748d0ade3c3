#!/bin/bash
# Per-rank work of the C3 row-sharded step at 2 / 4 / 8 ranks, simulated on one GPU
# (tools/shard_sim.py --one-rank: rank 0's kernels, the other shards' samples / floors
# precomputed, no communication).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sh
timeout -k 10 500 python tools/shard_sim.py --one-rank --ranks 2 4 8 --steps 20 > gpurun_out/sh/sim.out 2> gpurun_out/sh/sim.log
rc=$?
grep -v amdgpu.ids gpurun_out/sh/sim.out | tail -20
exit $rc
