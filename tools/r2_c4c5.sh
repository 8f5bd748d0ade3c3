#!/bin/bash
# Full-size single-GPU C4 / C5 bench lines (the N=1 anchors of the 8-GPU configurations), with
# the CPU baselines and the host-oracle parity sample over the full catalog.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c45
mkdir -p $O
cd $R
timeout -k 10 500 python -u bench.py --config C4 --steps 5 --warmup 2 --device-check 32 > $O/bench_C4.json 2> $O/bench_C4.log &&
timeout -k 10 600 python -u bench.py --config C5 --steps 3 --warmup 1 --device-check 32 > $O/bench_C5.json 2> $O/bench_C5.log
echo "c4c5 rc=$?"
