#!/bin/bash
# GEMM lab attribution variants + C2 / C3 bench lines of the current tree
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c2; mkdir -p $O
timeout -k 10 300 python tools/gemm_lab/run.py --rounds 4 base nozero nocoltest trivepi > $O/lab.jsonl 2> $O/lab.log &&
timeout -k 10 200 python bench.py --config C2 --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_C2.json 2> $O/bench_C2.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_C3.json 2> $O/bench_C3.log
rc=$?
cat $O/lab.jsonl; cut -c1-1500 $O/bench_C2.json; cut -c1-1200 $O/bench_C3.json
exit $rc
