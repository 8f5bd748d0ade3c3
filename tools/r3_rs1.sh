#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r3rs1}
mkdir -p $O
timeout -k 10 200 python -u tools/rank_sim.py --config C3 --world 8 > $O/rs8.jsonl 2> $O/rs8.log || { tail -5 $O/rs8.log; exit 1; }
cat $O/rs8.jsonl
