#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r3rs6}
mkdir -p $O
timeout -k 10 300 python -u tools/rank_sim.py --config C3 --world 8 --profile > $O/rs.json 2> $O/prof.txt || { tail -5 $O/prof.txt; exit 1; }
cat $O/rs.json
