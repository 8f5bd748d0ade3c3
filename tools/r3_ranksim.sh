#!/bin/bash
# rank 0's full N > 1 pipeline (tools/rank_sim.py) at 2, 4 and 8 ranks, and its kernel timeline at 8
export TMPDIR=/tmp
O=gpurun_out/${1:-r3rs}
mkdir -p $O
for w in 8 4 2; do
  timeout -k 10 200 python -u tools/rank_sim.py --config C3 --world $w > $O/rs_$w.jsonl 2> $O/rs_$w.log || { tail -5 $O/rs_$w.log; exit 1; }
  cat $O/rs_$w.jsonl
done
(cd $O && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d tl8 -o run -- python3 ../../tools/rank_sim.py --config C3 --world 8 --steps 20 > tl8.json 2> tl8.log) || exit 1
python3 tools/step_timeline.py $(find $O/tl8 -name "*kernel_trace.csv") --steps 2 --marker query_prep > $O/tl8.txt; tail -45 $O/tl8.txt
