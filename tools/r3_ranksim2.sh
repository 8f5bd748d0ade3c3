#!/bin/bash
# rank 0's full N > 1 pipeline (tools/rank_sim.py): C3/2, C4/8, C5/8
export TMPDIR=/tmp
O=gpurun_out/${1:-r3rs2}
mkdir -p $O
timeout -k 10 200 python -u tools/rank_sim.py --config C3 --world 2 > $O/rs_C3_2.jsonl 2> $O/rs_C3_2.log && cat $O/rs_C3_2.jsonl &&
timeout -k 10 400 python -u tools/rank_sim.py --config C4 --world 8 --steps 6 > $O/rs_C4_8.jsonl 2> $O/rs_C4_8.log && cat $O/rs_C4_8.jsonl &&
timeout -k 10 600 python -u tools/rank_sim.py --config C5 --world 8 --steps 3 > $O/rs_C5_8.jsonl 2> $O/rs_C5_8.log && cat $O/rs_C5_8.jsonl
rc=$?; [ $rc -ne 0 ] && tail -5 $O/*.log; exit $rc
