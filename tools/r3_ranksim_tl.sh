#!/bin/bash
# kernel timeline of rank 0's replayed C3/8 step (tools/rank_sim.py under rocprofv3)
export TMPDIR=/tmp
O=gpurun_out/${1:-r3rstl}
mkdir -p $O
(cd $O && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d tl -o run -- python3 $GRAFT_REPO_ROOT/tools/rank_sim.py --config C3 --world 8 --steps 20 > rs.json 2> rs.log) || { tail -5 $O/rs.log; exit 1; }
cat $O/rs.json
python3 tools/step_timeline.py $(find $O/tl -name "*kernel_trace.csv") --steps 2 --marker query_prep > $O/tl.txt; cat $O/tl.txt
