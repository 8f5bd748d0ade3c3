#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r3graph}
mkdir -p $O
for c in C2 C3; do
  timeout -k 10 200 python -u tools/graph_probe.py --config $c > $O/graph_$c.json 2> $O/graph_$c.log || { tail -5 $O/graph_$c.log; exit 1; }
  cat $O/graph_$c.json
done
