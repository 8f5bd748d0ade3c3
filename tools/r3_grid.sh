#!/bin/bash
# screening GEMM rate on a CU subset (ablation build _abl/libebert_grid.so, EBT_QP_GRID) with
# in-kernel clock stamps: does the chip's power limit give back clock when fewer CUs run it?
export TMPDIR=/tmp
O=gpurun_out/${1:-r3grid}
mkdir -p $O
for g in 256 240 224 192 256 240; do
  EBT_QP_GRID=$g timeout -k 10 120 python -u tools/clock_stamp.py --lib _abl/libebert_grid.so --secs 2 > $O/grid_$g.jsonl 2> $O/grid_$g.log || { tail -5 $O/grid_$g.log; exit 1; }
  echo "grid $g: $(head -1 $O/grid_$g.jsonl)"
done
