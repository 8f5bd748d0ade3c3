#!/bin/bash
# Filter GEMM per-launch rate vs segment rows (C3 N=1 segment 333,334 rows vs the 8-way shard's
# 125,000), with in-kernel clock stamps (_abl/libebert_stamp.so, tools/abl_build.sh stamp -DEBT_CLOCK_STAMP)
export TMPDIR=/tmp
O=gpurun_out/${1:-r3gn}
mkdir -p $O
for n in 333334 125000 62500; do
  timeout -k 10 120 python -u tools/clock_stamp.py --n $n --secs 2 > $O/stamp_$n.jsonl 2> $O/stamp_$n.log || { tail -5 $O/stamp_$n.log; exit 1; }
  cat $O/stamp_$n.jsonl
done
