#!/bin/bash
# MFMA issue order A/B (operand switching): i-outer (default) vs j-outer (_abl/libebert_ji.so),
# interleaved, in-kernel clock stamps on random C3-shaped operands
export TMPDIR=/tmp
O=gpurun_out/${1:-r3ji}
mkdir -p $O
for v in grid ji grid ji; do
  timeout -k 10 120 python -u tools/clock_stamp.py --lib _abl/libebert_$v.so --secs 2 > $O/$v.jsonl 2> $O/$v.log || { tail -5 $O/$v.log; exit 1; }
  echo "$v: $(head -2 $O/$v.jsonl | cut -c1-200)"
done
