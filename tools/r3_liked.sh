#!/bin/bash
# liked-user query prep at C3 (tools/liked_bench.py): vector form vs element form
export TMPDIR=/tmp
O=gpurun_out/${1:-r3liked}
mkdir -p $O
for L in 5 20 100; do
  for f in "" "--unaligned"; do
    timeout -k 10 200 python -u tools/liked_bench.py --liked $L $f > $O/liked_$L$f.json 2> $O/liked_$L$f.log || { tail -5 $O/liked_$L$f.log; exit 1; }
    cat $O/liked_$L$f.json
  done
done
