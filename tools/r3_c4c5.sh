#!/bin/bash
# C4 and C5 single-GPU lines on the current tree
export TMPDIR=/tmp
O=gpurun_out/${1:-r3c4c5}
mkdir -p $O
timeout -k 10 400 python -u bench.py --config C4 --no-cpu-baseline --steps 10 --device-check 32 > $O/bench_C4.json 2> $O/bench_C4.log || { tail -5 $O/bench_C4.log; exit 1; }
timeout -k 10 500 python -u bench.py --config C5 --no-cpu-baseline --steps 3 --device-check 32 > $O/bench_C5.json 2> $O/bench_C5.log || { tail -5 $O/bench_C5.log; exit 1; }
for f in C4 C5; do python3 -c "
import json
d=[json.loads(l) for l in open('$O/bench_$f.json') if l.startswith('{')][0]
print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('device_parity',{}).get('rows_bit_exact'), d.get('parity',{}).get('rows_bit_exact'))"; done
