#!/bin/bash
# C3 default bench (twice) and C2, after the load-scheduling fixes
export TMPDIR=/tmp
O=gpurun_out/${1:-r3c3c2}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_C3_$i.json 2> $O/bench_C3_$i.log || { tail -5 $O/bench_C3_$i.log; exit 1; }
done
timeout -k 10 200 python -u bench.py --config C2 --no-cpu-baseline --steps 50 > $O/bench_C2.json 2> $O/bench_C2.log || exit 1
for f in C3_1 C3_2 C2; do python3 -c "
import json
d=[json.loads(l) for l in open('$O/bench_$f.json') if l.startswith('{')][0]
print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['stage_ms_per_step'])"; done
