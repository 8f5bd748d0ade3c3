#!/bin/bash
# Round 3: the -m gpu suite, then the speculative sample scaled with the catalog (C4 / C5 full
# single-GPU lines, the C5/8 per-rank step simulated on one GPU), C2 / C3 regression lines.
export TMPDIR=/tmp
O=gpurun_out/${1:-r3e}
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s --maxfail=3 --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config C2 --no-cpu-baseline --steps 50 > $O/bench_C2.json 2> $O/bench_C2.log &&
timeout -k 10 200 python -u bench.py --config C3 --no-cpu-baseline > $O/bench_C3.json 2> $O/bench_C3.log &&
timeout -k 10 400 python -u bench.py --config C4 --no-cpu-baseline --steps 10 --device-check 32 > $O/bench_C4.json 2> $O/bench_C4.log &&
timeout -k 10 500 python -u bench.py --config C5 --no-cpu-baseline --steps 3 --device-check 32 > $O/bench_C5.json 2> $O/bench_C5.log &&
timeout -k 10 500 python -u tools/shard_sim.py --config C5 --one-rank --ranks 8 --steps 3 > $O/shard_sim_C5.jsonl 2> $O/shard_sim_C5.log
rc=$?
echo "r3_perf rc=$rc"
grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8
for f in C2 C3 C4 C5; do python -c "
import json,sys
try:
    d=[json.loads(l) for l in open('$O/bench_$f.json') if l.startswith('{')][0]
    print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['stage_ms_per_step'], d.get('plan',{}).get('spec'), d.get('device_parity',{}).get('rows_bit_exact'))
except Exception as e: print('$f', 'n/a', e)
"; done
cat $O/shard_sim_C5.jsonl 2>/dev/null
exit $rc
