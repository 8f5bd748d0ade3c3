#!/bin/bash
# Round 3 closing pass B: the other BASELINE configurations' single-GPU lines, rank 0's C3/8 and
# C5/8 work (tools/shard_sim.py), and the N = 8 --share-gpu rehearsal of the sharded path.
export TMPDIR=/tmp
O=gpurun_out/${1:-r3fb}
mkdir -p $O
timeout -k 10 200 python -u bench.py --config C2 --no-cpu-baseline --steps 50 > $O/bench_C2.json 2> $O/bench_C2.log &&
timeout -k 10 400 python -u bench.py --config C4 --no-cpu-baseline --steps 10 --device-check 32 > $O/bench_C4.json 2> $O/bench_C4.log &&
timeout -k 10 500 python -u bench.py --config C5 --no-cpu-baseline --steps 3 --device-check 32 > $O/bench_C5.json 2> $O/bench_C5.log &&
timeout -k 10 300 python -u tools/shard_sim.py --config C3 --one-rank --ranks 8 --steps 10 --only shared > $O/shard_C3.jsonl 2> $O/shard_C3.log &&
timeout -k 10 400 python -u tools/shard_sim.py --config C5 --one-rank --ranks 8 --steps 3 --only cut > $O/shard_C5.jsonl 2> $O/shard_C5.log &&
timeout -k 10 500 python -u bench.py --gpus 8 --share-gpu --config C3 --steps 2 --warmup 1 --cpu-budget 4 > $O/rehearse_n8.json 2> $O/rehearse_n8.log
rc=$?
echo "r3_finalB rc=$rc"
for f in C2 C4 C5; do python -c "
import json
d=[json.loads(l) for l in open('$O/bench_$f.json') if l.startswith('{')][0]
print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['stage_ms_per_step'], d.get('device_parity',{}).get('rows_bit_exact'))
" || true; done
cat $O/shard_C3.jsonl $O/shard_C5.jsonl 2>/dev/null
grep '^{' $O/rehearse_n8.json | cut -c1-300
exit $rc
