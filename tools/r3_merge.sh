#!/bin/bash
# Round 3: the block merge rewrite -- the GPU tests that run it (large-k' fused screens, the
# deferred tier, the C5-shaped workloads), then the C5/8 per-rank step with the sample at 1/200
# (default) and 1/100 of the rows (_abl/libebert_s100.so), then the C5 full single-GPU line.
export TMPDIR=/tmp
O=gpurun_out/${1:-r3h}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=3 --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
for v in s200; do
  if [ $v = s100 ]; then export EBERT_LIB=$PWD/_abl/libebert_s100.so; else unset EBERT_LIB; fi
  timeout -k 10 400 python -u tools/shard_sim.py --config C5 --one-rank --ranks 8 --steps 3 --only cut > $O/shard_C5_$v.jsonl 2> $O/shard_C5_$v.log || { tail -5 $O/shard_C5_$v.log; exit 1; }
  echo "$v"; cat $O/shard_C5_$v.jsonl
done
unset EBERT_LIB
timeout -k 10 500 python -u bench.py --config C5 --no-cpu-baseline --steps 3 --device-check 32 > $O/bench_C5.json 2> $O/bench_C5.log || exit 1
python -c "
import json
d=[json.loads(l) for l in open('$O/bench_C5.json') if l.startswith('{')][0]
print('C5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['stage_ms_per_step'], d.get('device_parity',{}).get('rows_bit_exact'))"
