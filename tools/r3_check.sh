#!/bin/bash
# the whole -m gpu suite, smoke(), the default bench line and the N = 8 --share-gpu rehearsal on the current tree
export TMPDIR=/tmp
O=gpurun_out/${1:-r3check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_C3.json 2> $O/bench_C3.log || { tail -5 $O/bench_C3.log; exit 1; }
timeout -k 10 500 python -u bench.py --gpus 8 --share-gpu --config C3 --steps 2 --warmup 1 --cpu-budget 4 > $O/rehearse_n8.json 2> $O/rehearse_n8.log || { tail -5 $O/rehearse_n8.log; exit 1; }
python3 -c "
import json
d=[json.loads(l) for l in open('$O/bench_C3.json') if l.startswith('{')][0]
print('C3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['rows_bit_exact'], d['cpu_baseline']['value'])
d=[json.loads(l) for l in open('$O/rehearse_n8.json') if l.startswith('{')][0]
print('N8', d['parity']['rows_bit_exact'], d['parity']['queries_checked'])"
