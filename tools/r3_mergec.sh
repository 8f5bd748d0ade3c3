#!/bin/bash
# union floor tests + merge bench (warm / cold inputs) + rank 0's replayed C3/8 step
export TMPDIR=/tmp
O=gpurun_out/${1:-r3mc}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_filter.py -m gpu -q -k "union_floor or merge" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 200 python -u tools/merge_bench.py > $O/mb.jsonl 2> $O/mb.log || { tail -5 $O/mb.log; exit 1; }
cat $O/mb.jsonl
timeout -k 10 200 python -u tools/rank_sim.py --config C3 --world 8 > $O/rs8.jsonl 2> $O/rs8.log || { tail -5 $O/rs8.log; exit 1; }
cat $O/rs8.jsonl
