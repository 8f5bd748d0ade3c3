#!/bin/bash
# block merge load batching: its tests, then rank 0's C5/8 step (merges) and the C5 line
export TMPDIR=/tmp
O=gpurun_out/${1:-r3bm}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "merge or block or large_kprime or deferred or workloads or sharded_scale" --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 400 python -u tools/shard_sim.py --config C5 --one-rank --ranks 8 --steps 3 --only cut > $O/shard_C5.jsonl 2> $O/shard_C5.log || { tail -5 $O/shard_C5.log; exit 1; }
cat $O/shard_C5.jsonl
