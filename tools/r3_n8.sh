#!/bin/bash
# Round 3: the sharded step's per-rank pieces at N = 8 on one MI355X -- the merge tests, the
# post-all-gather merge (co-rank vs bitonic), and rank 0's C3/8 and C4/8 work (tools/shard_sim.py).
export TMPDIR=/tmp
O=gpurun_out/${1:-r3n8}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py tests/test_gpu_capi_sharded.py -m gpu -v -k "merge or sharded" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 120 python -u tools/merge_bench.py > $O/merge_bench.jsonl 2> $O/merge_bench.log || { tail -5 $O/merge_bench.log; exit 1; }
cat $O/merge_bench.jsonl
timeout -k 10 300 python -u tools/shard_sim.py --config C3 --one-rank --ranks 8 --steps 5 > $O/shard_C3.jsonl 2> $O/shard_C3.log || { tail -5 $O/shard_C3.log; exit 1; }
cat $O/shard_C3.jsonl
