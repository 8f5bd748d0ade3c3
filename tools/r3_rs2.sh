#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r3rs2b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py tests/test_gpu_sharded.py tests/test_gpu_capi_sharded.py tests/test_gpu_parity.py -m gpu -q -k "merge or union_floor or sharded" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 200 python -u tools/rank_sim.py --config C3 --world 8 > $O/rs8.jsonl 2> $O/rs8.log || { tail -5 $O/rs8.log; exit 1; }
cat $O/rs8.jsonl
