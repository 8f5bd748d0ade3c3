#!/bin/bash
# merge kernel check + timing (tests, tools/merge_bench.py)
export TMPDIR=/tmp
O=gpurun_out/${1:-r3mb}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py tests/test_gpu_parity.py -m gpu -v -k "merge or golden or rescore" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 120 python -u tools/merge_bench.py > $O/merge_bench.jsonl 2> $O/merge_bench.log || { tail -5 $O/merge_bench.log; exit 1; }
cat $O/merge_bench.jsonl
