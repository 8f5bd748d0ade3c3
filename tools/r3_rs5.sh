#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r3rs5}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_capi_sharded.py tests/test_gpu_filter.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash tools/r3_ranksim_tl.sh r3rs5/tl > /dev/null 2>&1 || { tail -5 $O/tl/rs.log; exit 1; }
cat $O/tl/rs.json; grep -E "union_floor|rescore|merge|per step" $O/tl/tl.txt
