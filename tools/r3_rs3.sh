#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r3rs3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash tools/r3_ranksim_tl.sh r3rs3/tl > /dev/null 2>&1 || exit 1
cat $O/tl/rs.json; tail -24 $O/tl/tl.txt
