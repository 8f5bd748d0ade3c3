#!/bin/bash
# the whole -m gpu suite and smoke() on the current tree
export TMPDIR=/tmp
O=gpurun_out/${1:-r3suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
