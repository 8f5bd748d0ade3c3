#!/bin/bash
# Round 3: the -m gpu suite (verbose, per-test timeout) on the current tree.
export TMPDIR=/tmp
O=gpurun_out/${1:-r3t}
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s --maxfail=3 --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "r3_tests rc=$rc"
grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -15
exit $rc
