#!/bin/bash
# The -m gpu suite on the current tree (log under gpurun_out/$1, default t).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-t}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --durations=8 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed|Error|assert" $O/pytest.log | tail -15
exit $rc
