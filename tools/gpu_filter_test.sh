#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gf
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py -m gpu -x -q -rf -s --timeout 120 --timeout-method thread > gpurun_out/gf/pytest.log 2>&1
rc=$?
grep -E "hits per query|passed|failed|Error|assert" gpurun_out/gf/pytest.log | head -30
exit $rc
