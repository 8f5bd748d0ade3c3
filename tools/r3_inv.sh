#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r3inv}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_invariance.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" $O/pytest.log | head -20; exit $rc
