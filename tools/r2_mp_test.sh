#!/bin/bash
# The multi-process GPU test alone, then the whole -m gpu suite (as the driver runs it).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mp
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_multiprocess.py -x -v --timeout 240 --timeout-method thread > $O/mp.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --durations=5 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "rc=$rc"
tail -3 $O/mp.log; tail -8 $O/pytest.log
exit $rc
