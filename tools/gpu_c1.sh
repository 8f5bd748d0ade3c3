#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c1
bash tools/gemm_lab/gpu.sh base new > gpurun_out/c1/lab.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --durations=5 --timeout 300 --timeout-method thread > gpurun_out/c1/pytest.log 2>&1
rc=$?
cat gpurun_out/c1/lab.txt; tail -5 gpurun_out/c1/pytest.log
exit $rc
