#!/bin/bash
# Round-2 GPU test pass: MFMA rounding probe, full -m gpu suite (verbose, per-test timing), then
# the default bench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2t
mkdir -p $O
cd $R
timeout -k 10 120 python tools/mfma_rounding.py > $O/mfma_rounding.json 2> $O/mfma_rounding.log &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --durations=30 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] && timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_C3.json 2> $O/bench_C3.log
echo "r2_tests rc=$?"
