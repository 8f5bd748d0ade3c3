#!/bin/bash
# One GPU call: interleaved timing of the built variants (names as arguments), without and with
# row scales (the two filter epilogues).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gl
timeout -k 10 300 python tools/gemm_lab/run.py "$@" > gpurun_out/gl/run.jsonl 2> gpurun_out/gl/run.log &&
timeout -k 10 300 python tools/gemm_lab/run.py --cscale "$@" > gpurun_out/gl/run_cs.jsonl 2> gpurun_out/gl/run_cs.log
rc=$?
echo "gemm_lab rc=$rc"
cat gpurun_out/gl/run.jsonl gpurun_out/gl/run_cs.jsonl
exit $rc
