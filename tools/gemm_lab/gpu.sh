#!/bin/bash
# One GPU call: interleaved timing of the built variants (names as arguments).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gl
timeout -k 10 300 python tools/gemm_lab/run.py "$@" > gpurun_out/gl/run.jsonl 2> gpurun_out/gl/run.log
echo "gemm_lab rc=$?"
cat gpurun_out/gl/run.jsonl
