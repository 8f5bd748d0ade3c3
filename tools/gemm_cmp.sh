#!/bin/bash
# GEMM variant comparison on one GPU: default (pq) vs qp2 at several shapes.
set -o pipefail
for shape in 4096,262144,1536 4096,262144,768 4096,65536,1536 1024,100000,768; do
  for t in 0 2; do
    EBT_GEMM_TILE=$t timeout -k 10 120 python tools/kernel_bench.py --one --shape $shape || exit $?
  done
done
