#!/bin/bash
# rocprofv3 kernel stats + PMC traffic of the bench command for the given configs
export TMPDIR=/tmp
for c in "$@"; do
  steps=30; [ $c = C4 ] && steps=5; [ $c = C5 ] && steps=2
  bash tools/prof_bench.sh $c $steps || exit 1
done
