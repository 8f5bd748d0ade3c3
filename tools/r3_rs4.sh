#!/bin/bash
export TMPDIR=/tmp
bash tools/r3_ranksim_tl.sh r3rs4 > /dev/null 2>&1 || { tail -5 gpurun_out/r3rs4/rs.log; exit 1; }
cat gpurun_out/r3rs4/rs.json; tail -24 gpurun_out/r3rs4/tl.txt
