#!/bin/bash
# Consecutive batches on 1 vs 2 HIP streams (bench.py --streams), interleaved A/B at C2 and C3.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/streams
mkdir -p $O
cd $R
for rep in 1 2; do
  for c in C2 C3; do
    for s in 1 2; do
      timeout -k 10 240 python bench.py --config $c --streams $s --no-cpu-baseline --steps 50 > $O/${c}_s${s}_r$rep.json 2> $O/${c}_s${s}_r$rep.log || exit 1
      python -c "import json;d=json.load(open('$O/${c}_s${s}_r$rep.json'));print('$c s=$s rep=$rep', d['ms_per_step'], d['value'], d['roofline']['frac'], d['stage_ms_per_step'])"
    done
  done
done
