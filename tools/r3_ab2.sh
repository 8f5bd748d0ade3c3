#!/bin/bash
# Round 3 A/B on one box: (1) rescore by LDS-DMA batches (default build) vs the register gather
# (_abl/libebert_regs.so) at C2, interleaved; (2) the speculative sample at 1/200 of the rows
# (default) vs 1/100 (_abl/libebert_s100.so): the C5/8 per-rank step (tools/shard_sim.py).
export TMPDIR=/tmp
O=gpurun_out/${1:-r3g}
mkdir -p $O
for round in 1 2 3; do
  for v in lds regs; do
    if [ $v = regs ]; then export EBERT_LIB=$PWD/_abl/libebert_regs.so; else unset EBERT_LIB; fi
    timeout -k 10 200 python -u bench.py --config C2 --no-cpu-baseline --steps 50 > $O/C2_${v}_$round.json 2> $O/C2_${v}_$round.log || exit 1
    python -c "
import json
d=[json.loads(l) for l in open('$O/C2_${v}_$round.json') if l.startswith('{')][0]
print('C2 $v $round', d['ms_per_step'], 'rescore', d['stage_ms_per_step']['rescore'], 'merge', d['stage_ms_per_step']['merge_select'])"
  done
done
unset EBERT_LIB
for v in s200 s100; do
  if [ $v = s100 ]; then export EBERT_LIB=$PWD/_abl/libebert_s100.so; else unset EBERT_LIB; fi
  timeout -k 10 400 python -u tools/shard_sim.py --config C5 --one-rank --ranks 8 --steps 3 --only cut > $O/shard_C5_$v.jsonl 2> $O/shard_C5_$v.log || exit 1
  echo "$v"; cat $O/shard_C5_$v.jsonl
done
unset EBERT_LIB
