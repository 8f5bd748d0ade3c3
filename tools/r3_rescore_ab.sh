#!/bin/bash
# Round 3: rescore through LDS-DMA batches (default) vs the register gather (_abl/libebert_regs.so,
# -DEBT_RESCORE_REGISTERS): the GPU tests that exercise the rescore on the default build, then
# C2 / C3 bench lines interleaved A B A B, and the C3/8 per-rank step of each.
export TMPDIR=/tmp
O=gpurun_out/${1:-r3g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_sharded.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for round in 1 2; do
  for v in lds regs; do
    if [ $v = regs ]; then export EBERT_LIB=$PWD/_abl/libebert_regs.so; else unset EBERT_LIB; fi
    for c in C2 C3; do
      timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 30 > $O/${c}_${v}_$round.json 2> $O/${c}_${v}_$round.log || exit 1
      python -c "
import json
d=[json.loads(l) for l in open('$O/${c}_${v}_$round.json') if l.startswith('{')][0]
print('$c $v $round', d['ms_per_step'], 'rescore', d['stage_ms_per_step']['rescore'], 'merge', d['stage_ms_per_step']['merge_select'])"
    done
  done
done
unset EBERT_LIB
