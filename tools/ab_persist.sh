#!/bin/bash
# Interleaved A/B on one box of the C5 per-rank step and the C4 step: _abl/libebert_pre.so
# (pre-persistent screening GEMM) vs _abl/libebert_cur.so (persistent + compacted hit path).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/abp; mkdir -p $O
for rep in 1 2; do
for v in pre cur; do
  EBERT_LIB=$GRAFT_REPO_ROOT/_abl/libebert_$v.so timeout -k 10 300 python bench.py --config C5 --n 6250000 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.log || exit 1
  python -c "import json;d=json.load(open('$O/c5_${v}_$rep.json'));print('$v C5r', d['ms_per_step'], d['roofline']['frac'], d['stage_ms_per_step'])"
  EBERT_LIB=$GRAFT_REPO_ROOT/_abl/libebert_$v.so timeout -k 10 300 python bench.py --config C4 --n 2500000 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.log || exit 1
  python -c "import json;d=json.load(open('$O/c4_${v}_$rep.json'));print('$v C4q', d['ms_per_step'], d['roofline']['frac'], d['stage_ms_per_step'])"
done
done
