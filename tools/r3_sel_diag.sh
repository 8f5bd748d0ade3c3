#!/bin/bash
# Streaming select: the select-path GPU tests on an ablation build (_abl/libebert_room5.so,
# -DEBT_SEL_ROOM=5 -DEBT_SEL_WGS=3), then its timing interleaved with the shipped build, each
# beside torch.amax over the same 4096 x 1M matrix (tools/sel_diag.py). Log under gpurun_out/seldiag.
export TMPDIR=/tmp
O=gpurun_out/seldiag; mkdir -p $O
EBERT_LIB=_abl/libebert_room5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_room5.log 2>&1 || { tail -20 $O/pytest_room5.log; exit 1; }
tail -1 $O/pytest_room5.log
for r in 1 2; do
for v in ship room5; do
  if [ $v = ship ]; then L=robot_ebert_amd/libebert.so; else L=_abl/libebert_$v.so; fi
  [ -f $L ] || continue
  EBERT_LIB=$L timeout -k 10 120 python -u tools/sel_diag.py --tag $v >> $O/diag.jsonl 2>$O/$v.err || { tail -5 $O/$v.err; exit 1; }
done
done
cat $O/diag.jsonl
