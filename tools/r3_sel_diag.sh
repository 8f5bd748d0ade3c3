#!/bin/bash
# Streaming select diagnostics: the shipped build, the previous build (_abl/libebert_old.so) and
# the stream-only diagnostic (_abl/libebert_d1.so, -DEBT_SEL_DIAG=1), each beside torch.amax over
# the same 4096 x 1M matrix; then the select-path GPU tests. Log under gpurun_out/seldiag.
export TMPDIR=/tmp
O=gpurun_out/seldiag; mkdir -p $O
for r in 1 2; do
for v in ship tpi1 tpi3 d1; do
  if [ $v = ship ]; then L=robot_ebert_amd/libebert.so; else L=_abl/libebert_$v.so; fi
  [ -f $L ] || continue
  EBERT_LIB=$L timeout -k 10 120 python -u tools/sel_diag.py --tag $v >> $O/diag.jsonl 2>$O/$v.err || { tail -5 $O/$v.err; exit 1; }
done
done
cat $O/diag.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
