#!/bin/bash
# Streaming select A/B: tiles in flight per workgroup (EBT_SEL_TPI 1 / 2 / 4), interleaved,
# plus the select-path GPU tests on the shipped build. Log under gpurun_out/sel.
export TMPDIR=/tmp
O=gpurun_out/sel; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in tpi1 ship tpi4; do
    if [ $v = ship ]; then L=robot_ebert_amd/libebert.so; else L=_abl/libebert_$v.so; fi
    EBERT_LIB=$L timeout -k 10 240 python -u tools/topk_evidence.py --iters 10 > $O/$v.$r.jsonl 2>&1 || { tail -5 $O/$v.$r.jsonl; exit 1; }
    echo "$v $r: $(grep select_topk $O/$v.$r.jsonl | tr '\n' ' ')"
  done
done
