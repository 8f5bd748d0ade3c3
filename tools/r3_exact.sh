#!/bin/bash
# the float64 large-k path and exact fallback screen: tests, then old (_abl/libebert_old.so) vs new timing
export TMPDIR=/tmp
O=gpurun_out/${1:-r3exact}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_large_k.py tests/test_gpu_parity.py tests/test_gpu_capi.py -m gpu -q -k "large or exact or golden or 10000 or certif" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
for v in old new old new; do
  if [ $v = old ]; then export EBERT_LIB=$PWD/_abl/libebert_old.so; else unset EBERT_LIB; fi
  timeout -k 10 300 python -u tools/exact_bench.py > $O/exact_$v.json 2> $O/exact_$v.log || { tail -5 $O/exact_$v.log; exit 1; }
  cat $O/exact_$v.json
done
