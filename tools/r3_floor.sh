#!/bin/bash
# union floor kernels: the GPU tests, then rank 0's full N > 1 pipeline (tools/rank_sim.py)
export TMPDIR=/tmp
O=gpurun_out/${1:-r3fl}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_capi_sharded.py tests/test_gpu_sharded_scale.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
for w in 8 4; do
  timeout -k 10 200 python -u tools/rank_sim.py --config C3 --world $w > $O/rs_$w.jsonl 2> $O/rs_$w.log || { tail -5 $O/rs_$w.log; exit 1; }
  cat $O/rs_$w.jsonl
done
