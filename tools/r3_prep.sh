#!/bin/bash
# query prep (wave kernel) tests + one-step kernel timelines of C2 and C3 bench runs
export TMPDIR=/tmp
O=gpurun_out/${1:-r3prep}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_certificate.py tests/test_gpu_sharded.py tests/test_gpu_capi_sharded.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
for c in C2 C3; do
  (cd $O && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d tl_$c -o run -- python3 ../../bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > tl_$c.json 2> tl_$c.log) || exit 1
  python3 tools/step_timeline.py $(find $O/tl_$c -name "*kernel_trace.csv") --steps 2 > $O/tl_$c.txt || exit 1
  tail -40 $O/tl_$c.txt
done
