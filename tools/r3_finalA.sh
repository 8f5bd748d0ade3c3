#!/bin/bash
# Round 3 closing pass A: the whole -m gpu suite, smoke(), the default bench line (C3, N = 1,
# CPU baseline + parity), and the rocprofv3 evidence of the same command (kernel stats + the
# FETCH_SIZE / WRITE_SIZE passes behind roofline.traffic).
export TMPDIR=/tmp
O=gpurun_out/${1:-r3fa}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_C3.json 2> $O/bench_C3.log || { tail -5 $O/bench_C3.log; exit 1; }
cut -c1-400 $O/bench_C3.json
bash tools/prof_bench.sh C3 5 || exit 1
