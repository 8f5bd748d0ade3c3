#!/bin/bash
# Round 3: the fixed CSR-sort test, the in-kernel clock stamps of the screening GEMM
# (tools/clock_stamp.py on _abl/libebert_stamp.so), the default C3 bench line with its
# rocprofv3 kernel stats, and the C3 N = 8 --share-gpu rehearsal line.
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "sort_exclusions or offset_start" -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/clock_stamp.py > $O/clock_stamp.jsonl 2> $O/clock_stamp.log &&
timeout -k 10 300 python -u bench.py > $O/bench_C3.json 2> $O/bench_C3.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o C3 -- python3 bench.py --no-cpu-baseline --steps 20 > $O/bench_C3_prof.json 2> $O/bench_C3_prof.log &&
timeout -k 10 500 python -u bench.py --gpus 8 --share-gpu --config C3 --steps 2 --warmup 1 --cpu-budget 4 > $O/rehearse_n8.json 2> $O/rehearse_n8.log
rc=$?
echo "r3_clock rc=$rc"
tail -3 $O/pytest.log
cat $O/clock_stamp.jsonl
cut -c1-400 $O/bench_C3.json
exit $rc
