#!/bin/bash
# Round 3, first GPU pass: the whole -m gpu suite (incl. the 8-rank sharded tests at the C3/C4/C5
# shapes and the 8-process --share-gpu rehearsal), the default N = 1 bench line, and the C3
# N = 8 --share-gpu rehearsal line.
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s --maxfail=3 --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_C3.json 2> $O/bench_C3.log &&
timeout -k 10 500 python -u bench.py --gpus 8 --share-gpu --config C3 --steps 2 --warmup 1 --cpu-budget 4 > $O/rehearse_n8.json 2> $O/rehearse_n8.log
rc=$?
echo "r3_first rc=$rc"
tail -15 $O/pytest.log
cut -c1-600 $O/bench_C3.json
exit $rc
