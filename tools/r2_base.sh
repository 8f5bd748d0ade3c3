#!/bin/bash
# Round-2 baseline call: GPU tests, then the default bench (C3) and C2 under rocprofv3 stats.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2b
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_C3.json 2> $O/bench_C3.log &&
timeout -k 10 200 python bench.py --config C2 --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_C2.json 2> $O/bench_C2.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_C3 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_C3.json 2> $O/prof_C3.log
echo "r2_base rc=$?"
