#!/bin/bash
# One GPU pass on the current tree: the -m gpu suite, then the C3 and C2 bench lines and a
# rocprofv3 kernel-stats run of the C3 bench. Output under gpurun_out/$1 (default r2p).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r2p}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --durations=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_C3.json 2> $O/bench_C3.log &&
timeout -k 10 200 python bench.py --config C2 --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_C2.json 2> $O/bench_C2.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_C3 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_C3.json 2> $O/prof_C3.log
rc=$?
echo "r2_gpu_pass rc=$rc"
tail -3 $O/pytest.log
cat $O/bench_C3.json $O/bench_C2.json 2>/dev/null | cut -c1-400
exit $rc
