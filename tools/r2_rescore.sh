#!/bin/bash
# rescore_kernel gathering 4 rows per wave: the -m gpu suite, C2 and C3 bench lines, rocprofv3
# kernel stats of the C2 bench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rs4r
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline --steps 50 > $O/c2.json 2> $O/c2.log &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3.json 2> $O/c3.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config C2 --no-cpu-baseline --steps 50 > $O/prof.json 2> $O/prof.log
rc=$?
echo "rc=$rc"
tail -2 $O/pytest.log
cut -c1-300 $O/c2.json; cut -c1-300 $O/c3.json
exit $rc
