#!/bin/bash
# Final round-2 pass on the tree: the -m gpu suite, smoke(), the default bench line (as the
# driver runs it) and a rocprofv3 kernel-stats run of the same command.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --durations=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof.json 2> $O/prof.log
rc=$?
echo "r2_final rc=$rc"
tail -2 $O/pytest.log; tail -1 $O/smoke.log
cut -c1-600 $O/bench.json
exit $rc
