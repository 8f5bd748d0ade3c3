#!/bin/bash
# Round-2 closing pass on the tree: the -m gpu suite, smoke(), the default bench line (as the
# driver runs it), rocprofv3 kernel stats of the same command, C2 and C4 lines.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final2
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --durations=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof.json 2> $O/prof.log &&
timeout -k 10 300 python bench.py --config C2 --steps 50 --cpu-budget 4 > $O/c2.json 2> $O/c2.log &&
timeout -k 10 500 python bench.py --config C4 --steps 5 --warmup 2 --cpu-budget 4 > $O/c4.json 2> $O/c4.log
rc=$?
echo "final2 rc=$rc"
tail -2 $O/pytest.log; tail -1 $O/smoke.log
for f in bench c2 c4; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['ms_per_step'], d['value'], d['roofline']['frac'], d['stage_ms_per_step'], d.get('parity',{}).get('rows_bit_exact'), d.get('parity',{}).get('queries_checked'))"; done
exit $rc
