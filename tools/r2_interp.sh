#!/bin/bash
# Wave merge with the interpolated cut search: the -m gpu suite,
# C2 and C3 bench lines, rocprofv3 kernel stats of the C2 and C3 benches.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/interp
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline --steps 50 > $O/c2.json 2> $O/c2.log &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3.json 2> $O/c3.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --config C2 --no-cpu-baseline --steps 50 > $O/prof2.json 2> $O/prof2.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3 -o run -- python3 bench.py --no-cpu-baseline > $O/prof3.json 2> $O/prof3.log
rc=$?
echo "rc=$rc"
tail -2 $O/pytest.log
for f in c2 c3; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['ms_per_step'], d['value'], d['roofline']['frac'], d['stage_ms_per_step'])"; done
exit $rc
