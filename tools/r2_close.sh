#!/bin/bash
# Round-2 closing pass on the final tree: the -m gpu suite, smoke(), the default bench line (as
# the driver runs it), rocprofv3 kernel stats of the same command, and the two-rank multi-process
# rehearsal (one GPU, gloo) with its oracle parity.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/close
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --durations=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof.json 2> $O/prof.log &&
timeout -k 10 400 python -u bench.py --gpus 2 --share-gpu --steps 5 --warmup 2 > $O/n2.json 2> $O/n2.log
rc=$?
echo "close rc=$rc"
tail -2 $O/pytest.log; tail -1 $O/smoke.log
python3 -c "import json;d=json.load(open('$O/bench.json'));print('C3', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['per_launch']['avg_ms'], d['stage_ms_per_step'], d['parity']['rows_bit_exact'], d['parity']['queries_checked'])"
grep '^{' $O/n2.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('N2', d['n_gpus'], d['ms_per_step'], d['parity']['rows_bit_exact'], d['parity']['queries_checked'])"
exit $rc
