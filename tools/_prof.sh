# kernel trace of one bench configuration: tools/_prof.sh NAME [bench args...]
set -e
NAME=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$NAME -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > /dev/null 2>&1
python3 - $GRAFT_REPO_ROOT/gpurun_out/prof_$NAME/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:10.1f}us {float(r['Percentage']):6.2f}%")
PY
