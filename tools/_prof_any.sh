# kernel trace of any python command: tools/_prof_any.sh NAME script.py [args...]
set -e
NAME=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$NAME -o run -- python3 "$@" > $R/gpurun_out/prof_$NAME.out 2>&1
python3 - $R/gpurun_out/prof_$NAME/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:10.1f}us {float(r['TotalDurationNs'])/1e3:10.1f}us")
PY
