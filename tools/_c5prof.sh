export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o run -- python3 $R/bench.py --config C5 --n 6250000 --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c5.json 2> $R/gpurun_out/prof_c5.log
echo rc=$?
python3 - <<PY
import csv
rows=list(csv.DictReader(open("$R/gpurun_out/prof_c5/run_kernel_stats.csv")))
for r in rows[:14]:
    print(r["Name"][:80], r["Calls"], round(float(r["TotalDurationNs"])/1e6,2), round(float(r["AverageNs"])/1e3,1))
PY
