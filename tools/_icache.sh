export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1
grep -io "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQC_TC_INST[A-Z_]*\|SQ_INSTS_[A-Z_]*" $R/gpurun_out/counters.txt | sort -u | tr '\n' ' '
echo
for h in 0 1024; do
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex qp2 --output-format csv -d $R/gpurun_out/ic_$h -o run -- python3 $R/tools/seg_bench.py --n 131072 --hits $h --no-inf > $R/gpurun_out/ic_$h.log 2>&1
echo "h=$h rc=$?"
python3 - <<PY
import csv,glob,collections
tot=collections.defaultdict(float); n=collections.defaultdict(set)
for f in glob.glob("$R/gpurun_out/ic_$h/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]]+=float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
print({k: tot[k]/max(len(n[k]),1) for k in tot})
PY
done
