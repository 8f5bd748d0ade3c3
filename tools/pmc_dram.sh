# L2 -> fabric read requests vs the ones that reach DRAM, for the screening GEMM (no-hit launch
# over 524288 rows): does FETCH_SIZE's traffic come from the Infinity Cache or from HBM?
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-include-regex qp2 --output-format csv -d $R/gpurun_out/pmc_dram -o run -- python3 $R/tools/seg_bench.py --n 524288 --hits 0 --no-inf > $R/gpurun_out/pmc_dram.log 2>&1
echo "rc=$?"
python3 - <<PY
import csv,glob,collections
tot=collections.defaultdict(float); n=collections.defaultdict(set)
for f in glob.glob("$R/gpurun_out/pmc_dram/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]]+=float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
print({k: (tot[k]/max(len(n[k]),1), len(n[k])) for k in tot})
PY
