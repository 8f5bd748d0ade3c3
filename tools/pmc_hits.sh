export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for h in 0 128 1024; do
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-include-regex qp2 --output-format csv -d $R/gpurun_out/hp_$h -o run -- python3 $R/tools/seg_bench.py --n 131072 --hits $h --no-inf > $R/gpurun_out/hp_$h.log 2>&1
echo "h=$h rc=$?"
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_LDS_ATOMIC SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-include-regex qp2 --output-format csv -d $R/gpurun_out/hq_$h -o run -- python3 $R/tools/seg_bench.py --n 131072 --hits $h --no-inf > $R/gpurun_out/hq_$h.log 2>&1
python3 - <<PY
import csv,glob,collections
tot=collections.defaultdict(float); n=collections.defaultdict(set)
for d in ("hp","hq"):
  for f in glob.glob("$R/gpurun_out/%s_$h/**/*counter_collection.csv" % d, recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]]+=float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
print("$h", {k: round(tot[k]/max(len(n[k]),1)/65536, 1) for k in sorted(tot)})
PY
done
