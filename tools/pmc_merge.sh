#!/bin/bash
# PMC pass over the C2 bench: where the wave merge's time goes (waits vs issue).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_merge
mkdir -p $O
cd $R
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $O/p1 -o run -- python3 bench.py --config C2 --no-cpu-baseline --steps 10 --warmup 2 > $O/p1.json 2> $O/p1.log &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 bench.py --config C2 --no-cpu-baseline --steps 10 --warmup 2 > $O/p2.json 2> $O/p2.log
rc=$?
python3 - <<'PY'
import csv, glob, collections
for p in ("p1", "p2"):
    fs = glob.glob(f"gpurun_out/pmc_merge/{p}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print(p, "no csv"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for row in csv.DictReader(open(fs[0])):
        name = row["Kernel_Name"][:50]
        acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
        n[(name, row["Counter_Name"])] += 1
    for name, d in acc.items():
        if "merge_wave" in name or "rescore" in name or "qp2" in name:
            print(p, name, {k: round(v / n[(name, k)]) for k, v in d.items()})
PY
exit $rc
