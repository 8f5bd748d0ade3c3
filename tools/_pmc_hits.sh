set -e
R=$GRAFT_REPO_ROOT
for h in 0 1024; do
  bash tools/prof_kernel.sh h$h qp2 python3 $R/tools/seg_bench.py --n 524288 --hits $h --no-inf
  timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex qp2 --output-format csv -d $R/gpurun_out/pmc_h$h/p5 -o run -- python3 $R/tools/seg_bench.py --n 524288 --hits $h --no-inf > /dev/null 2>&1
  python3 tools/pmc_summary.py gpurun_out/pmc_h$h qp2 > gpurun_out/pmc_h$h.json
done
python3 - <<'PY'
import json
a = json.load(open("gpurun_out/pmc_h0.json")); b = json.load(open("gpurun_out/pmc_h1024.json"))
for k in sorted(set(a) | set(b)):
    if k == "kernel": continue
    print(f"{k:32s} {a.get(k)!s:>24} {b.get(k)!s:>24}")
PY
