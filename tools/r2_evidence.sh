#!/bin/bash
# Evidence pass on the current tree: rocprofv3 kernel stats + HBM PMC of the C3 and C2 bench
# commands (tools/prof_bench.sh), and one clock / MFMA-busy PMC pass of the C3 bench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/clk_C3
mkdir -p $O
bash tools/prof_bench.sh C3 5 &&
bash tools/prof_bench.sh C2 20 &&
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA --kernel-include-regex screen_gemm --output-format csv -d $O/p1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/p1.json 2> $O/p1.log
rc=$?
echo "r2_evidence rc=$rc"
exit $rc
