#!/bin/bash
# Round-2 first GPU call: GPU tests after the tree clean-up, HBM-kernel evidence under
# rocprofv3 (kernel trace + stats), the PMC clock / MFMA-busy pass on the screening GEMM.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2a
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/topk -o run -- python3 tools/topk_evidence.py > $O/topk.json 2> $O/topk.log &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex qp2 --output-format csv -d $O/pmc_clk -o run -- python3 tools/kernel_bench.py --one > $O/pmc_clk.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gemm_trace -o run -- python3 tools/kernel_bench.py --one > $O/gemm_trace.log 2>&1
echo "r2_first rc=$?"
