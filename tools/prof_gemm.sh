#!/bin/bash
# PMC passes over one screening-GEMM configuration (tools/kernel_bench.py --one), one counter
# group per rocprofv3 run (no traces combined with --pmc). Usage: prof_gemm.sh NAME [B,N,d]
# (EBT_KB_THR=inf: the filter epilogue appends nothing.)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
NAME=${1:-gemm}
SHAPE=${2:-4096,262144,1536}
O=$R/gpurun_out/pmc_$NAME
mkdir -p $O
KB="python3 $R/tools/kernel_bench.py --one --shape $SHAPE"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $KB > $O/trace.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex screen_gemm --output-format csv -d $O/p1 -o run -- $KB > $O/p1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex screen_gemm --output-format csv -d $O/p2 -o run -- $KB > $O/p2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE --kernel-include-regex screen_gemm --output-format csv -d $O/p3 -o run -- $KB > $O/p3.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU --kernel-include-regex screen_gemm --output-format csv -d $O/p4 -o run -- $KB > $O/p4.log 2>&1
echo "prof_gemm $NAME rc=$?"
