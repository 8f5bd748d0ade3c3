export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_qp2
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/kernel_bench.py --one > $O/trace.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex screen_gemm --output-format csv -d $O/p1 -o run -- python3 $R/tools/kernel_bench.py --one > $O/p1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex screen_gemm --output-format csv -d $O/p2 -o run -- python3 $R/tools/kernel_bench.py --one > $O/p2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE --kernel-include-regex screen_gemm --output-format csv -d $O/p3 -o run -- python3 $R/tools/kernel_bench.py --one > $O/p3.log 2>&1
echo done $?
