#!/bin/bash
# PMC passes over any kernel: prof_kernel.sh NAME REGEX CMD... -- a kernel-trace + stats pass,
# then one counter group per rocprofv3 run (no traces combined with --pmc), restricted to the
# kernels matching REGEX. Summarise with: python tools/pmc_summary.py gpurun_out/pmc_NAME REGEX
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
NAME=$1; RX=$2; shift 2
O=$R/gpurun_out/pmc_$NAME
mkdir -p $O
P="--kernel-include-regex $RX --output-format csv"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- "$@" > $O/trace.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES $P -d $O/p1 -o run -- "$@" > $O/p1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE $P -d $O/p2 -o run -- "$@" > $O/p2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS $P -d $O/p3 -o run -- "$@" > $O/p3.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM $P -d $O/p4 -o run -- "$@" > $O/p4.log 2>&1
echo "prof_kernel $NAME rc=$?"
