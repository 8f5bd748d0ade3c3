#!/bin/bash
# rocprofv3 evidence for one bench.py configuration: a kernel-trace + stats pass, then one PMC
# pass per TCC counter (FETCH_SIZE and WRITE_SIZE do not fit one pass) restricted to the
# screening GEMM. Usage: prof_bench.sh CONFIG [STEPS]. Summarise with tools/bench_profile.py.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CFG=${1:-C3}
STEPS=${2:-5}
O=$R/gpurun_out/prof_$CFG
mkdir -p $O
B="python3 $R/bench.py --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.json 2> $O/trace.log &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex screen_gemm --output-format csv -d $O/fetch -o run -- $B > $O/fetch.json 2> $O/fetch.log &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex screen_gemm --output-format csv -d $O/write -o run -- $B > $O/write.json 2> $O/write.log
echo "prof_bench $CFG rc=$?"
