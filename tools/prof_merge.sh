export TMPDIR=/tmp
mkdir -p gpurun_out/profm
cd gpurun_out/profm && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d . -o merge -- python3 ../../tools/merge_bench.py > mb.log 2>&1; rc=$?; cd ../..; find gpurun_out/profm -name "*kernel_stats.csv" | head -3; exit $rc
