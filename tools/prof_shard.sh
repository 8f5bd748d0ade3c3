set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_sh8 -o run -- python3 $R/tools/shard_sim.py --one-rank --ranks 8 --steps 10 --only shared > $R/gpurun_out/prof_sh8.out 2>&1
grep one_rank gpurun_out/prof_sh8.out
