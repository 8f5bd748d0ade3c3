set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log
cat gpurun_out/bench_default.json
bash tools/prof_bench.sh C3 5
cd tools && timeout -k 10 400 python shard_sim.py --one-rank --ranks 2 4 8 --steps 10 > ../gpurun_out/shard_sim.out 2>&1; grep one_rank ../gpurun_out/shard_sim.out
