set -e
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
cd tools
timeout -k 10 300 python seg_bench.py --n 524288 --hits 0,64,256,1024 2>&1 | grep -v amdgpu.ids | cut -c1-110
cd ..
for n in 1000000 125000; do
  timeout -k 10 300 python bench.py --n $n --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pp_$n.json 2> gpurun_out/pp_$n.log
  python -c "import json;d=json.load(open('gpurun_out/pp_$n.json'));print('$n', d['ms_per_step'], d['value'], d['stage_ms_per_step'])"
done
cd tools && timeout -k 10 300 python shard_sim.py --one-rank --ranks 8 --steps 10 --only cut 2>&1 | grep -v amdgpu.ids | tail -1
