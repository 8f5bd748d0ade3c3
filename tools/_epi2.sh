set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
cd tools
for n in 524288 131072; do
timeout -k 10 200 python seg_bench.py --n $n --hits 0,128,256,1024 2>&1 | grep -v amdgpu.ids | cut -c1-140
done
cd ..
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/e2_c3.json 2> gpurun_out/e2_c3.log
python -c "import json;d=json.load(open('gpurun_out/e2_c3.json'));print('C3', d['ms_per_step'], d['value'], d['roofline']['frac'], d['stage_ms_per_step'])"
cd tools && timeout -k 10 400 python shard_sim.py --one-rank --ranks 8 --steps 10 --only shared 2>&1 | grep -v amdgpu.ids
