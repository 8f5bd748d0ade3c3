set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 500 python bench.py --config C5 --n 6250000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5r.json 2> gpurun_out/c5r.log
python -c "import json;d=json.load(open('gpurun_out/c5r.json'));print('C5r', d['ms_per_step'], d['value'], d['roofline']['frac'], d['plan'], d['stage_ms_per_step'])"
timeout -k 10 300 python bench.py --config C4 --n 1250000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c4r.json 2> gpurun_out/c4r.log
python -c "import json;d=json.load(open('gpurun_out/c4r.json'));print('C4r', d['ms_per_step'], d['value'], d['roofline']['frac'], d['stage_ms_per_step'])"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c3.json 2> gpurun_out/c3.log
python -c "import json;d=json.load(open('gpurun_out/c3.json'));print('C3', d['ms_per_step'], d['value'], d['roofline']['frac'], d['stage_ms_per_step'])"
