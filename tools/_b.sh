set -e
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c3.json 2> gpurun_out/c3.log || { tail -20 gpurun_out/c3.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3.json'));print('C3', d['ms_per_step'], d['value'], d['roofline'], d['stage_ms_per_step'])"
