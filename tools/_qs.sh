set -e
for b in 4096 2048 1024 512; do
  timeout -k 10 300 python bench.py --b $b --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/qs_$b.json 2> gpurun_out/qs_$b.log
  echo "$b $(python -c "import json;d=json.load(open('gpurun_out/qs_$b.json'));print(d['ms_per_step'], d['value'])")"
done
