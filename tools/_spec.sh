set -e
for spec in 1 0; do
for n in 1000000 125000; do
  EBT_SPEC=$spec timeout -k 10 300 python bench.py --n $n --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sp_$spec_$n.json 2> gpurun_out/sp_$spec_$n.log
  python -c "import json;d=json.load(open('gpurun_out/sp_$spec_$n.json'));print('spec=$spec', '$n', d['ms_per_step'], d['value'], d['stage_ms_per_step'])"
done
done
