set -e
for v in oldepi fast fast2 noepi oldepi fast fast2; do
  echo "$v $(EBT_KB_THR=inf EBERT_LIB=_abl/libebert_$v.so timeout -k 10 120 python tools/kernel_bench.py --one 2>/dev/null | grep kernel | cut -c60-200)"
done
for v in oldepi fast fast2; do
  echo "hits $v $(EBERT_LIB=_abl/libebert_$v.so timeout -k 10 120 python tools/kernel_bench.py --one 2>/dev/null | grep kernel | cut -c60-230)"
done
timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/t.log 2>&1
tail -2 gpurun_out/t.log
for v in oldepi fast2; do
EBERT_LIB=_abl/libebert_$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.log
python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$v', d['ms_per_step'], d['value'], d['stage_ms_per_step'])"
done
