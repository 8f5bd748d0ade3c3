# A/B of the filter GEMM: _abl/libebert_prev.so (the previous build) vs the tree's libebert.so,
# interleaved on one box: seg_bench hit curve + the C3 bench (no CPU baseline)
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
for v in prev new; do
  if [ $v = new ]; then L=$GRAFT_REPO_ROOT/robot_ebert_amd/libebert.so; else L=$GRAFT_REPO_ROOT/_abl/libebert_prev.so; fi
  echo "$v $(cd tools && EBERT_LIB=$L timeout -k 10 120 python seg_bench.py --n 524288 --hits 0,128,1024 --no-inf 2>/dev/null | python3 -c '
import sys,json
out=[]
for l in sys.stdin:
    d=json.loads(l)
    if "hits" in d: out.append("%s:%.4f" % (round(d["hits"]), d["ms"]))
print(" ".join(out))')"
  EBERT_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.log
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v C3', d['ms_per_step'], d['value'], d['roofline']['achieved'])"
done
done
