# A/B of the whole C3 step: _abl/libebert_prev.so vs the tree's libebert.so, interleaved on one box
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2 3; do
for v in prev new; do
  if [ $v = new ]; then L=$GRAFT_REPO_ROOT/robot_ebert_amd/libebert.so; else L=$GRAFT_REPO_ROOT/_abl/libebert_prev.so; fi
  EBERT_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.log
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v C3', d['ms_per_step'], d['value'], d.get('stage_ms_per_step'))"
done
done
